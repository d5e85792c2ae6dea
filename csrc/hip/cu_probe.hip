// Where a CU-mask bit lands (codename_symbiont_amd/parallel/cu_partition.py): every workgroup of
// a launch on a stream masked to ONE CU records the hardware ids of the CU it ran on -- HW_ID
// (cu / sh / se fields) and XCC_ID, read with s_getreg -- so the host can build a reserve that is
// balanced over XCDs and shader engines from the mapping the runtime actually uses.
#include "common.h"

namespace symb {

__global__ __launch_bounds__(64) void cu_probe_kernel(uint32_t* __restrict__ out) {
  if (threadIdx.x == 0) {
    // s_getreg_b32 immediates: id | offset << 6 | (size - 1) << 11 -- HW_REG_HW_ID (4) and
    // HW_REG_XCC_ID (20), all 32 bits
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}

}  // namespace symb

// out: 2 x n_blocks uint32 (HW_ID, XCC_ID per workgroup)
int symb_cu_probe(uint32_t* out, int n_blocks, hipStream_t st) {
  if (n_blocks <= 0) return -1;
  hipLaunchKernelGGL(symb::cu_probe_kernel, dim3(n_blocks), dim3(64), 0, st, out);
  return (int)hipGetLastError();
}
