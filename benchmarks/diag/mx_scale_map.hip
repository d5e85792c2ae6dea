// Diagnostic: which lane's E8M0 scale does v_mfma_scale_f32_16x16x128_f8f6f4 apply to which
// A bytes?  A = e4m3 1.0 only in lane group g's VGPR half h (bytes 16h..16h+15 of the lane's 32),
// B = 1.0 everywhere, scale_a(lane) = 127 + (lane >> 4) + 4 * (lane & 1).  C[row][0] then equals
// 16 * 2^(exponent the hardware applied to those bytes for that row).
//
// Result on MI355X (row 0; lane groups 0..3 carry exponents 0..3):
//   group 0 half 0 -> 16 (group 0's scale)   group 0 half 1 -> 64  (group 2's)
//   group 1 half 0 -> 16 (group 0's)         group 1 half 1 -> 64  (group 2's)
//   group 2 half 0 -> 32 (group 1's)         group 2 half 1 -> 128 (group 3's)
//   group 3 half 0 -> 32 (group 1's)         group 3 half 1 -> 128 (group 3's)
// i.e. lane group g, VGPR half h holds k = 64h + 16g .. +15, and lane group b's scale covers
// k block 32b .. 32b+31.  gemm.hip's fp8 fragment reads follow this order.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void k(float* out) {
  const int lane = threadIdx.x;
  for (int g = 0; g < 4; ++g)
    for (int h = 0; h < 2; ++h) {
      i32x8 a, b;
      for (int r = 0; r < 8; ++r) {
        const bool on = (lane >> 4) == g && (r >> 2) == h;
        a[r] = on ? 0x38383838 : 0;
        b[r] = 0x38383838;
      }
      f32x4 c = {0, 0, 0, 0};
      const int sa = 127 + (lane >> 4) + 4 * (lane & 1);
      c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, 127);
      // C/D: col = lane & 15, row = (lane >> 4) * 4 + reg
      if ((lane & 15) == 0)
        for (int r = 0; r < 4; ++r) out[(g * 2 + h) * 16 + (lane >> 4) * 4 + r] = c[r];
    }
}

int main() {
  float* d;
  (void)hipMalloc(&d, 8 * 16 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float o[128];
  (void)hipMemcpy(o, d, sizeof o, hipMemcpyDeviceToHost);
  for (int gh = 0; gh < 8; ++gh) {
    printf("A in lane group %d half %d: C[row 0..15][0] =", gh / 2, gh % 2);
    for (int r = 0; r < 16; ++r) printf(" %g", o[gh * 16 + r]);
    printf("\n");
  }
  return 0;
}
