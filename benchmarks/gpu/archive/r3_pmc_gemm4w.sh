# PMC passes (SQ, TCC, GRBM each in its own run) for the FFN2 / QKV shapes: gemm4w vs the 8-wave tile vs hipBLASLt.
set -o pipefail
O=gpurun_out/${1:-r3_pmc_gemm4w}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
TCC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
run() {  # tag, args
  local tag=$1; shift
  timeout -k 5 60 python benchmarks/gemm_one.py --iters 20 "$@" > $O/$tag.time.json 2>&1 &&
  timeout -s KILL 60 rocprofv3 --pmc $SQ --output-format csv -d $O/$tag.sq -o p -- python3 benchmarks/gemm_one.py --iters 5 "$@" > $O/$tag.sq.log 2>&1 &&
  timeout -s KILL 60 rocprofv3 --pmc $TCC --output-format csv -d $O/$tag.tcc -o p -- python3 benchmarks/gemm_one.py --iters 5 "$@" > $O/$tag.tcc.log 2>&1 &&
  timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/$tag.grbm -o p -- python3 benchmarks/gemm_one.py --iters 5 "$@" > $O/$tag.grbm.log 2>&1
}
run ffn2_w4 --n 768 --k 3072 --epi 0 --w4 256 &&
run ffn2_t3 --n 768 --k 3072 --epi 0 --tile 3 &&
run ffn2_lt --n 768 --k 3072 --epi 0 --torch &&
run qkv_w4 --n 2304 --k 768 --epi 0 --w4 256 &&
run qkv_lt --n 2304 --k 768 --epi 0 --torch
echo done $?
