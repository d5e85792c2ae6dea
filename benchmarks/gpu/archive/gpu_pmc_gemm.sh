# PMC counters of one GEMM configuration per pass (SQ block, then GRBM clock); see gemm_one.py
set -o pipefail
O=gpurun_out/${1:-pmc_gemm}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
run() {  # tag, args
  local tag=$1; shift
  timeout -k 5 60 python benchmarks/gemm_one.py --iters 20 "$@" > $O/$tag.time.json 2>&1 &&
  timeout -s KILL 60 rocprofv3 --pmc $SQ --output-format csv -d $O/$tag.sq -o p -- python3 benchmarks/gemm_one.py --iters 5 "$@" > $O/$tag.sq.log 2>&1 &&
  timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/$tag.grbm -o p -- python3 benchmarks/gemm_one.py --iters 5 "$@" > $O/$tag.grbm.log 2>&1
}
run qkv9 --n 2304 --k 768 --epi 0 --tile 9 &&
run qkv2 --n 2304 --k 768 --epi 0 --tile 2 &&
run ffn2_9 --n 768 --k 3072 --epi 0 --tile 9 &&
run ffn1_9 --n 3072 --k 768 --epi 1 --tile 9
echo done $?
