#!/bin/bash
# Round 4: deep-ring GEMM v2 (buffer-descriptor DMA, 2x unrolled loop, write-through split-K
# hand-off) vs the round-3 tiles, plus a PMC pass per kernel on the e5 FFN2 / bge out shapes.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_b
mkdir -p $O
timeout -k 10 200 python -u benchmarks/diag/deep_debug.py > $O/diag.txt 2>&1; cat $O/diag.txt
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm_deep" > $O/tests_gemm.log 2>&1 || { tail -40 $O/tests_gemm.log; exit 1; }
tail -2 $O/tests_gemm.log
timeout -k 10 300 python -u benchmarks/gemm_sweep.py --models bge-base,e5-large \
  --variants d4,d5,d4nosk,t10,lt > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
run() {  # tag, args
  local tag=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc $SQ --output-format csv -d $O/$tag.sq -o p -- python3 benchmarks/gemm_one.py --iters 5 "$@" > $O/$tag.sq.log 2>&1 &&
  timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/$tag.grbm -o p -- python3 benchmarks/gemm_one.py --iters 5 "$@" > $O/$tag.grbm.log 2>&1
}
run ffn2e5_d4 --n 1024 --k 4096 --epi 0 --tile 3 --ns 4 --sk 0 &&
run ffn2e5_t10 --n 1024 --k 4096 --epi 0 --tile 10 &&
run ffn2e5_lt --n 1024 --k 4096 --epi 0 --torch &&
for t in ffn2e5_d4 ffn2e5_t10 ffn2e5_lt; do
  python benchmarks/pmc_kernel.py $(find $O/$t.sq $O/$t.grbm -name "*counter_collection.csv") --match "gemm|Cijk" > $O/$t.pmc.txt 2>&1; echo "== $t"; cat $O/$t.pmc.txt
done
