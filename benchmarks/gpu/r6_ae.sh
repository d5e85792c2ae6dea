#!/bin/bash
# Round 6, run ae: the grouped tile order's band height (group_m) for the 256-row GEMM tiles on
# the bge / e5 shapes this repo's kernels run by default (FFN1 with the GELU epilogue) and the
# plain ones, interleaved in one process.
set -o pipefail
O=gpurun_out/r6_ae
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 400 python benchmarks/gemm_sweep.py --models bge-base,e5-large --variants t3g1,t3g2,t3g4,t3g8,t3g16,t3g32 \
  --rounds 3 --iters 10 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
