#!/bin/bash
# Round 4: the 8-wave single-split skinny GEMM + residual/LayerNorm in the split-sum kernel at
# H >= 768 -- tests, then bge / MiniLM / e5 query-path latency and a bge 8 x 32 kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_u2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "skinny or graph or encoder" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in bge-base minilm-l6 e5-large; do for bs in "8 32" "4 32" "1 128" "1 16"; do set -- $bs
  timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --graph >> $O/lat.jsonl 2>> $O/lat.err || exit 1
done; done
cat $O/lat.jsonl
d=$O/prof_bge_8x32
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python benchmarks/lat_trace.py --model bge-base --b 8 --s 32 --iters 50 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
