#!/bin/bash
# Round 4: 8-wave small-M workgroups for multi-split K too (gemm_skinny_nw8 8 / 16 / 32) -- tests,
# then query-path latency A/B and a trace of the bge 8 x 32 forward at the best setting.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_v
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "skinny" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do for m in bge-base minilm-l6 e5-large; do for bs in "8 32" "1 16"; do set -- $bs
  for kg in 8 16 32; do
    timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --nw8-max-kg $kg >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  done
done; done; done
cat $O/lat.jsonl
d=$O/prof_bge_8x32_kg32
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python benchmarks/lat_trace.py --model bge-base --b 8 --s 32 --iters 50 --nw8-max-kg 32 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
