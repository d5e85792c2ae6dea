#!/bin/bash
# Round 4: small-M query path -- eager latency with the z-blocked skinny GEMM (max M 256) vs the
# tiled GEMMs above M = 64, graph replay vs eager, and kernel traces of one 8 x 32 forward each way.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "skinny or graph" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in minilm-l6 bge-base; do for bs in "1 16" "1 128" "4 32" "8 32" "16 16" "8 64"; do set -- $bs
  for sk in 256 64; do
    timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --skinny-max-m $sk >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  done
  timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --skinny-max-m 256 --graph >> $O/lat.jsonl 2>> $O/lat.err || exit 1
done; done
cat $O/lat.jsonl
for g in "" "--graph"; do
  d=$O/prof_minilm_8x32${g:+_graph}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python benchmarks/lat_trace.py --model minilm-l6 --b 8 --s 32 --skinny-max-m 256 --iters 50 $g > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
