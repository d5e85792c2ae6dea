#!/bin/bash
# Round 4: skinny GEMMs up to M = 256 by default and graph buckets that keep 256 tokens at 256;
# MX-fp4 128-row tiles A/B; then the scan PMC (r4_m) and the CU partition (r4_n).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_s
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -k "skinny or graph or encoder or mx4 or pruned or test_gemm" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in minilm-l6 bge-base; do for bs in "1 16" "4 32" "8 32" "16 16" "1 128"; do set -- $bs
  for g in "" "--graph"; do
    timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 $g >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  done
done; done
cat $O/lat.jsonl
for r in 1 2; do for t in 64 128; do
  timeout -k 10 400 python -u bench.py --steps 40 --warmup 5 --mx4-tile-rows $t > $O/head_t${t}_r$r.json 2> $O/head_t${t}_r$r.err || { tail -20 $O/head_t${t}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/head_t${t}_r$r.json | sed "s/^/head mx4 tile $t r$r /"
done; done
bash benchmarks/gpu/r4_m.sh && bash benchmarks/gpu/r4_n.sh
