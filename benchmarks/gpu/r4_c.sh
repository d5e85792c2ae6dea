#!/bin/bash
# Round 4: 256x192 big tile (whole waves for N = 768 / 2304), z-blocked skinny GEMM for
# 65..256-token query bursts, encoder A/B (bge / e5 / mpnet), headline bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_c
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T -k "test_gemm or skinny or encoder" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u benchmarks/gemm_sweep.py --models bge-base,e5-large \
  --variants t3,t10,lt > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
for m in bge-base e5-large mpnet-multi; do
  timeout -k 10 300 python -u benchmarks/micro.py encoder --model $m --tiles 3,12 > $O/enc_$m.json 2> $O/enc_$m.err || { tail -20 $O/enc_$m.err; exit 1; }
  cat $O/enc_$m.json
done
for m in minilm-l6 bge-base; do for bs in "1 128" "4 32" "8 32" "16 16"; do set -- $bs
  for sk in 256 64; do
    timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --skinny-max-m $sk >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  done
done; done
cat $O/lat.jsonl
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
