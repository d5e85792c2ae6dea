#!/bin/bash
# Round 4: the deep-ring GEMM (gemm_deep.hip) -- exactness, shape sweep vs the round-3 routes, and
# the bge-base / e5-large encoder forwards with every projection on our kernels.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_gemm
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm_deep or test_gemm" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u benchmarks/gemm_sweep.py --models bge-base,e5-large \
  --variants d5,d4,d5nosk,t10,lt,torch > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
for m in bge-base e5-large; do
  timeout -k 10 300 python -u benchmarks/micro.py encoder --model $m --tiles 3,10,12 > $O/enc_$m.json 2> $O/enc_$m.err || { tail -20 $O/enc_$m.err; exit 1; }
  cat $O/enc_$m.json
done
