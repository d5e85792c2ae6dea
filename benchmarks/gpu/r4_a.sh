#!/bin/bash
# Round 4, first box: the deep-ring GEMM (exactness, sweep vs the round-3 routes, encoder A/B)
# and the 768 / 1024-d search kernels (exactness).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_a
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 500 $T -k "gemm_deep or test_gemm" > $O/tests_gemm.log 2>&1 || { tail -40 $O/tests_gemm.log; exit 1; }
tail -2 $O/tests_gemm.log
timeout -k 10 500 $T -k "wide or 768 or quant_rows_i8 or prune_qprep or prefilter_shard or racing or mq_exact or pruned_search_is_exact" > $O/tests_index.log 2>&1 || { tail -40 $O/tests_index.log; exit 1; }
tail -2 $O/tests_index.log
timeout -k 10 300 python -u benchmarks/gemm_sweep.py --models bge-base,e5-large \
  --variants d5,d4,d5nosk,t10,lt,torch > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
for m in bge-base e5-large; do
  timeout -k 10 300 python -u benchmarks/micro.py encoder --model $m --tiles 3,10,12 > $O/enc_$m.json 2> $O/enc_$m.err || { tail -20 $O/enc_$m.err; exit 1; }
  cat $O/enc_$m.json
done
