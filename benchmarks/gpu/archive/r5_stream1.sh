#!/bin/bash
# Round 5: first GPU run of the stream scan (csrc/hip/index_stream.hip) and the glue-free pre-pass
# (csrc/hip/prepass.hip): their numerics tests and the pruned-search exactness tests, then the old
# (SYMB_PRUNE_STREAM=0) vs new first-pass scan at 100M x 384 (held-out int8 tier, self-query
# MX-fp4 tier), then the default bench (held-out searches included) on the new path.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_stream1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "quant_stream or scan_stream or test_extension or dense_scores or append_rows or prune or mx4" > $O/tests_stream.log 2>&1 || { tail -40 $O/tests_stream.log; exit 1; }
tail -8 $O/tests_stream.log
for v in 0 1; do
  SYMB_PRUNE_STREAM=$v timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 > $O/scan_i8_s$v.json 2> $O/scan_i8_s$v.err || { tail -20 $O/scan_i8_s$v.err; exit 1; }
  cat $O/scan_i8_s$v.json
  SYMB_PRUNE_STREAM=$v timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 --tier mx4 --queries self > $O/scan_mx4_s$v.json 2> $O/scan_mx4_s$v.err || { tail -20 $O/scan_mx4_s$v.err; exit 1; }
  cat $O/scan_mx4_s$v.json
done
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 --tier mx4 --queries self --variant 1 > $O/scan_mx4_v1.json 2> $O/scan_mx4_v1.err || { tail -20 $O/scan_mx4_v1.err; exit 1; }
cat $O/scan_mx4_v1.json
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
