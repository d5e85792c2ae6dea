#!/bin/bash
# Round 5: the MX-fp4 tier's query-side centroid test -- numerics, the 100M x 384 fp4 scan with
# near-duplicate queries (the headline's kind) with / without it on both stream forms, and the
# default bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_scan5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread \
  -k "centroid or scan_stream or mx4_tier" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --rounds 3 --tier mx4 --queries near --ab 0:0:0:0:0,0:0:0:0:1,0:0:0:1:0,0:0:0:1:1 > $O/ab_mx4_near.jsonl 2> $O/ab_mx4_near.err || { tail -20 $O/ab_mx4_near.err; exit 1; }
cat $O/ab_mx4_near.jsonl
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
