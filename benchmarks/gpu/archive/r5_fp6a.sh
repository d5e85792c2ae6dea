#!/bin/bash
# Round 5: the MX-fp6 (e2m3) middle tier -- writer / scan / tier numerics, then the 100M x 384
# held-out scan on the int8 tier vs the fp6 tier, then the default bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_fp6a
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread \
  -k "quant_stream_images or append_rows or scan_stream or mx6 or mx4_tier" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 > $O/scan_i8.jsonl 2> $O/scan_i8.err || { tail -20 $O/scan_i8.err; exit 1; }
cat $O/scan_i8.jsonl
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier mx6 > $O/scan_mx6.jsonl 2> $O/scan_mx6.err || { tail -20 $O/scan_mx6.err; exit 1; }
cat $O/scan_mx6.jsonl
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
