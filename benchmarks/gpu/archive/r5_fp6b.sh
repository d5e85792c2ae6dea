#!/bin/bash
# Round 5: MX-fp6 tier numerics and the fp6 vs fp4 vs int8 stream-scan kernels at 100M x 384.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_fp6b
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread \
  -k "quant_stream_images or append_rows or scan_stream or mx6 or mx4_tier" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for t in "i8 heldout" "mx6 near" "mx4 near"; do set -- $t
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier $1 --queries $2 --ab 0:0:0:0:0 --rounds 3 >> $O/scan.jsonl 2> $O/scan_$1.err || { tail -20 $O/scan_$1.err; exit 1; }
done
cat $O/scan.jsonl
