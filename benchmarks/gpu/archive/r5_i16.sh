#!/bin/bash
# Round 5: the int8 stream scan on the 16 x 16 x 64 MFMA shape (i8 variant 4) vs 32 x 32 x 32.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_i16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread -k "scan_stream_emits" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 --queries heldout --ab 0:0:0:0,0:4:0:0 --rounds 3 > $O/scan.jsonl 2> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 --queries heldout --thr-add 1e6 --ab 0:0:0:0,0:4:0:0 --rounds 3 >> $O/scan.jsonl 2>> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
cat $O/scan.jsonl
