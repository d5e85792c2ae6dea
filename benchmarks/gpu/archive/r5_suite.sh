#!/bin/bash
# Round 5: the BASELINE config suite on the round-5 tree (config #5 at the 1B / 8 per-rank sizing:
# 125M x 1024 fp8 rows), plus the 100M x 768 held-out int8 scan (stream scan vs LDS-query form).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_suite
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "scan_stream_emits" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --dim 768 --iters 5 --tier i8 --queries heldout --ab 0:0:0:0,0:5:0:0 --rounds 3 > $O/scan768.jsonl 2> $O/scan768.err || { tail -20 $O/scan768.err; exit 1; }
cat $O/scan768.jsonl
timeout -k 10 1150 python -u benchmarks/suite.py --fp8-rows 125000000 --out $O/suite_1gpu.jsonl > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
cat $O/suite_1gpu.jsonl | cut -c1-400
