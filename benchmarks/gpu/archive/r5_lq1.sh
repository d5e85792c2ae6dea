#!/bin/bash
# Round 5: the LDS-query int8 scan (csrc/hip/index_lq.hip, stream i8 variants 5/6/7): numerics,
# then 100M x 384 held-out A/B against the default stream scan in one process.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_lq1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "scan_stream_emits" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 --queries heldout --ab 0:0:0:0,0:5:0:0,0:6:0:0 --rounds 3 > $O/scan.jsonl 2> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 --queries heldout --thr-add 1e6 --ab 0:0:0:0,0:5:0:0,0:6:0:0,0:7:0:0,0:8:0:0 --rounds 3 >> $O/scan.jsonl 2>> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
cat $O/scan.jsonl
