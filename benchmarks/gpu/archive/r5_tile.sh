#!/bin/bash
# Round 5: int8 stream image with one scale per sub-tile -- the full GPU suite, the 100M x 384
# int8 scan (held-out thresholds and no-emission), the default bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_tile
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 --queries heldout --ab 0:0:0:0 --rounds 3 > $O/scan.jsonl 2> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 --queries heldout --thr-add 1e6 --ab 0:0:0:0,0:0:1:0 --rounds 3 >> $O/scan.jsonl 2>> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
cat $O/scan.jsonl
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
