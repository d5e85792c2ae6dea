#!/bin/bash
# Round 5: int8 stream scan cost split at 100M x 384 with no row emitting (thresholds + 1e6):
# the full hit test (abl 0), the max-then-one-scale test (abl 3), no test (abl 1); then the
# default bench on the VGPR-form build.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_abl
mkdir -p $O
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 --queries heldout --thr-add 1e6 \
  --ab 0:0:0:0,0:0:3:0,0:0:1:0 --rounds 3 > $O/scan.jsonl 2> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
cat $O/scan.jsonl
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
