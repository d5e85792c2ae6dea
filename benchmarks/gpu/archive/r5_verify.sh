#!/bin/bash
# Round 5 (re-entry): the full GPU suite and the driver's default bench on the rebuilt tree.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_verify
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
