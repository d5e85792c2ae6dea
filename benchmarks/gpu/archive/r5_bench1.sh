#!/bin/bash
# Round 5: the driver's default bench (headline + held-out searches) and a rocprofv3 step trace
# of it (kernel stats + the per-step gap between scans).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_bench1
mkdir -p $O
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o step -- python3 bench.py --steps 10 --warmup 3 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
tail -2 $O/step.log
