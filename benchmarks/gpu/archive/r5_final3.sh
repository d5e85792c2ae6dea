#!/bin/bash
# Round 5 final validation on the round-5 end tree (pre-pass rewrites + select floor): the full GPU suite, smoke(), the driver's default
# bench (headline + held-out) and a rocprofv3 kernel-stats pass of the headline step.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o step -- python3 bench.py --steps 10 --warmup 3 --opt heldout_searches=0 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
python3 benchmarks/step_gap.py $(find $O/step -name "*kernel_trace.csv") > $O/step_gap.txt
python3 benchmarks/step_timeline.py $(find $O/step -name "*kernel_trace.csv") --steps 1 > $O/timeline.txt
head -3 $O/step_gap.txt
