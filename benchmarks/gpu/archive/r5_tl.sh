#!/bin/bash
# Round 5: headline step timeline (rocprofv3 kernel trace) -- the serial chain between scans.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_tl
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o step -- python3 bench.py --steps 10 --warmup 3 --opt heldout_searches=0 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
tail -1 $O/step.log | cut -c1-300
python3 benchmarks/step_timeline.py $(find $O/step -name "*kernel_trace.csv") --steps 2 > $O/timeline.txt
python3 benchmarks/step_gap.py $(find $O/step -name "*kernel_trace.csv") > $O/step_gap.txt
cat $O/timeline.txt | head -80
