#!/bin/bash
# Round 5: step timeline of the co-scheduling form (mx4 variant 5, two-GEMM FFN).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_cosched_tl
mkdir -p $O
SYMB_AB_MX4V=5 SYMB_AB_MLP=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/step -o step -- python3 bench.py --steps 8 --warmup 3 --opt heldout_searches=0 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
python3 benchmarks/step_timeline.py $(find $O/step -name "*kernel_trace.csv") --steps 1 > $O/timeline.txt
head -60 $O/timeline.txt
