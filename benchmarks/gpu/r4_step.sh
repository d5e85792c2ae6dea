#!/bin/bash
# Round 4: kernel trace of the final-tree headline step (gap between consecutive scans).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_step
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o h -- python bench.py --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python benchmarks/step_trace.py $O/prof/h_kernel_trace.csv > $O/step_trace.txt 2>&1; head -30 $O/step_trace.txt
python benchmarks/step_gap.py $O/prof/h_kernel_trace.csv --steps 8 > $O/step_gap.txt; head -20 $O/step_gap.txt
find $O/prof -name "*kernel_trace.csv" -size +8M -delete
