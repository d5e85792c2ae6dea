#!/bin/bash
# End tree: the suite configs whose search runs the pruned pre-pass (index-100m = config #3,
# mpnet-full = the reference's 768-d deployment).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_suite2
mkdir -p $O
timeout -k 10 800 python -u benchmarks/suite.py --only index-100m,mpnet-full --out $O/suite_1gpu.jsonl > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
cut -c1-400 $O/suite_1gpu.jsonl
