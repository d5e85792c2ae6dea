#!/bin/bash
# Round 4: the BASELINE config suite re-run on the final tree (fused FFN block, small-M changes).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_suite2
mkdir -p $O
timeout -k 10 1000 python -u benchmarks/suite.py --out $O/suite_1gpu.jsonl > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
cat $O/suite_1gpu.jsonl
