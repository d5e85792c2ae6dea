#!/bin/bash
# Round 6, run q: the BASELINE config suite on the round-6 tree (config #5 at the 1B / 8 per-rank
# sizing: 125M x 1024 fp8 rows).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6_q
mkdir -p $O
timeout -k 10 1150 python -u benchmarks/suite.py --fp8-rows 125000000 --out $O/suite_1gpu.jsonl > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
cut -c1-300 $O/suite_1gpu.jsonl
