#!/bin/bash
# Round 5: stream-scan A/B in one process per tier (depth variants, the MX-fp4 128-query form,
# timing ablations: no emission test / no loads after the prologue), and the f8f6f4 operand
# layout probe (fp6 e2m3 / e3m2, fp4, fp8).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_scan3
mkdir -p $O
timeout -k 10 120 python -u benchmarks/diag/f6_layout.py > $O/f6_layout.jsonl 2> $O/f6_layout.err || { tail -20 $O/f6_layout.err; exit 1; }
cat $O/f6_layout.jsonl
timeout -k 10 400 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --rounds 3 --ab 0:0:0,0:2:0,0:3:0,0:0:1,0:0:2 > $O/ab_i8.jsonl 2> $O/ab_i8.err || { tail -20 $O/ab_i8.err; exit 1; }
cat $O/ab_i8.jsonl
timeout -k 10 400 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --rounds 3 --tier mx4 --queries self --ab 0:0:0,1:0:0,2:0:0,3:0:0,0:0:1,0:0:2 > $O/ab_mx4.jsonl 2> $O/ab_mx4.err || { tail -20 $O/ab_mx4.err; exit 1; }
cat $O/ab_mx4.jsonl
