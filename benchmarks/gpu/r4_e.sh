#!/bin/bash
# Round 4: 100M x 768 held-out search (pruned vs plain top-10, top-100), the reference's default
# deployment (mpnet-multi --mode full), and the per-rank anisotropic shapes of N = 2 / 4 / 8.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_e
mkdir -p $O
B="python -u bench.py --mode search --queries heldout --verify --steps 20 --warmup 3"
for p in i8 none; do
  timeout -k 10 500 $B --model mpnet-multi --index-prune $p > $O/s768_k10_$p.json 2> $O/s768_k10_$p.err || { tail -20 $O/s768_k10_$p.err; exit 1; }
  cat $O/s768_k10_$p.json
done
timeout -k 10 500 $B --model mpnet-multi --k 100 > $O/s768_k100.json 2> $O/s768_k100.err || { tail -20 $O/s768_k100.err; exit 1; }
cat $O/s768_k100.json
timeout -k 10 500 python -u bench.py --model mpnet-multi --mode full --steps 20 --warmup 5 > $O/mpnet_full.json 2> $O/mpnet_full.err || { tail -20 $O/mpnet_full.err; exit 1; }
cat $O/mpnet_full.json
