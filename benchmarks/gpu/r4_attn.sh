#!/bin/bash
# Round 4: attention configs at the MiniLM headline shape (256 x 128 tokens, 12 heads of 32).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_attn
mkdir -p $O
timeout -k 10 300 python benchmarks/micro.py attn --head-dim 32 --seq 128 --batch 256 > $O/attn.json 2> $O/attn.err || { tail $O/attn.err; exit 1; }
cat $O/attn.json
