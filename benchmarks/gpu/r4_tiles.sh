#!/bin/bash
# Round 4: MiniLM forward with the fused FFN block -- gemm tile modes for the remaining GEMMs
# (QKV, out-projection + LN), and the residual + LN tile height.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_tiles
mkdir -p $O
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --tiles 3,0,10 --rounds 5 > $O/enc_tiles.json 2> $O/enc_tiles.err || { tail $O/enc_tiles.err; exit 1; }
cat $O/enc_tiles.json
