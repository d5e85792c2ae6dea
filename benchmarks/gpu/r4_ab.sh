#!/bin/bash
# Round 4: fused FFN block on / off -- headline (3 interleaved rounds) and embed-only mode.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_ab
mkdir -p $O
for r in 1 2 3; do for m in 1 0; do
  timeout -k 10 400 python -u bench.py --mlp-fused $m > $O/head_mlp${m}_r$r.json 2> $O/head_mlp${m}_r$r.err || { tail -20 $O/head_mlp${m}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/head_mlp${m}_r$r.json | sed "s/^/head mlp$m r$r /"
done; done
for r in 1 2; do for m in 1 0; do
  timeout -k 10 300 python -u bench.py --mode embed --mlp-fused $m > $O/embed_mlp${m}_r$r.json 2> $O/embed_mlp${m}_r$r.err || { tail -20 $O/embed_mlp${m}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/embed_mlp${m}_r$r.json | sed "s/^/embed mlp$m r$r /"
done; done
