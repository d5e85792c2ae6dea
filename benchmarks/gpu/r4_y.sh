#!/bin/bash
# Round 4: the headline step with the fused FFN block on / off (same box, interleaved).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_y
mkdir -p $O
for r in 1 2; do for m in 1 0; do
  timeout -k 10 400 python -u bench.py --mlp-fused $m > $O/head_mlp${m}_r$r.json 2> $O/head_mlp${m}_r$r.err || { tail -20 $O/head_mlp${m}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/head_mlp${m}_r$r.json | paste - - | sed "s/^/mlp$m r$r /"
done; done
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --mlp 1,0 --rounds 5 > $O/enc_ab.json 2> $O/enc_ab.err || { tail $O/enc_ab.err; exit 1; }
cat $O/enc_ab.json
