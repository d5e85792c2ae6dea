#!/bin/bash
# Round 4: fused FFN v2 (2 k-tiles per phase-A stage) -- kernel trace and headline A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_z
mkdir -p $O
d=$O/prof_minilm_mlp1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run -- python benchmarks/micro.py encoder --model minilm-l6 --mlp 1 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
for r in 1 2; do for m in 1 0; do
  timeout -k 10 400 python -u bench.py --mlp-fused $m > $O/head_mlp${m}_r$r.json 2> $O/head_mlp${m}_r$r.err || { tail -20 $O/head_mlp${m}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/head_mlp${m}_r$r.json | paste - - | sed "s/^/mlp$m r$r /"
done; done
