#!/bin/bash
# Round 6, run w: the headline's threshold-sample density under the MX-fp4 tier (2^7 default vs
# 2^8 / 2^9), interleaved, with verify.
set -o pipefail
O=gpurun_out/r6_w
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
for r in 1 2; do
  for s in 7 8 9; do
    $T 200 python bench.py --verify --opt prune_shift_mx4=$s > $O/bench_s${s}_$r.json 2> $O/bench_s${s}_$r.err || { tail -20 $O/bench_s${s}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_s${s}_$r.json'));print('shift $s', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'], 'exact', d.get('verify_exact'), 'mx4', d.get('search_mx4_tier_batches'))"
  done
done
echo done
