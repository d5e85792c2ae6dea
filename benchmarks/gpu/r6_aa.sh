#!/bin/bash
# Round 6, run aa: the headline with the encoder stream at high priority (its workgroups take CUs
# as the scan's retire) against the default, interleaved, with verify.
# (The enc_priority option was removed after this run: profiles/r6_step/README.md.)
set -o pipefail
O=gpurun_out/r6_aa
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
for r in 1 2 3; do
  for p in 0 -1; do
    $T 200 python bench.py --verify --opt enc_priority=$p > $O/bench_p${p}_$r.json 2> $O/bench_p${p}_$r.err || { tail -20 $O/bench_p${p}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_p${p}_$r.json'));print('enc_priority $p', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'], 'exact', d.get('verify_exact'))"
  done
done
echo done
