#!/bin/bash
# Same-box A/B of the reference's 768-d deployment (mpnet-multi embed + top-10 over 100M x 768):
# this tree vs the commit before the pre-pass rewrites (_ab_old, a git worktree), alternated.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_mpnet_ab
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model mpnet-multi > $O/new_$i.json 2> $O/new_$i.err || { tail -20 $O/new_$i.err; exit 1; }
  (cd _ab_old && timeout -k 10 300 python -u bench.py --model mpnet-multi) > $O/old_$i.json 2> $O/old_$i.err || { tail -20 $O/old_$i.err; exit 1; }
  python3 -c "import json; [print(t, $i, json.loads(open('$O/'+t+'_$i.json').read())['value'], json.loads(open('$O/'+t+'_$i.json').read())['heldout_topk_qps']) for t in ('new','old')]"
done
