#!/bin/bash
# Round 6, run e: GPU suite on the current tree; then the 768-d int8-tier A/B on one box:
# the LDS-query stream form (default) vs the round-4 LDS-ring scan beside the stream fp4 tier
# (SYMB_PRUNE_I8=ring), in the reference's deployment (mpnet-multi embed + top-10 over 100M x 768,
# with the held-out search rate), alternated twice.
set -o pipefail
O=gpurun_out/r6_e
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for k in stream ring; do
    SYMB_PRUNE_I8=$k $T 300 python bench.py --model mpnet-multi --steps 20 --warmup 5 \
      > $O/mpnet_${k}_$r.json 2> $O/mpnet_${k}_$r.err || { tail -20 $O/mpnet_${k}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/mpnet_${k}_$r.json'));print('$k', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'], d['heldout_ms_per_search'], d['config']['index_scan'])"
  done
done
