#!/bin/bash
# Round 6, run ad: last check of the committed tree -- the GPU suite and smoke().
set -o pipefail
O=gpurun_out/r6_ad
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
$T 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
$T 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('headline', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'])"
