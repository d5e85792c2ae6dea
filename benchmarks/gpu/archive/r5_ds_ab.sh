#!/bin/bash
# A/B on one box: dense_scores with resident query fragments (this tree) vs the previous commit
# (_ab_old, a git worktree built the same way), the driver's default bench alternated 3x.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_ds_ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "dense or select or prune or pruned" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py > $O/new_$i.json 2> $O/new_$i.err || { tail -30 $O/new_$i.err; exit 1; }
  (cd _ab_old && timeout -k 10 400 python -u bench.py) > $O/old_$i.json 2> $O/old_$i.err || { tail -30 $O/old_$i.err; exit 1; }
  python3 - $O $i <<'PY'
import json, sys
o, i = sys.argv[1], sys.argv[2]
for t in ("new", "old"):
    d = json.loads(open(f"{o}/{t}_{i}.json").read())
    print(t, i, d["value"], d["ms_per_step"], "heldout", d["heldout_topk_qps"], d["heldout_ms_per_search"], d["verify_exact"] if "verify_exact" in d else "")
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ho -o ho -- python3 bench.py --mode search --steps 6 --warmup 2 > $O/ho.log 2>&1 || { tail -20 $O/ho.log; exit 1; }
python3 benchmarks/step_timeline.py $(find $O/ho -name "*kernel_trace.csv") --steps 1 > $O/ho_timeline.txt
grep -E "dense_scores|topk_select|mx4_select|prune_route" $O/ho_timeline.txt
