#!/bin/bash
# A/B on one box: mx4_select with direct probe enumeration (this tree) vs the previous commit
# (_ab_old, a git worktree built the same way), the driver's default bench alternated 3x.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_m4s_ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "select or prune or pruned or mx4" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
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
