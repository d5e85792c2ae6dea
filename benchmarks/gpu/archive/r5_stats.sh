#!/bin/bash
# The one-launch search statistics (prune_stats_kernel): the full GPU suite and smoke() on the
# end tree, config #3 (bench.py --mode search, statistics on) twice, and the driver's default bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_stats
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --mode search --steps 20 --warmup 3 > $O/search_$i.json 2> $O/search_$i.err || { tail -20 $O/search_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/search_$i.json').read()); print('search', d['value'], d['ms_per_step'], d.get('search_max_candidates'), d.get('search_dense_route_batches'))"
done
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read()); print('bench', d['value'], d['ms_per_step'], d['heldout_topk_qps'], d['heldout_ms_per_search'], d['verify_exact'])"
