#!/bin/bash
# Round 5: the headline sustained over 1000 steps (exactness checked at the end), and config #2
# (MiniLM embed) twice on the final tree.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_sustain
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 1000 --warmup 10 --verify > $O/sustained_1000.json 2> $O/sustained.err || { tail -20 $O/sustained.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/sustained_1000.json').read()); print('sustained', d['value'], d['ms_per_step'], d['search_mx4_tier_batches'], d['verify_exact'], d['heldout_topk_qps'])"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --mode embed > $O/embed_$r.json 2> $O/embed_$r.err || { tail -20 $O/embed_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/embed_$r.json').read()); print('embed', d['value'], d['ms_per_step'])"
done
# the held-out search's own timeline (config #3 shape): what runs besides the int8 scan
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ho -o ho -- python3 bench.py --mode search --steps 6 --warmup 2 > $O/ho.log 2>&1 || { tail -20 $O/ho.log; exit 1; }
python3 benchmarks/step_timeline.py $(find $O/ho -name "*kernel_trace.csv") --steps 1 > $O/ho_timeline.txt
head -40 $O/ho_timeline.txt
