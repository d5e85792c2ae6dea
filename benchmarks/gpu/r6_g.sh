#!/bin/bash
# Round 6, run g: the tree after the round-6 cleanup (stream-scan variants and the LDS-query scan
# removed, the LDS-ring int8 tier default at 768): GPU suite, headline x2 with verify, the
# reference's deployment (mpnet full), config #4 (bge embed) x2, and a headline step timeline.
set -o pipefail
O=gpurun_out/r6_g
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  $T 200 python bench.py --verify > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$r.json'));print('headline', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'], d['heldout_ms_per_search'], 'exact', d.get('verify_exact'))"
done
$T 300 python bench.py --model mpnet-multi > $O/mpnet.json 2> $O/mpnet.err || { tail -20 $O/mpnet.err; exit 1; }
python -c "import json;d=json.load(open('$O/mpnet.json'));print('mpnet full', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'], d['heldout_ms_per_search'])"
for r in 1 2; do
  $T 150 python bench.py --mode embed --model bge-base --steps 30 --warmup 5 > $O/bge_$r.json 2> $O/bge_$r.err || { tail -20 $O/bge_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bge_$r.json'));print('bge embed', d['value'], d['ms_per_step'])"
done
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o step -- python3 bench.py --steps 10 --warmup 3 --opt heldout_searches=0 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
python3 benchmarks/step_timeline.py $(find $O/step -name "*kernel_trace.csv") --steps 2 > $O/timeline.txt
head -70 $O/timeline.txt
