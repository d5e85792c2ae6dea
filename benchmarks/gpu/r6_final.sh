#!/bin/bash
# Round 6, run final: validation of the end tree -- the GPU
# suite, smoke(), headline x2 with verify, MiniLM embed x2 and mpnet full.
set -o pipefail
O=gpurun_out/r6_final
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
$T 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  $T 200 python bench.py --verify > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$r.json'));print('headline', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'], d['heldout_ms_per_search'], 'exact', d.get('verify_exact'))"
done
for r in 1 2; do
  $T 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed_$r.json 2> $O/embed_$r.err || { tail -20 $O/embed_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/embed_$r.json'));print('minilm embed', d['value'], d['ms_per_step'])"
done
$T 300 python bench.py --model mpnet-multi > $O/mpnet.json 2> $O/mpnet.err || { tail -20 $O/mpnet.err; exit 1; }
python -c "import json;d=json.load(open('$O/mpnet.json'));print('mpnet full', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'], d['heldout_ms_per_search'])"
echo done
