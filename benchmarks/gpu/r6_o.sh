#!/bin/bash
# Round 6, run o: headline with the compute / pre-pass streams at high priority (--opt
# stream_prio=0|1|2, interleaved), then a kernel trace of the default step (scan_after_encode=0).
set -o pipefail
O=gpurun_out/r6_o
mkdir -p $O
T="timeout -k 10"
for r in 1 2; do
  for p in 0 1 2; do
    $T 200 python bench.py --opt stream_prio=$p > $O/bench_p${p}_$r.json 2> $O/bench_p${p}_$r.err || { tail -20 $O/bench_p${p}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_p${p}_$r.json'));print('prio $p', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --output-format csv -d $O/step -o step -- python3 bench.py --steps 10 --warmup 3 --opt heldout_searches=0 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
python3 benchmarks/step_timeline.py $(find $O/step -name "*kernel_trace.csv") --steps 2 > $O/timeline.txt
head -70 $O/timeline.txt
echo done
