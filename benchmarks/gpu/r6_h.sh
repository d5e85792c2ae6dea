#!/bin/bash
# Round 6, run h: the headline with batch i's scan ordered after batch i + 1's encoder
# (--opt scan_after_encode, default 1) vs the round-5 order, alternated; its step timeline; the
# simulated 8-GPU per-rank step (both orders) and whether the RCCL kernels co-reside with the scan.
set -o pipefail
O=gpurun_out/r6_h
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
for r in 1 2 3; do
  for v in 1 0; do
    $T 200 python bench.py --opt scan_after_encode=$v > $O/bench_sae${v}_$r.json 2> $O/bench_sae${v}_$r.err || { tail -20 $O/bench_sae${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_sae${v}_$r.json'));print('scan_after_encode=$v', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'])"
  done
done
for v in 1 0; do
  $T 300 python bench.py --opt simulate_world=8 --opt scan_after_encode=$v > $O/sim8_sae$v.json 2> $O/sim8_sae$v.err || { tail -20 $O/sim8_sae$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sim8_sae$v.json'));print('sim8 scan_after_encode=$v', d['value'], d['ms_per_step'])"
done
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o step -- python3 bench.py --steps 10 --warmup 3 --opt heldout_searches=0 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
python3 benchmarks/step_timeline.py $(find $O/step -name "*kernel_trace.csv") --steps 2 > $O/timeline.txt
head -60 $O/timeline.txt
$T 300 rocprofv3 --kernel-trace --output-format csv -d $O/sim8 -o sim8 -- python3 bench.py --steps 6 --warmup 2 --opt heldout_searches=0 --opt simulate_world=8 > $O/sim8_prof.log 2>&1 || { tail -30 $O/sim8_prof.log; exit 1; }
python3 benchmarks/rccl_overlap.py $(find $O/sim8 -name "*kernel_trace.csv") | tee $O/rccl_overlap.json
