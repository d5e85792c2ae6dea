#!/bin/bash
# Round 6, run k: the forced-collective probe with every stream on its own hardware queue
# (GPU_MAX_HW_QUEUES=8; run i showed the probe's search stream and RCCL's stream sharing queue 4,
# which serialises them FIFO whatever the CUs allow), and the headline / simulate_world=8 step with
# 4 (the box default) vs 8 hardware queues.
set -o pipefail
O=gpurun_out/r6_k
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
GPU_MAX_HW_QUEUES=8 $T 300 rocprofv3 --kernel-trace --output-format csv -d $O/probe8 -o probe -- python3 benchmarks/rccl_coresident.py \
  --rows 50000000 --rounds 8 > $O/probe8.log 2>&1 || { tail -30 $O/probe8.log; exit 1; }
python3 benchmarks/rccl_overlap.py $(find $O/probe8 -name "*kernel_trace.csv") | tee $O/probe8_overlap.json
for r in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q $T 200 python bench.py > $O/bench_q${q}_$r.json 2> $O/bench_q${q}_$r.err || { tail -20 $O/bench_q${q}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_q${q}_$r.json'));print('hwq $q', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'])"
  done
done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q $T 300 python bench.py --opt simulate_world=8 > $O/sim8_q$q.json 2> $O/sim8_q$q.err || { tail -20 $O/sim8_q$q.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sim8_q$q.json'));print('sim8 hwq $q', d['value'], d['ms_per_step'])"
done
GPU_MAX_HW_QUEUES=8 $T 300 rocprofv3 --kernel-trace --output-format csv -d $O/sim8 -o sim8 -- python3 bench.py --steps 6 --warmup 2 --opt heldout_searches=0 --opt simulate_world=8 > $O/sim8_prof.log 2>&1 || { tail -30 $O/sim8_prof.log; exit 1; }
python3 benchmarks/rccl_overlap.py $(find $O/sim8 -name "*kernel_trace.csv") | tee $O/sim8_overlap.json
echo done
