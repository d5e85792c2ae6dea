#!/bin/bash
# Round 6, run x: the end tree's headline sustained over 1000 steps (verify), and a kernel trace of
# the step with the fused QKV + attention kernel.
set -o pipefail
O=gpurun_out/r6_x
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 400 python bench.py --steps 1000 --warmup 10 --verify > $O/sustained_1000.json 2> $O/sustained.err || { tail -20 $O/sustained.err; exit 1; }
python -c "import json;d=json.load(open('$O/sustained_1000.json'));print('sustained', d['value'], d['ms_per_step'], 'exact', d.get('verify_exact'), 'heldout', d['heldout_topk_qps'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --output-format csv -d $O/step -o step -- python3 bench.py --steps 10 --warmup 3 --opt heldout_searches=0 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
python3 benchmarks/step_timeline.py $(find $O/step -name "*kernel_trace.csv") --steps 2 > $O/timeline.txt
head -3 $O/timeline.txt
echo done
