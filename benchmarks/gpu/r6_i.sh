#!/bin/bash
# Round 6, run i: fp8 scan ring-depth variants (config #5, D = 1024) + the L2-source compute
# ceiling; the forced-collective RCCL co-residency probe; the headline with the reverted default.
set -o pipefail
O=gpurun_out/r6_i
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "fp8" > $O/t_fp8.log 2>&1 || { tail -40 $O/t_fp8.log; exit 1; }
tail -2 $O/t_fp8.log
$T 400 python benchmarks/micro.py scanfp8 --rows 100000000 --dim 1024 --rounds 3 --iters 5 \
  > $O/scanfp8.json 2> $O/scanfp8.err || { tail -20 $O/scanfp8.err; exit 1; }
cat $O/scanfp8.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fp8prof -o fp8 -- python3 benchmarks/micro.py scanfp8 \
  --rows 100000000 --dim 1024 --rounds 1 --iters 2 > $O/fp8prof.log 2>&1 || { tail -30 $O/fp8prof.log; exit 1; }
$T 300 rocprofv3 --kernel-trace --output-format csv -d $O/probe -o probe -- python3 benchmarks/rccl_coresident.py \
  --rows 50000000 --rounds 8 > $O/probe.log 2>&1 || { tail -30 $O/probe.log; exit 1; }
tail -1 $O/probe.log
python3 benchmarks/rccl_overlap.py $(find $O/probe -name "*kernel_trace.csv") | tee $O/probe_overlap.json
$T 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('headline', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'])"
echo done
