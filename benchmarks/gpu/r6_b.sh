#!/bin/bash
# Round 6, run b: deferred-LayerNorm numerics, the whole GPU suite, the headline, the embed-only
# mode (3 runs), and a same-box A/B of the wide encoders: deferred LN (this repo's GEMMs only) vs
# SYMB_DEFERRED_LN=0 (hipBLASLt plain projections + add_ln), plus a kernel trace of bge's embed.
set -o pipefail
O=gpurun_out/r6_b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "deferred or partial_subtile" > $O/t_new.log 2>&1 || { tail -40 $O/t_new.log; exit 1; }
tail -2 $O/t_new.log
$T 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
$T 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for i in 1 2 3; do
  $T 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed$i.json 2> $O/embed$i.err \
    || { tail -20 $O/embed$i.err; exit 1; }
  cat $O/embed$i.json
done
for m in bge-base mpnet-multi e5-large; do
  for d in 1 0; do
    SYMB_DEFERRED_LN=$d $T 150 python bench.py --mode embed --model $m --steps 30 --warmup 5 \
      > $O/embed_${m}_d$d.json 2> $O/embed_${m}_d$d.err || { tail -20 $O/embed_${m}_d$d.err; exit 1; }
    echo "$m deferred=$d"; python -c "import json,sys;d=json.load(open('$O/embed_${m}_d$d.json'));print(d['value'],d['ms_per_step'],d['embed_ms_per_step_rank0'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 200 rocprofv3 --kernel-trace --stats -d $O/prof_bge -o bge -- python bench.py --mode embed \
  --model bge-base --steps 10 --warmup 3 --opt graph=0 > $O/prof_bge.out 2>&1 || { tail -20 $O/prof_bge.out; exit 1; }
find $O/prof_bge -name "*kernel_stats.csv" | head -3
