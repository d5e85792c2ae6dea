#!/bin/bash
# Round 6, run c: the register-resident FFN block (mlp_reg_kernel) and the deferred-LN epilogue
# with coalesced statistics loads -- numerics, then same-box A/Bs (MiniLM FFN form 1 vs 2, wide
# encoders deferred vs hipBLASLt + add_ln), the headline, and a MiniLM embed kernel trace.
set -o pipefail
O=gpurun_out/r6_c
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "mlp or deferred or encoder_matches" > $O/t_new.log 2>&1 || { tail -40 $O/t_new.log; exit 1; }
tail -2 $O/t_new.log
for r in 1 2; do
  for f in 1 2; do
    SYMB_MLP_FORM=$f $T 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed_f${f}_$r.json \
      2> $O/embed_f${f}_$r.err || { tail -20 $O/embed_f${f}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/embed_f${f}_$r.json'));print('minilm form $f', d['value'], d['ms_per_step'])"
  done
done
for m in bge-base e5-large; do
  for d in 1 0; do
    SYMB_DEFERRED_LN=$d $T 150 python bench.py --mode embed --model $m --steps 30 --warmup 5 \
      > $O/embed_${m}_d$d.json 2> $O/embed_${m}_d$d.err || { tail -20 $O/embed_${m}_d$d.err; exit 1; }
    python -c "import json;d=json.load(open('$O/embed_${m}_d$d.json'));print('$m deferred=$d', d['value'], d['ms_per_step'])"
  done
done
$T 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('headline', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 200 rocprofv3 --kernel-trace --stats -d $O/prof_minilm -o minilm -- python bench.py --mode embed \
  --steps 10 --warmup 3 --opt graph=0 > $O/prof_minilm.out 2>&1 || { tail -20 $O/prof_minilm.out; exit 1; }
$T 200 rocprofv3 --kernel-trace --stats -d $O/prof_bge -o bge -- python bench.py --mode embed \
  --model bge-base --steps 10 --warmup 3 --opt graph=0 > $O/prof_bge.out 2>&1 || { tail -20 $O/prof_bge.out; exit 1; }
echo done
