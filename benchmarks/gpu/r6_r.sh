#!/bin/bash
# Round 6, run r: the QKV projection fused into the attention (attention.hip qkv_attn_kernel):
# numerics, then same-box A/Bs (SYMB_QKV_ATTN=1 fused vs 0 the GEMM + attention pair) of the
# MiniLM embed step and the headline, and a kernel trace of the fused embed step.
set -o pipefail
O=gpurun_out/r6_r
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "qkv_attention or encoder or attention" > $O/t_new.log 2>&1 || { tail -40 $O/t_new.log; exit 1; }
tail -2 $O/t_new.log
for r in 1 2; do
  for f in 1 0; do
    SYMB_QKV_ATTN=$f $T 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed_f${f}_$r.json 2> $O/embed_f${f}_$r.err || { tail -20 $O/embed_f${f}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/embed_f${f}_$r.json'));print('embed fused=$f', d['value'], d['ms_per_step'])"
  done
done
for r in 1 2; do
  for f in 1 0; do
    SYMB_QKV_ATTN=$f $T 200 python bench.py > $O/bench_f${f}_$r.json 2> $O/bench_f${f}_$r.err || { tail -20 $O/bench_f${f}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_f${f}_$r.json'));print('headline fused=$f', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 200 rocprofv3 --kernel-trace --stats -d $O/prof -o embed -- python3 bench.py --mode embed \
  --steps 10 --warmup 3 --opt graph=0 > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -12 | cut -c1-160
echo done
