#!/bin/bash
# Round 6, run d: 256 x 128 3-stage GEMM tiles (t20 / t21) vs the round-4 tiles (t3) vs hipBLASLt
# (lt) on bge / e5 shapes; the register-resident FFN after the barrier-drain fix.
set -o pipefail
O=gpurun_out/r6_d
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python benchmarks/gemm_sweep.py --models bge-base,e5-large --variants t3,t20,t21,lt \
  --rounds 3 --iters 10 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
for f in 1 2; do
  SYMB_MLP_FORM=$f $T 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed_f$f.json \
    2> $O/embed_f$f.err || { tail -20 $O/embed_f$f.err; exit 1; }
  python -c "import json;d=json.load(open('$O/embed_f$f.json'));print('minilm form $f', d['value'], d['ms_per_step'])"
done
