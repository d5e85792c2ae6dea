#!/bin/bash
# Round 6, run f: the fused FFN block's ring filled by register staging (SYMB_MLP_VS=1) vs LDS-DMA:
# numerics, then MiniLM embed and the headline, alternated.
set -o pipefail
O=gpurun_out/r6_f
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "mlp or encoder_matches" > $O/t_new.log 2>&1 || { tail -40 $O/t_new.log; exit 1; }
tail -2 $O/t_new.log
for r in 1 2; do
  for v in 0 1; do
    SYMB_MLP_VS=$v $T 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed_vs${v}_$r.json \
      2> $O/embed_vs${v}_$r.err || { tail -20 $O/embed_vs${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/embed_vs${v}_$r.json'));print('minilm vs=$v', d['value'], d['ms_per_step'])"
  done
done
for v in 0 1; do
  SYMB_MLP_VS=$v $T 200 python bench.py > $O/bench_vs$v.json 2> $O/bench_vs$v.err || { tail -20 $O/bench_vs$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_vs$v.json'));print('headline vs=$v', d['value'], d['ms_per_step'], 'heldout', d['heldout_topk_qps'])"
done
