#!/bin/bash
# Round 4: fused FFN block with the out-projection prologue (mode 2) -- numerics, encoder A/B,
# kernel trace, headline A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_x8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mlp_fused or encoder_matches" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --mlp 2,1,0 --rounds 5 > $O/enc_ab.json 2> $O/enc_ab.err || { tail $O/enc_ab.err; exit 1; }
cat $O/enc_ab.json
d=$O/prof_minilm_mlp2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run -- python benchmarks/micro.py encoder --model minilm-l6 --mlp 2 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
for r in 1 2; do for m in 2 1; do
  timeout -k 10 400 python -u bench.py --mlp-fused $m > $O/head_mlp${m}_r$r.json 2> $O/head_mlp${m}_r$r.err || { tail -20 $O/head_mlp${m}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/head_mlp${m}_r$r.json | sed "s/^/head mlp$m r$r /"
done; done
