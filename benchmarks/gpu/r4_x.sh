#!/bin/bash
# Round 4: the fused 384-wide FFN block (mlp_fused.hip) -- numerics, encoder A/B, kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_x2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mlp_fused or encoder" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --mlp 1,0 --rounds 5 > $O/enc_ab.json 2> $O/enc_ab.err || { tail $O/enc_ab.err; exit 1; }
cat $O/enc_ab.json
d=$O/prof_minilm_mlp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run -- python benchmarks/micro.py encoder --model minilm-l6 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
