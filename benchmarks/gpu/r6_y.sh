#!/bin/bash
# Round 6, run y: the ping-pong main loop of the 256-row GEMM tiles -- exactness (oracle and
# bit-identity with the 2-stage loop), then the bge / e5 shapes: 2-stage (t3), ping-pong (p3),
# 256 x 256 ping-pong (p2), hipBLASLt (lt), interleaved in one process.
# (Ran against commit d5ba24c; gemm_pp_config and the p / q sweep variants were removed after it.)
set -o pipefail
O=gpurun_out/r6_y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "pingpong or test_gemm_deferred_ln or (test_gemm and not fp8 and not skinny)" > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
$T 300 python benchmarks/gemm_sweep.py --models bge-base,e5-large --variants t3,p3,q3,q2,lt \
  --rounds 3 --iters 10 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
