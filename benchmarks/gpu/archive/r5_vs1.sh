#!/bin/bash
# Round 5: the VGPR-staged 4-wave GEMM (csrc/hip/gemm_vs.hip): oracle tests, then the encoder GEMM
# shapes at M = 32768 against this repo's tiles (t3) and the hipBLASLt route (lt), one process.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_vs1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "vgpr_staged" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u benchmarks/gemm_sweep.py --models bge-base,e5-large --variants vs,t3,lt --rounds 3 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 200 python -u bench.py --mode embed > $O/embed.json 2> $O/embed.err || { tail -20 $O/embed.err; exit 1; }
cut -c1-300 $O/embed.json
