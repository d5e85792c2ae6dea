#!/bin/bash
# Round 5: the ping-pong GEMM (csrc/hip/gemm_pp.hip) -- numerics, then the encoder-shape sweep
# against hipBLASLt and the round-4 tiles; the MX-fp4 768 diagnosis; the stream vs LDS-ring scan.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_pp1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "pingpong" > $O/tests_pp.log 2>&1 || { tail -40 $O/tests_pp.log; exit 1; }
tail -4 $O/tests_pp.log
timeout -k 10 400 python -u benchmarks/gemm_sweep.py --variants pp,pp256,pp128,t3,lt --rounds 5 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 300 python -u benchmarks/diag/mx4_768.py > $O/mx4_768.txt 2>&1 || { tail -30 $O/mx4_768.txt; exit 1; }
cat $O/mx4_768.txt
for v in 0 1; do
  SYMB_PRUNE_STREAM=$v timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 > $O/scan_i8_s$v.json 2> $O/scan_i8_s$v.err || { tail -20 $O/scan_i8_s$v.err; exit 1; }
  cat $O/scan_i8_s$v.json
  SYMB_PRUNE_STREAM=$v timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 --tier mx4 --queries self > $O/scan_mx4_s$v.json 2> $O/scan_mx4_s$v.err || { tail -20 $O/scan_mx4_s$v.err; exit 1; }
  cat $O/scan_mx4_s$v.json
done
