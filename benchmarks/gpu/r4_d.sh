#!/bin/bash
# Round 4: the split int8 image (PCA basis, 64 fp16 + 320 int8 dims) for anisotropic corpora --
# kernel / search exactness tests, then the r3_real anisotropic rows pruned vs plain; then the
# r4_c GEMM / encoder / skinny / headline measurements.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_d
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 500 $T -k "split or quant_rows or prune or pruned or index_scan_i8 or wide" > $O/tests_split.log 2>&1 || { tail -40 $O/tests_split.log; exit 1; }
tail -2 $O/tests_split.log
B="python -u bench.py --mode search --queries heldout --verify --steps 20 --warmup 3"
for c in anisotropic random; do for p in i8 none; do
  timeout -k 10 400 $B --corpus $c --index-prune $p > $O/real_${c}_$p.json 2> $O/real_${c}_$p.err || { tail -20 $O/real_${c}_$p.err; exit 1; }
  cat $O/real_${c}_$p.json
done; done
timeout -k 10 400 $T -k "test_gemm or skinny or encoder" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u benchmarks/gemm_sweep.py --models bge-base,e5-large \
  --variants t3,t10,lt > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
for m in bge-base e5-large mpnet-multi; do
  timeout -k 10 300 python -u benchmarks/micro.py encoder --model $m --tiles 3,12 > $O/enc_$m.json 2> $O/enc_$m.err || { tail -20 $O/enc_$m.err; exit 1; }
  cat $O/enc_$m.json
done
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
