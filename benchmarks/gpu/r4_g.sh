#!/bin/bash
# Round 4: split-image A/B (sample 1/32 vs 1/64 tiles), the per-rank anisotropic shapes of
# N = 2 / 4 / 8, then the 768-d table and the mpnet deployment row (r4_e).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_g
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 500 $T -k "split or quant_rows or prune or pruned or index_scan_i8 or test_gemm or hipblaslt" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="python -u bench.py --mode search --queries heldout --verify --steps 20 --warmup 3"
for v in "i8 0" "i8 5" "none 0"; do set -- $v
  timeout -k 10 400 $B --corpus anisotropic --index-prune $1 --prune-sample-shift $2 > $O/aniso_256_$1_s$2.json 2> $O/aniso_256_$1_s$2.err || { tail -20 $O/aniso_256_$1_s$2.err; exit 1; }
  cat $O/aniso_256_$1_s$2.json
done
for shape in "50000000 512" "25000000 1024" "12500000 2048"; do set -- $shape
  for p in i8 none; do
    timeout -k 10 300 $B --corpus anisotropic --index-rows $1 --batch $2 --index-prune $p > $O/aniso_$2_$p.json 2> $O/aniso_$2_$p.err || { tail -20 $O/aniso_$2_$p.err; exit 1; }
    cat $O/aniso_$2_$p.json
  done
done
bash benchmarks/gpu/r4_e.sh
