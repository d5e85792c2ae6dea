# fixed-vs-per-k-tile cost: one shape family at K = 384 .. 3072 for the 8-phase, 2-stage and torch
set -o pipefail
O=gpurun_out/${1:-ksweep}; mkdir -p $O
for k in 384 768 1536 3072; do
  for v in "--tile 9" "--tile 2" "--torch"; do
    timeout -k 5 60 python benchmarks/gemm_one.py --n 2304 --k $k --iters 30 $v 2>/dev/null | tee -a $O/ksweep.jsonl || exit 1
  done
done
echo done
