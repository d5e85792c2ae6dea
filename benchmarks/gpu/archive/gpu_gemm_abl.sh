# gemm256 ablation: full / no stores / no epilogue at K = 384, 768, 3072
set -o pipefail
O=gpurun_out/${1:-gabl}; mkdir -p $O
for k in 384 768 3072; do
  for abl in 0 1 2; do
    timeout -k 5 60 python benchmarks/gemm_one.py --n 2304 --k $k --iters 30 --tile 9 --abl $abl 2>/dev/null | tee -a $O/abl.jsonl || exit 1
  done
done
echo done
