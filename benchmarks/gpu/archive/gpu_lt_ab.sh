# hipBLASLt route for the plain projections: numerics, encoder A/B (tile 3 vs 12), kernel stats
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_lt}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "hipblaslt or test_gemm" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
for m in bge-base e5-large minilm-l6; do
  timeout -k 10 300 python benchmarks/micro.py encoder --model $m --tiles 3,12 --rounds 5 --iters 10 > $O/enc_$m.json 2>&1 && tail -1 $O/enc_$m.json || exit 1
done
echo done
