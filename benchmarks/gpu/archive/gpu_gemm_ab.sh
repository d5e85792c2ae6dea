# GEMM A/B on one MI355X: numerics first, then the micro-benchmarks (writes gpurun_out/gemm_ab/)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/gemm_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "test_gemm and not fp8" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 300 python benchmarks/micro.py gemm > $O/gemm.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --tiles 3,6,7 > $O/enc_minilm.json 2>&1
echo done $?
