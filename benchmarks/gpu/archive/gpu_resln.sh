# RES_LN tile 8 vs 16 waves (gpurun_out/resln/)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/resln; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "test_gemm and not fp8" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -1 $O/tests.log &&
timeout -k 10 300 python benchmarks/micro.py gemm > $O/gemm.json 2>&1
echo done $?
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --tiles 3,8 > gpurun_out/resln/enc_minilm.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base --tiles 3,8 > gpurun_out/resln/enc_bge.json 2>&1
echo done2 $?
