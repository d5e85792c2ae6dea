# GEMM A/B on one MI355X: numerics first, then the micro-benchmarks (writes gpurun_out/gemm_ab/)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/gemm_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "gemm or encoder" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 300 python benchmarks/micro.py gemm > $O/gemm.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py gemmfp8 > $O/gemmfp8.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base --tiles 0,2,3 > $O/enc_bge.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --tiles 0,3 > $O/enc_minilm.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model e5-large --precision bf16,fp8 --tiles 0,3 > $O/enc_e5.json 2>&1
echo done $?
