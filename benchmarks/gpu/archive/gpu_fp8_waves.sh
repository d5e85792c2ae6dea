# fp8 GEMM 4 vs 8 waves (gpurun_out/fp8w/)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/fp8w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fp8 or mx" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -1 $O/tests.log &&
timeout -k 10 300 python benchmarks/micro.py gemmfp8 > $O/gemmfp8.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model e5-large --precision fp8 --fp8-waves 8,257 --rounds 7 > $O/enc_e5.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base --precision fp8 --fp8-waves 8,257 --rounds 7 > $O/enc_bge.json 2>&1
echo done $?
