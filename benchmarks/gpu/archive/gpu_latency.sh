set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/lat; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "gemm or encoder" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -1 $O/tests.log &&
timeout -k 10 300 python benchmarks/micro.py latency > $O/latency.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --rounds 7 > $O/enc_minilm.json 2>&1
echo done $?
