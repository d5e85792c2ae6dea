set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/tiles; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "encoder" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -1 $O/tests.log &&
for m in minilm-l6 bge-base e5-large; do timeout -k 10 300 python benchmarks/micro.py encoder --model $m --tiles 3,7 --rounds 7 > $O/enc_$m.json 2>&1 || exit 1; done
echo done $?
