# encoder numerics + forward timings after an epilogue change
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_encval}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or encoder or hf or gelu or fp8" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 --rounds 5 --iters 10 > $O/enc_minilm.json 2>&1 && tail -1 $O/enc_minilm.json &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base --rounds 5 --iters 10 > $O/enc_bge.json 2>&1 && tail -1 $O/enc_bge.json
echo done $?
