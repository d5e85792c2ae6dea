# gemm4w (persistent 4-wave 256x256 GEMM): numerics, then the per-shape sweep against the other routes.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_gemm4w}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "test_gemm4w" > $O/tests.log 2>&1 &&
timeout -k 10 500 python benchmarks/gemm_sweep.py --models bge-base,e5-large --variants ${VARIANTS:-t3,w4,w4_192,lt,torch} > $O/sweep.jsonl 2> $O/sweep.err
rc=$?; tail -3 $O/tests.log; echo done $rc
