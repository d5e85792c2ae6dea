set -o pipefail
mkdir -p gpurun_out/s4
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s4/gpu_tests.log 2>&1 && tail -3 gpurun_out/s4/gpu_tests.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4/smoke.log 2>&1 && tail -1 gpurun_out/s4/smoke.log &&
timeout -k 10 400 python bench.py > gpurun_out/s4/bench.json 2> gpurun_out/s4/bench.err && cat gpurun_out/s4/bench.json &&
timeout -k 10 300 python benchmarks/micro.py gemm > gpurun_out/s4/gemm.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py gemmfp8 > gpurun_out/s4/gemmfp8.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base > gpurun_out/s4/enc_bge.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model e5-large --precision bf16,fp8 > gpurun_out/s4/enc_e5.json 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s4/prof_e5 -o e5 -- python benchmarks/micro.py encoder --model e5-large --precision bf16,fp8 --rounds 2 --iters 3 > gpurun_out/s4/prof_e5.log 2>&1
echo done $?
