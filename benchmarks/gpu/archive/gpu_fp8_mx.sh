# fp8 MX hand-off A/B on one MI355X: numerics first, then micro-benchmarks (gpurun_out/fp8_mx/)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/fp8_mx; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fp8 or gemm or add_ln or encoder" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 300 python benchmarks/micro.py gemmfp8 > $O/gemmfp8.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model e5-large --precision bf16,fp8 > $O/enc_e5.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base --precision bf16,fp8 > $O/enc_bge.json 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_e5 -o e5 -- python benchmarks/micro.py encoder --model e5-large --precision fp8 --rounds 2 --iters 3 > $O/prof_e5.log 2>&1
echo done $?
