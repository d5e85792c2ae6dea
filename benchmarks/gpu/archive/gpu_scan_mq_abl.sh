# index_scan_mq_kernel numerics + ablations + in-kernel clock at the per-rank shapes of N = 8, 2
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_mq_abl}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mq" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py scanmqabl --rows 12500000 --nq 2048 > $O/abl_12.5M_2048.json 2>&1 && tail -1 $O/abl_12.5M_2048.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 > $O/mq_12.5M_2048.json 2>&1 && tail -1 $O/mq_12.5M_2048.json &&
timeout -k 10 300 python benchmarks/micro.py scanmqabl --rows 50000000 --nq 512 > $O/abl_50M_512.json 2>&1 && tail -1 $O/abl_50M_512.json
echo done $?
