# multi-query-block scan (index_mq.hip): numerics tests + A/B vs the 256-query kernel at the
# per-rank shapes of the sharded search (N = 2, 4, 8)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_mq}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "mq or seeded or xcd or index" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 > $O/mq_12.5M_2048.json 2>&1 && tail -1 $O/mq_12.5M_2048.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 --qmode near > $O/mq_12.5M_2048_near.json 2>&1 && tail -1 $O/mq_12.5M_2048_near.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 25000000 --nq 1024 > $O/mq_25M_1024.json 2>&1 && tail -1 $O/mq_25M_1024.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 50000000 --nq 512 > $O/mq_50M_512.json 2>&1 && tail -1 $O/mq_50M_512.json
echo done $?
