# emitting scan in its 2-set (256 queries / workgroup) form at the 1-GPU shape vs the list kernel
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_mq_n1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mq" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 100000000 --nq 256 > $O/mq_100M_256.json 2>&1 && tail -1 $O/mq_100M_256.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 100000000 --nq 256 --qmode near > $O/mq_100M_256_near.json 2>&1 && tail -1 $O/mq_100M_256_near.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 > $O/mq_12.5M_2048.json 2>&1 && tail -1 $O/mq_12.5M_2048.json
echo done $?
