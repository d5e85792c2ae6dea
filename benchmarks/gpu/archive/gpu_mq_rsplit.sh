# row-split 256-query emitting scan: exactness tests, ablations at the 1-GPU headline shape,
# search A/B against the 2-set form, headline bench
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_rsplit}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mq" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py scanmqabl --rows 100000000 --nq 256 --sets 4 --rsplit 2 > $O/abl_rsplit_100M_256.json 2>&1 && tail -1 $O/abl_rsplit_100M_256.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 100000000 --nq 256 > $O/mq_100M_256.json 2>&1 && tail -1 $O/mq_100M_256.json &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json
echo done $?
