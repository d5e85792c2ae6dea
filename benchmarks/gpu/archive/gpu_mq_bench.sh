# emitting-scan integration: MQ tests, headline bench with candidate stats, list-kernel A/B
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_mq_bench}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "mq or index" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
SYMB_MQ_STATS=1 timeout -k 10 400 python bench.py > $O/bench_stats.json 2> $O/bench_stats.err && cat $O/bench_stats.json && grep emitting $O/bench_stats.err &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 100000000 --nq 256 > $O/mq_100M_256.json 2>&1 && tail -1 $O/mq_100M_256.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 > $O/mq_12.5M_2048.json 2>&1 && tail -1 $O/mq_12.5M_2048.json
echo done $?
