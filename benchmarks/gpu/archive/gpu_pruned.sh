# exact int8 bound-pruned search: numerics (exactness vs the bf16 scan), A/B, headline with it
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_pruned}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "i8 or pruned" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 100000000 --nq 256 --prune > $O/mq_100M_256.json 2>&1 && tail -1 $O/mq_100M_256.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 --prune > $O/mq_12.5M_2048.json 2>&1 && tail -1 $O/mq_12.5M_2048.json &&
timeout -k 10 300 python bench.py --index-prune i8 > $O/bench_pruned.json 2> $O/bench_pruned.err && cat $O/bench_pruned.json
echo done
