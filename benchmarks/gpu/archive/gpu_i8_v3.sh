# int8-pruned search, integer pre-test + fused 512-query chains: tests, both shapes, headline
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_i8_v3}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "i8 or pruned" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py scani8abl --rows 100000000 --nq 256 > $O/abl_100M_256.json 2>&1 && tail -1 $O/abl_100M_256.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 --prune > $O/mq_12.5M_2048.json 2>&1 && tail -1 $O/mq_12.5M_2048.json &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json
echo done
