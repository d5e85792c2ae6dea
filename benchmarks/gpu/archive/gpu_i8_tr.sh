# int8-pruned search: 64- vs 128-row tiles -- exactness tests, ablations, headline
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_i8_tr}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "i8 or pruned" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py scani8abl --rows 100000000 --nq 256 --i8-tr 128 > $O/abl_128.json 2>&1 && tail -1 $O/abl_128.json &&
timeout -k 10 300 python benchmarks/micro.py scani8abl --rows 100000000 --nq 256 --i8-tr 64 > $O/abl_64.json 2>&1 && tail -1 $O/abl_64.json &&
timeout -k 10 300 python bench.py --i8-tile-rows 128 > $O/bench_128.json 2> $O/bench_128.err && python -c "import json; d=json.load(open('$O/bench_128.json')); print('128', d['value'], d['ms_per_step'])" &&
timeout -k 10 300 python bench.py --i8-tile-rows 64 > $O/bench_64.json 2> $O/bench_64.err && python -c "import json; d=json.load(open('$O/bench_64.json')); print('64', d['value'], d['ms_per_step'])"
echo done
