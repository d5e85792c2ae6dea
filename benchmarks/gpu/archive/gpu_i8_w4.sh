# int8 pruned scan: 8-wave (one per CU) vs 4-wave (two per CU) workgroups
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_i8_w4}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "i8 or pruned" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py scani8abl --rows 100000000 --nq 256 --i8-waves 4 > $O/abl_w4.json 2>&1 && tail -1 $O/abl_w4.json &&
timeout -k 10 300 python benchmarks/micro.py scani8abl --rows 100000000 --nq 256 --i8-waves 8 > $O/abl_w8.json 2>&1 && tail -1 $O/abl_w8.json &&
timeout -k 10 300 python bench.py --i8-waves 4 > $O/bench_w4.json 2> $O/bench_w4.err && python -c "import json; d=json.load(open('$O/bench_w4.json')); print('w4', d['value'], d['ms_per_step'])" &&
timeout -k 10 300 python bench.py --i8-waves 8 > $O/bench_w8.json 2> $O/bench_w8.err && python -c "import json; d=json.load(open('$O/bench_w8.json')); print('w8', d['value'], d['ms_per_step'])"
echo done
