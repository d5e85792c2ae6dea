# int8 quantiser with in-kernel bounds: tests, headline, config-2 embed step
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_i8_q}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_services_gpu.py -x -q --timeout 200 --timeout-method thread -k "i8 or pruned or service or vector" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && python -c "import json; d=json.load(open('$O/bench.json')); print('headline', d['value'], d['ms_per_step'])" &&
timeout -k 10 300 python bench.py --mode embed > $O/bench_embed.json 2> $O/bench_embed.err && python -c "import json; d=json.load(open('$O/bench_embed.json')); print('embed', d['value'], d['ms_per_step'])"
echo done
