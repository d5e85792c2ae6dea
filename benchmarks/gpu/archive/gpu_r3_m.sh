# Round 3 batch M: the exact tail counted in the per-block route -- kernel tests, headline
# stats, headline A/B timing, sustained 1000 steps.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "route or prune or pruned or crowded or split_across or large_k or radix or mq" > $O/tests_route.log 2>&1 || { tail -60 $O/tests_route.log; exit 1; }
tail -2 $O/tests_route.log
SYMB_MQ_STATS=1 timeout -k 10 300 python bench.py --verify > $O/w20v.json 2> $O/w20v.err || { tail -30 $O/w20v.err; exit 1; }
python -c "import json;r=json.loads(open('$O/w20v.json').read().strip().splitlines()[-1]);print('w20v',r['ms_per_step'],r['value'],{k:v for k,v in r.items() if k.startswith('verify') or k.startswith('search_')})"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/w20_$r.json 2> $O/w20_$r.err || { tail -30 $O/w20_$r.err; exit 1; }
  python -c "import json;r=json.loads(open('$O/w20_$r.json').read().strip().splitlines()[-1]);print('w20 $r',r['ms_per_step'],r['value'],r['search_ms_per_step_rank0'])"
done
SYMB_MQ_STATS=1 timeout -k 10 500 python bench.py --steps 1000 --warmup 5 --timeline $O/timeline_1000.jsonl > $O/s1000.json 2> $O/s1000.err || { tail -30 $O/s1000.err; exit 1; }
python -c "import json;r=json.loads(open('$O/s1000.json').read().strip().splitlines()[-1]);print('s1000',r['ms_per_step'],r['value'],r.get('step_ms_first_decile'),r.get('step_ms_last_decile'),{k:v for k,v in r.items() if k.startswith('search_')})"
