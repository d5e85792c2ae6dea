# Round 3 batch J: the per-block route (crowded row blocks to the bf16 scan, the rest int8):
# its kernel tests, the headline, the sustained 1000-step headline and the realistic corpora.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_j}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "route or prune or pruned or crowded or split_across or large_k or radix" > $O/tests_route.log 2>&1 || { tail -60 $O/tests_route.log; exit 1; }
tail -3 $O/tests_route.log
timeout -k 10 300 python bench.py > $O/w20.json 2> $O/w20.err || { tail -30 $O/w20.err; exit 1; }
python -c "import json;r=json.loads(open('$O/w20.json').read().strip().splitlines()[-1]);print('w20',r['ms_per_step'],r['value'])"
SYMB_MQ_STATS=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --verify > $O/w20v.json 2> $O/w20v.err || { tail -30 $O/w20v.err; exit 1; }
python -c "import json;r=json.loads(open('$O/w20v.json').read().strip().splitlines()[-1]);print('w20v',r['ms_per_step'],r['value'],{k:v for k,v in r.items() if k.startswith('verify') or k.startswith('search_')})"
SYMB_MQ_STATS=1 timeout -k 10 500 python bench.py --steps 1000 --warmup 5 --timeline $O/timeline_1000.jsonl > $O/s1000.json 2> $O/s1000.err || { tail -30 $O/s1000.err; exit 1; }
python -c "import json;r=json.loads(open('$O/s1000.json').read().strip().splitlines()[-1]);print('s1000',r['ms_per_step'],r['value'],r.get('step_ms_first_decile'),r.get('step_ms_last_decile'),{k:v for k,v in r.items() if k.startswith('search_')})"
for c in random anisotropic; do
  timeout -k 10 300 python bench.py --mode search --corpus $c --steps 20 --warmup 3 --verify > $O/search_$c.json 2> $O/search_$c.err || { tail -30 $O/search_$c.err; exit 1; }
  python -c "import json;r=json.loads(open('$O/search_$c.json').read().strip().splitlines()[-1]);print('search $c',r['ms_per_step'],{k:v for k,v in r.items() if k.startswith('verify') or k.startswith('search_')})"
done
