# Final round-3 validation: every GPU test, smoke, the default bench (20 steps), an exactness
# check (--verify), and a sustained 1000-step run with the clock timeline.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_final}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --verify > $O/bench_verify.json 2> $O/bench_verify.err &&
timeout -k 10 600 python bench.py --steps 1000 --warmup 10 --timeline $O/timeline_1000.jsonl > $O/sustained_1000.json 2> $O/sustained_1000.err
rc=$?; tail -2 $O/gpu_tests.log; tail -1 $O/smoke.log
for f in bench bench_verify sustained_1000; do python -c "import json;r=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',r['value'],r['ms_per_step'],{k:r.get(k) for k in ('verify_exact','verify_ids_identical','step_ms_first_decile','step_ms_last_decile','search_overflow_batches')})" || true; done
echo done $rc
