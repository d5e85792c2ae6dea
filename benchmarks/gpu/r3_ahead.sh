# Headline step with batch i + 2 encoded during step i (encode-ahead 2) vs i + 1 (round-3 form).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_ahead}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_services_gpu.py -x -q --timeout 300 --timeout-method thread -k "bench" > $O/tests.log 2>&1 &&
for r in 1 2; do
  for a in 2 1; do
    timeout -k 10 300 python bench.py --encode-ahead $a > $O/a${a}_r$r.json 2> $O/a${a}_r$r.err || { tail -20 $O/a${a}_r$r.err; exit 1; }
    python -c "import json;r=json.loads(open('$O/a${a}_r$r.json').read().strip().splitlines()[-1]);print('ahead $a r$r',r['value'],r['ms_per_step'],r['search_ms_per_step_rank0'])"
  done
done &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o h -- python bench.py --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err &&
python benchmarks/step_trace.py $O/prof/h_kernel_trace.csv
rc=$?; tail -2 $O/tests.log; echo done $rc
