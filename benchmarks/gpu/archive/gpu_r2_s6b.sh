# session 6: cached tile-sample index + rank-0 gid fast path -- GPU tests, headline x3, kernel trace
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_s6b}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  echo "run $i: $(python -c "import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1
echo done $?
