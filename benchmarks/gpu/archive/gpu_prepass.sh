# Pre-pass list scans at 1 tile per workgroup (HbmIndexShard.prepass_min_tiles): GPU tests, then
# headline A/B against the old 16-tile floor (interleaved, one box) and a kernel trace.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_prepass}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for t in 16 0 16 0 16 0 16 0; do
  i=$((i+1)); f=$O/bench_${i}_p$t
  timeout -k 10 300 python bench.py --prepass-min-tiles $t > $f.json 2> $f.err || exit 1
  echo "prepass_min_tiles $t: $(python -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1
echo done $?
