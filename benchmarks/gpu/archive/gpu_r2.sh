# round-2 validation: pytest -m gpu, smoke, headline bench, rocprof kernel stats of the headline
# usage: bash benchmarks/gpu/archive/gpu_r2.sh <tag>
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -1 $O/gpu_tests.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1
echo done $?
