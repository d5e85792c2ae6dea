# Re-validation after a container rebuild (fresh in-tree .so files): every GPU test, smoke, the
# default bench (the query-path latency runs are r3_skinny.sh).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_reval}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k skinny -x -q --timeout 120 --timeout-method thread > $O/skinny_tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/gpu_tests.log; tail -1 $O/smoke.log; cat $O/bench.json
echo done $rc
