# Late-round-3 validation: every GPU test, smoke, the default headline bench.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_validate2}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/gpu_tests.log; tail -1 $O/smoke.log; tail -1 $O/bench.json; echo done $rc
