# session-5 validation after the hipBLASLt route: GPU tests, smoke, BASELINE config suite
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 900 python benchmarks/suite.py --out $O/suite_1gpu.jsonl > $O/suite.log 2>&1; tail -3 $O/suite.log
cut -c1-400 $O/suite_1gpu.jsonl
echo done
