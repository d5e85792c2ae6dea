# BASELINE config suite on the session-6 final state
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_s6c_suite}; mkdir -p $O
timeout -k 10 900 python benchmarks/suite.py --out $O/suite_1gpu.jsonl > $O/suite.log 2>&1 && cut -c1-260 $O/suite_1gpu.jsonl
echo done $?
