# round-2 BASELINE config suite + end-to-end service benchmark on one MI355X
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2suite}; mkdir -p $O
timeout -k 10 900 python benchmarks/suite.py --out $O/suite_1gpu.jsonl > $O/suite.log 2>&1; tail -3 $O/suite.log
cat $O/suite_1gpu.jsonl | cut -c1-300
timeout -k 10 600 python benchmarks/e2e_service.py > $O/e2e.json 2> $O/e2e.err; tail -c 1500 $O/e2e.json
echo done
