set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/graph; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_services_gpu.py -m gpu -x -v --timeout 280 --timeout-method thread -k "bench_contract" > $O/tests.log 2>&1 && tail -1 $O/tests.log &&
for r in 1 2; do
  timeout -k 10 300 python bench.py --mode embed > $O/embed_graph_$r.json 2>/dev/null &&
  timeout -k 10 300 python bench.py --mode embed --no-graph > $O/embed_eager_$r.json 2>/dev/null || exit 1
done
timeout -k 10 400 python bench.py > $O/headline.json 2>/dev/null
echo done $?
