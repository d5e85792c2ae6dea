# Round 3 batch L: end-to-end service over the 100M-row index with the per-block route.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_l}; mkdir -p $O
for c in 256 512; do
  SYMB_SEARCH_MAX_BATCH=512 SYMB_SCAN_CUS=224 timeout -k 10 600 python benchmarks/e2e_service.py --index-rows 100000000 --requests 40000 --warmup-requests 8000 --concurrency $c > $O/e2e_c$c.json 2> $O/e2e_c$c.err || { tail -30 $O/e2e_c$c.err; exit 1; }
  tail -1 $O/e2e_c$c.json | python -c "import json,sys;r=json.loads(sys.stdin.read());print('e2e c$c',r['value'],r['search_latency_ms'],r['gateway_hops_ms']);print(json.dumps(r['service_stages_ms']['vector_memory_service']))"
done
