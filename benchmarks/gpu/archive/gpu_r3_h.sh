# Round 3 batch H: pipelined headline vs threshold-sample rate; e2e at 100M with the native burst
# reply encoder at two concurrencies; the sustained pipelined headline.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_h}; mkdir -p $O
for r in 5 6 5 6; do
  timeout -k 10 300 python bench.py --prune-sample-shift $r > $O/h_ts$r.json 2> $O/h_ts$r.err || { tail $O/h_ts$r.err; exit 1; }
  python -c "import json;r=json.loads(open('$O/h_ts$r.json').read().strip().splitlines()[-1]);print('ts $r',r['ms_per_step'],r['value'],r['search_ms_per_step_rank0'])"
done
for c in 256 512; do
  SYMB_SEARCH_MAX_BATCH=512 SYMB_SCAN_CUS=224 timeout -k 10 600 python benchmarks/e2e_service.py --index-rows 100000000 --requests 40000 --warmup-requests 8000 --concurrency $c > $O/e2e_c$c.json 2> $O/e2e_c$c.err || { tail -30 $O/e2e_c$c.err; exit 1; }
  tail -1 $O/e2e_c$c.json | python -c "import json,sys;r=json.loads(sys.stdin.read());print('e2e c$c',r['value'],r['search_latency_ms'],r['gateway_hops_ms']);print(json.dumps(r['service_stages_ms']['vector_memory_service']))"
done
bash benchmarks/gpu/archive/gpu_r3_sustain.sh r3_h/sustain 1000
