# Round 3 batch G: pipelined headline with CU headroom for the pre-pass; end-to-end at 100M with
# per-service stage timers; the realistic-distribution table with the final search code.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_g}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_rccl_gpu.py tests/test_kernels_gpu.py -k "rccl or split" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 0 248 240 0 248 240; do
  timeout -k 10 300 python bench.py --scan-cus $r > $O/h_cus$r.json 2> $O/h_cus$r.err || { tail $O/h_cus$r.err; exit 1; }
  python -c "import json;r=json.loads(open('$O/h_cus$r.json').read().strip().splitlines()[-1]);print('cus $r',r['ms_per_step'],r['value'],r['search_ms_per_step_rank0'])"
done
SYMB_SEARCH_MAX_BATCH=512 SYMB_SCAN_CUS=224 timeout -k 10 600 python benchmarks/e2e_service.py --index-rows 100000000 --requests 40000 --warmup-requests 8000 --concurrency 256 > $O/e2e.json 2> $O/e2e.err || { tail -30 $O/e2e.err; exit 1; }
tail -1 $O/e2e.json | python -c "import json,sys;r=json.loads(sys.stdin.read());print(r['value'],r['search_latency_ms']);print(json.dumps(r['service_stages_ms']));print(json.dumps(r['service_counters']))"
bash benchmarks/gpu/archive/gpu_r3_real.sh r3_g/real
