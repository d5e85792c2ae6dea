# Service search pipelined over two streams (VectorStore._search_pipelined): GPU test, then the
# e2e A/B at 2048 in flight with aligned bursts (pipeline on = default, off).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_e2e_pipe}; mkdir -p $O
run() {  # tag, pipeline
  SYMB_SEARCH_PIPELINE=$2 SYMB_SEARCH_ALIGN=256 SYMB_SEARCH_MAX_BATCH=512 SYMB_SCAN_CUS=224 timeout -k 10 420 python benchmarks/e2e_service.py --index-rows 100000000 --requests 40000 --warmup-requests 8000 --concurrency 512 > $O/e2e_$1.json 2> $O/e2e_$1.err || { tail -30 $O/e2e_$1.err; return 1; }
  tail -1 $O/e2e_$1.json | python -c "import json,sys;r=json.loads(sys.stdin.read());vm=r['service_stages_ms']['vector_memory_service'];c=r['service_counters']['vector_memory_service'];print('$1',r['value'],r['search_latency_ms'],'q/launch',round(c['search.batched_queries']/c['search.launches'],1),'scan p50',round(vm['stage.index_search']['p50'],1))"
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "pipelined_search or concurrent" > $O/tests.log 2>&1 &&
run pipe_on 1 &&
run pipe_off 0
rc=$?; tail -2 $O/tests.log; echo done $rc
