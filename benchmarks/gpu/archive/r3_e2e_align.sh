# End-to-end service over the 100M-row index: bursts aligned to the int8 scan's 256-query block
# (SYMB_SEARCH_ALIGN=256, the new default) at 2048 and 1024 in flight; then the unaligned round-3
# setting (ALIGN=0) at 2048 for the A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_e2e_align}; mkdir -p $O
run() {  # tag, align, max_batch, concurrency
  SYMB_SEARCH_ALIGN=$2 SYMB_SEARCH_MAX_BATCH=$3 SYMB_SCAN_CUS=224 timeout -k 10 420 python benchmarks/e2e_service.py --index-rows 100000000 --requests 40000 --warmup-requests 8000 --concurrency $4 > $O/e2e_$1.json 2> $O/e2e_$1.err || { tail -30 $O/e2e_$1.err; return 1; }
  tail -1 $O/e2e_$1.json | python -c "import json,sys;r=json.loads(sys.stdin.read());vm=r['service_stages_ms']['vector_memory_service'];c=r['service_counters']['vector_memory_service'];print('$1',r['value'],r['search_latency_ms'],'q/launch',round(c['search.batched_queries']/c['search.launches'],1),'scan p50',round(vm['stage.index_search']['p50'],1))"
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefilter" > $O/prefilter_tests.log 2>&1 &&
run a256_b512_c512 256 512 512 &&
run a256_b512_c256 256 512 256 &&
run a0_b512_c512 0 512 512
echo done $?
