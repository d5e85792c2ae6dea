# Round 3 batch F: pipelined search (batch i+1's query-side work under batch i's scan) A/B on the
# headline + kernel trace; end-to-end at 100M rows with bigger search bursts and CU headroom for
# the encoder sharing the GPU.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_f}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "split or pruned or route" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in pipe nopipe pipe2 nopipe2; do
  extra=""; [ "${r#nopipe}" != "$r" ] && extra="--no-search-pipeline"
  timeout -k 10 300 python bench.py $extra > $O/h_$r.json 2> $O/h_$r.err || { tail $O/h_$r.err; exit 1; }
  python -c "import json;r=json.load(open('$O/h_$r.json'));print('$r',r['ms_per_step'],r['value'],r['search_ms_per_step_rank0'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o h -- python bench.py --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err || exit 1
python benchmarks/step_trace.py $O/prof/h_kernel_trace.csv || true
for v in "c256_b512:256:512:0" "c256_b512_cu224:256:512:224"; do
  IFS=: read name c b cus <<< "$v"
  SYMB_SEARCH_MAX_BATCH=$b SYMB_SCAN_CUS=$cus timeout -k 10 600 python benchmarks/e2e_service.py --index-rows 100000000 --requests 40000 --warmup-requests 8000 --concurrency $c > $O/e2e_$name.json 2> $O/e2e_$name.err || { tail -30 $O/e2e_$name.err; exit 1; }
  python -c "import json;r=json.load(open('$O/e2e_$name.json'));print('$name',r['value'],r['search_latency_ms'],r['gateway_hops_ms'])"
done
