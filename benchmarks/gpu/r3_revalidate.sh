# Re-validation after a container rebuild (fresh in-tree .so files): every GPU test, smoke, the
# default bench, then the small-batch query-path encoder latency with a kernel trace.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_reval}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k skinny -x -q --timeout 120 --timeout-method thread > $O/skinny_tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
for bs in "1 16" "1 64" "4 16" "8 32"; do set -- $bs
  timeout -k 10 120 python benchmarks/lat_trace.py --b $1 --s $2 >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  timeout -k 10 120 python benchmarks/lat_trace.py --b $1 --s $2 --skinny-max-m 0 >> $O/lat.jsonl 2>> $O/lat.err || exit 1
done &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_b1s16_tiled -o run -- python benchmarks/lat_trace.py --b 1 --s 16 --skinny-max-m 0 > $O/prof_b1s16_tiled.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_b1s16 -o run -- python benchmarks/lat_trace.py --b 1 --s 16 > $O/prof_b1s16.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; tail -1 $O/smoke.log; cat $O/bench.json $O/lat.jsonl
echo done $rc
