# fp8 prefilter + exact bf16 rescore: numerics (fp8 D=256/384 scans, recall), then the headline
# step with --index-prefilter fp8 next to the exact default, and --mode search for both
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-pref}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fp8 or prefilter or concurrent" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; tail -1 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -qE "[0-9]+ failed" $O/tests.log || { tail -40 $O/tests.log; exit 1; }
timeout -k 10 400 python bench.py --index-prefilter fp8 > $O/bench_prefilter.json 2> $O/bench.err && cat $O/bench_prefilter.json &&
timeout -k 10 400 python bench.py --mode search --index-prefilter fp8 > $O/search_prefilter.json 2>> $O/bench.err && cat $O/search_prefilter.json &&
timeout -k 10 400 python bench.py --mode search > $O/search_exact.json 2>> $O/bench.err && cat $O/search_exact.json
echo done $?
