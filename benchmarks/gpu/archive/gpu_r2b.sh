# validation after the GEMM / hub changes: GPU tests, smoke, headline bench, encoder A/B
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2b}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -1 $O/gpu_tests.log
grep -q " passed" $O/gpu_tests.log && ! grep -qE "[0-9]+ failed" $O/gpu_tests.log || { tail -40 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
timeout -k 10 400 python bench.py --no-overlap > $O/bench_nooverlap.json 2>> $O/bench.err && cat $O/bench_nooverlap.json &&
for m in bge-base e5-large; do
  timeout -k 10 300 python benchmarks/micro.py encoder --model $m --tiles 3,10 > $O/enc_$m.json 2>&1 || exit 1
  tail -1 $O/enc_$m.json
done
echo done
