# encoder forward A/B: tile 3 (auto incl. the 8-phase GEMM) vs 10 (round-1 auto), plus numerics
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-encab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or encoder" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; tail -1 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "failed" $O/tests.log || { tail -30 $O/tests.log; exit 1; }
for m in minilm-l6 bge-base e5-large; do
  timeout -k 10 300 python benchmarks/micro.py encoder --model $m --tiles 3,10 > $O/enc_$m.json 2>&1 || exit 1
  cat $O/enc_$m.json | tail -1
done
echo done
