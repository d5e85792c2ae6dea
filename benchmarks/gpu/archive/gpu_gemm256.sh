# 8-phase 256x256 GEMM: numerics (tile 9), then isolated single-config timings (gemm_one.py):
# K sweep and epilogues for the 8-phase kernel, the 2-stage 256x256 and hipBLASLt (torch)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-g256}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "test_gemm[" --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1; tail -1 $O/gemm_tests.log
grep -q " passed" $O/gemm_tests.log && ! grep -q "failed" $O/gemm_tests.log || { tail -30 $O/gemm_tests.log; exit 1; }
for k in 384 768 3072; do
  for v in "--tile 9" "--tile 9 --abl 1" "--tile 2" "--torch"; do
    timeout -k 5 60 python benchmarks/gemm_one.py --n 2304 --k $k --iters 30 $v 2>/dev/null | tee -a $O/ksweep.jsonl || exit 1
  done
done
for e in "--n 3072 --k 768 --epi 1" "--n 768 --k 3072 --epi 2" "--n 768 --k 768 --epi 2" "--n 1536 --k 384 --epi 1"; do
  for v in "--tile 9" "--tile 3" "--torch"; do
    timeout -k 5 60 python benchmarks/gemm_one.py $e --iters 30 $v 2>/dev/null | tee -a $O/epi.jsonl || exit 1
  done
done
echo done
