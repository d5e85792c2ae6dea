# Small-M GEMM with 64-row blocks in grid z (max_m up to 256): tests, then eager latency of
# 65..256-token forwards with max_m 256 / 64 (tiled) for MiniLM and bge-base.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_skinny_rows}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "skinny or graph_replay or encoder" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
for m in minilm-l6 bge-base; do for bs in "1 128" "4 32" "8 16" "8 32" "16 16"; do set -- $bs
  for sk in 256 64; do
    timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --skinny-max-m $sk >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  done
done; done
rc=$?; tail -2 $O/tests.log; cat $O/lat.jsonl
echo done $rc
