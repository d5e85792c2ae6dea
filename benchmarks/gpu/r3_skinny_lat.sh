# Small-M GEMM, default form: its GPU tests, eager query-path latency (skinny / tiled) for MiniLM
# and bge-base, and kernel traces of the 1 x 16 forwards.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_skinny3}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "skinny or graph_replay" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
for m in minilm-l6 bge-base; do for bs in "1 16" "1 32" "1 64" "4 16" "8 32"; do set -- $bs
  for sk in 64 0; do
    timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --skinny-max-m $sk >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  done
done; done &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_minilm -o run -- python benchmarks/lat_trace.py --b 1 --s 16 > $O/prof_minilm.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_bge -o run -- python benchmarks/lat_trace.py --model bge-base --b 1 --s 16 > $O/prof_bge.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_bge_tiled -o run -- python benchmarks/lat_trace.py --model bge-base --b 1 --s 16 --skinny-max-m 0 > $O/prof_bge_tiled.log 2>&1
rc=$?; tail -2 $O/tests.log; cat $O/lat.jsonl
echo done $rc
