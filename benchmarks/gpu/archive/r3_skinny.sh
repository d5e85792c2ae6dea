# Small-M split-K GEMM (gemm_skinny.hip): its GPU tests, then query-path encoder latency
# (eager and hipGraph replay) with the skinny path on / off, and a kernel trace of each.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_skinny}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "skinny or graph_replay or gemm or encoder" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
for m in minilm-l6 bge-base; do for bs in "1 16" "1 64" "4 16" "8 32"; do set -- $bs
  for sk in 64 0; do
    timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --skinny-max-m $sk >> $O/lat.jsonl 2>> $O/lat.err || exit 1
    timeout -k 10 120 python benchmarks/lat_trace.py --model $m --b $1 --s $2 --skinny-max-m $sk --graph >> $O/lat.jsonl 2>> $O/lat.err || exit 1
  done
done; done &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_tiled -o run -- python benchmarks/lat_trace.py --b 1 --s 16 --skinny-max-m 0 > $O/prof_tiled.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_skinny -o run -- python benchmarks/lat_trace.py --b 1 --s 16 > $O/prof_skinny.log 2>&1
rc=$?; tail -2 $O/tests.log; cat $O/lat.jsonl
echo done $rc
