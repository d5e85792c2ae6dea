#!/bin/bash
# DPP wave-pop top-k select (topk_select_counted_kernel rewrite): its oracle tests and the
# pruned-search exactness tests, then the driver's default bench (headline + held-out) and the
# headline / held-out timelines.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_sel
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "select or prune or pruned or dense or mx4 or stream_emits or large_k or second_segment or search" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o step -- python3 bench.py --steps 10 --warmup 3 --opt heldout_searches=0 > $O/step.log 2>&1 || { tail -30 $O/step.log; exit 1; }
python3 benchmarks/step_gap.py $(find $O/step -name "*kernel_trace.csv") > $O/step_gap.txt
python3 benchmarks/step_timeline.py $(find $O/step -name "*kernel_trace.csv") --steps 1 > $O/timeline.txt
head -12 $O/step_gap.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ho -o ho -- python3 bench.py --mode search --steps 6 --warmup 2 > $O/ho.log 2>&1 || { tail -20 $O/ho.log; exit 1; }
python3 benchmarks/step_timeline.py $(find $O/ho -name "*kernel_trace.csv") --steps 1 > $O/ho_timeline.txt
head -30 $O/ho_timeline.txt
