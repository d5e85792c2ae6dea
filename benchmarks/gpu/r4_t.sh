#!/bin/bash
# Round 4: kernel trace of the bge-base 8 x 32 query-path forward (eager, small-M path to 256).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_t
mkdir -p $O
timeout -k 10 120 python benchmarks/lat_trace.py --model bge-base --b 8 --s 32 >> $O/lat.jsonl 2>> $O/lat.err || exit 1
cat $O/lat.jsonl
d=$O/prof_bge_8x32
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python benchmarks/lat_trace.py --model bge-base --b 8 --s 32 --iters 50 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
find $O -name "*.db" | head
