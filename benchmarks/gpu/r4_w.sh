#!/bin/bash
# Round 4: kernel breakdown of the MiniLM-L6 256 x 128 forward (the headline's encoder work).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_w
mkdir -p $O
timeout -k 10 200 python benchmarks/micro.py encoder --model minilm-l6 > $O/enc.json 2> $O/enc.err || { tail $O/enc.err; exit 1; }
cat $O/enc.json
d=$O/prof_minilm_256x128
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run -- python benchmarks/micro.py encoder --model minilm-l6 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
