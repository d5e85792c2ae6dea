#!/bin/bash
# Round 5 baseline on the round-4 tree: the default bench, held-out 100M x 384 search (random and
# anisotropic corpora), the int8 scan kernel alone, and a kernel-stats profile of the held-out search.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_base
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --mode search --steps 20 --warmup 3 > $O/heldout_random.json 2> $O/heldout_random.err || { tail -20 $O/heldout_random.err; exit 1; }
cat $O/heldout_random.json
timeout -k 10 300 python -u bench.py --mode search --corpus anisotropic --steps 20 --warmup 3 > $O/heldout_aniso.json 2> $O/heldout_aniso.err || { tail -20 $O/heldout_aniso.err; exit 1; }
cat $O/heldout_aniso.json
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 > $O/scan_one_random.json 2> $O/scan_one.err || { tail -20 $O/scan_one.err; exit 1; }
cat $O/scan_one_random.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_heldout -o run -- python3 -u bench.py --mode search --steps 10 --warmup 2 > $O/prof_heldout.log 2>&1 || { tail -20 $O/prof_heldout.log; exit 1; }
find $O/prof_heldout -name '*kernel_stats.csv' | head -1 | xargs -I{} head -25 {}
