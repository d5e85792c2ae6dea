#!/bin/bash
# Round 4: kernel statistics of the exact searches (split image on the anisotropic corpus at the
# 1-GPU and 8-GPU per-rank shapes, plain image on random rows) -- rocprofv3 --kernel-trace --stats,
# traces deleted, stats kept.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_l
mkdir -p $O
for v in "anisotropic 100000000 256" "anisotropic 12500000 2048" "random 100000000 256" "random 12500000 2048"; do set -- $v
  d=$O/prof_$1_$3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python -u bench.py --mode search --queries heldout --corpus $1 --index-rows $2 --batch $3 --steps 10 --warmup 2 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  find $d -name "*kernel_trace.csv" -delete
  f=$(find $d -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-6
done
