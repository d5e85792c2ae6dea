#!/bin/bash
# Held-out search (bench.py --mode search: 100M x 384, 256 fresh held-out queries per search) at
# threshold-sample densities 1 in 2^5 (default) / 2^6 / 2^4, alternated, after the pre-pass rewrites.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_shift
mkdir -p $O
for i in 1 2; do
  for s in 5 6 4; do
    timeout -k 10 300 python -u bench.py --mode search --steps 20 --warmup 3 --opt prune_sample_shift=$s > $O/s${s}_$i.json 2> $O/s${s}_$i.err || { tail -20 $O/s${s}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/s${s}_$i.json').read()); print('shift $s run $i', d['value'], d['ms_per_step'])"
  done
done
