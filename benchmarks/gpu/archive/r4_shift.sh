#!/bin/bash
# Round 4: the threshold sample's density (1 tile in 2^shift) under the MX-fp4 tier -- headline A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_shift
mkdir -p $O
for r in 1 2; do for sh in 5 6 7 4; do
  timeout -k 10 400 python -u bench.py --prune-sample-shift $sh --steps 30 > $O/head_s${sh}_r$r.json 2> $O/head_s${sh}_r$r.err || { tail -20 $O/head_s${sh}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*' $O/head_s${sh}_r$r.json | tr '\n' ' ' | sed "s/^/shift $sh r$r /"; echo
done; done
