#!/bin/bash
# Round 4: threshold sample density on held-out searches (int8 / split tiers) and the verified
# headline at the sparser sample.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_shift2
mkdir -p $O
B="python -u bench.py --mode search --queries heldout --verify --steps 20 --warmup 3"
for c in random anisotropic; do for sh in 5 7; do
  timeout -k 10 400 $B --corpus $c --prune-sample-shift $sh > $O/${c}_s$sh.json 2> $O/${c}_s$sh.err || { tail -20 $O/${c}_s$sh.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*' $O/${c}_s$sh.json | tr '\n' ' ' | sed "s/^/$c shift $sh /"; echo
done; done
for sh in 7 8 6; do
  timeout -k 10 400 python -u bench.py --prune-sample-shift $sh --steps 40 --verify > $O/head_s$sh.json 2> $O/head_s$sh.err || { tail -20 $O/head_s$sh.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*' $O/head_s$sh.json | tr '\n' ' ' | sed "s/^/head shift $sh /"; echo
done
