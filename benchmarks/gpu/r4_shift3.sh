#!/bin/bash
# Round 4: the MX-fp4-tier sample density (2^7 while recent searches took the fp4 tier) --
# index tests, headline A/B against the fixed 2^5 sample, held-out random / anisotropic searches.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_shift3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "index or prune or mx4 or split" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for sh in 0 5; do
  timeout -k 10 400 python -u bench.py --prune-sample-shift $sh --steps 40 --verify > $O/head_s${sh}_r$r.json 2> $O/head_s${sh}_r$r.err || { tail -20 $O/head_s${sh}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*\|"search_mx4_tier_batches": [0-9]*' $O/head_s${sh}_r$r.json | tr '\n' ' ' | sed "s/^/head shift-arg $sh r$r /"; echo
done; done
B="python -u bench.py --mode search --queries heldout --verify --steps 20 --warmup 3"
for c in random anisotropic; do
  timeout -k 10 400 $B --corpus $c > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*\|"search_mx4_tier_batches": [0-9]*' $O/$c.json | tr '\n' ' ' | sed "s/^/$c default /"; echo
done
