#!/bin/bash
# Round 4: enqueue only the likely tier scan (TIER_SKIP) -- index tests, headline A/B, held-out.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_skip
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_services_gpu.py -x -q --timeout 120 --timeout-method thread -k "index or prune or mx4 or split or store or search" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for sk in 1 0; do
  SYMB_TIER_SKIP=$sk timeout -k 10 400 python -u bench.py --steps 40 --verify > $O/head_skip${sk}_r$r.json 2> $O/head_skip${sk}_r$r.err || { tail -20 $O/head_skip${sk}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*' $O/head_skip${sk}_r$r.json | tr '\n' ' ' | sed "s/^/head skip=$sk r$r /"; echo
done; done
B="python -u bench.py --mode search --queries heldout --verify --steps 20 --warmup 3"
for c in random anisotropic; do
  timeout -k 10 400 $B --corpus $c > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*' $O/$c.json | tr '\n' ' ' | sed "s/^/$c /"; echo
done
