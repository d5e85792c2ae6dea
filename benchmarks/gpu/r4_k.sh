#!/bin/bash
# Round 4: pair pre-test of the fused int8 chains (one test over both sub-tiles, then the
# per-sub-tile tests) vs the per-sub-tile tests alone -- exactness, then same-box A/B on the
# headline, the random and the anisotropic held-out searches.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_k
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 500 $T -k "split or prune or pruned or index_scan_i8" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u benchmarks/diag/split_emit.py > $O/split_emit.jsonl 2>&1 || { tail -20 $O/split_emit.jsonl; exit 1; }
cut -c1-120 $O/split_emit.jsonl
B="python -u bench.py --mode search --queries heldout --steps 20 --warmup 3"
for r in 1 2; do for p in 1 0; do
  timeout -k 10 400 python -u bench.py --i8-pair $p > $O/head_p${p}_r$r.json 2> $O/head_p${p}_r$r.err || { tail -20 $O/head_p${p}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/head_p${p}_r$r.json | sed "s/^/head p$p r$r /"
  for c in random anisotropic; do
    timeout -k 10 400 $B --corpus $c --i8-pair $p > $O/${c}_p${p}_r$r.json 2> $O/${c}_p${p}_r$r.err || { tail -20 $O/${c}_p${p}_r$r.err; exit 1; }
    grep -o '"ms_per_step": [0-9.]*' $O/${c}_p${p}_r$r.json | sed "s/^/$c p$p r$r /"
  done
done; done
