#!/bin/bash
# Round 4: the MX-fp4 first tier -- exactness tests, same-box headline A/B (SYMB_PRUNE_MX4 on /
# off), held-out random / anisotropic searches (the int8 / split tier must still be chosen), and
# a kernel trace of the headline step.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_o
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -k "mx4 or split or prune or pruned or index_scan_i8 or index" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for m in 1 0; do
  SYMB_PRUNE_MX4=$m timeout -k 10 400 python -u bench.py --steps 40 --warmup 5 --verify > $O/head_mx${m}_r$r.json 2> $O/head_mx${m}_r$r.err || { tail -20 $O/head_mx${m}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*\|"search_mx4_tier_batches": [0-9]*' $O/head_mx${m}_r$r.json | tr '\n' ' ' | sed "s/^/head mx4=$m r$r /"; echo
done; done
B="python -u bench.py --mode search --queries heldout --verify --steps 20 --warmup 3"
for c in random anisotropic; do
  timeout -k 10 400 $B --corpus $c > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"verify_exact": [a-z]*\|"search_mx4_tier_batches": [0-9]*' $O/$c.json | tr '\n' ' ' | sed "s/^/$c /"; echo
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o h -- python bench.py --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python benchmarks/step_trace.py $O/prof/h_kernel_trace.csv
python benchmarks/step_gap.py $O/prof/h_kernel_trace.csv --steps 8 > $O/step_gap.txt; head -12 $O/step_gap.txt
find $O/prof -name "*kernel_trace.csv" -size +8M -delete
