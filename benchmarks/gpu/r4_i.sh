#!/bin/bash
# Round 4: one pre-test per fused chain (8 rows per lane) in the int8 / split scans -- exactness
# tests, the headline, the random and anisotropic 100M x 256 searches, one per-rank shape, and
# kernel statistics of the split and plain searches.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_i
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 500 $T -k "split or quant_rows or prune or pruned or index_scan_i8 or wide or index" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u benchmarks/diag/split_emit.py > $O/split_emit.jsonl 2>&1 || { tail -20 $O/split_emit.jsonl; exit 1; }
cut -c1-200 $O/split_emit.jsonl
timeout -k 10 400 python bench.py --verify > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
B="python -u bench.py --mode search --queries heldout --verify --steps 20 --warmup 3"
for v in "anisotropic i8 100000000 256" "anisotropic none 100000000 256" "random i8 100000000 256" "anisotropic i8 50000000 512" "anisotropic none 50000000 512"; do set -- $v
  timeout -k 10 400 $B --corpus $1 --index-prune $2 --index-rows $3 --batch $4 > $O/$1_$4_$2.json 2> $O/$1_$4_$2.err || { tail -20 $O/$1_$4_$2.err; exit 1; }
  cat $O/$1_$4_$2.json
done
for c in anisotropic random; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python -u bench.py --mode search --queries heldout --corpus $c --steps 10 --warmup 2 > $O/prof_$c.log 2>&1 || { tail -20 $O/prof_$c.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
