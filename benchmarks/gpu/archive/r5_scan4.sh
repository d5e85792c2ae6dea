#!/bin/bash
# Round 5: the LDS-landing stream scan (per-wave LDS-DMA ring, asm DMAs, counted vmcnt) -- its
# numerics, then an interleaved A/B against the register ring, with the timing ablations.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_scan4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread \
  -k "scan_stream or mx4_tier or pruned_search_is_exact or crowded" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --rounds 3 --ab 0:0:0:0,0:0:0:1,0:0:1:1,0:0:2:1 > $O/ab_i8.jsonl 2> $O/ab_i8.err || { tail -20 $O/ab_i8.err; exit 1; }
cat $O/ab_i8.jsonl
timeout -k 10 400 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --rounds 3 --tier mx4 --queries self --ab 0:0:0:0,0:0:0:1,0:0:1:1,0:0:2:1 > $O/ab_mx4.jsonl 2> $O/ab_mx4.err || { tail -20 $O/ab_mx4.err; exit 1; }
cat $O/ab_mx4.jsonl
