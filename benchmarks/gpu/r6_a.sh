#!/bin/bash
# Round 6, first run: GPU suite on the tree with the partial-sub-tile fix, the MX-fp6 tier off,
# gemm_vs removed; headline bench; the new embed-only mode (three runs, MiniLM) and bge embed.
set -o pipefail
O=gpurun_out/r6_a
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed$i.json 2> $O/embed$i.err \
    || { tail -20 $O/embed$i.err; exit 1; }
  cat $O/embed$i.json
done
timeout -k 10 120 python bench.py --mode embed --model bge-base --steps 30 --warmup 5 > $O/embed_bge.json \
  2> $O/embed_bge.err || { tail -20 $O/embed_bge.err; exit 1; }
cat $O/embed_bge.json
