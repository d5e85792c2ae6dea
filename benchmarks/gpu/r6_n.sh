#!/bin/bash
# Round 6, run n: fp8 scan, register-staged tile loads (variant 18, exact, checked against the
# default) vs the LDS-DMA default, with the no-load diagnostic (11) for the floor; 100M x 1024.
set -o pipefail
O=gpurun_out/r6_n
mkdir -p $O
T="timeout -k 10"
for r in 1 2; do
  for v in 0 18 11; do
    $T 200 python benchmarks/fp8_one.py --rows 100000000 --variant $v --iters 10 --check $([ $v = 18 ] && echo 1 || echo 0) > $O/fp8_v${v}_$r.json 2> $O/fp8_v${v}_$r.err || { tail -20 $O/fp8_v${v}_$r.err; exit 1; }
    cat $O/fp8_v${v}_$r.json
  done
done
echo done
