#!/bin/bash
# Round 6, run m: fp8 scan DMA placement A/B (index_fp8.hip variants 15-17, exact forms checked
# against the default) at 100M x 1024, interleaved.
set -o pipefail
O=gpurun_out/r6_m
mkdir -p $O
T="timeout -k 10"
for r in 1 2; do
  for v in 0 15 16 17; do
    $T 200 python benchmarks/fp8_one.py --rows 100000000 --variant $v --iters 10 --check 1 > $O/fp8_v${v}_$r.json 2> $O/fp8_v${v}_$r.err || { tail -20 $O/fp8_v${v}_$r.err; exit 1; }
    cat $O/fp8_v${v}_$r.json
  done
done
echo done
