#!/bin/bash
# Round 6, run l: where the fp8 scan's non-MFMA time goes -- timing diagnostics of the default
# geometry (index_fp8.hip variants 9, 11-14) at 100M x 1024.
set -o pipefail
O=gpurun_out/r6_l
mkdir -p $O
T="timeout -k 10"
for v in 0 9 11 12 13 14 0; do
  $T 200 python benchmarks/fp8_one.py --rows 100000000 --variant $v --iters 10 > $O/fp8_v$v.json 2> $O/fp8_v$v.err || { tail -20 $O/fp8_v$v.err; exit 1; }
  cat $O/fp8_v$v.json
done
echo done
