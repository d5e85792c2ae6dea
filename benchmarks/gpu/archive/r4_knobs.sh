#!/bin/bash
# Round 4: headline knob sweep on the final tree (each knob against the default, same box).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_knobs
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 400 python -u bench.py --steps 40 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/$tag.json | sed "s/^/$tag /"
}
for r in 1 2; do
  run default_r$r
  run mx4tr64_r$r --mx4-tile-rows 64
  run smt8_r$r --scan-min-tiles 8
  run smt32_r$r --scan-min-tiles 32
  run pmt4_r$r --prepass-min-tiles 4
done
