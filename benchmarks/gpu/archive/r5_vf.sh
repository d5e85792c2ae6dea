#!/bin/bash
# Round 5: VGPR-form MFMA build (-mllvm -amdgpu-mfma-vgpr-form=1, _hip_vf.so) vs the default one
# on the stream scans at 100M x 384, plus the int8 scan's shared-scale hit-test ablation (abl 3).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_vf
mkdir -p $O
for build in default vf; do
  if [ $build = vf ]; then export SYMB_HIP_SO=$PWD/codename_symbiont_amd/_hip_vf.so; fi
  for t in "i8 heldout 0:0:0:0,0:0:3:0" "mx4 near 0:0:0:0:1,0:0:0:0:0" "mx6 near 0:0:0:0"; do set -- $t
    timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier $1 --queries $2 --ab $3 --rounds 3 \
      | sed "s/^{/{\"build\": \"$build\", /" >> $O/scan.jsonl 2> $O/scan_${build}_$1.err || { tail -20 $O/scan_${build}_$1.err; exit 1; }
  done
done
cat $O/scan.jsonl
