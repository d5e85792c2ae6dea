#!/bin/bash
# Round 6, run t: where the fused QKV + attention kernel's time goes (SYMB_QKV_ATTN_ABL: 1 = no
# attention phase, 2 = no projection MFMAs; timing only), kernel traces of the embed step.
set -o pipefail
O=gpurun_out/r6_t
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for a in 0 1 2; do
  SYMB_QKV_ATTN_ABL=$a $T 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/abl$a -o e -- python3 bench.py --mode embed \
    --steps 10 --warmup 3 --opt graph=0 > $O/abl$a.out 2>&1 || { tail -20 $O/abl$a.out; exit 1; }
  grep -h "qkv_attn" $(find $O/abl$a -name "*kernel_stats.csv") | cut -c1-160
done
echo done
