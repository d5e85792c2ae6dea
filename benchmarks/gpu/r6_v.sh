#!/bin/bash
# Round 6, run v: fused QKV + attention with (SYMB_QKV_ATTN=1) and without (2) the out-projection
# + LayerNorm, and the unfused pair (0): embed A/B and kernel traces, same box.
set -o pipefail
O=gpurun_out/r6_v
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
for r in 1 2; do
  for f in 1 2 0; do
    SYMB_QKV_ATTN=$f $T 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed_f${f}_$r.json 2> $O/embed_f${f}_$r.err || { tail -20 $O/embed_f${f}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/embed_f${f}_$r.json'));print('embed mode=$f', d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 1 2; do
  SYMB_QKV_ATTN=$f $T 200 rocprofv3 --kernel-trace --stats -d $O/prof$f -o embed -- python3 bench.py --mode embed \
    --steps 10 --warmup 3 --opt graph=0 > $O/prof$f.out 2>&1 || { tail -20 $O/prof$f.out; exit 1; }
done
echo done
