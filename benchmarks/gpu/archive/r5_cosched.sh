#!/bin/bash
# Round 5: co-scheduling the next batch's encoder under the headline's fp4 scan -- the MX-fp4
# scan form held to 256 VGPRs (mx4 variant 5: a second wave fits on every SIMD) x the FFN as the
# fused 160-KiB-LDS block (1) or as two GEMMs whose workgroups fit beside the scan (0).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_cosched
mkdir -p $O
for cfg in "0 1" "5 1" "5 0"; do set -- $cfg
  SYMB_AB_MX4V=$1 SYMB_AB_MLP=$2 timeout -k 10 300 python -u bench.py --verify --opt heldout_searches=0 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -20 $O/b_$1_$2.err; exit 1; }
  echo "mx4v=$1 mlp=$2 $(python3 -c "import json; d=json.loads(open('$O/b_$1_$2.json').read()); print(d['value'], d['ms_per_step'], d['search_mx4_tier_batches'], d['verify_exact'])")"
done
