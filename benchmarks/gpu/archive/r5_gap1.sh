#!/bin/bash
# Round 5: shrinking the gap between headline scans -- the 4-wave centroid kernel (test), then the
# headline with / without the pre-pass stream at high priority and with / without the MX-fp6 tier.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_gap1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "centroid or mx6 or stream_emits" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for cfg in "auto 0" "auto 1" "0 0" "0 1"; do set -- $cfg
  SYMB_PRUNE_MX6=$1 timeout -k 10 300 python -u bench.py --opt heldout_searches=0 --opt pre_priority=$2 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -20 $O/b_$1_$2.err; exit 1; }
  echo "mx6=$1 prio=$2 $(python3 -c "import json,sys; d=json.load(open('$O/b_$1_$2.json')); print(d['value'], d['ms_per_step'])")"
done
