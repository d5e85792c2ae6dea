#!/bin/bash
# Round 4: CU partition with the MEASURED mask-bit -> (XCC, SE, CU) map -- GPU tests, the map,
# and a same-box A/B of the reserve size (CUs per XCD) on the headline.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_n
mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_cu_partition_gpu.py -x -q --timeout 60 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 60 python -c "
import json
from codename_symbiont_amd.parallel.cu_partition import probe_cu_map, reserve_from_map
m = probe_cu_map('cuda')
print(json.dumps({'bit_to_xcc_se_cu': m, 'reserve_2': reserve_from_map(m, 2), 'reserve_4': reserve_from_map(m, 4)}))
" > $O/cu_map.json 2>&1 || { cat $O/cu_map.json; exit 1; }
cut -c1-300 $O/cu_map.json
for r in 1 2; do for v in 0 2 4 6 8; do
  timeout -k 10 400 python -u bench.py --steps 40 --warmup 5 --scan-cu-reserve $v > $O/cu_${v}_r$r.json 2> $O/cu_${v}_r$r.err || { tail -20 $O/cu_${v}_r$r.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/cu_${v}_r$r.json | sed "s/^/reserve $v r$r /"
done; done
