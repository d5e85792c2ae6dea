#!/bin/bash
# Round 5: PMC of the int8 stream scan (tile-scale image, VGPR-form build) at 100M x 384 held-out.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_pmc_i8
mkdir -p $O
P="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for t in "i8 heldout" "mx4 near"; do set -- $t
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $P -d $O/pmc_$1 -o run -- python3 benchmarks/scan_one.py --rows 100000000 --iters 3 --tier $1 --queries $2 > $O/pmc_$1.log 2>&1 || { tail -20 $O/pmc_$1.log; exit 1; }
  python3 benchmarks/pmc_kernel.py $(find $O/pmc_$1 -name "*counter_collection.csv") --match scan_stream > $O/pmc_$1.txt
  cat $O/pmc_$1.txt
done
