#!/bin/bash
# Round 5: the LDS-query int8 scan's compute path -- ablations (no refills, no LDS reads) timed in
# one process, then one PMC pass each (effective clock, MFMA busy, wave wait shares).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_lq2
mkdir -p $O
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier i8 --queries heldout --thr-add 1e6 --ab 0:5:0:0,0:7:0:0,0:9:0:0 --rounds 3 > $O/scan.jsonl 2> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 5 --tier mx6 --queries heldout >> $O/scan.jsonl 2>> $O/scan.err || { tail -20 $O/scan.err; exit 1; }
cat $O/scan.jsonl
P="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for f in 5 7 9; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $P -d $O/pmc_$f -o run -- python3 benchmarks/scan_one.py --rows 100000000 --iters 3 --tier i8 --queries heldout --thr-add 1e6 --ab 0:$f:0:0 --rounds 1 > $O/pmc_$f.log 2>&1 || { tail -20 $O/pmc_$f.log; exit 1; }
  python3 benchmarks/pmc_kernel.py $(find $O/pmc_$f -name "*counter_collection.csv") --match scan_lq > $O/pmc_$f.txt
  cat $O/pmc_$f.txt
done
