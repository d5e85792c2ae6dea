#!/bin/bash
# Round 4: where the int8 scan's time goes -- ablations (micro.py scani8abl: full, no DMA, no
# emission test, DMA ring only, in-kernel clock) at 100M x 256, and PMC passes (SQ occupancy /
# waits, TCC, GRBM clock) of the plain and split scans (benchmarks/scan_one.py).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_m
mkdir -p $O
timeout -k 10 300 python -u benchmarks/micro.py scani8abl --rows 100000000 --nq 256 > $O/abl.json 2> $O/abl.err || { tail -20 $O/abl.err; exit 1; }
cat $O/abl.json
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"
TCC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
for c in random anisotropic; do
  A="benchmarks/scan_one.py --rows 25000000 --nq 256 --corpus $c --iters 5"
  timeout -k 5 120 python -u $A > $O/$c.time.json 2>&1 && cat $O/$c.time.json &&
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/$c.sq -o p -- python3 $A > $O/$c.sq.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $SQ2 --output-format csv -d $O/$c.sq2 -o p -- python3 $A > $O/$c.sq2.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $TCC --output-format csv -d $O/$c.tcc -o p -- python3 $A > $O/$c.tcc.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/$c.grbm -o p -- python3 $A > $O/$c.grbm.log 2>&1 || exit 1
  python3 benchmarks/pmc_kernel.py $(find $O/$c.sq $O/$c.sq2 $O/$c.tcc $O/$c.grbm -name "*counter_collection.csv") --match index_scan_i8 > $O/$c.pmc.txt 2>&1
  cat $O/$c.pmc.txt
  find $O/$c.* -name "*.csv" -size +4M -delete
done
