#!/bin/bash
# Round 6, run z: counters of the 256-row GEMM tiles' 2-stage vs ping-pong main loops and of
# hipBLASLt on e5-large FFN2 (M 32768, N 1024, K 4096: the longest k-loop).
# (Ran against commit d5ba24c; gemm_pp_config and the p / q sweep variants were removed after it.)
set -o pipefail
O=gpurun_out/r6_z
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"
TCC="TCC_HIT_sum TCC_MISS_sum"
for v in pp0 pp1 lt; do
  case $v in
    pp0) A="benchmarks/gemm_one.py --m 32768 --n 1024 --k 4096 --epi 2 --tile 3 --pp 0 --iters 5"; MT=gemm_bf16;;
    pp1) A="benchmarks/gemm_one.py --m 32768 --n 1024 --k 4096 --epi 2 --tile 3 --pp 1 --iters 5"; MT=gemm_bf16;;
    lt) A="benchmarks/gemm_one.py --m 32768 --n 1024 --k 4096 --epi 2 --tile 3 --lt 1 --iters 5"; MT=Cijk;;
  esac
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/$v.sq -o p -- python3 $A > $O/$v.sq.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $SQ2 --output-format csv -d $O/$v.sq2 -o p -- python3 $A > $O/$v.sq2.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $TCC --output-format csv -d $O/$v.tcc -o p -- python3 $A > $O/$v.tcc.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/$v.grbm -o p -- python3 $A > $O/$v.grbm.log 2>&1 || { echo "pmc $v failed"; tail -20 $O/$v.*.log; exit 1; }
  python3 benchmarks/pmc_kernel.py $(find $O/$v.sq $O/$v.sq2 $O/$v.tcc $O/$v.grbm -name "*counter_collection.csv") --match $MT > $O/$v.pmc.txt
  cat $O/$v.pmc.txt
done
