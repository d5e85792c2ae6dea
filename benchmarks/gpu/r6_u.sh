#!/bin/bash
# Round 6, run u: counters of the fused QKV + attention kernel (MiniLM embed step, eager).
set -o pipefail
O=gpurun_out/r6_u
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"
A="bench.py --mode embed --steps 4 --warmup 2 --opt graph=0"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o p -- python3 $A > $O/sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $SQ2 --output-format csv -d $O/sq2 -o p -- python3 $A > $O/sq2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/grbm -o p -- python3 $A > $O/grbm.log 2>&1 || { echo "pmc failed"; tail -20 $O/*.log; exit 1; }
python3 benchmarks/pmc_kernel.py $(find $O/sq $O/sq2 $O/grbm -name "*counter_collection.csv") --match qkv_attn > $O/qkv_attn.pmc.txt
cat $O/qkv_attn.pmc.txt
python3 benchmarks/pmc_kernel.py $(find $O/sq $O/sq2 $O/grbm -name "*counter_collection.csv") --match attn_varlen > $O/attn.pmc.txt || true
echo done
