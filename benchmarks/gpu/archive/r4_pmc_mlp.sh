#!/bin/bash
# Round 4: SQ / TCC / GRBM counter passes over the MiniLM 256 x 128 forward with the fused FFN
# block (v2): the fused kernel against the two-GEMM path's FFN1 GEMM.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_pmc_mlp
mkdir -p $O
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"
TCC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
for m in 1 0; do
  A="benchmarks/micro.py encoder --model minilm-l6 --mlp $m --rounds 1 --iters 3"
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/m$m.sq -o p -- python3 $A > $O/m$m.sq.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $SQ2 --output-format csv -d $O/m$m.sq2 -o p -- python3 $A > $O/m$m.sq2.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $TCC --output-format csv -d $O/m$m.tcc -o p -- python3 $A > $O/m$m.tcc.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/m$m.grbm -o p -- python3 $A > $O/m$m.grbm.log 2>&1 || exit 1
done
F1=$(find $O/m1.sq $O/m1.sq2 $O/m1.tcc $O/m1.grbm -name "*counter_collection.csv")
F0=$(find $O/m0.sq $O/m0.sq2 $O/m0.tcc $O/m0.grbm -name "*counter_collection.csv")
python3 benchmarks/pmc_kernel.py $F1 --match mlp_fused > $O/fused.pmc.txt 2>&1; echo "== fused"; cat $O/fused.pmc.txt
python3 benchmarks/pmc_kernel.py $F0 --match "gemm_bf16_kernel<128, 128, 2, 4, 1" > $O/ffn1.pmc.txt 2>&1; echo "== ffn1 gemm"; cat $O/ffn1.pmc.txt
python3 benchmarks/pmc_kernel.py $F0 --match "gemm_bf16_kernel<128, 384" > $O/resln.pmc.txt 2>&1; echo "== res+ln gemm"; cat $O/resln.pmc.txt
find $O -name "*.csv" -size +4M -delete
