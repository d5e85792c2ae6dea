#!/bin/bash
# Round 6, run j: config #5's fp8 scan -- counters of the default kernel and of its L2-source
# compute ceiling (variant 9); then the end-to-end service with the block-filling search bursts
# and the pipelined embed batcher.
set -o pipefail
O=gpurun_out/r6_j
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "fp8" > $O/t_fp8.log 2>&1 || { tail -40 $O/t_fp8.log; exit 1; }
tail -1 $O/t_fp8.log
for v in 0 9; do
  $T 200 python benchmarks/fp8_one.py --rows 100000000 --variant $v --iters 10 > $O/fp8_v$v.json 2> $O/fp8_v$v.err || { tail -20 $O/fp8_v$v.err; exit 1; }
  cat $O/fp8_v$v.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU"
for v in 0 9; do
  A="benchmarks/fp8_one.py --rows 25000000 --variant $v --iters 3"
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/v$v.sq -o p -- python3 $A > $O/v$v.sq.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $SQ2 --output-format csv -d $O/v$v.sq2 -o p -- python3 $A > $O/v$v.sq2.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/v$v.grbm -o p -- python3 $A > $O/v$v.grbm.log 2>&1 || { echo "pmc v$v failed"; tail -20 $O/v$v.*.log; exit 1; }
  python3 benchmarks/pmc_kernel.py $(find $O/v$v.sq $O/v$v.sq2 $O/v$v.grbm -name "*counter_collection.csv") --match index_scan_fp8 > $O/v$v.pmc.txt
  cat $O/v$v.pmc.txt
done
$T 600 python -u benchmarks/e2e_service.py --model minilm-l6 --index-rows 100000000 --requests 40000 \
  --warmup-requests 8000 --concurrency 512 > $O/minilm_100m_c512.json 2> $O/minilm_100m_c512.err || { tail -30 $O/minilm_100m_c512.err; exit 1; }
tail -1 $O/minilm_100m_c512.json | cut -c1-400
SYMB_PRUNE_MX4=0 $T 600 python -u benchmarks/e2e_service.py --model mpnet-multi --index-rows 100000000 --requests 20000 \
  --warmup-requests 4000 --concurrency 512 > $O/mpnet_100m_c512.json 2> $O/mpnet_100m_c512.err || { tail -30 $O/mpnet_100m_c512.err; exit 1; }
tail -1 $O/mpnet_100m_c512.json | cut -c1-400
echo done
