#!/bin/bash
# Round 5: tests, the 100M x 768 held-out int8 scan (LDS-query default vs stream form, XCD order),
# then PMC of the VGPR-staged GEMM (gemm_vs.hip) vs the hipBLASLt route on e5 FFN2 and bge QKV.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_vs2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "scan_stream_emits or vgpr_staged" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --dim 768 --iters 5 --tier i8 --queries heldout --ab 0:0:0:0,0:2:0:0 --rounds 3 > $O/scan768.jsonl 2> $O/scan768.err || { tail -20 $O/scan768.err; exit 1; }
cut -c1-260 $O/scan768.jsonl
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for shape in "1024 4096 2" "2304 768 0"; do set -- $shape
  for v in vs lt; do
    if [ $v = vs ]; then X="--vs 0"; M="gemm_vs"; else X="--lt 1"; M="Cijk"; fi
    for pi in 1 2; do eval P=\$P$pi
      timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $P -d $O/p_${1}_${v}_$pi -o run -- python3 benchmarks/gemm_one.py --n $1 --k $2 --epi $3 --iters 20 $X > $O/p_${1}_${v}_$pi.log 2>&1 || { tail -20 $O/p_${1}_${v}_$pi.log; exit 1; }
      python3 benchmarks/pmc_kernel.py $(find $O/p_${1}_${v}_$pi -name "*counter_collection.csv") --match $M > $O/pmc_${1}_${v}_$pi.txt
      echo "== $1 $2 $v pass $pi"; cat $O/pmc_${1}_${v}_$pi.txt
    done
  done
done
