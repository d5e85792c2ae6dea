#!/bin/bash
# Round 5: stream scan with the integer pre-test -- numerics (stream + 768/1024 tiers + list-mode
# route fix), 100M x 384 timings of both tiers against the LDS-ring scan, one PMC pass per kernel.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_scan2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread \
  -k "quant_stream or scan_stream or append_rows or dense_scores or pruned_search_768 or mx4_tier or crowded" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -4 $O/tests.log
for v in 1 0; do
  SYMB_PRUNE_STREAM=$v timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 > $O/scan_i8_s$v.json 2> $O/scan_i8_s$v.err || { tail -20 $O/scan_i8_s$v.err; exit 1; }
  cat $O/scan_i8_s$v.json
  SYMB_PRUNE_STREAM=$v timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 --tier mx4 --queries self > $O/scan_mx4_s$v.json 2> $O/scan_mx4_s$v.err || { tail -20 $O/scan_mx4_s$v.err; exit 1; }
  cat $O/scan_mx4_s$v.json
done
timeout -k 10 300 python -u benchmarks/scan_one.py --rows 100000000 --iters 10 --dim 768 > $O/scan_i8_768.json 2> $O/scan_i8_768.err || { tail -20 $O/scan_i8_768.err; exit 1; }
cat $O/scan_i8_768.json
P="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for t in i8 mx4; do
  q=heldout; [ $t = mx4 ] && q=self
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $P -d $O/pmc_$t -o run -- python3 benchmarks/scan_one.py --rows 25000000 --iters 3 --tier $t --queries $q > $O/pmc_$t.log 2>&1 || { tail -20 $O/pmc_$t.log; exit 1; }
  python3 benchmarks/pmc_kernel.py $(find $O/pmc_$t -name "*counter_collection.csv") --match scan_stream > $O/pmc_$t.txt
  cat $O/pmc_$t.txt
done
