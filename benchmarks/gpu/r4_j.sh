#!/bin/bash
# Round 4: CU-partitioned streams for the headline (the scan on a CU-masked stream,
# the encoder / pre-pass with a reserve) -- A/B against the default, then a kernel trace of the
# default step (gap between consecutive int8 scans).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4_j
mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_cu_partition_gpu.py -x -q --timeout 60 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "0 all" "1 all" "2 all" "4 all" "2 reserve" "0 all"; do set -- $v
  timeout -k 10 400 python -u bench.py --steps 40 --warmup 5 --scan-cu-reserve $1 --side-cus $2 > $O/cu_$1_$2.json 2> $O/cu_$1_$2.err || { tail -20 $O/cu_$1_$2.err; exit 1; }
  cut -c1-120 $O/cu_$1_$2.json; grep -o '"ms_per_step": [0-9.]*\|"host_phase_ms_per_step_rank0": {[^}]*}' $O/cu_$1_$2.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o h -- python bench.py --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python benchmarks/step_trace.py $O/prof/h_kernel_trace.csv
find $O/prof -name "*kernel_trace.csv" -size +8M -delete
