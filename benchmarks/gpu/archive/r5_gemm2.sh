#!/bin/bash
# Round 5: where the ping-pong GEMM v1 loses -- timing ablations (no k-loop vmcnt; no k-loop DMA),
# the half-tile ring (v2), its numerics, a sweep, and one PMC pass each for pp / round-4 tiles /
# hipBLASLt on the e5 FFN2 shape.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_gemm2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "pingpong" > $O/tests_pp.log 2>&1 || { tail -40 $O/tests_pp.log; exit 1; }
tail -3 $O/tests_pp.log
for s in "32768 3072 1024" "32768 1024 4096"; do
  set -- $s
  for v in "--pp 256" "--pp 256 --ring 0" "--pp 257 --ring 0" "--pp 258 --ring 0" "--tile 3" "--lt 1"; do
    timeout -k 10 120 python -u benchmarks/gemm_one.py --m $1 --n $2 --k $3 --epi 0 --iters 50 $v >> $O/abl.jsonl 2>> $O/abl.err || { tail -20 $O/abl.err; exit 1; }
  done
done
cat $O/abl.jsonl
timeout -k 10 400 python -u benchmarks/gemm_sweep.py --variants pp256,pp256v1,t3,lt --rounds 5 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
P="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for v in "pp --pp 256" "t3 --tile 3" "lt --lt 1"; do
  set -- $v; name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $P -d $O/pmc_$name -o run -- python3 benchmarks/gemm_one.py --m 32768 --n 1024 --k 4096 --epi 0 --iters 20 "$@" > $O/pmc_$name.log 2>&1 || { tail -20 $O/pmc_$name.log; exit 1; }
  python3 benchmarks/pmc_kernel.py $(find $O/pmc_$name -name "*counter_collection.csv") --match "gemm|Cijk" > $O/pmc_$name.txt
  cat $O/pmc_$name.txt
done
