#!/bin/bash
# Round 4 validation on the final tree: the >2 GiB fp32 GEMM probe, the full GPU suite (as the driver runs it), smoke(),
# the default bench, a sustained 1000-step run with a clock timeline.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_final
mkdir -p $O
timeout -k 10 120 python -u benchmarks/diag/gemm_2g.py > $O/gemm_2g.log 2>&1 || { tail -20 $O/gemm_2g.log; exit 1; }
cat $O/gemm_2g.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_gpu.log 2>&1 || { tail -60 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 python -u bench.py --steps 1000 --warmup 10 --verify --timeline $O/timeline.jsonl > $O/sustained_1000.json 2> $O/sustained_1000.err || { tail -20 $O/sustained_1000.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*\|"verify_exact": [a-z]*\|"step_ms_first_decile": [0-9.]*\|"step_ms_last_decile": [0-9.]*' $O/sustained_1000.json
