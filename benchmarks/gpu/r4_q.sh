#!/bin/bash
# Round 4: dense exact tail up to 2048 queries (the MX-fp4 tier for the N = 4 / 8 per-rank
# shapes) -- tests, projections, headline; the MiniLM embed step vs the bare encoder; then the
# CU-reserve sweep, small-M latency and scan PMC (r4_n / r4_h / r4_m).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_q
mkdir -p $O
T="python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T -k "mx4 or prune or pruned or index" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 4 8; do
  timeout -k 10 400 python -u bench.py --simulate-world $n --steps 30 --warmup 5 > $O/proj_n$n.json 2> $O/proj_n$n.err || { tail -20 $O/proj_n$n.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/proj_n$n.json | sed "s/^/proj n=$n /"
done
timeout -k 10 400 python -u bench.py --steps 40 --warmup 5 > $O/head.json 2> $O/head.err || { tail -20 $O/head.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/head.json | sed "s/^/head /"
timeout -k 10 300 python -u benchmarks/micro.py encoder --model minilm-l6 --tiles 3 > $O/enc_minilm.json 2> $O/enc_minilm.err || { tail -20 $O/enc_minilm.err; exit 1; }
cat $O/enc_minilm.json
for g in "" "--no-graph"; do
  timeout -k 10 300 python -u bench.py --mode embed --steps 40 --warmup 5 $g > $O/embed$g.json 2> $O/embed$g.err || { tail -20 $O/embed$g.err; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"host_phase_ms_per_step_rank0": {[^}]*}\|"embed_ms_per_step_rank0": [0-9.]*' $O/embed$g.json | tr '\n' ' ' | sed "s/^/embed $g /"; echo
done
bash benchmarks/gpu/r4_n.sh && bash benchmarks/gpu/r4_h.sh && bash benchmarks/gpu/r4_m.sh
