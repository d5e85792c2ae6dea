#!/bin/bash
# Round 5: the simulated N-GPU per-rank step (--opt simulate_world=N: a 100M/N shard and 256*N
# gathered queries on ONE GPU; a projection, not a multi-GPU measurement) at N = 2, 4, 8.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_sim
mkdir -p $O
for n in 2 4 8; do
  timeout -k 10 300 python -u bench.py --opt simulate_world=$n --opt heldout_searches=5 > $O/sim_$n.json 2> $O/sim_$n.err || { tail -20 $O/sim_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/sim_$n.json').read()); print($n, d['ms_per_step'], d.get('projected_job_rate'), d.get('heldout_ms_per_search'), d.get('search_mx4_tier_batches'))"
done
