#!/bin/bash
# Round 5: config #2 (MiniLM embed step) host-bound check -- hipGraph replay vs eager launches,
# alternated twice on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5_embed_ab
mkdir -p $O
for r in 1 2; do for g in 1 0; do
  timeout -k 10 200 python -u bench.py --mode embed --steps 50 --opt graph=$g > $O/e_${g}_$r.json 2> $O/e_${g}_$r.err || { tail -20 $O/e_${g}_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/e_${g}_$r.json').read()); print('graph=$g', d['value'], d['ms_per_step'], d['embed_ms_per_step_rank0'], d['host_enqueue_ms_per_step_rank0'])"
done; done
