#!/bin/bash
# Round 4: per-rank projection of the N-GPU headline on one GPU (bench.py --simulate-world N:
# 100M/N-row shard, 256 N gathered queries, the result all_to_all through a single-rank RCCL
# group), next to the real 1-GPU step; then the BASELINE config suite.
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_f
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 > $O/proj_n1.json 2> $O/proj_n1.err || { tail -20 $O/proj_n1.err; exit 1; }
cat $O/proj_n1.json
for n in 2 4 8; do
  timeout -k 10 400 python -u bench.py --simulate-world $n --steps 30 --warmup 5 > $O/proj_n$n.json 2> $O/proj_n$n.err || { tail -20 $O/proj_n$n.err; exit 1; }
  cat $O/proj_n$n.json
done
timeout -k 10 600 python -u bench.py --steps 1000 --warmup 10 --verify > $O/sustained_1000.json 2> $O/sustained_1000.err || { tail -20 $O/sustained_1000.err; exit 1; }
cat $O/sustained_1000.json
timeout -k 10 400 python -u bench.py --corpus anisotropic --queries heldout --verify > $O/full_aniso.json 2> $O/full_aniso.err || { tail -20 $O/full_aniso.err; exit 1; }
cat $O/full_aniso.json
timeout -k 10 900 python -u benchmarks/suite.py --out $O/suite_1gpu.jsonl > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
cat $O/suite_1gpu.jsonl
