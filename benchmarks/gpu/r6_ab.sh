#!/bin/bash
# Round 6, run ab: the end-to-end service on the end tree (fused QKV + attention in the MiniLM
# encoder), same harness as run j.
set -o pipefail
O=gpurun_out/r6_ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 600 python -u benchmarks/e2e_service.py --model minilm-l6 --index-rows 100000000 --requests 40000 \
  --warmup-requests 8000 --concurrency 512 > $O/minilm_100m_c512.json 2> $O/minilm_100m_c512.err || { tail -30 $O/minilm_100m_c512.err; exit 1; }
tail -1 $O/minilm_100m_c512.json | cut -c1-400
SYMB_PRUNE_MX4=0 $T 600 python -u benchmarks/e2e_service.py --model mpnet-multi --index-rows 100000000 --requests 20000 \
  --warmup-requests 4000 --concurrency 512 > $O/mpnet_100m_c512.json 2> $O/mpnet_100m_c512.err || { tail -30 $O/mpnet_100m_c512.err; exit 1; }
tail -1 $O/mpnet_100m_c512.json | cut -c1-400
echo done
