#!/bin/bash
# MX-fp4 emission diagnostic, then the r4_o validation / A/B.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 200 python -u benchmarks/diag/mx4_emit.py > gpurun_out/mx4_emit.jsonl 2>&1 || { tail -20 gpurun_out/mx4_emit.jsonl; exit 1; }
cut -c1-300 gpurun_out/mx4_emit.jsonl
bash benchmarks/gpu/r4_o.sh
