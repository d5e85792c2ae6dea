#!/bin/bash
# small-M latency (r4_h), scan PMC (r4_m), then the CU partition with the measured map (r4_n).
cd "$(dirname "$0")/../.."
bash benchmarks/gpu/r4_h.sh && bash benchmarks/gpu/r4_m.sh && bash benchmarks/gpu/r4_n.sh
