#!/bin/bash
# r4_n (CU partition, measured map) + r4_h (small-M latency, graph vs eager) + r4_m (scan PMC).
cd "$(dirname "$0")/../.."
bash benchmarks/gpu/r4_n.sh && bash benchmarks/gpu/r4_h.sh && bash benchmarks/gpu/r4_m.sh
