# Round 3: end-to-end service benchmark at the headline index size (100M x 384 bf16, one GPU):
# gateway -> NATS -> HIP encoder -> NATS -> 100M-row HBM index, C++ load generator.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_e2e}; mkdir -p $O
for c in ${3:-64 128}; do
  timeout -k 10 600 python benchmarks/e2e_service.py --index-rows ${2:-100000000} --requests 24000 --warmup-requests 4000 --concurrency $c > $O/e2e_c$c.json 2> $O/e2e_c$c.err || { tail -30 $O/e2e_c$c.err; exit 1; }
  tail -c 1200 $O/e2e_c$c.json; echo
done
