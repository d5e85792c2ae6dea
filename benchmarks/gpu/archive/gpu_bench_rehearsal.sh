# Rehearsal of bench.py's multi-rank path (the driver's N = 2 / 4 scaling runs) on ONE GPU: every
# rank on cuda:0 over gloo (RCCL refuses two ranks on one device).  Checks the contract (one JSON
# line from rank 0, whole-job value, n_gpus) and that the per-rank shapes run; the timings are NOT
# scaling numbers (N ranks share one GPU).
set -o pipefail
export PYTHONUNBUFFERED=1 SYMB_DIST_BACKEND=gloo SYMB_DEVICE_INDEX=0
O=gpurun_out/${1:-r2_rehearsal}; mkdir -p $O
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 \
      > $O/bench_n$n.json 2> $O/bench_n$n.err || { tail -30 $O/bench_n$n.err; exit 1; }
  tail -c 700 $O/bench_n$n.json
done
echo done
