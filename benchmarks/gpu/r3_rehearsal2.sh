# Late round 3: the driver's scaling launch form rehearsed on one GPU (gloo ranks on cuda:0,
# torch.distributed.run, N = 2 and 4) with the current tree.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_rehearsal2}; mkdir -p $O
for n in 2 4; do
  SYMB_DIST_BACKEND=gloo SYMB_DEVICE_INDEX=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n \
      --steps 5 --warmup 2 > $O/trun_n$n.json 2> $O/trun_n$n.err || { tail -30 $O/trun_n$n.err; exit 1; }
  tail -c 400 $O/trun_n$n.json; echo
done
echo done
