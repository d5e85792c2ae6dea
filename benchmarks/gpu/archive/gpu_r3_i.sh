# Round 3 batch I: the driver's scaling-run shapes rehearsed on one GPU (gloo ranks, both launch
# forms: torch.distributed.run and bench.py's own self-launch), then the full GPU test suite and
# smoke.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_i}; mkdir -p $O
for n in 2 4; do
  SYMB_DIST_BACKEND=gloo SYMB_DEVICE_INDEX=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n \
      --steps 5 --warmup 2 > $O/trun_n$n.json 2> $O/trun_n$n.err || { tail -30 $O/trun_n$n.err; exit 1; }
  tail -c 600 $O/trun_n$n.json; echo
done
SYMB_DIST_BACKEND=gloo SYMB_DEVICE_INDEX=0 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 \
    > $O/self_n2.json 2> $O/self_n2.err || { tail -30 $O/self_n2.err; exit 1; }
tail -c 600 $O/self_n2.json; echo
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
