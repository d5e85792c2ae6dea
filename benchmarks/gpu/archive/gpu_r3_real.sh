# Round 3: realistic-distribution search table (random / clustered / anisotropic corpora,
# held-out queries) for the exact int8-pruned search (with its sampled route) vs the plain bf16
# emitting scan, ids verified against the full bf16 list scan, at the 1-GPU headline shape and the
# per-rank shapes of the N = 2 / 4 / 8 sharded search (rows / N per rank, 256 N gathered queries).
# usage: bash benchmarks/gpu/archive/gpu_r3_real.sh <out-subdir> ["rows:batch ..."]
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_real}; mkdir -p $O
SHAPES=${2:-"100000000:256 50000000:512 25000000:1024 12500000:2048"}
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -20 $O/$name.err; exit 1; }
  echo "$name $(python -c "import json,sys;r=json.load(open('$O/$name.json'));print(r['ms_per_step'],r['value'],r.get('search_overflow_batches'),r.get('search_max_candidates'),r.get('search_dense_route_batches'),r.get('verify_exact'),r.get('verify_ids_identical'))")"
}
echo "name ms_per_search qps overflow_batches max_candidates dense_routed exact ids_identical"
for shape in $SHAPES; do
  ROWS=${shape%%:*}; NQ=${shape##*:}
  S="--mode search --steps 20 --warmup 3 --index-rows $ROWS --batch $NQ --verify"
  for c in "random" "clustered --clusters 100000 --cluster-spread 0.6" "clustered --clusters 10000 --cluster-spread 0.5" "anisotropic"; do
    tag=${ROWS}x${NQ}_$(echo $c | sed 's/--clusters /c/;s/ --cluster-spread /s/' | tr -d ' ')
    run ${tag}_i8 $S --corpus $c
    run ${tag}_bf16 $S --corpus $c --index-prune none
  done
done
echo done
