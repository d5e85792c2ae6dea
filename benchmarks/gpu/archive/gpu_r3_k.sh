# Round 3 batch K: same-box interleaved A/B of the per-block route (default) against the
# whole-batch route only (--prune-block-frac 1): headline (pipelined) and held-out random search.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_k}; mkdir -p $O
for r in 1 2; do
  for v in blk whole; do
    F=""; [ $v = whole ] && F="--prune-block-frac 1"
    timeout -k 10 300 python bench.py $F > $O/w20_${v}_$r.json 2> $O/w20_${v}_$r.err || { tail -30 $O/w20_${v}_$r.err; exit 1; }
    python -c "import json;r=json.loads(open('$O/w20_${v}_$r.json').read().strip().splitlines()[-1]);print('w20 $v $r',r['ms_per_step'],r['value'],r['search_ms_per_step_rank0'])"
  done
done
for r in 1 2; do
  for v in blk whole; do
    F=""; [ $v = whole ] && F="--prune-block-frac 1"
    timeout -k 10 300 python bench.py --mode search --corpus random --steps 20 --warmup 3 $F > $O/sr_${v}_$r.json 2> $O/sr_${v}_$r.err || { tail -30 $O/sr_${v}_$r.err; exit 1; }
    python -c "import json;r=json.loads(open('$O/sr_${v}_$r.json').read().strip().splitlines()[-1]);print('search $v $r',r['ms_per_step'])"
  done
done
