# Threshold-sample rate at the per-rank shapes of the N = 8 / 2 headline (12.5M x 2048, 50M x 512
# gathered queries, bench-like "near" queries): exactness vs the full scan, candidate counts,
# overflow, and the pruned search time, shifts 5 / 6 / 7.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_prune_shift_rank}; mkdir -p $O
for shape in "12500000 2048" "50000000 512"; do
  set -- $shape
  for s in 5 6 7; do
    timeout -k 10 300 python benchmarks/micro.py scanmq --rows $1 --nq $2 --prune --qmode near \
        --prune-shift $s --rounds 3 --iters 5 > $O/mq_${1}_${2}_s$s.json 2> $O/mq_${1}_${2}_s$s.err || exit 1
    python -c "import json; d=json.load(open('$O/mq_${1}_${2}_s$s.json')); print('$1 x $2 shift $s', d['results']['pruned_i8'], 'cand', round(d['pruned_cand_mean']), d['pruned_cand_max'], 'ovf', d['pruned_overflow'], 'ids', d['ids_equal_frac'])"
  done
done
echo done
