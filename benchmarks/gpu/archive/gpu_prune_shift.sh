# A/B of the exact pruned search's threshold sample rate (1 tile in 2^shift): a sparser sample is
# a cheaper pre-pass but a lower T (more int8 emissions and bf16 re-scores).  Headline step, one box.
set -o pipefail
export PYTHONUNBUFFERED=1 SYMB_MQ_STATS=1
O=gpurun_out/${1:-r2_prune_shift}; mkdir -p $O
i=0
for s in 5 6 7 4 5 6; do
  i=$((i+1)); f=$O/bench_${i}_s$s
  timeout -k 10 300 python bench.py --prune-sample-shift $s > $f.json 2> $f.err || exit 1
  echo "shift $s: $(python -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['search_ms_per_step_rank0'])") $(grep overflowed $f.err)"
done
echo done
