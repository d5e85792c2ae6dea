# headline step A/B: small-scan row blocks, search-stream priority
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_step_ab}; mkdir -p $O
for v in "base:" "mt2:--scan-min-tiles 2" "prio:--search-priority" "mt2prio:--scan-min-tiles 2 --search-priority" "base2:"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python bench.py $f > $O/bench_$n.json 2> $O/bench_$n.err || exit 1
  python -c "import json,sys; d=json.load(open('$O/bench_$n.json')); print('$n', d['value'], d['ms_per_step'], d['search_ms_per_step_rank0'])"
done
echo done
