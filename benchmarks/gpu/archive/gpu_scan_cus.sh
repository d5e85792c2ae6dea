# headline step with the scan on fewer CUs than the chip (the encoder overlaps on the rest)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_cus}; mkdir -p $O
for c in 0 240 224 192; do
  timeout -k 10 300 python bench.py --scan-cus $c > $O/bench_cus$c.json 2> $O/bench_cus$c.err || exit 1
  python -c "import json;d=json.load(open('$O/bench_cus$c.json'));print($c, d['value'], d['ms_per_step'], d['search_ms_per_step_rank0'])"
done
for c in 0 224; do
  timeout -k 10 300 python bench.py --scan-cus $c --no-overlap > $O/bench_noov_cus$c.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$O/bench_noov_cus$c.json'));print('noov', $c, d['value'], d['ms_per_step'], d['search_ms_per_step_rank0'])"
done
echo done
