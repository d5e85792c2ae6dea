# Headline with the int8 scan limited to fewer CUs so batch i+1's encoder and pre-pass run beside
# batch i's scan (kernel trace: they otherwise wait for the scan, 2.6-2.9 ms per step).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_scan_cus}; mkdir -p $O
for r in 1 2; do
  for c in 0 224 240; do
    timeout -k 10 300 python bench.py --scan-cus $c > $O/c${c}_r$r.json 2> $O/c${c}_r$r.err || { tail -20 $O/c${c}_r$r.err; exit 1; }
    python -c "import json;r=json.loads(open('$O/c${c}_r$r.json').read().strip().splitlines()[-1]);print('cus $c r$r',r['value'],r['ms_per_step'],r['search_ms_per_step_rank0'])"
  done
done
echo done
