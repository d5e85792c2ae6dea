# Batch i's scan waits for batch i+1's encoder (so the encoder runs beside batch i's pre-pass).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_scanwait}; mkdir -p $O
for r in 1 2; do
  for w in 1 0; do
    timeout -k 10 300 python bench.py --scan-waits-encoder $w > $O/w${w}_r$r.json 2> $O/w${w}_r$r.err || { tail -20 $O/w${w}_r$r.err; exit 1; }
    python -c "import json;r=json.loads(open('$O/w${w}_r$r.json').read().strip().splitlines()[-1]);print('wait $w r$r',r['value'],r['ms_per_step'],r['search_ms_per_step_rank0'])"
  done
done &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o h -- python bench.py --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err &&
python benchmarks/step_trace.py $O/prof/h_kernel_trace.csv
echo done $?
