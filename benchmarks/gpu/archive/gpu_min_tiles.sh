# A/B of the row-block floor of the 256-query list scans (HbmIndexShard.scan_min_tiles) in the
# headline step.  The exact pruned search's pre-pass runs two SMALL list scans on the critical
# path (the seed sub-sample, ~49k rows, and the fresh-row tail, 4096-8191 rows); with 16 tiles
# per workgroup they get only 48 / <= 8 workgroups (111 / 206 us in profiles/r2_s6's trace).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_min_tiles}; mkdir -p $O
i=0
for t in 16 2 1 16 2 1 16 2 1; do
  i=$((i+1)); f=$O/bench_${i}_t$t
  timeout -k 10 300 python bench.py --scan-min-tiles $t > $f.json 2> $f.err || exit 1
  echo "min_tiles $t: $(python -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_t1 -o bench -- python bench.py --steps 10 --warmup 3 --scan-min-tiles 1 > $O/prof_t1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_t16 -o bench -- python bench.py --steps 10 --warmup 3 --scan-min-tiles 16 > $O/prof_t16.log 2>&1
echo done $?
