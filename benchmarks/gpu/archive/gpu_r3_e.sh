# Round 3 batch E: why the sustained headline slows -- 400-step runs with search statistics
# (overflows, dense routes) for the pruned and the plain scan, and a kernel trace of the pruned one.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_e}; mkdir -p $O
for v in i8 none; do
  SYMB_MQ_STATS=1 timeout -k 10 300 python bench.py --steps 400 --warmup 5 --index-prune $v --timeline $O/tl_$v.jsonl > $O/s400_$v.json 2> $O/s400_$v.err || { tail $O/s400_$v.err; exit 1; }
  python -c "import json;r=json.load(open('$O/s400_$v.json'));print('$v',r['ms_per_step'],r.get('step_ms_first_decile'),r.get('step_ms_last_decile'),r.get('search_overflow_batches'),r.get('search_max_candidates'),r.get('search_dense_route_batches'))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o s -- python bench.py --steps 400 --warmup 5 > $O/prof.json 2> $O/prof.err || exit 1
echo done
