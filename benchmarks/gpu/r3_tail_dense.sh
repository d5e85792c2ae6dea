# Dense exact tail for the pruned search's route: pruned-search GPU tests, headline A/B
# (tail_dense_max_nq 512 vs 0 = the emitting tail scan) and a kernel trace of the new step.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_tail_dense}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "prune or pruned or route or topk or mq" > $O/tests.log 2>&1 &&
for r in 1 2; do
  for m in 512 0; do
    SYMB_TAIL_DENSE_MAX_NQ=$m timeout -k 10 300 python bench.py > $O/td${m}_r$r.json 2> $O/td${m}_r$r.err || { tail -20 $O/td${m}_r$r.err; exit 1; }
    python -c "import json;r=json.loads(open('$O/td${m}_r$r.json').read().strip().splitlines()[-1]);print('tail_dense $m r$r',r['value'],r['ms_per_step'],r['search_ms_per_step_rank0'])"
  done
done &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o h -- python bench.py --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err &&
python benchmarks/step_trace.py $O/prof/h_kernel_trace.csv
rc=$?; tail -2 $O/tests.log; echo done $rc
