# headline A/B: encode/search stream overlap vs back-to-back (gpurun_out/overlap/)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/overlap; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_services_gpu.py -m gpu -x -q -k "bench_contract" --timeout 280 --timeout-method thread > $O/tests.log 2>&1 && tail -1 $O/tests.log &&
for r in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_overlap_$r.json 2> $O/bench_overlap_$r.err &&
  timeout -k 10 300 python bench.py --no-overlap > $O/bench_serial_$r.json 2> $O/bench_serial_$r.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1
echo done $?
