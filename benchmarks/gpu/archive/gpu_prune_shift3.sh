# Threshold-sample rate of the exact pruned search, re-measured after the cheaper pre-pass
# (profiles/r2_prepass/): 6 interleaved pairs of shift 6 vs 7, one box, + a shift-7 trace.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_prune_shift3}; mkdir -p $O
i=0
for s in 6 7 6 7 6 7 6 7 6 7; do
  i=$((i+1)); f=$O/bench_${i}_s$s
  timeout -k 10 300 python bench.py --prune-sample-shift $s > $f.json 2> $f.err || exit 1
  echo "shift $s: $(python -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_s7 -o bench -- python bench.py --steps 20 --warmup 3 --prune-sample-shift 7 > $O/prof.log 2>&1
echo done $?
