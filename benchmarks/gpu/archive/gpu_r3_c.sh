# Round 3 batch C: full GPU tests, kernel traces of the dense-routed pruned search vs the plain
# scan (anisotropic corpus), the headline with fresh batches every step, sustained 1000 steps.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in i8 none; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_aniso_$v -o s -- python bench.py --mode search --corpus anisotropic --steps 10 --warmup 2 --index-prune $v > $O/aniso_$v.json 2> $O/aniso_$v.err || exit 1
  tail -c 400 $O/aniso_$v.json; echo
done
bash benchmarks/gpu/archive/gpu_r3_sustain.sh r3_c/sustain 1000
