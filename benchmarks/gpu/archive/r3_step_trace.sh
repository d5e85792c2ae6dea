# Kernel trace of the headline step (30 steps): gap between consecutive int8 scans and what runs in it.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_step_trace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o h -- python bench.py --steps 30 --warmup 5 > $O/prof.json 2> $O/prof.err
rc=$?; python benchmarks/step_trace.py $O/prof/h_kernel_trace.csv; echo done $rc
