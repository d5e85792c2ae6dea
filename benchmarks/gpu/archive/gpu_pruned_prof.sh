# kernel trace of the headline step with the exact int8-pruned search
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_pruned_prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 10 --warmup 3 --index-prune i8 > $O/prof.log 2>&1
echo done $?
