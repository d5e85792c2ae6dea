# int8-pruned search: parts and scan-kernel ablations at the 1-GPU and 8-GPU per-rank shapes
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_i8_abl}; mkdir -p $O
timeout -k 10 300 python benchmarks/micro.py scani8abl --rows 100000000 --nq 256 > $O/abl_100M_256.json 2>&1 && tail -1 $O/abl_100M_256.json &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 10 --warmup 3 --index-prune i8 > $O/prof.log 2>&1
echo done $?
