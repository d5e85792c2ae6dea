# kernel-level split of the multi-query-block search (seed sample gather, seed scan, MQ scan,
# select, gated fallback) at the 8-rank per-rank shape
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_mq_prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o mq -- python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 --rounds 2 --iters 3 > $O/prof.log 2>&1
echo done $?
