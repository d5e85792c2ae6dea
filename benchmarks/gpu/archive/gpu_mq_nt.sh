# emitting scan: default vs non-temporal row stream at the 1-GPU and 8-GPU per-rank shapes
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_mq_nt}; mkdir -p $O
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 100000000 --nq 256 > $O/mq_100M_256.json 2>&1 && tail -1 $O/mq_100M_256.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 > $O/mq_12.5M_2048.json 2>&1 && tail -1 $O/mq_12.5M_2048.json
echo done $?
