# emitting scan ablations at the 1-GPU headline shape (100M x 256 queries, 2-set form) and the
# 8-GPU per-rank shape (12.5M x 2048, 4-set form): full / no DMA / no emission / DMA ring only
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_mq_n1_abl}; mkdir -p $O
timeout -k 10 300 python benchmarks/micro.py scanmqabl --rows 100000000 --nq 256 --sets 2 > $O/abl_100M_256.json 2>&1 && tail -1 $O/abl_100M_256.json &&
timeout -k 10 300 python benchmarks/micro.py scanmqabl --rows 12500000 --nq 2048 --sets 4 > $O/abl_12.5M_2048.json 2>&1 && tail -1 $O/abl_12.5M_2048.json
echo done $?
