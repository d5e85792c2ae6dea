# int8 pruned scan at the 8-GPU per-rank shape: 512-query vs 256-query (fused) workgroups
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_i8_rs2}; mkdir -p $O
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 12500000 --nq 2048 --prune > $O/mq_12.5M_2048.json 2>&1 && tail -1 $O/mq_12.5M_2048.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 25000000 --nq 1024 --prune > $O/mq_25M_1024.json 2>&1 && tail -1 $O/mq_25M_1024.json &&
timeout -k 10 300 python benchmarks/micro.py scanmq --rows 50000000 --nq 512 --prune > $O/mq_50M_512.json 2>&1 && tail -1 $O/mq_50M_512.json
echo done
