set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r2_wide; mkdir -p $O
timeout -k 10 300 python benchmarks/micro.py scanabl --rows 12500000 --nq 2048 --rounds 5 --iters 5 > $O/abl_12.5M_2048.json 2>&1 && tail -1 $O/abl_12.5M_2048.json &&
timeout -k 10 300 python benchmarks/micro.py scanabl --rows 25000000 --nq 1024 --rounds 5 --iters 5 > $O/abl_25M_1024.json 2>&1 && tail -1 $O/abl_25M_1024.json
