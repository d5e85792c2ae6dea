# attention: XCD-contiguous (sequence, head) order -- numerics, micro A/B (d = 32 / 64), encoders
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_attn_xcd}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python benchmarks/micro.py attn --head-dim 32 > $O/attn_d32.json 2>&1 && tail -1 $O/attn_d32.json &&
timeout -k 10 300 python benchmarks/micro.py attn --head-dim 64 > $O/attn_d64.json 2>&1 && tail -1 $O/attn_d64.json &&
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 > $O/enc_minilm.json 2>&1 && tail -1 $O/enc_minilm.json &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base > $O/enc_bge.json 2>&1 && tail -1 $O/enc_bge.json
echo done
