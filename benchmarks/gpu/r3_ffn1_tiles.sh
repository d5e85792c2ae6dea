# Every gemm.hip tile mode on the GELU FFN1 shapes (our own fused op on every route).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_ffn1_tiles}; mkdir -p $O
timeout -k 10 400 python benchmarks/gemm_sweep.py --models minilm-l6,bge-base,e5-large --only ffn1 --variants t3,t0,t1,t2,t4,t5,t6,t7,t8,t9,w4,torch > $O/sweep.jsonl 2> $O/sweep.err
echo done $?
