# Kernel names / launch geometry hipBLASLt picks for the encoder shapes (torch.matmul, bf16).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_lt_names}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o lt -- python benchmarks/gemm_sweep.py --models minilm-l6,bge-base,e5-large --variants torch --rounds 2 --iters 5 > $O/sweep.jsonl 2> $O/sweep.err
echo done $?
