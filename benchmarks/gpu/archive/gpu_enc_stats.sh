# per-kernel time of the MiniLM and bge-base encoder forwards (batch 256 x 128, varlen)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_enc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/minilm -o enc -- python benchmarks/micro.py encoder --model minilm-l6 --rounds 3 --iters 10 > $O/minilm.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bge -o enc -- python benchmarks/micro.py encoder --model bge-base --rounds 3 --iters 10 > $O/bge.log 2>&1
echo done $?
