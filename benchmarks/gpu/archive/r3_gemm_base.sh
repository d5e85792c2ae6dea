# Round-3 GEMM baseline: smoke, per-shape sweep of every route, bge/e5 encoder A/B (gemm.hip
# everywhere vs the hipBLASLt route) and per-kernel stats of the bge forward on gemm.hip only.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_gemm_base}; mkdir -p $O
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python benchmarks/gemm_sweep.py --models minilm-l6,bge-base,e5-large > $O/sweep.jsonl 2> $O/sweep.err &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base --tiles 3,12 --rounds 5 --iters 10 > $O/enc_bge.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model e5-large --tiles 3,12 --rounds 3 --iters 5 > $O/enc_e5.json 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bge -o enc -- python benchmarks/micro.py encoder --model bge-base --tiles 3 --rounds 3 --iters 10 > $O/bge_prof.log 2>&1
echo done $?
