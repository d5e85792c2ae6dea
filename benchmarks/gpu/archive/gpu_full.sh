# full GPU validation: pytest -m gpu, smoke, headline bench, encoder micro-benchmarks (gpurun_out/full/)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -1 $O/gpu_tests.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
timeout -k 10 300 python benchmarks/micro.py encoder --model minilm-l6 > $O/enc_minilm.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model bge-base --precision bf16,fp8 > $O/enc_bge.json 2>&1 &&
timeout -k 10 300 python benchmarks/micro.py encoder --model e5-large --precision bf16,fp8 > $O/enc_e5.json 2>&1 &&
timeout -k 10 400 python bench.py --mode embed > $O/bench_embed.json 2> $O/bench_embed.err
echo done $?
