# prefilter recall/speed at 100M x 384 (random and near-duplicate queries), 256 and 2048 queries
set -o pipefail
O=gpurun_out/${1:-pref2}; mkdir -p $O
for qm in random near; do
  timeout -k 10 300 python benchmarks/micro.py prefilter --rows 100000000 --nq 256 --qmode $qm --rounds 3 --iters 3 2>/dev/null | tee -a $O/prefilter.jsonl || exit 1
done
timeout -k 10 300 python benchmarks/micro.py prefilter --rows 12500000 --nq 2048 --qmode random --rounds 3 --iters 3 2>/dev/null | tee -a $O/prefilter.jsonl
echo done $?
