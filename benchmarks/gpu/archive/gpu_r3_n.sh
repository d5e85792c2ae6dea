# Round 3 batch N: encoder hipGraph in the headline step, interleaved A/B against eager launches.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_n}; mkdir -p $O
for r in 1 2 3; do
  for v in graph eager; do
    F=""; [ $v = eager ] && F="--no-graph"
    timeout -k 10 300 python bench.py $F > $O/w20_${v}_$r.json 2> $O/w20_${v}_$r.err || { tail -30 $O/w20_${v}_$r.err; exit 1; }
    python -c "import json;r=json.loads(open('$O/w20_${v}_$r.json').read().strip().splitlines()[-1]);print('w20 $v $r',r['ms_per_step'],r['value'],r['search_ms_per_step_rank0'],r['host_enqueue_ms_per_step_rank0'],r['config']['encoder_hipgraph'])"
  done
done
