# Round 3: the headline step sustained for 1000+ steps (power-bound scan: does the clock settle?)
# next to the driver's 20-step window, with per-step GPU times and rocm-smi clock/power samples.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_sustain}; mkdir -p $O
STEPS=${2:-1000}
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/w20.json 2> $O/w20.err || exit 1
timeout -k 10 400 python bench.py --steps $STEPS --warmup 5 --timeline $O/timeline.jsonl > $O/sustained.json 2> $O/sustained.err || exit 1
python - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("w20", "sustained"):
    r = json.load(open(f"{o}/{f}.json"))
    print(f, r["steps"], r["ms_per_step"], r["value"], r.get("step_ms_first_decile"), r.get("step_ms_last_decile"), r.get("sclk_mhz_samples"))
PY
