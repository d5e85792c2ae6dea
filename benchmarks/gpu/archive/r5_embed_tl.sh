#!/bin/bash
# Round 5: config #2 step trace (what the GPU runs per MiniLM embed step besides the forward).
set -o pipefail
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r5_embed_tl
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/t -o t -- python3 bench.py --mode embed --steps 30 > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r5_embed_tl/t/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50], r["Queue_Id"]) for r in csv.DictReader(open(f)))
emb = [r for r in rows if "embed_ln" in r[2]]
a, b = emb[-3][0], emb[-2][0]
print("step span us", (b - a) / 1e3)
for st, en, nm, q in rows:
    if a <= st < b:
        print(f"{(st - a) / 1e3:8.1f} {(en - st) / 1e3:8.1f} q{q} {nm}")
PY
