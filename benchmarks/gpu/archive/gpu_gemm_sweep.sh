# Per-shape GEMM sweep for the wide encoders (M = 256 x 128 tokens): auto tiles, the 8-phase
# 256x256 kernel, the hipBLASLt route and torch.matmul (hipBLASLt, no epilogue).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-gemm_sweep}; mkdir -p $O
: > $O/sweep.jsonl
for shape in "2304 768 0" "768 768 2" "3072 768 1" "768 3072 2" "3072 1024 0" "1024 1024 2" "4096 1024 1" "1024 4096 2" "1152 384 0" "1536 384 1"; do
  set -- $shape
  for v in "--tile 3" "--tile 9" "--tile 3 --lt 1" "--torch"; do
    timeout -k 10 120 python benchmarks/gemm_one.py --m 32768 --n $1 --k $2 --epi $3 $v --iters 30 >> $O/sweep.jsonl 2>> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
  done
done
python - "$O" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1] + "/sweep.jsonl")]
for r in rows:
    v = "torch" if r["torch"] else f"tile{r['tile']}" + ("+lt" if r["lt"] else "")
    print(f"N={r['n']:5d} K={r['k']:5d} epi={r['epi']} {v:10s} {r['ms']*1000:8.1f} us {r['TFLOPs']:6d} TF")
PY
