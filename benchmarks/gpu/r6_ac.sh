#!/bin/bash
# Round 6, run ac: the fused FFN block's MFMA sections at s_setprio 1 (SYMB_MLP_PRIO) -- output
# identity, then MiniLM embed and the headline, interleaved.
set -o pipefail
O=gpurun_out/r6_ac
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="timeout -k 10"
$T 120 python - > $O/identity.log 2>&1 <<'PY' || { tail -20 $O/identity.log; exit 1; }
import math, torch
from codename_symbiont_amd.ops._ext import hip
from codename_symbiont_amd.ops.kernels import mlp_fused
g = torch.Generator(device="cuda").manual_seed(0)
M = 32768
x = torch.nn.functional.layer_norm(torch.randn(M, 384, device="cuda", generator=g), (384,)).bfloat16()
w1 = (torch.randn(1536, 384, device="cuda", generator=g) / math.sqrt(384)).bfloat16()
w2 = (torch.randn(384, 1536, device="cuda", generator=g) / math.sqrt(1536)).bfloat16()
b1, b2 = torch.randn(1536, device="cuda", generator=g), torch.randn(384, device="cuda", generator=g)
ga, be = torch.ones(384, device="cuda"), torch.zeros(384, device="cuda")
outs = []
for p in (0, 1):
    hip().mlp_prio_config(p)
    outs.append(mlp_fused(x, w1, b1, w2, b2, ga, be, 1e-12).clone())
hip().mlp_prio_config(0)
torch.cuda.synchronize()
assert torch.equal(outs[0], outs[1])
print("identical")
PY
cat $O/identity.log
for r in 1 2 3; do
  for p in 0 1; do
    SYMB_MLP_PRIO=$p $T 120 python bench.py --mode embed --steps 50 --warmup 10 > $O/embed_p${p}_$r.json 2> $O/embed_p${p}_$r.err || { tail -20 $O/embed_p${p}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/embed_p${p}_$r.json'));print('prio $p embed', d['value'], d['ms_per_step'])"
  done
done
for r in 1 2; do
  for p in 0 1; do
    SYMB_MLP_PRIO=$p $T 200 python bench.py > $O/bench_p${p}_$r.json 2> $O/bench_p${p}_$r.err || { tail -20 $O/bench_p${p}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_p${p}_$r.json'));print('prio $p headline', d['value'], d['ms_per_step'])"
  done
done
echo done
