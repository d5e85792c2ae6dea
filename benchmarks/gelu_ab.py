#!/usr/bin/env python3
"""GELU epilogue cost: the same GEMM with the bias epilogue vs the bias+GELU epilogue on the
MiniLM / bge FFN1 shapes (varlen batch 256 x ~80 tokens)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.micro import ab  # noqa: E402
from codename_symbiont_amd.ops import kernels as K  # noqa: E402

out = {}
for name, M, N, Kd in (("minilm.ffn1", 20480, 1536, 384), ("bge.ffn1", 20480, 3072, 768),
                       ("minilm.qkv", 20480, 1152, 384)):
    x = torch.randn(M, Kd, device="cuda").bfloat16()
    w = (torch.randn(N, Kd, device="cuda") / math.sqrt(Kd)).bfloat16()
    b = torch.randn(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    from codename_symbiont_amd.ops._ext import hip
    h = hip()

    def gelu(poly):
        h.gemm_gelu_config(poly)
        K.gemm(x, w, b, K.EPI_GELU, out=y)
        h.gemm_gelu_config(0)

    ref = (x.float() @ w.float().t() + b)
    ref = torch.nn.functional.gelu(ref)
    errs = {}
    for poly in (0, 1):
        gelu(poly)
        torch.cuda.synchronize()
        errs[f"gelu_poly{poly}_max_abs_err_vs_fp32"] = float((y.float() - ref).abs().max())
    r = ab({"bias": lambda: K.gemm(x, w, b, K.EPI_BIAS, out=y),
            "gelu_erf": lambda: gelu(0), "gelu_poly": lambda: gelu(1),
            "torch_matmul": lambda: torch.matmul(x, w.t(), out=y)}, rounds=5, iters=20)
    fl = 2 * M * N * Kd
    out[name] = {k: dict(us=round(m * 1e3, 1), TFLOPs=round(fl / (m / 1e3) / 1e12)) for k, (m, _) in r.items()}
    out[name].update(errs)
print(json.dumps({"bench": "gelu_epilogue_ab", "results": out}))
