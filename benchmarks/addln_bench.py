#!/usr/bin/env python3
"""add_ln (residual + LayerNorm, bf16 in/out) at encoder shapes: time and effective bandwidth,
against torch's layer_norm on the same tensors."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.micro import ab  # noqa: E402
from codename_symbiont_amd.ops import kernels as K  # noqa: E402

out = {}
for T, H in ((32768, 768), (32768, 1024), (32768, 384)):
    x = torch.randn(T, H, device="cuda").bfloat16()
    r = torch.randn(T, H, device="cuda").bfloat16()
    g = torch.randn(H, device="cuda")
    b = torch.randn(H, device="cuda")
    y = torch.empty_like(x)
    ref = torch.nn.functional.layer_norm((x.float() + r.float()), (H,), g, b, 1e-12)
    K.add_ln(x, r, g, b, 1e-12, out=y)
    torch.cuda.synchronize()
    err = float((y.float() - ref).abs().max())
    res = ab({"hip_add_ln": lambda: K.add_ln(x, r, g, b, 1e-12, out=y),
              "hip_ln_only": lambda: K.add_ln(x, None, g, b, 1e-12, out=y),
              "torch_layer_norm": lambda: torch.nn.functional.layer_norm(x, (H,), g.bfloat16(),
                                                                        b.bfloat16(), 1e-12)},
             rounds=5, iters=20)
    nbytes = {"hip_add_ln": 3 * T * H * 2, "hip_ln_only": 2 * T * H * 2, "torch_layer_norm": 2 * T * H * 2}
    out[f"{T}x{H}"] = {k: dict(us=round(m * 1e3, 1), TBps=round(nbytes[k] / (m / 1e3) / 1e12, 2))
                       for k, (m, _) in res.items()}
    out[f"{T}x{H}"]["max_abs_err_vs_fp32"] = err
print(json.dumps({"bench": "add_ln", "results": out}))
