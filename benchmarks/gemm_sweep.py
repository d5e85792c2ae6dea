#!/usr/bin/env python3
"""Encoder GEMM shapes, every route in ONE process with interleaved rounds (A/B discipline).

    python benchmarks/gemm_sweep.py [--models bge-base,e5-large] [--variants t3,t9,lt,torch]

Variants: tN = symb_gemm with tile mode N (3 = auto with the 256x192 tile, 10 = the round-3
auto rule, 2 = the 256x256 tile wherever N % 256 == 0), hipBLASLt route off; tNgG = the same with
a G-row grouped tile order (default 8); lt = the hipBLASLt route for the plain projections (the
default);
torch = torch.matmul (hipBLASLt, no epilogue).
Operands are random (the clock the chip holds depends on the data).  One JSON line per
(shape, variant): median / min us over the rounds and TFLOP/s at the median.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, N, K, epi) per model at M = batch x seq tokens; epi 0 bias, 1 GELU, 2 bias + residual
SHAPES = {
    "minilm-l6": [("qkv", 1152, 384, 0), ("ffn1", 1536, 384, 1)],
    "bge-base": [("qkv", 2304, 768, 0), ("out", 768, 768, 2), ("ffn1", 3072, 768, 1), ("ffn2", 768, 3072, 2)],
    "e5-large": [("qkv", 3072, 1024, 0), ("out", 1024, 1024, 2), ("ffn1", 4096, 1024, 1), ("ffn2", 1024, 4096, 2)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="bge-base,e5-large")
    ap.add_argument("--variants", default="t3,t10,lt,torch")
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="comma list of GEMM names to keep (e.g. ffn1)")
    a = ap.parse_args()
    from codename_symbiont_amd.ops import kernels as K
    from codename_symbiont_amd.ops._ext import hip

    g = torch.Generator(device="cuda").manual_seed(0)
    for model in a.models.split(","):
        for name, n, k, epi in SHAPES[model]:
            if a.only and name not in a.only.split(","):
                continue
            x = torch.randn(a.m, k, device="cuda", generator=g).bfloat16()
            w = (torch.randn(n, k, device="cuda", generator=g) / math.sqrt(k)).bfloat16()
            b = torch.randn(n, device="cuda", generator=g)
            r = torch.randn(a.m, n, device="cuda", generator=g).bfloat16() if epi >= 2 else None
            y = torch.empty(a.m, n, device="cuda", dtype=torch.bfloat16)

            def mk(v):
                if v == "torch":
                    return lambda: torch.matmul(x, w.t(), out=y)
                if v == "lt":
                    return lambda: (hip().gemm_config(128, 10, 8),
                                    hip().gemm_lt_config(1), K.gemm(x, w, b, epi, r, out=y),
                                    hip().gemm_lt_config(0))
                t, _, gm = v[1:].partition("g")     # tN or tNgG (grouped tile order, G rows)
                t, gm = int(t), int(gm or 8)
                return lambda: (hip().gemm_config(128, t, gm), hip().gemm_lt_config(0),
                                K.gemm(x, w, b, epi, r, out=y))

            fns = {v: mk(v) for v in a.variants.split(",")}
            times = {v: [] for v in fns}
            for f in fns.values():
                for _ in range(3):
                    f()
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for v, f in fns.items():
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    f()
                    s.record()
                    for _ in range(a.iters):
                        f()
                    e.record()
                    torch.cuda.synchronize()
                    times[v].append(s.elapsed_time(e) / a.iters * 1e3)
            for v, ts in times.items():
                med = statistics.median(ts)
                print(json.dumps({"model": model, "gemm": name, "m": a.m, "n": n, "k": k, "epi": epi,
                                  "variant": v, "us_med": round(med, 1), "us_min": round(min(ts), 1),
                                  "TFLOPs": round(2 * a.m * n * k / med / 1e6)}), flush=True)
    hip().gemm_config(128, 3, 8)
    hip().gemm_lt_config(1)


if __name__ == "__main__":
    main()
