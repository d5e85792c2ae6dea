#!/usr/bin/env python3
"""Run ONE encoder GEMM configuration repeatedly (for rocprofv3 --pmc / kernel-trace passes).

    python benchmarks/gemm_one.py --m 32768 --n 3072 --k 768 --epi 1 --tile 3 --iters 50
    tile: symb_gemm_config tile mode (3 = auto with the 256x192 tile, 10 = round-3 auto,
    2 = 256x256 wherever N % 256 == 0);
    --torch runs torch.matmul (hipBLASLt) on the same operands instead.
Prints one JSON line: ms per call and TFLOP/s.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--n", type=int, default=3072)
    ap.add_argument("--k", type=int, default=768)
    ap.add_argument("--epi", type=int, default=0)
    ap.add_argument("--tile", type=int, default=3)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--lt", type=int, default=0,
                    help="hipBLASLt route for plain projections (gemm_lt_config: 0 off, 1 auto)")
    a = ap.parse_args()
    from codename_symbiont_amd.ops import kernels as K
    from codename_symbiont_amd.ops._ext import hip

    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(a.m, a.k, device="cuda", generator=g).bfloat16()
    w = (torch.randn(a.n, a.k, device="cuda", generator=g) / math.sqrt(a.k)).bfloat16()
    b = torch.randn(a.n, device="cuda", generator=g)
    r = torch.randn(a.m, a.n, device="cuda", generator=g).bfloat16() if a.epi >= 2 else None
    y = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
    hip().gemm_config(128, a.tile, 8)
    hip().gemm_lt_config(a.lt)
    f = (lambda: torch.matmul(x, w.t(), out=y)) if a.torch else (lambda: K.gemm(x, w, b, a.epi, r, out=y))
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    print(json.dumps({"lt": a.lt, "m": a.m, "n": a.n, "k": a.k, "epi": a.epi, "tile": a.tile, "torch": a.torch,
                      "ms": round(ms, 4), "TFLOPs": round(2 * a.m * a.n * a.k / ms / 1e9)}))


if __name__ == "__main__":
    main()
