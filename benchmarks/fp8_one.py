#!/usr/bin/env python3
"""Repeat the fp8 (e4m3) list scan of config #5 (index_fp8.hip) on one shard -- the target of
rocprofv3 --pmc passes (benchmarks/pmc_kernel.py --match index_scan_fp8).

    python benchmarks/fp8_one.py [--rows 25000000] [--dim 1024] [--nq 256] [--variant 0] [--iters 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=25_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--seed-threshold", type=int, default=1)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--check", type=int, default=0, help="compare ids / scores with variant 0")
    a = ap.parse_args()
    from codename_symbiont_amd.index.shard import HbmIndexShard

    shard = HbmIndexShard(a.dim, a.rows, device="cuda", dtype="fp8")
    shard.fill_random(a.rows, seed=1)
    shard.seed_threshold = bool(a.seed_threshold)
    g = torch.Generator(device="cuda").manual_seed(5)
    q = torch.nn.functional.normalize(torch.randn(a.nq, a.dim, device="cuda", generator=g),
                                      dim=-1).bfloat16()
    match = None
    if a.check:   # the default kernel's answer, for the exact A/B forms
        shard.scan_variant = 0
        ref = shard.search(q, 10)
        shard.scan_variant = a.variant
        got = shard.search(q, 10)
        match = bool(torch.equal(ref[1], got[1]) and torch.equal(ref[0], got[0]))
    shard.scan_variant = a.variant
    shard.search(q, 10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        shard.search(q, 10)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.iters * 1e3
    print(json.dumps({"bench": "fp8_one", "rows": a.rows, "dim": a.dim, "nq": a.nq,
                      "variant": a.variant, "ms": round(ms, 3), "matches_v0": match,
                      "GBps": round(a.rows * a.dim / (ms / 1e3) / 1e9)}))


if __name__ == "__main__":
    main()
