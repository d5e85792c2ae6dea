"""Small-batch encoder forwards in a loop, for a rocprofv3 kernel trace of the query path.

    rocprofv3 --kernel-trace --stats -d gpurun_out/lat -- python benchmarks/lat_trace.py --b 1 --s 16

Prints the host-timed eager latency (us per forward, synchronised) as one JSON line.
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
    ap.add_argument("--model", default="minilm-l6")
    ap.add_argument("--b", type=int, default=1)
    ap.add_argument("--s", type=int, default=16)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--skinny-max-m", type=int, default=256,
                    help="largest M of the small-M split-K GEMM path (0: tiled GEMMs only)")
    ap.add_argument("--nw8-max-kg", type=int, default=8,
                    help="8-wave small-M workgroups for 4 < K/128 <= this (gemm_skinny_nw8)")
    ap.add_argument("--nw8-min-wgs", type=int, default=128,
                    help="... and above that K for M > 64 while the grid keeps this many workgroups")
    ap.add_argument("--graph", action="store_true",
                    help="replay the bucketed hipGraph (HipEncoder.forward_graphed) instead of eager")
    a = ap.parse_args()
    from codename_symbiont_amd.ops._ext import hip

    hip().gemm_skinny_config(a.skinny_max_m)
    hip().gemm_skinny_nw8(a.nw8_max_kg, a.nw8_min_wgs)
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch

    cfg = get_config(a.model)
    enc = HipEncoder(cfg, seed=0)
    b = synthetic_batch(cfg, a.b, a.s, seed=1).to("cuda")
    fwd = enc.forward_graphed if a.graph else enc.forward_packed
    for _ in range(20):
        fwd(b)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        fwd(b)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(json.dumps({"bench": "encoder_latency_us", "model": a.model, "B": a.b, "S": a.s,
                      "tokens": int(b.num_tokens), "skinny_max_m": a.skinny_max_m, "nw8_max_kg": a.nw8_max_kg, "nw8_min_wgs": a.nw8_min_wgs,
                      "graph": a.graph,
                      "p50_us": round(ts[len(ts) // 2] * 1e6, 1),
                      "p10_us": round(ts[len(ts) // 10] * 1e6, 1)}))


if __name__ == "__main__":
    main()
