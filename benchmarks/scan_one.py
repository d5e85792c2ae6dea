#!/usr/bin/env python3
"""Repeat the pruned search's full-shard first-pass scan on the inputs one real search prepared --
the target of timing A/Bs and rocprofv3 --pmc passes (benchmarks/pmc_kernel.py --match scan).

    python benchmarks/scan_one.py [--rows 25000000] [--nq 256] [--corpus random] [--iters 10]
                                  [--tier i8|mx4|mx6] [--queries heldout|self]

The shard's scan is the stream scan (index_stream.hip) unless SYMB_PRUNE_STREAM=0 (the round-4
LDS-ring scan, index_i8.hip).  --tier mx4 times the MX-fp4 first tier on the same block grid with
the thresholds the tier choice computed (--queries self: stored rows as queries; near: near-duplicate queries, whose sets the centroid
test skips; both at the headline's fp4 threshold 0.74).  --tier mx6 times the MX-fp6 middle tier
(SYMB_PRUNE_MX6) at the thresholds its tier choice computed.
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
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--corpus", default="random")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tier", choices=["i8", "mx4", "mx6"], default="i8")
    ap.add_argument("--queries", choices=["heldout", "self", "near"], default="heldout")
    ap.add_argument("--ab", default="",
                    help="stream forms timed in one process, interleaved: comma list of "
                         "ablation[:centroid] (ablation: stream_config; centroid 0 = the MX-fp4 "
                         "centroid test off), e.g. 0:1,0:0")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--thr-add", type=float, default=0.0,
                    help="added to the scan's thresholds (e.g. 10: no row emits -- kernel-only timing)")
    a = ap.parse_args()
    from codename_symbiont_amd.index.shard import STREAM_SUB, HbmIndexShard
    from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    h, st = hip(), stream_handle()
    gen = CorpusGen(a.corpus, a.dim, "cuda")
    shard = HbmIndexShard(a.dim, a.rows + 8192, device="cuda", prune="i8")
    t0 = time.perf_counter()
    fill_corpus(shard, gen, a.rows, seed=1)
    torch.cuda.synchronize()
    fill_s = time.perf_counter() - t0
    if a.queries == "self":
        idx = torch.randint(0, a.rows, (a.nq,), device="cuda")
        q = shard.rows[idx].clone()
    elif a.queries == "near":   # near-duplicate queries (cos ~0.99), like the headline's embeddings
        g = torch.Generator(device="cuda").manual_seed(7)
        c = torch.nn.functional.normalize(torch.randn(a.dim, device="cuda", generator=g), dim=0)
        q = torch.nn.functional.normalize(
            c + 0.1 * torch.randn(a.nq, a.dim, device="cuda", generator=g) / a.dim ** 0.5, dim=-1).bfloat16()
    else:
        q = gen.unit(a.nq, seed=7).bfloat16()
    shard.mq_stats = True
    shard.search(q, 10)
    torch.cuda.synchronize()
    P, n = shard._pruned_last, shard.visible
    rsplit = 2 if a.nq < 512 else 1
    heavy = P["heavy"]
    m4, m6 = P["m4"], P.get("m6")
    if a.tier == "mx4" and m4 is None:
        raise SystemExit("no MX-fp4 tier on this shard")
    if a.tier == "mx6" and m6 is None:
        raise SystemExit("no MX-fp6 tier on this shard")
    if a.tier == "mx4" and a.queries in ("self", "near"):
        # the headline's batches take the fp4 tier because their k-th scores sit near 0.99 (fresh
        # near-duplicate embeddings): T - margin4 ~ 0.74.  Stored random rows as queries have
        # k-th scores ~0.2 (only the row itself scores high), for which the tier is never chosen;
        # time the kernel at the headline's threshold instead
        m4["thr4"].fill_(0.74)
    if a.tier == "mx6" and a.queries in ("self", "near"):
        m6["thr6"].fill_(0.74)   # (kernel timing at the headline's threshold, as for mx4)
    if a.thr_add:
        for t in (P["thr"], m4 and m4.get("thr4"), m6 and m6.get("thr6")):
            if t is not None:
                t.add_(a.thr_add)
    nbytes = 0

    def scan():
        if a.tier == "mx6":
            P["cnt"].zero_()
            h.index_scan_stream(shard.img_mx6.data_ptr(), n, shard.img_mx6.shape[0] * STREAM_SUB,
                                P["rows_per_blk"], P["n_rblk"], m6["q6"].data_ptr(),
                                m6["qs6"].data_ptr(), a.nq, m6["thr6"].data_ptr(),
                                P["cs"].data_ptr(), P["ci"].data_ptr(), P["cnt"].data_ptr(),
                                P["cap"], 1, st, dim=a.dim, form=2)
        elif a.tier == "mx4":
            P["cnt"].zero_()
            if shard.img_mx4 is not None:
                h.index_scan_stream(shard.img_mx4.data_ptr(), n, shard.img_mx4.shape[0] * STREAM_SUB,
                                    P["rows_per_blk"], P["n_rblk"], m4["q4"].data_ptr(),
                                    m4["qs4"].data_ptr(), a.nq, m4["thr4"].data_ptr(),
                                    P["cs"].data_ptr(), P["ci"].data_ptr(), P["cnt"].data_ptr(),
                                    P["cap"], 1, st, dim=a.dim, form=1,
                                    **(shard._cent_args(m4) if cent[0] else {}))
            else:
                h.index_scan_i8(shard.rows_mx4.data_ptr(), shard.sc_mx4.data_ptr(), n,
                                shard.rows_mx4.shape[0], P["rows_per_blk"], P["n_rblk"],
                                m4["q4"].data_ptr(), a.nq, m4["thr4"].data_ptr(), P["cs"].data_ptr(),
                                P["ci"].data_ptr(), P["cnt"].data_ptr(), P["cap"], 1, st, rsplit,
                                dim=a.dim, sq=m4["qs4"].data_ptr(), form=1)
        elif shard.img_i8 is not None and not heavy:
            h.index_scan_stream(shard.img_i8.data_ptr(), n, shard.img_i8.shape[0] * STREAM_SUB,
                                P["rows_per_blk"], P["n_rblk"], P["q8"].data_ptr(), 0, a.nq,
                                P["thr"].data_ptr(), P["cs"].data_ptr(), P["ci"].data_ptr(),
                                P["cnt"].data_ptr(), P["cap"], 1, st, dim=a.dim, form=0)
        else:
            h.index_scan_i8(shard.rows_i8.data_ptr(), shard.sx_i8.data_ptr(), n,
                            shard.rows_i8.shape[0], P["rows_per_blk"], P["n_rblk"],
                            P["q8"].data_ptr(), a.nq, P["thr"].data_ptr(), P["cs"].data_ptr(),
                            P["ci"].data_ptr(), P["cnt"].data_ptr(), P["cap"], 1, st, rsplit,
                            dim=a.dim, heavy=heavy, sq=P["sq"].data_ptr() if heavy else 0)

    if a.tier == "mx6":
        nbytes, kernel = shard.img_mx6.shape[1] / STREAM_SUB, "stream-mx6"
    elif a.tier == "mx4":
        nbytes = (shard.img_mx4.shape[1] / STREAM_SUB if shard.img_mx4 is not None
                  else a.dim // 2 + 16)
        kernel = "stream-mx4" if shard.img_mx4 is not None else "ldsring-mx4"
    elif shard.img_i8 is not None and not heavy:
        nbytes, kernel = shard.img_i8.shape[1] / STREAM_SUB, "stream-i8"
    else:
        nbytes, kernel = shard.rows_i8.shape[1] + 4, "ldsring-" + ("split" if heavy else "i8")
    forms = [tuple(int(x) for x in f.split(":")) for f in a.ab.split(",")] if a.ab else [None]
    cent = [True]   # the MX-fp4 centroid test (a 5th form field: 0 = off)
    times = {f: [] for f in forms}
    for _ in range(a.rounds if a.ab else 1):
        for f in forms:
            if f is not None:
                h.stream_config(f[0])
                cent[0] = len(f) < 2 or bool(f[1])
            scan()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                scan()
            torch.cuda.synchronize()
            times[f].append((time.perf_counter() - t0) * 1e3 / a.iters)
    if a.ab:
        h.stream_config(0)
    for f, ts in times.items():
        ms = sorted(ts)[len(ts) // 2]
        print(json.dumps({"bench": "scan_one", "kernel": kernel, "form": f, "rows": n, "nq": a.nq,
                          "dim": a.dim, "corpus": a.corpus, "queries": a.queries,
                          "image": "split" if heavy else "plain",
                          "ms": round(ms, 3), "TBps": round(n * nbytes / ms / 1e9, 2),
                          "n_rblk": P["n_rblk"], "rows_per_blk": P["rows_per_blk"],
                          "cand_mean": round(float(P["cnt"].float().mean()), 1),
                          "cand_max": int(P["cnt"].max()), "fill_s": round(fill_s, 1),
                          "tier_flag": None if shard._tier_last is None else int(shard._tier_last.item())}),
              flush=True)


if __name__ == "__main__":
    main()
