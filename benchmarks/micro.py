#!/usr/bin/env python3
"""Kernel micro-benchmarks on one MI355X (interleaved A/B rounds in ONE process).

  python benchmarks/micro.py scan   [--rows 100000000] [--nq 256]   fused scan+top-k variants
  python benchmarks/micro.py gemm                                   encoder GEMMs vs torch (hipBLASLt)
  python benchmarks/micro.py encoder [--batch 256 --seq 128]        whole encoder forward
  python benchmarks/micro.py attn                                   varlen attention

Prints one JSON line per measurement (median / min over rounds).
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


def timeit(fn, iters=10):
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def ab(variants: dict, rounds=5, iters=10):
    for f in variants.values():  # warm
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for k, f in variants.items():
            res[k].append(timeit(f, iters))
    return {k: (statistics.median(v), min(v)) for k, v in res.items()}


def cmd_scan(a):
    from codename_symbiont_amd.index.shard import HbmIndexShard, _round_up
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    D = a.dim
    shard = HbmIndexShard(D, a.rows, device="cuda")
    shard.fill_random(a.rows, seed=1)
    q = torch.nn.functional.normalize(torch.randn(a.nq, D, device="cuda"), dim=-1).bfloat16()
    h = hip()
    kmax = 16
    lists, qpb = h.topk_geometry(D, kmax)
    n_qblk = math.ceil(a.nq / qpb)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    out = {}
    for mult in (1, 2):
        n_rblk = max(1, round(ncu * mult / n_qblk))
        rpb = _round_up(math.ceil(a.rows / n_rblk), 64)
        n_rblk = math.ceil(a.rows / rpb)
        ncand = n_rblk * lists * kmax
        cs = torch.empty(a.nq, ncand, device="cuda")
        ci = torch.empty(a.nq, ncand, dtype=torch.int32, device="cuda")
        st = stream_handle()
        variants = {}
        for ns in ((2, 3) if D == 384 else (0,)):
            for aux in (0, 2):
                for xcd in ((0, 1) if n_qblk > 1 else (0,)):
                    def f(ns=ns, aux=aux, xcd=xcd):
                        h.index_scan(shard.rows.data_ptr(), a.rows, D, rpb, n_rblk, q.data_ptr(),
                                     a.nq, kmax, cs.data_ptr(), ci.data_ptr(), st, ns, aux, 0, xcd)
                    variants[f"blk{mult}x_ns{ns}_aux{aux}_xcd{xcd}"] = f
        if mult == 1:
            def srch(seed):
                shard.seed_threshold = seed
                return shard.search(q, 10)
            ref = srch(False)
            got = srch(True)
            out["seeded_matches_unseeded"] = bool(torch.equal(ref[1], got[1]))
            variants["search_k10_seeded"] = lambda: srch(True)
            variants["search_k10_unseeded"] = lambda: srch(False)
        r = ab(variants, rounds=a.rounds, iters=a.iters)
        for k, (med, mn) in r.items():
            gbs = a.rows * D * 2 / (med / 1e3) / 1e9
            tf = 2 * a.rows * D * a.nq / (med / 1e3) / 1e12
            out[k] = dict(ms=round(med, 3), min_ms=round(mn, 3), GBps=round(gbs), TFLOPs=round(tf))
    print(json.dumps({"bench": "scan", "rows": a.rows, "dim": D, "nq": a.nq, "results": out}))


def cmd_scanmq(a):
    """512-query-per-workgroup emitting scan (index_mq.hip) vs the 256-query list kernel on the
    per-rank shape of the sharded search (rows/N x 256*N queries), seeded top-10 searches."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    D, k = 384, 10
    shard = HbmIndexShard(D, a.rows + 8192, device="cuda", prune="i8" if a.prune else None)
    if a.prune_shift:
        shard.PRUNE_TILE_SHIFT = a.prune_shift
    shard.fill_random(a.rows, seed=1)
    q = torch.nn.functional.normalize(torch.randn(a.nq, D, device="cuda"), dim=-1).bfloat16()
    if a.qmode == "near":   # bench-like: fresh embeddings appended last, queries near them
        near = torch.nn.functional.normalize(q.float() + 0.05 * torch.randn_like(q.float()), dim=-1)
        shard.append_unit(near.bfloat16())

    shard.mq_min_nq = min(shard.mq_min_nq, a.nq)

    prune = shard.prune

    def srch(mq, rsplit=True, pr=False):
        shard.scan_mq = mq
        shard.mq_rsplit = rsplit
        shard.prune = prune if pr else None
        return shard.search(q, k)

    ref = srch(False)
    got = srch(True)
    torch.cuda.synchronize()
    cnt, ovf = shard._mq_last
    ids_equal = float((ref[1] == got[1]).float().mean())
    max_score_diff = float((ref[0] - got[0]).abs().max())
    variants = {"list256": lambda: srch(False), "mq512": lambda: srch(True)}
    if prune:   # exact int8 bound-pruned scan + bf16 re-score (index_i8.hip)
        got4 = srch(True, True, True)
        torch.cuda.synchronize()
        pc, po = shard._mq_last
        ids_equal = min(ids_equal, float((ref[1] == got4[1]).float().mean()))
        max_score_diff = max(max_score_diff, float((ref[0] - got4[0]).abs().max()))
        variants["pruned_i8"] = lambda: srch(True, True, True)
        if a.nq >= 512:   # the 256-query fused form for big batches too
            def rs2():
                shard.i8_rsplit2 = True
                try:
                    return srch(True, True, True)
                finally:
                    shard.i8_rsplit2 = False
            got5 = rs2()
            torch.cuda.synchronize()
            ids_equal = min(ids_equal, float((ref[1] == got5[1]).float().mean()))
            variants["pruned_i8_rs2"] = rs2
    from codename_symbiont_amd.ops._ext import hip

    def srch_nt():   # non-temporal row stream
        hip().mq_config(2)
        try:
            return srch(True)
        finally:
            hip().mq_config(0)

    got3 = srch_nt()
    torch.cuda.synchronize()
    ids_equal = min(ids_equal, float((ref[1] == got3[1]).float().mean()))
    variants["mq_nt"] = srch_nt
    if a.nq < 512:   # the two 256-query forms: row-split 4-set ("mq512") and 2-set
        got2 = srch(True, False)
        torch.cuda.synchronize()
        ids_equal = min(ids_equal, float((ref[1] == got2[1]).float().mean()))
        max_score_diff = max(max_score_diff, float((ref[0] - got2[0]).abs().max()))
        variants["mq_2set"] = lambda: srch(True, False)
    r = ab(variants, rounds=a.rounds, iters=a.iters)
    flop = 2 * shard.visible * D * a.nq
    out = {n: dict(ms=round(m, 3), min_ms=round(mn, 3), TFLOPs=round(flop / (m / 1e3) / 1e12))
           for n, (m, mn) in r.items()}
    extra = {}
    if prune:
        extra = {"pruned_overflow": int(po.item()), "pruned_cand_mean": float(pc.float().mean()),
                 "pruned_cand_max": int(pc.max()), "i8_bounds": [float(v) for v in shard.i8_bounds]}
    print(json.dumps({"bench": "scanmq", "rows": shard.visible, "nq": a.nq, "qmode": a.qmode, **extra,
                      "ids_equal_frac": ids_equal, "max_score_diff": max_score_diff,
                      "overflow": int(ovf.item()), "cand_mean": float(cnt.float().mean()),
                      "cand_max": int(cnt.max()), "results": out}))


def cmd_scanmqabl(a):
    """index_scan_mq_kernel ablations (abl 0 full, 1 no DMA, 2 no emission test) and its in-kernel
    clock (abl 3 stamps), same thresholds and grid as shard.search."""
    from codename_symbiont_amd.index.shard import HbmIndexShard, TILE_ROWS, _round_up
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    D, k = 384, 10
    shard = HbmIndexShard(D, a.rows, device="cuda")
    shard.fill_random(a.rows, seed=1)
    q = torch.nn.functional.normalize(torch.randn(a.nq, D, device="cuda"), dim=-1).bfloat16()
    h = hip()
    n = shard.visible
    ms, sample = shard._block_sample(n)
    pre_s, _ = shard._scan(ms, q, 16, k, None, None, sample, "bf16")
    thr = pre_s[:, k - 1].contiguous() - shard.MQ_THR_MARGIN
    n_qblk = math.ceil(a.nq / h.mq_queries_per_blk(a.sets, a.rsplit))
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    n_rblk = max(1, round(ncu / n_qblk))
    rpb = _round_up(math.ceil(n / n_rblk), TILE_ROWS)
    n_rblk = math.ceil(n / rpb)
    cap = shard.MQ_CAP
    cs = torch.zeros(a.nq, cap, device="cuda")
    ci = torch.empty(a.nq, cap, dtype=torch.int32, device="cuda")
    cnt = torch.empty(a.nq, dtype=torch.int32, device="cuda")
    st = stream_handle()

    def run(abl):
        h.index_scan_mq_ablate(shard.rows.data_ptr(), n, rpb, n_rblk, q.data_ptr(), a.nq,
                               thr.data_ptr(), cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap,
                               1, st, abl, a.sets, a.rsplit)
    variants = {f"abl{m}": (lambda m=m: run(m)) for m in (0, 1, 2, 4)}
    flat = shard.rows[:n].view(torch.int64)
    variants["torch_int64_sum"] = lambda: flat.sum()   # plain streaming read of the same bytes
    r = ab(variants, rounds=a.rounds, iters=a.iters)
    flop = 2 * n * D * a.nq
    out = {nm: dict(ms=round(m, 3), TFLOPs=round(flop / (m / 1e3) / 1e12),
                    TBps=round(n * D * 2 / (m / 1e3) / 1e12, 2)) for nm, (m, _) in r.items()}
    timeit(lambda: run(3), 10)
    run(3)
    torch.cuda.synchronize()
    st_ = cs.view(-1)[: 2 * n_rblk * n_qblk].view(-1, 2).double()
    ghz = (st_[:, 0] / st_[:, 1] * 0.1).median().item()
    out["in_kernel_clock_GHz"] = round(ghz, 3)
    out["cycles_per_tile"] = round((st_[:, 0] / math.ceil(rpb / TILE_ROWS)).median().item(), 1)
    print(json.dumps({"bench": "scanmq_ablation", "rows": n, "nq": a.nq, "sets": a.sets, "rsplit": a.rsplit,
                      "n_rblk": n_rblk, "n_qblk": n_qblk, "results": out}))


def cmd_scani8abl(a):
    """Exact int8-pruned search (index_i8.hip): its parts (whole search, scan kernel, re-score)
    and the scan kernel's ablations (0 full, 1 no DMA, 2 no emission test, 4 DMA ring only) plus
    its in-kernel clock (3), on the grid and thresholds shard.search uses."""
    from codename_symbiont_amd.index.shard import HbmIndexShard, TILE_ROWS
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    D, k = 384, 10
    shard = HbmIndexShard(D, a.rows + 8192, device="cuda", prune="i8")
    shard.fill_random(a.rows, seed=1)
    q = torch.nn.functional.normalize(torch.randn(a.nq, D, device="cuda"), dim=-1).bfloat16()
    hip().i8_config(a.i8_tr, a.i8_waves)
    shard.mq_stats = True      # keeps _pruned_last (the scan's inputs and grid)
    shard.search(q, k)
    torch.cuda.synchronize()
    P = shard._pruned_last
    h, st, n = hip(), stream_handle(), shard.visible

    def scan(abl):
        h.index_scan_i8_ablate(shard.rows_i8.data_ptr(), shard.sx_i8.data_ptr(), n,
                               shard.rows_i8.shape[0], P["rows_per_blk"], P["n_rblk"],
                               P["q8"].data_ptr(), a.nq,
                               P["thr"].data_ptr(), P["cs"].data_ptr(), P["ci"].data_ptr(),
                               P["cnt"].data_ptr(), P["cap"], 1, st, abl)

    ci0, cnt0, cs0 = P["ci"].clone(), P["cnt"].clone(), torch.empty_like(P["cs"])

    def rescore():   # on the first search's candidates (the ablations overwrite P's buffers)
        h.rescore_bf16(shard.rows.data_ptr(), P["q"].data_ptr(), a.nq, D, ci0.data_ptr(),
                       cnt0.data_ptr(), P["cap"], cs0.data_ptr(), st)

    variants = {"search": lambda: shard.search(q, k), "rescore": rescore}
    variants.update({f"abl{m}": (lambda m=m: scan(m)) for m in ((0, 2, 4) if a.i8_waves == 4 else (0, 1, 2, 4))})
    r = ab(variants, rounds=a.rounds, iters=a.iters)
    out = {nm: dict(ms=round(m, 3), TBps=round(n * D / (m / 1e3) / 1e12, 2)) for nm, (m, _) in r.items()}
    cnt = cnt0
    timeit(lambda: scan(3), 10)
    scan(3)
    torch.cuda.synchronize()
    nb = P["n_rblk"] * math.ceil(a.nq / 256)
    st_ = P["cs"].view(-1)[: 2 * nb].view(-1, 2).double()
    out["in_kernel_clock_GHz"] = round((st_[:, 0] / st_[:, 1] * 0.1).median().item(), 3)
    out["cycles_per_64_rows"] = round((st_[:, 0] / math.ceil(P["rows_per_blk"] / TILE_ROWS)).median().item(), 1)
    hip().i8_config(64)
    print(json.dumps({"bench": "scani8_ablation", "rows": n, "nq": a.nq, "tile_rows": a.i8_tr, "waves": a.i8_waves,
                      "cand_mean": float(cnt.float().mean()),
                      "cand_max": int(cnt.max()), "results": out}))


def cmd_scanabl(a):
    """DMA-only vs compute-only vs full scan (D=384), plus a plain torch streaming read."""
    from codename_symbiont_amd.index.shard import HbmIndexShard, _round_up
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    D = 384
    shard = HbmIndexShard(D, a.rows, device="cuda")
    shard.fill_random(a.rows, seed=1)
    q = torch.nn.functional.normalize(torch.randn(a.nq, D, device="cuda"), dim=-1).bfloat16()
    h = hip()
    n_qblk = math.ceil(a.nq / 256)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    n_rblk = max(1, round(ncu / n_qblk))
    rpb = _round_up(math.ceil(a.rows / n_rblk), 64)
    n_rblk = math.ceil(a.rows / rpb)
    cs = torch.empty(a.nq, n_rblk * 2 * 16, device="cuda")
    ci = torch.empty(a.nq, n_rblk * 2 * 16, dtype=torch.int32, device="cuda")
    st = stream_handle()
    flat = shard.rows[:a.rows].view(torch.int64)
    pre_s, _ = shard._scan(a.rows // 64, q, 16, 10, None, None)
    thr = torch.nextafter(pre_s[:, 9].contiguous(), torch.tensor(-math.inf, device="cuda"))
    tp = thr.data_ptr() if a.seed else 0
    variants = {f"abl{m}": (lambda m=m: h.index_scan_ablate(shard.rows.data_ptr(), a.rows, rpb, n_rblk,
                                                            q.data_ptr(), a.nq, cs.data_ptr(),
                                                            ci.data_ptr(), st, m, tp)) for m in (0, 1, 2, 3, 4, 5)}
    variants["torch_int64_sum"] = lambda: flat.sum()
    # correctness: the 8-wave (abl0) and the wide 4-wave (abl3) kernels give the same merged top-k
    merged = {}
    for m in (0, 3, 4):
        variants[f"abl{m}"]()
        os_ = torch.empty(a.nq, 10, device="cuda")
        oi = torch.empty(a.nq, 10, dtype=torch.int32, device="cuda")
        h.topk_merge(cs.data_ptr(), ci.data_ptr(), a.nq, n_rblk * 2 * 16, 16, 10,
                     os_.data_ptr(), oi.data_ptr(), 0, 0, st)
        torch.cuda.synchronize()
        merged[m] = (os_.clone(), oi.clone())
    same_var = {m: bool(torch.equal(merged[0][1], merged[m][1])) for m in (3, 4)}
    r = ab(variants, rounds=a.rounds, iters=a.iters)
    out = {k: dict(ms=round(m, 3), GBps=round(a.rows * D * 2 / (m / 1e3) / 1e9)) for k, (m, _) in r.items()}
    print(json.dumps({"bench": "scan_ablation", "rows": a.rows, "nq": a.nq, "seeded": bool(a.seed), "variants_match_abl0": same_var,
                      "results": out}))


def cmd_scanstamp(a):
    """Per-segment s_memtime stamps of the D=384 scan (diagnostic builds: full, L2-source, compute)."""
    from codename_symbiont_amd.index.shard import HbmIndexShard, _round_up
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    D = 384
    shard = HbmIndexShard(D, a.rows, device="cuda")
    shard.fill_random(a.rows, seed=1)
    q = torch.nn.functional.normalize(torch.randn(a.nq, D, device="cuda"), dim=-1).bfloat16()
    h = hip()
    n_rblk = max(1, round(torch.cuda.get_device_properties(0).multi_processor_count / math.ceil(a.nq / 256)))
    rpb = _round_up(math.ceil(a.rows / n_rblk), 64)
    n_rblk = math.ceil(a.rows / rpb)
    cs = torch.zeros(a.nq, n_rblk * 2 * 16, device="cuda")
    ci = torch.empty(a.nq, n_rblk * 2 * 16, dtype=torch.int32, device="cuda")
    st = stream_handle()
    names = ["vmcnt_wait", "barrier", "chain0+dma", "pro1+topk0", "chain1", "topk1", "cyc_per_tile", "GHz"]
    out = {}
    pre_s, _ = shard._scan(a.rows // 64, q, 16, 10, None, None)
    thr = torch.nextafter(pre_s[:, 9].contiguous(), torch.tensor(-math.inf, device="cuda"))
    for m, label, tp in ((8, "full", 0), (8, "full_seeded", thr.data_ptr()), (9, "l2_source", 0),
                         (10, "compute_only", 0)):
        run = lambda: h.index_scan_ablate(shard.rows.data_ptr(), a.rows, rpb, n_rblk, q.data_ptr(), a.nq,
                                          cs.data_ptr(), ci.data_ptr(), st, m, tp)
        ms = timeit(run, 20)  # also warms the clock
        run()
        torch.cuda.synchronize()
        v = cs.view(-1)[: n_rblk * 8 * 8].view(n_rblk, 8, 8)
        med = v.median(dim=0).values  # [wave, seg]
        out[label] = dict(ms=round(ms, 3), per_wave={f"w{w}": [round(float(x), 1) for x in med[w]] for w in range(8)},
                          mean={n: round(float(v[:, :, i].mean()), 1) for i, n in enumerate(names)})
    print(json.dumps({"bench": "scan_stamps", "rows": a.rows, "segments": names, "results": out}))


def cmd_scanfp8(a):
    """fp8 (e4m3) index scan, D=1024 by default (BASELINE config #5 geometry), seeded top-10."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    D = a.dim if a.dim != 384 else 1024
    shard = HbmIndexShard(D, a.rows, device="cuda", dtype="fp8")
    shard.fill_random(a.rows, seed=1)
    q = torch.nn.functional.normalize(torch.randn(a.nq, D, device="cuda"), dim=-1).bfloat16()
    out = {}

    def run(variant, seed):
        shard.scan_variant, shard.seed_threshold = variant, seed
        return shard.search(q, 10)

    ref = run(0, False)
    vs = (0,)
    out["variants_match"] = all(torch.equal(ref[1], run(v, sd)[1]) for v in vs for sd in (0, 1))
    variants = {f"v{v}_seed{sd}": (lambda v=v, sd=sd: run(v, sd)) for v in vs for sd in (False, True)}
    # v9: the default geometry re-reading 8 tiles per row block from L2 (compute ceiling)
    variants["v9_l2src_seedTrue"] = lambda: run(9, True)
    r = ab(variants, rounds=a.rounds, iters=a.iters)
    for k, (med, mn) in r.items():
        out[k] = dict(ms=round(med, 3), GBps=round(a.rows * D / (med / 1e3) / 1e9),
                      TFLOPs=round(2 * a.rows * D * a.nq / (med / 1e3) / 1e12))
    print(json.dumps({"bench": "scan_fp8", "rows": a.rows, "dim": D, "nq": a.nq, "results": out}))


def cmd_gemm(a):
    from codename_symbiont_amd.ops import kernels as K

    M = a.batch * a.seq
    shapes = [("qkv", 1152, 384, K.EPI_BIAS), ("out+ln", 384, 384, K.EPI_RES_LN),
              ("ffn1", 1536, 384, K.EPI_GELU), ("ffn2+ln", 384, 1536, K.EPI_RES_LN),
              ("bge.qkv", 2304, 768, K.EPI_BIAS), ("bge.out+res", 768, 768, K.EPI_RES),
              ("bge.ffn1", 3072, 768, K.EPI_GELU), ("bge.ffn2+res", 768, 3072, K.EPI_RES)]
    out = {}
    for name, N, Kd, epi in shapes:
        x = torch.randn(M, Kd, device="cuda").bfloat16()
        w = (torch.randn(N, Kd, device="cuda") / math.sqrt(Kd)).bfloat16()
        b = torch.randn(N, device="cuda")
        r = torch.randn(M, N, device="cuda").bfloat16()
        g = torch.ones(N, device="cuda")
        be = torch.zeros(N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        from codename_symbiont_amd.ops._ext import hip as _hip
        rr = r if epi >= 2 else None
        var = {"torch_matmul_only": lambda: torch.matmul(x, w.t(), out=y)}
        if epi == K.EPI_RES_LN:
            tmp = torch.empty_like(y)
            var["hip_res+add_ln"] = lambda: (K.gemm(x, w, b, K.EPI_RES, rr, out=tmp),
                                             K.add_ln(tmp, None, g, be, 1e-12, out=y))
            var["hip_bm64"] = lambda: (_hip().gemm_config(64, 0), K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_bm128"] = lambda: (_hip().gemm_config(128, 3), K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_bm128_8w"] = lambda: (_hip().gemm_config(128, 3), _hip().gemm_resln_config(8),
                                           K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y),
                                           _hip().gemm_resln_config(16))
        else:
            var["hip_128x128"] = lambda: (_hip().gemm_config(128, 0, 8), K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_128x128_rowmajor"] = lambda: (_hip().gemm_config(128, 0, 0),
                                                   K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_128x128_g16"] = lambda: (_hip().gemm_config(128, 0, 16),
                                              K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_256x128_3st"] = lambda: (_hip().gemm_config(128, 1, 8),
                                              K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_128x128_8w_32x64"] = lambda: (_hip().gemm_config(128, 6, 8),
                                                   K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_128x128_8w_64x32"] = lambda: (_hip().gemm_config(128, 7, 8),
                                                   K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_128x128_16w"] = lambda: (_hip().gemm_config(128, 8, 8),
                                              K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_128x128_3st"] = lambda: (_hip().gemm_config(128, 4, 8),
                                              K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            var["hip_128x128_4st"] = lambda: (_hip().gemm_config(128, 5, 8),
                                              K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
            if N % 256 == 0:
                var["hip_256x256"] = lambda: (_hip().gemm_config(128, 2, 8),
                                              K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
                var["hip_256_8phase"] = lambda: (_hip().gemm_config(128, 9, 8),
                                                 K.gemm(x, w, b, epi, rr, g, be, 1e-12, out=y))
        res = ab(var, rounds=a.rounds, iters=a.iters)
        _hip().gemm_config(128, 3, 8)
        fl = 2 * M * N * Kd
        out[name] = {k: dict(ms=round(m, 4), TFLOPs=round(fl / (m / 1e3) / 1e12)) for k, (m, _) in res.items()}
    print(json.dumps({"bench": "gemm", "M": M, "results": out}))


def cmd_encoder(a):
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch

    cfg = get_config(a.model)
    b = synthetic_batch(cfg, a.batch, a.seq, seed=0).to("cuda")
    o1 = torch.empty(a.batch, cfg.hidden, device="cuda")
    o2 = torch.empty(a.batch, cfg.hidden, device="cuda", dtype=torch.bfloat16)
    from codename_symbiont_amd.ops._ext import hip as _hip

    encs = {p: HipEncoder(cfg, seed=0, precision=p) for p in a.precision.split(",")}
    tiles = [int(t) for t in a.tiles.split(",")]
    fw = [int(t) for t in a.fp8_waves.split(",")]
    var = {}
    mlps = [int(m) for m in a.mlp.split(",")]
    for p, e in encs.items():
        for t in tiles:
            for w, m in [(w, m) for w in (fw if p == "fp8" else fw[:1]) for m in mlps]:
                name = p + ("" if len(tiles) == 1 else f"_tile{t}") + ("" if len(fw) == 1 else f"_w{w}") \
                    + ("" if len(mlps) == 1 else f"_mlp{m}")
                # w = 256 / 257: 8-wave fp8 tiles plus the 256x256 fp8 tile wherever the bf16
                # rule takes it / where the fp8 auto rule does (the default); else no 256x256
                # t = 12: tile rule 10 + hipBLASLt for the plain K, N >= 768 projections (the
                # default route); other t: symb_gemm_config tile modes, every projection ours
                var[name] = (lambda e=e, t=t, w=w, m=m: (_hip().gemm_config(128, 10 if t == 12 else t, 8),
                                                    _hip().mlp_fused_config(m),
                                                    _hip().gemm_lt_config(1 if t == 12 else 0),
                                                    _hip().gemm_fp8_config(8 if w >= 256 else w,
                                                                           {256: 1, 257: 2}.get(w, 0)),
                                                    e.forward_packed(b, o1, o2)))
    res = ab(var, rounds=a.rounds, iters=a.iters)
    _hip().gemm_config(128, 3, 8)
    _hip().gemm_lt_config(1)
    _hip().gemm_fp8_config(8)
    _hip().mlp_fused_config(1)
    toks = a.batch * a.seq
    fl = cfg.flops_per_token(a.seq) * toks
    out = {p: dict(ms=round(m, 3), embeds_per_s=round(a.batch / (m / 1e3)),
                   TFLOPs=round(fl / (m / 1e3) / 1e12)) for p, (m, _) in res.items()}
    print(json.dumps({"bench": "encoder", "model": a.model, "batch": a.batch, "seq": a.seq,
                      "results": out}))


def cmd_latency(a):
    """Small-batch (query path) encoder latency: eager launches vs the captured hipGraph."""
    from codename_symbiont_amd.ops._ext import hip
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch

    cfg = get_config(a.model)
    enc = HipEncoder(cfg, seed=0)
    out = {}
    for B, S in ((1, 16), (1, 64), (8, 32), (32, 48)):
        b = synthetic_batch(cfg, B, S, seed=1).to("cuda")
        r = ab({"eager": lambda: enc.forward_packed(b), "graph": lambda: enc.forward_graphed(b),
                "eager_no_small_m_ring": lambda: (hip().gemm_config(128, 7, 8), enc.forward_packed(b),
                                                  hip().gemm_config(128, 3, 8))},
               rounds=a.rounds, iters=50)
        out[f"B{B}xS{S}"] = {k: round(m * 1e3, 1) for k, (m, _) in r.items()}
    print(json.dumps({"bench": "encoder_latency_us", "model": a.model, "results": out}))


def cmd_gemmfp8(a):
    """e4m3 GEMM (row quantiser + fp8 MFMA GEMM) vs the bf16 GEMM on encoder shapes."""
    from codename_symbiont_amd.models.encoder import quant_weight_fp8
    from codename_symbiont_amd.ops import kernels as K
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    M = a.batch * a.seq
    shapes = [("e5.qkv", 3072, 1024, 0), ("e5.out", 1024, 1024, 2), ("e5.ffn1", 4096, 1024, 1),
              ("e5.ffn2", 1024, 4096, 2), ("minilm.ffn1", 1536, 384, 1)]
    out = {}
    st = stream_handle()
    for name, N, Kd, epi in shapes:
        x = torch.randn(M, Kd, device="cuda").bfloat16()
        w = (torch.randn(N, Kd, device="cuda") / math.sqrt(Kd)).bfloat16()
        bias = torch.randn(N, device="cuda")
        r = torch.randn(M, N, device="cuda").bfloat16()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        a8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
        sa = torch.empty(M, device="cuda")
        w8, sw = quant_weight_fp8(w)
        h = hip()
        rr = r.data_ptr() if epi == 2 else 0

        def f8(with_quant=True):
            if with_quant:
                h.quant_rows_fp8(x.data_ptr(), Kd, a8.data_ptr(), Kd, sa.data_ptr(), M, Kd, st)
            h.gemm_fp8(epi, a8.data_ptr(), Kd, w8.data_ptr(), Kd, sa.data_ptr(), sw.data_ptr(),
                       bias.data_ptr(), rr, N, y.data_ptr(), N, M, N, Kd, st)
        # MX mode as the encoder uses it: GELU layers emit MX fp8 (EPI_GELU_MX8), the others take
        # an MX-scaled A (E8M0 per 32 k through the MFMA's scale operand), no quantiser pass
        aexp = torch.full((M, Kd // 32), 127, dtype=torch.uint8, device="cuda")
        y8 = torch.empty(M, N, dtype=torch.uint8, device="cuda")
        yexp = torch.empty(M, N // 32, dtype=torch.uint8, device="cuda")

        def fmx():
            if epi == 1:
                h.gemm_fp8(4, a8.data_ptr(), Kd, w8.data_ptr(), Kd, sa.data_ptr(), sw.data_ptr(),
                           bias.data_ptr(), 0, 0, y8.data_ptr(), N, M, N, Kd, st,
                           cscale=yexp.data_ptr())
            else:
                h.gemm_fp8(epi, a8.data_ptr(), Kd, w8.data_ptr(), Kd, 0, sw.data_ptr(),
                           bias.data_ptr(), rr, N, y.data_ptr(), N, M, N, Kd, st,
                           ascale=aexp.data_ptr())
        res = ab({"bf16": lambda: K.gemm(x, w, bias, epi, r if epi == 2 else None, out=y),
                  "fp8_with_quant": lambda: f8(True), "fp8_gemm_only": lambda: f8(False),
                  "fp8_gemm_only_rowmajor": lambda: (h.gemm_config(128, 0, 0), f8(False),
                                                     h.gemm_config(128, 3, 8)),
                  "fp8_mx": lambda: fmx(),
                  "fp8_mx_4w": lambda: (h.gemm_fp8_config(4, 0), fmx(), h.gemm_fp8_config(8)),
                  "fp8_gemm_only_4w": lambda: (h.gemm_fp8_config(4, 0), f8(False), h.gemm_fp8_config(8)),
                  "fp8_mx_128": lambda: (h.gemm_fp8_config(8, 0), fmx(), h.gemm_fp8_config(8)),
                  "fp8_mx_256": lambda: (h.gemm_fp8_config(8, 1), fmx(), h.gemm_fp8_config(8)),
                  "fp8_gemm_only_256": lambda: (h.gemm_fp8_config(8, 1), f8(False), h.gemm_fp8_config(8))},
                 rounds=a.rounds, iters=a.iters)
        fl = 2 * M * N * Kd
        out[name] = {k: dict(ms=round(m, 4), TFLOPs=round(fl / (m / 1e3) / 1e12)) for k, (m, _) in res.items()}
    print(json.dumps({"bench": "gemm_fp8", "M": M, "results": out}))


def cmd_attn(a):
    from codename_symbiont_amd.ops import kernels as K

    nh, hd = 12, a.head_dim
    cu = torch.arange(0, (a.batch + 1) * a.seq, a.seq, dtype=torch.int32, device="cuda")
    qkv = torch.randn(a.batch * a.seq, 3 * nh * hd, device="cuda").bfloat16()
    out = torch.empty(a.batch * a.seq, nh * hd, device="cuda", dtype=torch.bfloat16)
    from codename_symbiont_amd.ops._ext import hip

    def run(w, kv, x):
        hip().attention_config(w, kv, x)
        return K.attention(qkv, cu, a.seq, nh, hd, out=out)
    res = ab({f"waves{w}_kvt{kv}_xcd{x}": (lambda w=w, kv=kv, x=x: run(w, kv, x))
              for w in (4, 8) for kv in (64, 128) for x in (0, 1, 2)}, a.rounds, a.iters)
    hip().attention_config(8, 64, 2)
    fl = 4 * a.batch * nh * a.seq * a.seq * hd
    print(json.dumps({"bench": "attn", "head_dim": hd, "seq": a.seq, "results": {
        k: {"ms": round(m, 4), "TFLOPs": round(fl / (m / 1e3) / 1e12)} for k, (m, _) in res.items()}}))


def cmd_prefilter(a):
    """Exact bf16 scan vs fp8 prefilter + exact bf16 rescore on the SAME rows and queries:
    time per search, recall@k of the prefilter against the exact scan, and whether every returned
    score is the exact bf16 cosine.  --qmode random: isotropic queries; --qmode near: queries are
    noisy copies of index rows (a real corpus: true neighbours well above the bulk)."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    k = 10
    sh = HbmIndexShard(a.dim, a.rows, device="cuda", prefilter="fp8")
    sh.fill_random(a.rows, seed=3)
    g = torch.Generator(device="cuda").manual_seed(4)
    q = torch.randn(a.nq, a.dim, device="cuda", generator=g)
    if a.qmode == "near":
        idx = torch.randint(0, a.rows, (a.nq,), device="cuda", generator=g)
        q = sh.rows[idx].float() + 0.6 * q / math.sqrt(a.dim)
    q = torch.nn.functional.normalize(q, dim=-1).bfloat16()

    def exact():
        sh.prefilter = None
        try:
            return sh.search(q, k)
        finally:
            sh.prefilter = "fp8"

    res = ab({"exact_bf16": exact, "prefilter_fp8": lambda: sh.search(q, k)}, rounds=a.rounds,
             iters=a.iters)
    es, ei = exact()
    ps, pi = sh.search(q, k)
    torch.cuda.synchronize()
    hits = sum(len(set(pi[i].tolist()) & set(ei[i].tolist())) for i in range(a.nq))
    true = torch.stack([(q[i].float() * sh.rows[pi[i].long()].float()).sum(-1) for i in range(a.nq)])
    print(json.dumps({"bench": "prefilter", "rows": a.rows, "dim": a.dim, "nq": a.nq, "k": k,
                      "qmode": a.qmode,
                      "ms": {n: round(m, 3) for n, (m, _) in res.items()},
                      "recall_at_k": round(hits / (a.nq * k), 5),
                      "max_abs_score_err_vs_exact_recompute": float((ps - true).abs().max()),
                      "top1_equal_frac": float((pi[:, 0] == ei[:, 0]).float().mean())}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["scan", "scanmq", "scanmqabl", "scani8abl", "scanabl", "scanstamp", "scanfp8", "gemm", "encoder", "attn", "latency", "gemmfp8", "prefilter"])
    ap.add_argument("--qmode", choices=["random", "near"], default="random", help="prefilter: query kind")
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--head-dim", type=int, default=32)
    ap.add_argument("--model", default="minilm-l6")
    ap.add_argument("--seed", type=int, default=1, help="scanabl: seed per-query thresholds")
    ap.add_argument("--precision", default="bf16", help="encoder: comma list of bf16,fp8")
    ap.add_argument("--mlp", default="1", help="encoder: comma list of mlp_fused_config values "
                    "(1: the fused 384-wide FFN block, 2: + the out-projection, 0: two GEMMs)")
    ap.add_argument("--tiles", default="3", help="encoder: comma list of gemm_config tile modes "
                    "(3 = the default auto tiles, 10 = round-3 auto, 12 = round-3 default with hipBLASLt)")
    ap.add_argument("--fp8-waves", default="8", help="encoder: comma list of fp8 GEMM wave counts")
    ap.add_argument("--sets", type=int, default=4, help="scanmqabl: 16-query sets per wave (2 or 4)")
    ap.add_argument("--rsplit", type=int, default=1, help="scanmqabl: waves per query group (1, 2)")
    ap.add_argument("--prune", action="store_true", help="scanmq: also the exact int8-pruned search")
    ap.add_argument("--prune-shift", type=int, default=0,
                    help="scanmq --prune: threshold sample 1 tile in 2^shift (0 = shard default)")
    ap.add_argument("--i8-tr", type=int, default=64, help="scani8abl: int8 scan tile rows (64, 128)")
    ap.add_argument("--i8-waves", type=int, default=8, help="scani8abl: int8 scan waves per workgroup (8, 4)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    {"scan": cmd_scan, "scanmq": cmd_scanmq, "scanmqabl": cmd_scanmqabl, "scani8abl": cmd_scani8abl, "scanabl": cmd_scanabl, "scanstamp": cmd_scanstamp, "scanfp8": cmd_scanfp8, "gemm": cmd_gemm, "encoder": cmd_encoder, "attn": cmd_attn, "latency": cmd_latency, "gemmfp8": cmd_gemmfp8, "prefilter": cmd_prefilter}[a.cmd](a)


if __name__ == "__main__":
    main()
