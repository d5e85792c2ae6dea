#!/usr/bin/env python3
"""Diagnose the MX-fp4 tier at D = 768 on the exactness test's data (tests/test_kernels_gpu.py
test_index_pruned_search_mx4_tier_is_exact): a 1M-row random shard plus a 5000-row near-duplicate
crowd, near queries.  Prints, for the queries whose result is wrong, where each missing top-k row
was lost: T and thr4 against the true k-th score, the row's fp4 estimate against thr4 (decoded
images), its block's route flag, and whether the scan emitted it."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from codename_symbiont_amd.index.shard import HbmIndexShard, STREAM_SUB  # noqa: E402
from codename_symbiont_amd.ops import reference as R  # noqa: E402


def main():
    D, nq, k = int(os.environ.get("D", "768")), 256, 10
    dev = torch.device("cuda")
    n = (1 << 20) + 555
    g = torch.Generator(device=dev).manual_seed(12)
    shard = HbmIndexShard(D, n + 8192, prune="i8")
    shard.fill_random(n, seed=6)
    c = torch.nn.functional.normalize(torch.randn(D, device=dev, generator=g), dim=0)
    crowd = c + 0.1 * torch.randn(5000, D, device=dev, generator=g) / math.sqrt(D)
    shard.append_f32(crowd)
    rows = shard.unit_rows().float()
    q = c + 0.1 * torch.randn(nq, D, device=dev, generator=g) / math.sqrt(D)
    q = torch.nn.functional.normalize(q, dim=-1).bfloat16()
    shard.mq_stats = True
    ts, ti = R.topk_ref(rows, q, k)
    ctx = shard._pruned_begin(q, k, None)
    out_s, out_i = shard._pruned_end(ctx)
    torch.cuda.synchronize()
    m4 = ctx["mx4"]
    print("nv", int(m4["nv"]), "dense", int(ctx["dense"]), "geo", ctx["geo"])
    T, thr4 = ctx["T"], m4["thr4"]
    kth = ts[:, k - 1]
    print("T <= kth all:", bool((T <= kth + 1e-6).all()), "max T - kth", float((T - kth).max()))
    bad = ((out_s - ts).abs() > 2e-5).any(1)
    print("wrong queries", int(bad.sum()), "of", nq)
    last = shard._pruned_last
    cnt, ci = last["cnt"], last["ci"]
    print("cand counts: min", int(cnt.min()), "max", int(cnt.max()), "cap", last["cap"])
    n_rows = shard.visible
    img = shard.img_mx4
    x4 = R.stream_mx4_decode(img[: (n_rows + STREAM_SUB - 1) // STREAM_SUB], n_rows, D)
    q4t = R.stream_mx4_query_decode(m4["q4"], m4["qs4"])
    blk = ctx["blk"]
    n_rblk = ctx["geo"][2]
    rpb = ctx["geo"][1]
    skip = blk[2 + n_rblk:].cpu()
    print("blocks routed:", int(skip.sum()), "list", blk[: 2 + int(blk[0])].tolist()[:12])
    for qi in bad.nonzero().flatten().tolist()[:4]:
        cand = set(ci[qi, : min(int(cnt[qi]), last["cap"])].tolist())
        est = (x4 @ q4t[qi].float())
        print(f"q{qi}: T {float(T[qi]):.5f} kth {float(kth[qi]):.5f} thr4 {float(thr4[qi]):.5f} "
              f"cnt {int(cnt[qi])} emitted>=thr4 {int((est >= thr4[qi]).sum())}")
        for r in ti[qi].tolist():
            if r in cand:
                continue
            b = r // rpb
            print(f"   missing row {r} score {float(rows[r] @ q[qi].float()):.5f} est {float(est[r]):.5f} "
                  f"block {b} skip {int(skip[b])}")


if __name__ == "__main__":
    main()
