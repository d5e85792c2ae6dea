#!/usr/bin/env python3
"""Diagnose the MX-fp6 tier choice (mx4_select_kernel stage 1) on the tier test's data: a 1M-row
random shard plus a 3000-row near-duplicate crowd, random held-out queries.  Prints the margins,
T, the select's band estimate per query (recomputed in torch from the same exact scores) against
its limit, and the fp6 scan's actual candidate counts at thr6."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from codename_symbiont_amd.index.shard import HbmIndexShard, STREAM_SUB, TILE_ROWS  # noqa: E402
from codename_symbiont_amd.ops._ext import hip, stream_handle  # noqa: E402


def q(t, p):
    return round(float(torch.quantile(t.float(), p)), 5)


def main():
    D, nq, k = int(os.environ.get("D", "384")), 256, 10
    n = int(os.environ.get("ROWS", str((1 << 20) + 555)))
    os.environ["SYMB_PRUNE_MX6"] = "1"
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(13)
    shard = HbmIndexShard(D, n + 8192, prune="i8")
    shard.fill_random(n, seed=7)
    c = torch.nn.functional.normalize(torch.randn(D, device=dev, generator=g), dim=0)
    shard.append_f32(c + 0.1 * torch.randn(3000, D, device=dev, generator=g) / math.sqrt(D))
    qq = torch.nn.functional.normalize(torch.randn(nq, D, device=dev, generator=g), dim=-1).bfloat16()
    print("bounds i8", shard.i8_bounds.tolist(), "mx4", shard.mx4_bounds.tolist(),
          "mx6", shard.mx6_bounds.tolist())
    ctx = shard._pruned_begin(qq, k, None)
    torch.cuda.synchronize()
    m6 = ctx["mx6"]
    T = ctx["T"]
    _, _, m8 = shard.prune_query_image(qq)
    mg6 = m6["m6"]
    print("flag", int(m6["nv"].item()), "T", q(T, 0.5), "m8", q(m8, 0.5), "m6", q(mg6, 0.5),
          "thr6", q(m6["thr6"], 0.5))
    # the select's estimate: exact scores of every 4th seed tile x rate + tail rows in the band
    sc = (qq.float() @ shard.unit_rows()[: shard.visible].float().t())
    lo, hi = T - mg6, T - m8
    band_all = ((sc >= lo[:, None]) & (sc < hi[:, None])).sum(1)
    above = (sc >= (T - mg6)[:, None]).sum(1)
    print(json.dumps({"band_true_median": q(band_all, 0.5), "band_true_max": int(band_all.max()),
                      "rows_above_thr6_median": q(above, 0.5), "rows_above_thr6_max": int(above.max()),
                      "limit": shard.MX6_LIMIT_FRAC * shard.PRUNE_CAP}))
    m6["nv"].fill_(1)          # force the fp6 tier: its real candidate counts
    shard.mq_stats = True
    out = shard._pruned_end(ctx)
    torch.cuda.synchronize()
    cnt = shard._pruned_last["cnt"]
    print(json.dumps({"fp6_cand_median": q(cnt, 0.5), "fp6_cand_max": int(cnt.max())}))


if __name__ == "__main__":
    main()
