"""Diagnostic: the pruned search on the anisotropic corpus (split image) with the MX-fp4 tier's
tile form 64 / 128 and with the tier off -- exact against torch.topk?"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, ".")
from codename_symbiont_amd.index.shard import HbmIndexShard  # noqa: E402
from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus  # noqa: E402
from codename_symbiont_amd.ops._ext import hip  # noqa: E402

n, k = (1 << 21) + 333, 10
gen = CorpusGen("anisotropic", 384, "cuda")
shard = HbmIndexShard(384, n + 4096, prune="i8")
fill_corpus(shard, gen, n, seed=3)
q = gen.unit(256, seed=17).bfloat16()
sc = q.float() @ shard.unit_rows().float().t()
ts, ti = torch.topk(sc, k, dim=1)
for form in ("t128", "t64", "off"):
    hip().mx4_config(64 if form == "t64" else 128)
    saved = shard.rows_mx4
    if form == "off":
        shard.rows_mx4 = None
    shard.mq_stats = True
    s1, r1 = shard.search(q, k)
    torch.cuda.synchronize()
    cnt, ovf = shard._mq_last
    nv = shard._mx4_last
    err = (s1 - ts).abs()
    bad = (err > 2e-5)
    rows_bad = bad.any(1).nonzero().flatten().tolist()[:8]
    print(json.dumps({"form": form, "nv": None if nv is None else int(nv.item()),
                      "ovf": int(ovf.item()), "bad": int(bad.sum()), "max_err": float(err.max()),
                      "bad_queries": rows_bad, "cnt_max": int(cnt.max()),
                      "geo": list(shard._i8_geometry(shard.visible, 256, shard._n_cus()))}), flush=True)
    shard.rows_mx4 = saved
