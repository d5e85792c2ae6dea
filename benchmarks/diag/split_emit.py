"""Diagnostic: index_scan_i8_kernel HK = 2 emission vs the torch split estimate, broken down by
row sub-tile / query wave / set (missing vs extra), for both row-split forms."""
import json
import sys

import torch

sys.path.insert(0, ".")
from codename_symbiont_amd.index.shard import HbmIndexShard  # noqa: E402
from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus  # noqa: E402
from codename_symbiont_amd.ops._ext import hip, stream_handle  # noqa: E402

n = 300_077
gen = CorpusGen("anisotropic", 384, "cuda")
shard = HbmIndexShard(384, n + 4096, prune="i8")
fill_corpus(shard, gen, n, seed=1)
h, st = hip(), stream_handle(shard.device)
for nq, rsplit in ((600, 1), (600, 2), (256, 1), (512, 1)):
    q = gen.unit(nq, seed=5).bfloat16()
    q8, sq, margin = shard.prune_query_image(q)
    est = shard.prune_estimate(q8, sq, 0, n)
    t = est.topk(40, dim=1).values[:, -1]
    thr = (t / sq).contiguous()
    _, rows_per_blk, n_rblk = shard._i8_geometry(n, nq, shard._n_cus())
    cap = 4096
    cs = torch.empty(nq, cap, device="cuda")
    ci = torch.empty(nq, cap, dtype=torch.int32, device="cuda")
    cnt = torch.empty(nq, dtype=torch.int32, device="cuda")
    h.index_scan_i8(shard.rows_i8.data_ptr(), shard.sx_i8.data_ptr(), n, shard.rows_i8.shape[0],
                    rows_per_blk, n_rblk, q8.data_ptr(), nq, thr.data_ptr(), cs.data_ptr(),
                    ci.data_ptr(), cnt.data_ptr(), cap, 1, st, rsplit, heavy=64, sq=sq.data_ptr())
    torch.cuda.synchronize()
    want = est >= t[:, None]
    near = (est - t[:, None]).abs() <= 1e-5 * est.abs().clamp_min(1.0)
    got = torch.zeros_like(want)
    scores = torch.full_like(est, float("nan"))
    for i in range(nq):
        c = int(cnt[i])
        got[i, ci[i, :c].long()] = True
        scores[i, ci[i, :c].long()] = cs[i, :c] * sq[i]
    miss = (want & ~got & ~near).nonzero()
    extra = (got & ~want & ~near).nonzero()
    rec = {"nq": nq, "rsplit": rsplit, "rows_per_blk": rows_per_blk, "n_rblk": n_rblk,
           "missing": len(miss), "extra": len(extra), "cnt_max": int(cnt.max())}
    for name, m in (("miss", miss), ("extra", extra)):
        if len(m):
            qi, ri = m[:, 0], m[:, 1]
            rec[name + "_by_subtile"] = torch.bincount((ri % 64) // 16, minlength=4).tolist()
            rec[name + "_by_rowin16"] = torch.bincount(ri % 16, minlength=16).tolist()
            rec[name + "_by_qwave"] = torch.bincount((qi % 512) // 64, minlength=8).tolist()
            rec[name + "_by_qset"] = torch.bincount((qi % 64) // 16, minlength=4).tolist()
            rec[name + "_by_qblk"] = torch.bincount(qi // (512 if rsplit == 1 else 256)).tolist()
            rec[name + "_by_tile_in_blk"] = torch.bincount(((ri % rows_per_blk) // 64).clamp_max(40)).tolist()
            rec[name + "_examples"] = [(int(a), int(b), float(est[a, b]), float(t[a]),
                                        float(scores[a, b])) for a, b in m[:5]]
    print(json.dumps(rec), flush=True)
