"""Diagnostic: index_scan_i8_kernel HK = MX4 emission vs the torch decode of the fp4 image,
broken down by row sub-tile / query wave / set / query block (missing vs extra), per row-split
form and batch size."""
import json
import sys

import torch

sys.path.insert(0, ".")
from codename_symbiont_amd.index.shard import HbmIndexShard  # noqa: E402
from codename_symbiont_amd.ops import reference as R  # noqa: E402
from codename_symbiont_amd.ops._ext import hip, stream_handle  # noqa: E402

n = 300_077
shard = HbmIndexShard(384, n + 4096, prune="i8")
shard.fill_random(n, seed=5)
xt = R.mx4_decode_ref(shard.rows_mx4[:n], shard.sc_mx4[:n])
h, st = hip(), stream_handle(shard.device)
for nq, rsplit in ((600, 1), (600, 2), (256, 1), (512, 1), (256, 2)):
    g = torch.Generator(device="cuda").manual_seed(nq)
    q = torch.nn.functional.normalize(torch.randn(nq, 384, device="cuda", generator=g), dim=-1).bfloat16()
    q4 = torch.empty(nq, 192, dtype=torch.uint8, device="cuda")
    qs4 = torch.empty(nq, 16, dtype=torch.uint8, device="cuda")
    m4 = torch.empty(nq, device="cuda")
    shard._mx4_image(q, q4, qs4, shard.mx4_bounds, margin=m4)
    est = R.mx4_decode_ref(q4, qs4) @ xt.t()
    t = est.topk(40, dim=1).values[:, -1].contiguous()
    _, rows_per_blk, n_rblk = shard._i8_geometry(n, nq, shard._n_cus())
    cap = 4096
    cs = torch.empty(nq, cap, device="cuda")
    ci = torch.empty(nq, cap, dtype=torch.int32, device="cuda")
    cnt = torch.empty(nq, dtype=torch.int32, device="cuda")
    h.index_scan_i8(shard.rows_mx4.data_ptr(), shard.sc_mx4.data_ptr(), n, shard.rows_mx4.shape[0],
                    rows_per_blk, n_rblk, q4.data_ptr(), nq, t.data_ptr(), cs.data_ptr(),
                    ci.data_ptr(), cnt.data_ptr(), cap, 1, st, rsplit, dim=384,
                    sq=qs4.data_ptr(), form=1)
    torch.cuda.synchronize()
    want = est >= t[:, None]
    near = (est - t[:, None]).abs() <= 1e-5 * est.abs().clamp_min(1.0)
    got = torch.zeros_like(want)
    sc = torch.full_like(est, float("nan"))
    for i in range(nq):
        c = min(int(cnt[i]), cap)
        got[i, ci[i, :c].long()] = True
        sc[i, ci[i, :c].long()] = cs[i, :c]
    miss = (want & ~got & ~near).nonzero()
    extra = (got & ~want & ~near).nonzero()
    qpb = 512 if rsplit == 1 else 256
    rec = {"nq": nq, "rsplit": rsplit, "missing": len(miss), "extra": len(extra),
           "cnt_max": int(cnt.max())}
    for name, m in (("miss", miss), ("extra", extra)):
        if len(m):
            qi, ri = m[:, 0], m[:, 1]
            rec[name + "_by_subtile"] = torch.bincount((ri % 64) // 16, minlength=4).tolist()
            rec[name + "_by_rowin16"] = torch.bincount(ri % 16, minlength=16).tolist()
            rec[name + "_by_qwave"] = torch.bincount((qi % qpb) // 64, minlength=8).tolist()
            rec[name + "_by_qset"] = torch.bincount((qi % 64) // 16, minlength=4).tolist()
            rec[name + "_by_qblk"] = torch.bincount(qi // qpb).tolist()
            rec[name + "_examples"] = [(int(a), int(b), float(est[a, b]), float(t[a]), float(sc[a, b]))
                                       for a, b in m[:4]]
    print(json.dumps(rec), flush=True)
