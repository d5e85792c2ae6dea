#!/usr/bin/env python3
"""Repeat the pruned search of tests/test_kernels_gpu.py::test_index_pruned_search_is_exact
[1100-random-128] on the same inputs, with and without the per-block route: per run the listed
blocks, the whole-batch flag, the overflow flag and how many scores differ from the exact scan."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from codename_symbiont_amd.index.shard import HbmIndexShard  # noqa: E402
from codename_symbiont_amd.ops._ext import hip  # noqa: E402

DEV = "cuda"
nq, tr, reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1100, 128, 12
n, k, D = (1 << 20) + 777, 10, 384
g = torch.Generator(device=DEV).manual_seed(71)
x = torch.randn(n, D, device=DEV, generator=g)
ref = HbmIndexShard(D, n + 4096)
shard = HbmIndexShard(D, n + 4096, prune="i8")
for sh in (ref, shard):
    sh.append_f32(x)
q = torch.nn.functional.normalize(torch.randn(nq, D, device=DEV, generator=g), dim=-1).bfloat16()
s0, r0 = ref.search(q, k)
hip().i8_config(tr, 8)
for route in (True, False):
    shard.prune_route = route
    for i in range(reps):
        s1, r1 = shard.search(q, k)
        cnt, ovf = shard._mq_last
        blk = shard._route_blk_last
        torch.cuda.synchronize()
        bad = ((s1.float() - s0.float()).abs() > 2e-5)
        rows = bad.any(1).nonzero().flatten().tolist()
        nrb = int(blk[1].item())
        listed = blk[2:2 + int(blk[0].item())].tolist() if route else []
        print(f"route={route} rep={i} listed={listed[:12]} n_rblk={nrb} dense={int(shard._route_last.item())} "
              f"ovf={int(ovf.item())} bad={int(bad.sum().item())} queries={rows[:8]} maxcnt={int(cnt.max().item())}",
              flush=True)
        if rows:
            qi = rows[0]
            miss = sorted(set(r0[qi].tolist()) - set(r1[qi].tolist()))
            print("   query", qi, "missing rows", miss, "blocks", [m // ((n + nrb - 1) // nrb) for m in miss],
                  "ref", s0[qi].tolist(), "got", s1[qi].tolist(), flush=True)
