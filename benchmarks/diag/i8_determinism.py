#!/usr/bin/env python3
"""Is the int8 pruned scan's candidate emission deterministic?  Same inputs, repeated searches per
(queries, tile rows, waves) configuration: the total candidate count must not change, and the
scores must equal the exact scan's."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from codename_symbiont_amd.index.shard import HbmIndexShard  # noqa: E402
from codename_symbiont_amd.ops._ext import hip  # noqa: E402

DEV = "cuda"
n, k, D = (1 << 20) + 777, 10, 384
g = torch.Generator(device=DEV).manual_seed(71)
x = torch.randn(n, D, device=DEV, generator=g)
ref = HbmIndexShard(D, n + 4096)
shard = HbmIndexShard(D, n + 4096, prune="i8")
for sh in (ref, shard):
    sh.append_f32(x)
shard.prune_route = False
qall = torch.nn.functional.normalize(torch.randn(2048, D, device=DEV, generator=g), dim=-1).bfloat16()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
for nq, tr, wv in [(256, 64, 8), (1100, 64, 8), (2048, 64, 8), (256, 128, 8), (1100, 128, 8),
                   (1100, 64, 4)]:
    q = qall[:nq].contiguous()
    s0, _ = ref.search(q, k)
    hip().i8_config(tr, wv)
    tots, bads = [], []
    for i in range(reps):
        s1, r1 = shard.search(q, k)
        cnt, ovf = shard._mq_last
        torch.cuda.synchronize()
        tots.append(int(cnt.sum().item()))
        bads.append(int(((s1.float() - s0.float()).abs() > 2e-5).sum().item()))
    hip().i8_config(64, 8)
    print(f"nq={nq} tile_rows={tr} waves={wv}: candidate totals {sorted(set(tots))} bad {bads}",
          flush=True)
