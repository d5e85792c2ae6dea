"""Multi-process rehearsal of the sharded headline search on ONE GPU: world_size 2 or 4 ranks,
all on cuda:0, over the gloo backend (RCCL refuses two ranks on one device, and the driver's
8-GPU node is not ours to launch).  Every rank holds a HIP shard with the exact int8-pruned scan
(csrc/hip/index_i8.hip), so the gathered 512 / 1024-query batch takes the 512-query-workgroup
path of the N = 2 / 4 headline; ShardedSearcher's all_gather -> local scan -> all_to_all -> merge
(parallel/sharded.py) must return, for every rank's queries, the rows and scores of ONE exact
bf16 scan over the union of the shards."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_PER_RANK, D, NQ, K = (1 << 20) + 4321, 384, 256, 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")   # every rank on cuda:0
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.parallel import dist as D_
    from codename_symbiont_amd.parallel.sharded import ShardedSearcher

    info = D_.init(backend="gloo", device_type="cuda")
    dev = info.device
    n = N_PER_RANK
    g = torch.Generator(device=dev).manual_seed(5)
    x_all = torch.randn(world * n, D, device=dev, generator=g)
    shard = HbmIndexShard(D, n + 4096, device=dev, prune="i8")
    shard.append_f32(x_all[rank * n:(rank + 1) * n])
    ref = HbmIndexShard(D, world * n + 4096, device=dev)   # plain exact bf16 scan of the union
    ref.append_f32(x_all)
    # half: noisy copies of rows held by the NEXT rank (the answer crosses ranks), half random
    gq = torch.Generator(device=dev).manual_seed(100 + rank)
    src = ((rank + 1) % world) * n + torch.randint(0, n, (NQ // 2,), device=dev, generator=gq)
    q = torch.cat([x_all[src] + (0.5 / D ** 0.5) * torch.randn(NQ // 2, D, device=dev, generator=gq),
                   torch.randn(NQ - NQ // 2, D, device=dev, generator=gq)])
    q = torch.nn.functional.normalize(q, dim=-1).bfloat16()
    s, gid = ShardedSearcher(shard, info).search(q, K)
    s0, r0 = ref.search(q, K)
    cnt, ovf = shard._mq_last
    torch.cuda.synchronize(dev)
    out[rank] = (s.float().cpu().numpy(), gid.cpu().numpy(), s0.cpu().numpy(),
                 r0.long().cpu().numpy(), int(ovf.item()), int(cnt.shape[0]))
    D_.barrier(info)
    D_.shutdown(info)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_pruned_search_matches_single_exact_scan(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        s, gid, s0, r0, ovf, nq_scanned = out[r]
        assert nq_scanned == world * NQ, "each rank scans the gathered query batch"
        assert ovf == 0, "random / near data must not overflow the candidate buffer"
        rows = (gid >> 40) * N_PER_RANK + (gid & ((1 << 40) - 1))
        assert (rows == r0).mean() > 0.999, f"rank {r}: sharded ids differ from the exact scan"
        np.testing.assert_allclose(s, s0, atol=2e-5, err_msg=f"rank {r}: scores")
        assert (rows[: NQ // 2, 0] // N_PER_RANK == (r + 1) % world).mean() > 0.9, \
            "the noisy-copy queries' best rows live on the next rank"
