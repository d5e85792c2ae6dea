"""Forced-collective probe: does an RCCL kernel co-reside with the pruned search's stream scan?


One GPU, a single-rank RCCL group.  Each round enqueues one exact pruned search of 256 held-out
queries on a side stream (its full-shard scan holds one 512-register wave per SIMD on every CU),
sleeps ``delay`` ms on the host so the scan is running, then issues the collectives an 8-GPU step
would issue under it -- the query all_gather (8 x 256 x D bf16 out), the result all_to_all (8 x
256 x k x 12 bytes) and, as the plain case, an all_reduce of the gathered-query size -- on the
default stream, which has no dependency on the search.  Run it under
``rocprofv3 --kernel-trace --output-format csv`` and read the trace with
``benchmarks/rccl_overlap.py``: a collective that starts inside a scan co-resides; one that starts
within a few us of a scan's end waited for it.

    python benchmarks/rccl_coresident.py --rows 50000000 --rounds 8
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50_000_000)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--world", type=int, default=8, help="payload sizes of this many ranks")
    ap.add_argument("--rounds", type=int, default=8)
    a = ap.parse_args()
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.parallel import dist as sd

    info = sd.init(single_rank_group=True)
    dev = info.device
    shard = HbmIndexShard(a.dim, a.rows, device=dev, prune="i8")
    shard.fill_random(a.rows, seed=3)
    g = torch.Generator(device=dev).manual_seed(11)
    qs = [torch.nn.functional.normalize(torch.randn(a.nq, a.dim, device=dev, generator=g), dim=-1)
          .bfloat16() for _ in range(a.rounds + 2)]
    W, nq, k = a.world, a.nq, a.k
    q_in = torch.randn(nq * W, a.dim, device=dev).bfloat16()        # what W ranks would gather
    q_out = torch.empty_like(q_in)
    r_in = torch.zeros(W * nq * k * 3, dtype=torch.int32, device=dev)  # (score, id lo, id hi)
    r_out = torch.empty_like(r_in)
    red = torch.randn(nq * W * a.dim, device=dev).bfloat16()
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        shard.search(qs[0], k)       # warm: kernels loaded, tier flags settled
    torch.cuda.synchronize()
    dist.all_to_all_single(r_out, r_in)
    dist.all_gather_into_tensor(q_out, q_in)
    dist.all_reduce(red)
    torch.cuda.synchronize()
    # alone: the same collectives with the GPU idle (the trace's reference durations)
    for _ in range(2):
        dist.all_to_all_single(r_out, r_in)
        dist.all_gather_into_tensor(q_out, q_in)
        dist.all_reduce(red)
        torch.cuda.synchronize()
    delays = []
    for r in range(a.rounds):
        delay = 0.5 + 0.25 * r       # ms after the search's enqueue
        with torch.cuda.stream(side):
            shard.search(qs[r + 1], k)
        time.sleep(delay / 1e3)
        dist.all_to_all_single(r_out, r_in)
        dist.all_gather_into_tensor(q_out, q_in)
        dist.all_reduce(red)
        torch.cuda.synchronize()
        delays.append(delay)
    print(json.dumps({"probe": "rccl_coresident", "rows": a.rows, "dim": a.dim, "nq": nq,
                      "payload_world": W, "host_delays_ms": delays,
                      "bytes": {"all_gather_out": q_out.numel() * 2, "all_to_all": r_in.numel() * 4,
                                "all_reduce": red.numel() * 2}}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
