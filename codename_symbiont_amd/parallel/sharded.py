"""Corpus-sharded top-k search across the GPUs of one node (RCCL over xGMI).

Replaces Qdrant's single-node HNSW (services/vector_memory_service/src/main.rs:261-308, which has
``shard_number: None`` at :50) with the retrieval analogue of context parallelism:

    queries of every rank --all_gather--> every rank scans ITS shard with the fused MFMA kernel
    --> per-rank top-k [world*nq, k] --all_to_all--> each query's owner --> k-way merge.

Message sizes are tiny (nq x D bf16 queries, nq x k x (f32+i64) results) and xGMI is a full mesh
of point-to-point links, so all_gather / all_to_all (direct, α-dominated) are used and
all_reduce is avoided entirely: exactly TWO collectives per search, the query all_gather and ONE
all_to_all of the packed (score, id) lists (12 bytes per entry as int32 triples).  Global point
ids are ``rank << 40 | row``.

Stream order of the pipelined step (bench.py: ``begin`` of batch i+1 on a pre-pass stream, then
``end`` of batch i on the compute stream).  Every rank issues the collectives in the same host
order -- all_gather(i+1), all_to_all(i), all_gather(i+2), ... -- which is what RCCL requires of
one communicator; torch's ProcessGroupNCCL runs them on the group's internal stream in that order,
each after the issuing stream's prior work (an event wait).  all_gather(i+1) depends only on
batch i+1's encoder, all_to_all(i) on batch i's scan, and neither stream waits on the other's
collective, so no rank can block on a peer that is itself blocked: the order is deadlock-free for
any world size (tests/test_parallel_cpu.py rehearses it on gloo up to 8 ranks).  Its cost: the
all_to_all of batch i queues behind the all_gather of batch i+1, which is issued under batch i's
scan; an RCCL kernel that waits for a late peer there occupies a few CUs of the scan.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..index.shard import HbmIndexShard
from .dist import DistInfo

RANK_SHIFT = 40


def encode_gid(rank: int, rows: torch.Tensor) -> torch.Tensor:
    r = rows.long()
    if rank == 0:   # (0 << 40) | r == r, and missing slots are already -1: one cast, no kernels more
        return r
    return torch.where(r >= 0, (rank << RANK_SHIFT) | r, torch.full_like(r, -1))


def decode_gid(gid: int) -> tuple[int, int]:
    return gid >> RANK_SHIFT, gid & ((1 << RANK_SHIFT) - 1)


class ShardedSearcher:
    def __init__(self, shard: HbmIndexShard, info: DistInfo, group=None):
        self.shard = shard
        self.info = info
        self.group = group
        # gloo has no bf16 collectives on every build: ship queries as f32 there
        self.wire_dtype = torch.bfloat16 if info.backend == "nccl" else torch.float32
        # a single-rank process group still runs the collective path (RCCL tests on one GPU)
        self.collective = info.world > 1 or info.backend != "none"

    def search(self, q_local: torch.Tensor, k: int):
        """Every rank calls this collectively with its own [nq, D] unit queries (same nq on all
        ranks).  Returns (scores f32 [nq, k], global ids int64 [nq, k]) for the LOCAL queries."""
        info = self.info
        if not self.collective:
            s, r = self.shard.search(q_local, k)
            return s, encode_gid(0, r)
        nq, D = q_local.shape
        q_send = q_local.to(self.wire_dtype).contiguous()
        q_all = torch.empty(info.world * nq, D, dtype=self.wire_dtype, device=q_send.device)
        dist.all_gather_into_tensor(q_all, q_send, group=self.group)
        s, r = self.shard.search(q_all.to(torch.bfloat16), k)
        self.collectives += 1
        return self._exchange(s, encode_gid(info.rank, r), nq, k)

    collectives = 0   # collectives issued (tests: 2 per search)

    def _exchange(self, s: torch.Tensor, gid: torch.Tensor, nq: int, k: int):
        """ONE all_to_all of the per-rank (score, id) lists packed as int32 triples [W*nq, k, 3]
        (score bits, id low, id high), then the k-way merge of what came back."""
        W = self.info.world
        packed = pack_results(s, gid)
        recv = torch.empty_like(packed)
        dist.all_to_all_single(recv, packed, group=self.group)
        self.collectives += 1
        s_recv, g_recv = unpack_results(recv)
        return merge_ranked(s_recv.view(W, nq, k), g_recv.view(W, nq, k), k)


    def begin(self, q_local: torch.Tensor, k: int) -> dict:
        """First half of ``search`` for a pipelined caller (bench.py): the query all_gather and
        the shard's query-side pre-pass run now, on the current stream; ``end`` runs the
        full-shard scan, the exchange and the merge (HbmIndexShard.search_begin)."""
        info = self.info
        if not self.collective:
            return {"ctx": self.shard.search_begin(q_local, k), "k": k}
        nq, D = q_local.shape
        q_send = q_local.to(self.wire_dtype).contiguous()
        q_all = torch.empty(info.world * nq, D, dtype=self.wire_dtype, device=q_send.device)
        dist.all_gather_into_tensor(q_all, q_send, group=self.group)
        self.collectives += 1
        return {"ctx": self.shard.search_begin(q_all.to(torch.bfloat16), k), "k": k, "nq": nq}

    def end(self, h: dict):
        info, k = self.info, h["k"]
        s, r = self.shard.search_end(h["ctx"])
        if not self.collective:
            return s, encode_gid(0, r)
        return self._exchange(s, encode_gid(info.rank, r), h["nq"], k)


class SimulatedShardedSearcher(ShardedSearcher):
    """The per-rank work of a ``vworld``-GPU sharded search, on ONE GPU (bench.py
    --simulate-world N): a PROJECTION, never a multi-GPU measurement.

    The real collectives run through a single-rank RCCL group, so their kernels are launched and
    contend for CUs with the scans exactly as on each rank of the real job, and each moves the
    payload ONE rank sends (its [nq, D] queries; its [vworld * nq, k] score + id lists).  What
    the other ranks would contribute is stood in for locally: the all_gathered batch is this
    rank's queries followed by (vworld - 1) * nq foreign queries from ``foreign`` (embeddings that
    are NOT in this shard, as the other ranks' are not), so the shard scan, the pre-pass and the
    merge see the per-rank shapes of the N-GPU step.  Not modelled: xGMI transfer time and the
    wait for the slowest peer."""

    def __init__(self, shard: HbmIndexShard, info: DistInfo, vworld: int, foreign: list,
                 group=None):
        super().__init__(shard, info, group)
        if info.world != 1:
            raise ValueError("a simulated world runs on exactly one rank")
        self.vworld = int(vworld)
        self.foreign = foreign      # list of [(vworld - 1) * nq, D] bf16 query blocks
        self._fi = 0

    def _gather(self, q_local: torch.Tensor) -> torch.Tensor:
        nq, D = q_local.shape
        q_send = q_local.to(self.wire_dtype).contiguous()
        q_own = torch.empty(nq, D, dtype=self.wire_dtype, device=q_send.device)
        if self.collective:
            dist.all_gather_into_tensor(q_own, q_send, group=self.group)
        else:
            q_own.copy_(q_send)
        f = self.foreign[self._fi % len(self.foreign)]
        self._fi += 1
        return torch.cat([q_own.to(torch.bfloat16), f[:(self.vworld - 1) * nq]])

    def _exchange(self, s: torch.Tensor, gid: torch.Tensor, nq: int, k: int):
        packed = pack_results(s, gid)
        recv = torch.empty_like(packed)
        if self.collective:
            dist.all_to_all_single(recv, packed, group=self.group)
        else:
            recv.copy_(packed)
        s_recv, g_recv = unpack_results(recv)
        return merge_ranked(s_recv.view(self.vworld, nq, k), g_recv.view(self.vworld, nq, k), k)

    def search(self, q_local: torch.Tensor, k: int):
        nq = q_local.shape[0]
        s, r = self.shard.search(self._gather(q_local), k)
        return self._exchange(s, encode_gid(0, r), nq, k)

    def begin(self, q_local: torch.Tensor, k: int) -> dict:
        return {"ctx": self.shard.search_begin(self._gather(q_local), k), "k": k,
                "nq": q_local.shape[0]}

    def end(self, h: dict):
        s, r = self.shard.search_end(h["ctx"])
        return self._exchange(s, encode_gid(0, r), h["nq"], h["k"])


def pack_results(s: torch.Tensor, gid: torch.Tensor) -> torch.Tensor:
    """[n, k] f32 scores + [n, k] int64 ids -> [n, k, 3] int32 (score bits, id lo, id hi): one
    buffer, one collective."""
    n, k = s.shape
    return torch.cat([s.contiguous().view(torch.int32).view(n, k, 1),
                      gid.contiguous().view(torch.int32).view(n, k, 2)], 2)


def unpack_results(p: torch.Tensor):
    """Inverse of pack_results: ([n, k] f32, [n, k] int64)."""
    n, k, _ = p.shape
    return (p[:, :, 0].contiguous().view(torch.float32),
            p[:, :, 1:].contiguous().view(torch.int64).view(n, k))


def merge_ranked(scores: torch.Tensor, gids: torch.Tensor, k: int):
    """[world, nq, k] per-rank sorted lists -> [nq, k] global top-k (ties: lower rank first)."""
    W, nq, kk = scores.shape
    s = scores.permute(1, 0, 2).reshape(nq, W * kk)
    g = gids.permute(1, 0, 2).reshape(nq, W * kk)
    top_s, idx = torch.topk(s, min(k, W * kk), dim=1, sorted=True)
    return top_s, torch.gather(g, 1, idx)
