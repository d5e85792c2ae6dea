"""EmbedGroup: data-parallel sentence embedding over RCCL, one process per GPU.

The reference embeds on ONE GPU in padded batches of 8 (services/preprocessing_service/src/
embedding_generator.rs:146, :75-91).  Here the preprocessing endpoint (rank 0) hands each packed
token batch to the group and every GPU of the node encodes a share of it:

  EMBED : header (op, B, T) -> broadcast cu_seqlens [B+1] and the ids/positions [2, T] (int32) ->
          every rank takes a token-balanced contiguous slice of the sentences (a pure function of
          cu_seqlens, so only the batch itself travels), encodes it with its own HIP encoder, pads
          the pooled f32 rows to the largest slice and all_gather_into_tensor's them over xGMI ->
          rank 0 reassembles [B, H] in input order.
  STOP  : header only.

Messages are tiny next to the work (a 256 x 128-token batch is 256 KB of ids in, 256 x H x 4 B of
embeddings out), so one broadcast + one all_gather per batch keeps every link's share small.  The
slice each rank encodes runs on its own compute stream; rank 0's H2D of the next batch overlaps
through the embed batcher's copy stream (services/batcher.py).  Ranks 1..N-1 run ``serve()``.
"""
from __future__ import annotations

import threading

import numpy as np
import torch
import torch.distributed as dist

from ..models.encoder import PackedBatch
from .dist import DistInfo

OP_STOP, OP_EMBED = 0, 1


def split_by_tokens(cu: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous sentence ranges [s, e) per rank with ~equal token counts (ranges may be empty)."""
    B = len(cu) - 1
    T = int(cu[-1])
    bounds = [0]
    for r in range(1, world):
        i = int(np.searchsorted(cu, T * r / world, side="left"))
        bounds.append(min(max(i, bounds[-1]), B))
    bounds.append(B)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


class EmbedGroup:
    def __init__(self, info: DistInfo, encoder, group=None):
        self.info = info
        self.enc = encoder
        self.group = group
        self.H = encoder.cfg.hidden
        self.comm_device = info.device if info.backend == "nccl" else torch.device("cpu")
        self._lock = threading.Lock()
        # a single-rank process group still runs every collective (RCCL tests on one GPU)
        self.collective = info.world > 1 or info.backend != "none"

    # ------------------------------------------------------------------ plumbing
    def _bcast(self, t: torch.Tensor) -> torch.Tensor:
        if self.collective:
            dist.broadcast(t, src=0, group=self.group)
        return t

    def _header(self, op: int, a: int = 0, b: int = 0) -> torch.Tensor:
        return self._bcast(torch.tensor([op, a, b, 0], dtype=torch.int64, device=self.comm_device))

    def _do_embed(self, cu: torch.Tensor, toks: torch.Tensor) -> torch.Tensor | None:
        info = self.info
        cu_np = cu.cpu().numpy()
        ranges = split_by_tokens(cu_np, info.world)
        s, e = ranges[info.rank]
        maxb = max(1, max(b - a for a, b in ranges))
        out = torch.zeros(maxb, self.H, dtype=torch.float32, device=self.comm_device)
        if e > s:
            t0, t1 = int(cu_np[s]), int(cu_np[e])
            dev = getattr(self.enc, "device", torch.device("cpu"))
            lens = np.diff(cu_np[s:e + 1])
            local = PackedBatch(toks[0, t0:t1].to(dev), toks[1, t0:t1].to(dev), None,
                                (cu[s:e + 1] - t0).to(dev, torch.int32), int(lens.max()))
            pooled, _ = self.enc.forward_packed(local)
            out[:e - s].copy_(pooled.float())
        if not self.collective:
            return out[:e - s]
        gathered = torch.empty(info.world * maxb, self.H, dtype=torch.float32, device=self.comm_device)
        dist.all_gather_into_tensor(gathered, out, group=self.group)
        if not info.is_root:
            return None
        return torch.cat([gathered[r * maxb: r * maxb + (b - a)] for r, (a, b) in enumerate(ranges)])

    # ------------------------------------------------------------------ collective entry points
    def embed(self, b: PackedBatch | None) -> torch.Tensor | None:
        """Collective: rank 0 passes the batch (any device), the others pass None (or run
        ``serve``).  Returns the pooled f32 embeddings [B, H] on rank 0, None elsewhere."""
        info = self.info
        with self._lock:
            if info.is_root:
                B, T = b.num_seqs, b.num_tokens
                self._header(OP_EMBED, B, T)
                cu = self._bcast(b.cu_seqlens.to(self.comm_device, torch.int32).contiguous())
                toks = self._bcast(torch.stack([b.ids.to(self.comm_device, torch.int32),
                                                b.pos.to(self.comm_device, torch.int32)]).contiguous())
            else:
                h = self._header(OP_STOP).tolist()
                if h[0] != OP_EMBED:
                    raise RuntimeError(f"embed group: expected EMBED, got op {h[0]}")
                B, T = h[1], h[2]
                cu = self._bcast(torch.empty(B + 1, dtype=torch.int32, device=self.comm_device))
                toks = self._bcast(torch.empty(2, T, dtype=torch.int32, device=self.comm_device))
            return self._do_embed(cu, toks)

    def stop(self) -> None:
        if self.info.is_root and self.info.world > 1:
            with self._lock:
                self._header(OP_STOP)

    def serve(self) -> None:
        """Ranks 1..N-1: execute rank 0's ops until STOP."""
        assert not self.info.is_root
        while True:
            h = self._header(OP_STOP).tolist()
            if h[0] == OP_STOP:
                return
            if h[0] != OP_EMBED:
                raise RuntimeError(f"unknown embed op {h[0]}")
            cu = self._bcast(torch.empty(h[1] + 1, dtype=torch.int32, device=self.comm_device))
            toks = self._bcast(torch.empty(2, h[2], dtype=torch.int32, device=self.comm_device))
            self._do_embed(cu, toks)


class GroupEncoder:
    """The encoder interface the embed batcher uses (cfg, device, forward_packed), backed by an
    EmbedGroup: every forward is spread over all GPUs of the node."""

    def __init__(self, group: EmbedGroup):
        self.group = group
        self.cfg = group.enc.cfg
        self.device = getattr(group.enc, "device", torch.device("cpu"))
        self.backend = f"{getattr(group.enc, 'backend', 'hip')}-dp{group.info.world}"

    def forward_packed(self, b: PackedBatch, out_f32=None, out_unit=None, pool=True):
        pooled = self.group.embed(b).to(self.device)
        unit = torch.nn.functional.normalize(pooled, dim=-1).to(torch.bfloat16)
        if out_f32 is not None:
            out_f32.copy_(pooled)
            pooled = out_f32
        if out_unit is not None:
            out_unit.copy_(unit)
            unit = out_unit
        return pooled, unit
