"""EmbedGroup: data-parallel sentence embedding over RCCL, one process per GPU.

The reference embeds on ONE GPU in padded batches of 8 (services/preprocessing_service/src/
embedding_generator.rs:146, :75-91).  Here the preprocessing endpoint (rank 0) hands each packed
token batch to the group and every GPU of the node encodes a share of it:

  EMBED : header (op, B, T, wire, the per-rank split) -> broadcast cu_seqlens [B+1] and the
          ids/positions [2, T] (int32) -> every rank encodes its token-balanced contiguous slice of
          the sentences (rank 0 computes the split from the host copy of cu_seqlens and sends it
          in the header, with each slice's longest sentence, so no rank reads cu_seqlens back
          from the device) -> the pooled rows, padded to the largest slice, are all_gathered over
          xGMI as bf16 (f32 on gloo) -> rank 0 reassembles [B, H] in input order as f32.
  STOP  : header only.

Messages are tiny next to the work (a 256 x 128-token batch is 256 KB of ids in, 256 x H x 2 B of
embeddings out), so one broadcast + one all_gather per batch keeps every link's share small.  The
slice each rank encodes runs on its own compute stream; rank 0's H2D of the next batch overlaps
through the embed batcher's copy stream (services/batcher.py).  Ranks 1..N-1 run ``serve()``.

Control plane: on RCCL the fixed-size header travels over a gloo (host TCP) group of the same
ranks, so learning a batch's shapes is a host receive that never synchronises a GPU stream --
a rank enqueues batch i + 1's receives and forward while batch i's are still running (a header
broadcast over RCCL would need a device read-back, which waits for everything queued before it).

The bf16 wire rounds each pooled value of ranks 1..N-1 once (relative 2^-9; cosine to the f32
rows >= 0.99999, tests/test_parallel_cpu.py); rank 0's own slice never crosses the wire and keeps
its f32 values.  ``wire_dtype`` = torch.float32 keeps every value exactly (the bench and the
service report which wire ran).
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


HDR_FIXED = 5    # op, B, T, wire (0 = f32, 1 = bf16), maxb
HDR_RANK = 5     # then per rank: sentences [s, e), tokens [t0, t1), the slice's longest sentence


class EmbedGroup:
    def __init__(self, info: DistInfo, encoder, group=None, wire_dtype=None):
        self.info = info
        self.enc = encoder
        self.group = group
        self.H = encoder.cfg.hidden
        self.comm_device = info.device if info.backend == "nccl" else torch.device("cpu")
        self._lock = threading.Lock()
        # a single-rank process group still runs every collective (RCCL tests on one GPU)
        self.collective = info.world > 1 or info.backend != "none"
        # the embeddings' wire format: bf16 over RCCL (half the bytes), f32 on gloo (no bf16
        # collectives on every build)
        if wire_dtype is None:
            wire_dtype = torch.bfloat16 if info.backend == "nccl" else torch.float32
        self.wire_dtype = wire_dtype
        self.hdr_len = HDR_FIXED + HDR_RANK * info.world
        # the header's group: gloo beside RCCL (host-only receive), else the data group itself
        self.ctrl = group
        if self.collective and info.backend == "nccl" and group is None:
            self.ctrl = dist.new_group(backend="gloo")
        self.ctrl_device = (torch.device("cpu") if self.ctrl is not group
                            else self.comm_device)

    @property
    def wire(self) -> str:
        """The embeddings' wire dtype (``bf16`` | ``f32``), for result records."""
        return "bf16" if self.wire_dtype == torch.bfloat16 else "f32"

    # ------------------------------------------------------------------ plumbing
    def _bcast(self, t: torch.Tensor) -> torch.Tensor:
        if self.collective:
            dist.broadcast(t, src=0, group=self.group)
        return t

    def _header(self, vals=None) -> list[int]:
        """Broadcast the op header from rank 0 (vals) / receive it (vals None); host ints."""
        if vals is not None:
            t = torch.tensor(vals + [0] * (self.hdr_len - len(vals)), dtype=torch.int64)
        else:
            t = torch.zeros(self.hdr_len, dtype=torch.int64)
        t = t.to(self.ctrl_device)
        if self.collective:
            dist.broadcast(t, src=0, group=self.ctrl)
        return vals if vals is not None else t.tolist()

    def _plan(self, cu_host: np.ndarray) -> list[int]:
        """Rank 0: the EMBED header for a batch with these (host) cu_seqlens."""
        B, T = len(cu_host) - 1, int(cu_host[-1])
        ranges = split_by_tokens(cu_host, self.info.world)
        maxb = max(1, max(e - s for s, e in ranges))
        per = []
        for s, e in ranges:
            ml = int(np.diff(cu_host[s:e + 1]).max()) if e > s else 0
            per += [s, e, int(cu_host[s]), int(cu_host[e]), ml]
        wire = 1 if self.wire_dtype == torch.bfloat16 else 0
        return [OP_EMBED, B, T, wire, maxb] + per

    def _do_embed(self, hdr: list[int], cu: torch.Tensor, toks: torch.Tensor) -> torch.Tensor | None:
        info = self.info
        maxb = hdr[4]
        wdt = torch.bfloat16 if hdr[3] else torch.float32
        def part(r):
            return hdr[HDR_FIXED + HDR_RANK * r:HDR_FIXED + HDR_RANK * (r + 1)]
        ranges = [tuple(part(r)[:2]) for r in range(info.world)]
        s, e, t0, t1, max_len = part(info.rank)
        out = torch.zeros(maxb, self.H, dtype=wdt, device=self.comm_device)
        pooled = None
        if e > s:
            dev = getattr(self.enc, "device", torch.device("cpu"))
            # the slice's sentences and tokens by the header's host offsets: no device read
            local = PackedBatch(toks[0, t0:t1].to(dev), toks[1, t0:t1].to(dev), None,
                                (cu[s:e + 1] - t0).to(dev, torch.int32), max_len)
            pooled, _ = self.enc.forward_packed(local)
            out[:e - s].copy_(pooled)
        if not self.collective:
            return out[:e - s].float()
        gathered = torch.empty(info.world * maxb, self.H, dtype=wdt, device=self.comm_device)
        dist.all_gather_into_tensor(gathered, out, group=self.group)
        if not info.is_root:
            return None
        # rank 0's own rows straight from its f32 output (they never crossed the wire)
        own = (pooled.float().to(self.comm_device) if pooled is not None
               else gathered[:0].float())
        return torch.cat([own] + [gathered[r * maxb: r * maxb + (b - a)].float()
                                  for r, (a, b) in enumerate(ranges) if r > 0])

    # ------------------------------------------------------------------ collective entry points
    def embed(self, b: PackedBatch | None, cu_host=None) -> torch.Tensor | None:
        """Collective: rank 0 passes the batch (any device) and, when it has one, a host copy of
        its cu_seqlens (``cu_host``: else rank 0 reads them back once); the others pass None (or
        run ``serve``).  Returns the pooled f32 embeddings [B, H] on rank 0, None elsewhere."""
        info = self.info
        with self._lock:
            if info.is_root:
                if cu_host is None:
                    cu_host = b.cu_seqlens.cpu()
                cu_np = np.asarray(cu_host, dtype=np.int64)
                hdr = self._header(self._plan(cu_np))
                cu = self._bcast(b.cu_seqlens.to(self.comm_device, torch.int32).contiguous())
                toks = self._bcast(torch.stack([b.ids.to(self.comm_device, torch.int32),
                                                b.pos.to(self.comm_device, torch.int32)]).contiguous())
            else:
                hdr = self._header()
                if hdr[0] != OP_EMBED:
                    raise RuntimeError(f"embed group: expected EMBED, got op {hdr[0]}")
                cu, toks = self._recv_batch(hdr)
            return self._do_embed(hdr, cu, toks)

    def _recv_batch(self, hdr):
        cu = self._bcast(torch.empty(hdr[1] + 1, dtype=torch.int32, device=self.comm_device))
        toks = self._bcast(torch.empty(2, hdr[2], dtype=torch.int32, device=self.comm_device))
        return cu, toks

    def stop(self) -> None:
        if self.info.is_root and self.info.world > 1:
            with self._lock:
                self._header([OP_STOP])

    def serve(self) -> None:
        """Ranks 1..N-1: execute rank 0's ops until STOP."""
        assert not self.info.is_root
        while True:
            hdr = self._header()
            if hdr[0] == OP_STOP:
                return
            if hdr[0] != OP_EMBED:
                raise RuntimeError(f"unknown embed op {hdr[0]}")
            cu, toks = self._recv_batch(hdr)
            self._do_embed(hdr, cu, toks)


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
