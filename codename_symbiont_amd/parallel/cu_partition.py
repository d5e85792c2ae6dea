"""CU partitioning of one GPU between concurrent streams (hipExtStreamCreateWithCUMask).

The headline step runs the full-shard scan on one stream while the next batches' encoder and the
query-side pre-pass run on others (bench.py).  A launch fills every CU it can get and the GPU
does not preempt, so work queued on a second stream waits for the scan's workgroups to retire.
A CU mask makes the partition a property of the STREAM: the scan stream's kernels are dispatched
only to its CUs, and the reserve stays free for the other streams whatever the grid sizes are
(unlike a grid-size cap, which the dispatcher may still place anywhere).

Which CUs to reserve: MI355X has 256 CUs in 8 XCDs.  The runtime numbers CUs 0..255; whether CU
i sits on XCD i // 32 or on XCD i % 8 is not documented here, so the reserve takes CUs
32 x + ((x + 8 j) mod 32) for XCD slot x and j < per_xcd -- exactly ``per_xcd`` CUs of every XCD
under either numbering, so each XCD's L2 keeps serving the same share of the scan.
"""
from __future__ import annotations

import torch


def balanced_reserve(n_cus: int, per_xcd: int, xcds: int = 8) -> list[int]:
    """CU ids of a reserve of ``per_xcd`` CUs on each of ``xcds`` XCDs (see the module doc)."""
    if per_xcd <= 0:
        return []
    per = n_cus // xcds
    # (under the round-robin numbering an XCD owns the ids = x mod xcds: per / xcds of each block)
    if per_xcd > per // xcds or n_cus % xcds or per % xcds:
        raise ValueError(f"cannot reserve {per_xcd} CUs per XCD of {n_cus} CUs / {xcds} XCDs "
                         f"balanced under both numberings (at most {per // xcds})")
    out = []
    for x in range(xcds):
        for j in range(per_xcd):
            out.append(per * x + (x + xcds * j) % per)
    return sorted(set(out))


def mask_words(n_cus: int, cus) -> list[int]:
    """The uint32 bit-vector of a CU set (bit i of word i // 32 = CU i)."""
    words = [0] * ((n_cus + 31) // 32)
    for c in cus:
        if not 0 <= c < n_cus:
            raise ValueError(f"CU {c} outside 0..{n_cus - 1}")
        words[c // 32] |= 1 << (c % 32)
    return words


class CuPartition:
    """CU-masked streams on ``device``: ``main`` on every CU but the reserve (the scans) and
    ``n_side`` side streams (``sides``; ``side`` = the first) on the reserve only
    (``side_all=True``: every CU, i.e. the side work may also use the main CUs whenever they are
    idle).  ``main_cus`` is the number of CUs the main stream owns (the scans size their grids to
    it)."""

    def __init__(self, device, per_xcd: int, side_all: bool = True, n_side: int = 1):
        from ..ops._ext import hip

        self.device = torch.device(device)
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = hip()
        self.n_cus = h.cu_count(idx)
        self.reserve = balanced_reserve(self.n_cus, per_xcd)
        rest = [c for c in range(self.n_cus) if c not in set(self.reserve)]
        self.main_cus = len(rest)
        side_mask = mask_words(self.n_cus, range(self.n_cus) if side_all else self.reserve)
        self._raw = [h.stream_with_cu_mask(idx, mask_words(self.n_cus, rest))]
        self._raw += [h.stream_with_cu_mask(idx, side_mask) for _ in range(max(1, n_side))]
        self.main = torch.cuda.ExternalStream(self._raw[0], device=self.device)
        self.sides = [torch.cuda.ExternalStream(r, device=self.device) for r in self._raw[1:]]
        self.side = self.sides[0]

    def masks(self) -> tuple[list[int], list[int]]:
        from ..ops._ext import hip

        w = (self.n_cus + 31) // 32
        return hip().cu_mask_of(self._raw[0], w), hip().cu_mask_of(self._raw[1], w)
