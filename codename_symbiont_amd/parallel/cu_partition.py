"""CU partitioning of one GPU between concurrent streams (hipExtStreamCreateWithCUMask).

The headline step runs the full-shard scan on one stream while the next batches' encoder and the
query-side pre-pass run on others (bench.py).  A launch fills every CU it can get and the GPU
does not preempt, so work queued on a second stream waits for the scan's workgroups to retire.
A CU mask makes the partition a property of the STREAM: the scan stream's kernels are dispatched
only to its CUs, and the reserve stays free for the other streams whatever the grid sizes are
(unlike a grid-size cap, which the dispatcher may still place anywhere).

Which CUs to reserve: MI355X has 256 CUs in 8 XCDs, and how the runtime's mask bits map onto
(XCD, shader engine, CU) is not documented here.  ``probe_cu_map`` measures it (one tiny launch per
mask bit reads the hardware ids of the CU it ran on) and the reserve takes ``per_xcd`` CUs of
every XCD, dealt over its shader engines, so every XCD keeps the same share of the scan's
workgroups (which are dealt round-robin over the XCDs).  Measured: it cannot -- a single-bit mask
let a launch run on 15 CUs across all 8 XCDs -- so the partition uses ``balanced_reserve`` (two
guessed numberings) and is an A/B knob, off by default: with 1-2 reserved CUs per XCD the
headline went from 11.0 to 16.1-16.7 ms, with 4 per XCD 10.84 ms (profiles/r4_cu_partition/).
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


_MAPS: dict = {}


def probe_cu_map(device, bits=None) -> list[list[tuple[int, int, int]]]:
    """The (xcc, se, cu) hardware ids the workgroups of a launch on a stream masked to ONE
    mask bit actually ran on, per bit (csrc/hip/cu_probe.hip: 16 workgroups each record HW_ID /
    XCC_ID).  Measured on MI355X / ROCm 7: a single-bit mask does NOT confine a launch to one CU
    -- bit 0's workgroups ran on 15 CUs across all 8 XCDs (profiles/r4_cu_partition/) -- so the
    result is a list of id sets, not a bijection.  Cached per device (all bits only)."""
    from ..ops._ext import hip, stream_handle

    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if bits is None and idx in _MAPS:
        return _MAPS[idx]
    h = hip()
    n = h.cu_count(idx)
    bits = list(range(n)) if bits is None else list(bits)
    out = torch.zeros(len(bits), 16, 2, dtype=torch.int32, device=torch.device("cuda", idx))
    torch.cuda.synchronize(idx)
    # one masked stream at a time: a CU mask is a property of a hardware queue, and 256 live
    # masked streams crashed the runtime (profiles/r4_cu_partition/README.md)
    for i, c in enumerate(bits):
        st = h.stream_with_cu_mask(idx, mask_words(n, [c]))
        h.cu_probe(out[i].data_ptr(), 16, st)
        torch.cuda.synchronize(idx)
        h.stream_destroy(st)
    ids = out.cpu().to(torch.int64) & 0xFFFFFFFF
    res = []
    for i in range(len(bits)):
        hw, xcc = ids[i, :, 0], ids[i, :, 1] & 0xF
        cu, se = (hw >> 8) & 0xF, (hw >> 13) & 0x7
        res.append(sorted({(int(a), int(b), int(d)) for a, b, d in zip(xcc, se, cu)}))
    if len(bits) == n:
        _MAPS[idx] = res
    return res


def reserve_from_map(cu_map, per_xcd: int) -> list[int]:
    """``per_xcd`` mask bits of every XCC, dealt round-robin over its shader engines, for a map
    in which every bit confines work to one CU (a list of (xcc, se, cu)); probe_cu_map shows
    that MI355X / ROCm 7 masks do not, so CuPartition uses balanced_reserve."""
    by_xcc: dict = {}
    for bit, (xcc, se, cu) in enumerate(cu_map):
        by_xcc.setdefault(xcc, {}).setdefault(se, []).append((cu, bit))
    out = []
    for xcc, ses in sorted(by_xcc.items()):
        lists = [sorted(v) for _, v in sorted(ses.items())]
        picked, j = [], 0
        while len(picked) < per_xcd:
            lst = lists[j % len(lists)]
            k = j // len(lists)
            if k >= len(lst):
                raise ValueError(f"XCC {xcc} has too few CUs for {per_xcd}")
            picked.append(lst[k][1])
            j += 1
        out += picked
    return sorted(out)


class CuPartition:
    """CU-masked streams on ``device``: ``main`` on every CU but the reserve (the scans) and
    ``n_side`` side streams (``sides``; ``side`` = the first) on the reserve only
    (``side_all=True``: every CU, i.e. the side work may also use the main CUs whenever they are
    idle).  ``main_cus`` is the number of CUs the main stream owns (the scans size their grids to
    it)."""

    def __init__(self, device, per_xcd: int, side_all: bool = True, n_side: int = 1,
                 probe: bool = False):
        from ..ops._ext import hip

        self.device = torch.device(device)
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = hip()
        self.n_cus = h.cu_count(idx)
        # (probe=True only with a driver whose masks confine work to single CUs, see probe_cu_map)
        self.cu_map = [m[0] for m in probe_cu_map(self.device)] if probe else None
        self.reserve = (reserve_from_map(self.cu_map, per_xcd) if probe
                        else balanced_reserve(self.n_cus, per_xcd))
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
