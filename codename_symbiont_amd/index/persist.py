"""Checkpoint / resume of an HBM index shard: snapshot + append-only WAL.

The reference persists through Qdrant (on-disk vectors + payload, vector_memory_service/src/main.rs
:39,52; docker volume ./data/qdrant_storage).  The HBM index is volatile, so each shard keeps:

  <dir>/CURRENT                        commit pointer: "snapshot.<gen>" (atomic replace + fsync)
  <dir>/snapshot.<gen>/meta.json       {"dim", "count", "format": 1}
  <dir>/snapshot.<gen>/vectors.npy     count x dim bf16 bit patterns (uint16 .npy, memory-
                                       mappable), or e4m3 bytes (uint8) for an fp8 shard
  <dir>/snapshot.<gen>/payloads.jsonl  one [point_id, doc_id, url, text, order, model, ts] per row
  <dir>/wal.log                        records appended (and fsync'd) per upsert batch

A snapshot is written to a fresh generation directory (files + directory fsync'd), committed by
replacing CURRENT, and only then are older generations deleted and the WAL truncated -- a crash
at any step boots from the previous committed generation + the untruncated WAL.

WAL record: magic u32 | n u32 | body_len u32 | crc32(body) u32 | body, body = n x
(u16 id_len, id, u32 payload_len, payload JSON, f32[dim]).  A torn tail record (crash mid-write)
fails its length/CRC check and is dropped on replay.  Boot = mmap snapshot -> HBM, replay WAL.
"""
from __future__ import annotations

import json
import os
import struct
import zlib

import numpy as np
import torch

from .shard import HbmIndexShard, Payload

MAGIC = 0x53594D42  # "SYMB"
_HDR = struct.Struct("<IIII")


class Wal:
    def __init__(self, path: str, dim: int):
        self.path = path
        self.dim = dim
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self._f = open(path, "ab")

    def append(self, point_ids: list[str], payloads: list[Payload], vecs: np.ndarray) -> None:
        vecs = np.ascontiguousarray(vecs, dtype=np.float32)
        assert vecs.shape == (len(point_ids), self.dim)
        parts = []
        for pid, p, v in zip(point_ids, payloads, vecs):
            b = pid.encode()
            pj = json.dumps([p.original_document_id, p.source_url, p.sentence_text,
                             p.sentence_order, p.model_name, p.processed_at_ms],
                            ensure_ascii=False).encode()
            parts += [struct.pack("<H", len(b)), b, struct.pack("<I", len(pj)), pj, v.tobytes()]
        body = b"".join(parts)
        self._f.write(_HDR.pack(MAGIC, len(point_ids), len(body), zlib.crc32(body)) + body)
        self._f.flush()
        os.fsync(self._f.fileno())

    def truncate(self) -> None:
        self._f.close()
        self._f = open(self.path, "wb")
        self._f.flush()
        os.fsync(self._f.fileno())

    def close(self) -> None:
        self._f.close()

    @staticmethod
    def repair(path: str) -> int:
        """Truncate a torn / corrupt tail so later appends stay reachable; returns valid bytes."""
        if not os.path.exists(path):
            return 0
        with open(path, "rb") as f:
            data = f.read()
        off = 0
        while off + _HDR.size <= len(data):
            magic, _n, blen, crc = _HDR.unpack_from(data, off)
            body = data[off + _HDR.size: off + _HDR.size + blen]
            if magic != MAGIC or len(body) != blen or zlib.crc32(body) != crc:
                break
            off += _HDR.size + blen
        if off != len(data):
            with open(path, "r+b") as f:
                f.truncate(off)
                f.flush()
                os.fsync(f.fileno())
        return off

    @staticmethod
    def replay(path: str, dim: int):
        """Yields (point_ids, payloads, vecs) per intact record."""
        if not os.path.exists(path):
            return
        with open(path, "rb") as f:
            data = f.read()
        off = 0
        while off + _HDR.size <= len(data):
            magic, n, blen, crc = _HDR.unpack_from(data, off)
            body = data[off + _HDR.size: off + _HDR.size + blen]
            if magic != MAGIC or len(body) != blen or zlib.crc32(body) != crc:
                break  # torn / corrupt tail
            off += _HDR.size + blen
            ids, pls, vs = [], [], []
            o = 0
            for _ in range(n):
                (lb,) = struct.unpack_from("<H", body, o)
                o += 2
                ids.append(body[o:o + lb].decode())
                o += lb
                (lp,) = struct.unpack_from("<I", body, o)
                o += 4
                a = json.loads(body[o:o + lp])
                o += lp
                pls.append(Payload(*a))
                vs.append(np.frombuffer(body, dtype=np.float32, count=dim, offset=o))
                o += 4 * dim
            yield ids, pls, np.stack(vs) if vs else np.zeros((0, dim), np.float32)


CURRENT = "CURRENT"        # commit pointer: names the live snapshot.<gen> directory
_SNAP_PREFIX = "snapshot."


def fsync_dir(path: str) -> None:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def fsync_file(path: str) -> None:
    with open(path, "rb+") as f:
        os.fsync(f.fileno())


def write_atomic(path: str, data: bytes) -> None:
    """tmp + fsync + rename + fsync(dir): after return ``path`` holds ``data`` durably, and a
    crash at any point leaves either the old or the new content."""
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    fsync_dir(os.path.dirname(path) or ".")


def _rmtree(path: str) -> None:
    if not os.path.isdir(path):
        return
    for fn in os.listdir(path):
        os.remove(os.path.join(path, fn))
    os.rmdir(path)


def _snap_gen(name: str) -> int:
    tail = name[len(_SNAP_PREFIX):]
    return int(tail) if name.startswith(_SNAP_PREFIX) and tail.isdigit() else -1


def committed_snapshot(directory: str) -> str | None:
    """Path of the committed snapshot directory, or None.  ``CURRENT`` names it; directories
    written by the pre-pointer format (``snapshot/``, or ``snapshot.old`` left by a crash in its
    two-rename swap) are still honoured when no pointer exists."""
    cur = os.path.join(directory, CURRENT)
    if os.path.exists(cur):
        with open(cur, encoding="utf-8") as f:
            name = f.read().strip()
        p = os.path.join(directory, name)
        if os.path.exists(os.path.join(p, "meta.json")):
            return p
        raise RuntimeError(f"snapshot pointer {cur} names {name!r}, which is incomplete")
    for legacy in ("snapshot", "snapshot.old"):
        p = os.path.join(directory, legacy)
        if os.path.exists(os.path.join(p, "meta.json")):
            return p
    return None


def save_snapshot(shard: HbmIndexShard, directory: str, chunk: int = 1 << 20,
                  _crash_before_commit: bool = False) -> None:
    """Write ``snapshot.<gen>/`` (every file fsync'd, then the directory), then commit it by
    atomically replacing ``CURRENT``; only then are older generations removed.  A crash anywhere
    leaves the previous committed snapshot (and the WAL, truncated by the caller only after
    this returns) intact.  ``_crash_before_commit`` stops right before the pointer swap (tests)."""
    os.makedirs(directory, exist_ok=True)
    names = os.listdir(directory)
    gen = max([_snap_gen(n) for n in names] + [0]) + 1
    final = os.path.join(directory, f"{_SNAP_PREFIX}{gen}")
    tmp = final + ".tmp"
    _rmtree(tmp)
    os.makedirs(tmp)
    n, D = shard.count, shard.dim
    fp8 = getattr(shard, "dtype", "bf16") == "fp8"
    mm = np.lib.format.open_memmap(os.path.join(tmp, "vectors.npy"), mode="w+",
                                   dtype=np.uint8 if fp8 else np.uint16, shape=(n, D)) if n else None
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        if fp8:
            mm[s:e] = shard.rows[s:e].cpu().numpy()
        else:
            mm[s:e] = shard.rows[s:e].view(torch.int16).cpu().numpy().view(np.uint16)
    if mm is not None:
        mm.flush()
        del mm
        fsync_file(os.path.join(tmp, "vectors.npy"))
    with open(os.path.join(tmp, "payloads.jsonl"), "w", encoding="utf-8") as f:
        ps = shard.payloads
        empty = None
        for r in range(n):
            if r not in ps.fields and r not in ps.point_ids:   # row without point (synthetic)
                if empty is None:
                    pid, p = ps.get(r)
                    empty = json.dumps([pid, p.original_document_id, p.source_url,
                                        p.sentence_text, p.sentence_order, p.model_name,
                                        p.processed_at_ms], ensure_ascii=False) + "\n"
                f.write(empty)
                continue
            pid, p = ps.get(r)
            f.write(json.dumps([pid, p.original_document_id, p.source_url, p.sentence_text,
                                p.sentence_order, p.model_name, p.processed_at_ms],
                               ensure_ascii=False) + "\n")
        f.flush()
        os.fsync(f.fileno())
    with open(os.path.join(tmp, "meta.json"), "w") as f:
        json.dump({"dim": D, "count": n, "format": 1, "dtype": "fp8" if fp8 else "bf16"}, f)
        f.flush()
        os.fsync(f.fileno())
    fsync_dir(tmp)
    os.replace(tmp, final)
    fsync_dir(directory)
    if _crash_before_commit:
        return
    write_atomic(os.path.join(directory, CURRENT), f"{_SNAP_PREFIX}{gen}\n".encode())
    # committed: drop older generations and the pre-pointer layout
    for name in os.listdir(directory):
        p = os.path.join(directory, name)
        if name == f"{_SNAP_PREFIX}{gen}" or not os.path.isdir(p):
            continue
        if name in ("snapshot", "snapshot.old", "snapshot.tmp") or name.startswith(_SNAP_PREFIX):
            _rmtree(p)


def load_snapshot(shard: HbmIndexShard, directory: str, chunk: int = 1 << 20) -> int:
    snap = committed_snapshot(directory)
    if snap is None:
        return 0
    meta_p = os.path.join(snap, "meta.json")
    with open(meta_p) as f:
        meta = json.load(f)
    if meta["dim"] != shard.dim:
        raise ValueError(f"snapshot dim {meta['dim']} != index dim {shard.dim}")
    fp8 = meta.get("dtype", "bf16") == "fp8"
    if fp8 != (getattr(shard, "dtype", "bf16") == "fp8"):
        raise ValueError(f"snapshot dtype {meta.get('dtype', 'bf16')} != index dtype {shard.dtype}")
    n = meta["count"]
    if n == 0:
        return 0
    mm = np.load(os.path.join(snap, "vectors.npy"), mmap_mode="r")
    r0 = shard._reserve(n)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        if fp8:
            t = torch.from_numpy(np.array(mm[s:e]))
        else:
            t = torch.from_numpy(np.array(mm[s:e]).view(np.int16)).view(torch.bfloat16)
        shard.rows[r0 + s:r0 + e].copy_(t.to(shard.device))
    shard.rows_written(r0, n)   # the fp8 prefilter image, if the shard keeps one
    with open(os.path.join(snap, "payloads.jsonl"), encoding="utf-8") as f:
        empty = None
        for r, line in enumerate(f):
            if line == empty:          # a row without point id or payload: nothing to store
                continue
            a = json.loads(line)
            if a[0] is None and a[1:] == ["", "", "", 0, "", 0]:
                empty = line
                continue
            shard.payloads.set(r0 + r, a[0], Payload(*a[1:]))
    shard.publish()
    return n
