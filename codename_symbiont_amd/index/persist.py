"""Checkpoint / resume of an HBM index shard: INCREMENTAL snapshots + a rotating append-only WAL.

The reference persists through Qdrant, which keeps vectors and payloads on disk and writes them
incrementally (vector_memory_service/src/main.rs:39,52; docker volume ./data/qdrant_storage).
The HBM index is volatile, so each shard directory holds a log-structured snapshot:

  CURRENT                   commit pointer: "manifest.<gen>.json" (atomic replace + fsync)
  manifest.<gen>.json       {"format": 2, gen, dim, dtype, count, segments, patches, payloads}
  seg.<gen>.npy             rows [row0, row0 + n) as captured at generation gen (bf16 bit patterns
                            as uint16, or e4m3 bytes; .npy, memory-mappable)
  patch.<gen>.rows.npy      overwritten rows (int64 row ids) of OLDER segments ...
  patch.<gen>.vecs.npy      ... and their contents at generation gen
  pay.<gen>.bin             payload delta: the rows whose point id / payload changed since the
                            previous generation (columnar binary, see write_payloads)
  wal.log, wal.<seq>.log    the live WAL and WAL files rotated out at a snapshot cut

A snapshot writes only what changed since the previous one -- the new rows (one segment), the
overwritten older rows (one patch) and the changed payloads (one delta) -- so its cost follows the
rows written since, not the shard size.  Segments and payload deltas are merged geometrically (a
new segment absorbs its predecessor while it holds at least half as many rows; likewise deltas),
so a shard of N rows is O(log N) files and every row is rewritten O(log N) times in total; too
many patched rows trigger one full rewrite.  Boot applies the files in generation order (a later
segment, patch or delta wins), so a merged segment supersedes the patches written before it.

The cut (``ShardPersister.cut``) runs under the caller's lock and captures only what is not on
disk yet: the rows appended since the last cut, the older rows overwritten since (D2H) and the
payload delta, plus the WAL rotation.  ``SnapshotJob.write`` then writes, fsyncs and commits from
a background thread while upserts continue; a merged segment is STREAMED there from the older
segment files (memory-mapped), their patches, the captured overwrites and the captured new rows
into an ``open_memmap`` output, a chunk at a time -- host memory never holds a whole segment.  A
snapshot with no committed base (the first one, or a shard from elsewhere) streams the shard D2H
in chunks straight into its segment file under the lock when it is larger than FULL_CAPTURE_MAX
bytes, else captures it in host memory and writes in the background.  A crash at any
point leaves the previous committed manifest and every WAL file it does not cover, so boot =
committed manifest -> HBM, then replay of the uncovered WAL files in order.

WAL record: magic u32 | n u32 | body_len u32 | crc32(body) u32 | body, body = n x
(u16 id_len, id, u32 payload_len, payload JSON, f32[dim]).  A torn tail record (crash mid-write)
fails its length/CRC check and is dropped on replay.

Directories written by the previous full-rewrite format (``snapshot.<gen>/`` with vectors.npy +
payloads.jsonl, CURRENT naming it, or the older ``snapshot/``) still load.
"""
from __future__ import annotations

import json
import logging
import os
import struct
import zlib

import numpy as np
import torch

from .shard import HbmIndexShard, Payload

log = logging.getLogger("symbiont.index")

MAGIC = 0x53594D42  # "SYMB"
_HDR = struct.Struct("<IIII")


class Wal:
    """Append-only WAL ``<dir>/wal.log``; ``rotate(seq)`` moves it to ``wal.<seq>.log`` at a
    snapshot cut (records before the cut) and starts a fresh one."""

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

    def rotate(self, seq: int) -> str:
        """wal.log -> wal.<seq>.log (durable rename), fresh wal.log; returns the rotated path."""
        self._f.close()
        d = os.path.dirname(self.path) or "."
        rotated = os.path.join(d, f"wal.{seq}.log")
        os.replace(self.path, rotated)
        self._f = open(self.path, "ab")
        fsync_dir(d)
        return rotated

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


def wal_files(directory: str, after_gen: int) -> list[str]:
    """The WAL files a boot over a snapshot of generation ``after_gen`` must replay, in order:
    every rotated wal.<seq>.log with seq > after_gen, then the live wal.log."""
    rot = []
    if os.path.isdir(directory):
        for fn in os.listdir(directory):
            parts = fn.split(".")
            if len(parts) == 3 and parts[0] == "wal" and parts[2] == "log" and parts[1].isdigit():
                if int(parts[1]) > after_gen:
                    rot.append((int(parts[1]), os.path.join(directory, fn)))
    return [p for _, p in sorted(rot)] + [os.path.join(directory, "wal.log")]


CURRENT = "CURRENT"        # commit pointer: names the live manifest (or a legacy snapshot dir)
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


# ------------------------------------------------------------------ payload files (columnar)
_PAY_MAGIC = b"SYMP"
_PAY_STR = ("pid", "doc", "url", "text", "model")


def write_payloads(path: str, keys: np.ndarray, entries: list) -> None:
    """Columnar payload file: ``keys`` int64 [m] (rows, or gids for a group table), per entry
    (point_id | None, fields tuple | None) in PayloadStore.FIELDS order.  Layout: magic, u32
    version, u64 m, keys, u8 flags (1 = has point id, 2 = has payload), i64 order, i64 ts, then
    for each of the 5 strings u64 offsets[m + 1] + utf-8 blob.  Written in one pass, fsync'd."""
    m = len(entries)
    flags = np.zeros(m, np.uint8)
    order = np.zeros(m, np.int64)
    ts = np.zeros(m, np.int64)
    cols = [[] for _ in _PAY_STR]
    for i, (pid, f) in enumerate(entries):
        if pid is not None:
            flags[i] |= 1
        cols[0].append((pid or "").encode())
        if f is not None:
            flags[i] |= 2
            doc, url, text, so, model, pts = f
            cols[1].append((doc or "").encode())
            cols[2].append((url or "").encode())
            cols[3].append((text or "").encode())
            cols[4].append((model or "").encode())
            order[i] = int(so or 0)
            ts[i] = int(pts or 0)
        else:
            for c in cols[1:]:
                c.append(b"")
    with open(path, "wb") as fh:
        fh.write(_PAY_MAGIC + struct.pack("<IQ", 1, m))
        fh.write(np.ascontiguousarray(keys, np.int64).tobytes())
        fh.write(flags.tobytes())
        fh.write(order.tobytes())
        fh.write(ts.tobytes())
        for c in cols:
            off = np.zeros(m + 1, np.uint64)
            if m:
                np.cumsum(np.fromiter((len(b) for b in c), np.uint64, m), out=off[1:])
            fh.write(off.tobytes())
            fh.write(b"".join(c))
        fh.flush()
        os.fsync(fh.fileno())


def read_payloads(path: str):
    """-> (keys int64 [m], entries list of (point_id | None, fields tuple | None))."""
    with open(path, "rb") as fh:
        data = fh.read()
    if data[:4] != _PAY_MAGIC:
        raise ValueError(f"{path}: not a payload file")
    _ver, m = struct.unpack_from("<IQ", data, 4)
    o = 16
    keys = np.frombuffer(data, np.int64, m, o)
    o += 8 * m
    flags = np.frombuffer(data, np.uint8, m, o)
    o += m
    order = np.frombuffer(data, np.int64, m, o)
    o += 8 * m
    ts = np.frombuffer(data, np.int64, m, o)
    o += 8 * m
    strs = []
    for _ in _PAY_STR:
        off = np.frombuffer(data, np.uint64, m + 1, o).astype(np.int64)
        o += 8 * (m + 1)
        base = o
        blob = data
        strs.append((off, base, blob))
        o += int(off[-1]) if m else 0

    def col(j, i):
        off, base, blob = strs[j]
        return blob[base + off[i]: base + off[i + 1]].decode()

    entries = []
    for i in range(m):
        fl = int(flags[i])
        pid = col(0, i) if fl & 1 else None
        f = ((col(1, i), col(2, i), col(3, i), int(order[i]), col(4, i), int(ts[i]))
             if fl & 2 else None)
        entries.append((pid, f))
    return keys.copy(), entries


def merge_payload_files(paths: list[str], out: str) -> int:
    """Union of payload deltas, later files winning per key, into one file; returns its size."""
    merged: dict[int, tuple] = {}
    for p in paths:
        keys, ents = read_payloads(p)
        for k, e in zip(keys.tolist(), ents):
            merged[k] = e
    ks = np.fromiter(sorted(merged), np.int64, len(merged))
    write_payloads(out, ks, [merged[k] for k in ks.tolist()])
    return len(merged)


# ------------------------------------------------------------------ shard snapshots
def _rows_to_host(shard: HbmIndexShard, r0: int, r1: int, chunk: int = 1 << 20) -> np.ndarray:
    """Rows [r0, r1) as host bytes (uint16 bf16 patterns, or uint8 e4m3)."""
    fp8 = shard.dtype == "fp8"
    out = np.empty((r1 - r0, shard.dim), np.uint8 if fp8 else np.uint16)
    for s in range(r0, r1, chunk):
        e = min(r1, s + chunk)
        t = shard.rows[s:e]
        t = t if fp8 else t.view(torch.int16)
        out[s - r0:e - r0] = t.cpu().numpy().view(out.dtype)
    return out


def _host_to_rows(shard: HbmIndexShard, r0: int, a: np.ndarray, chunk: int = 1 << 20) -> None:
    fp8 = shard.dtype == "fp8"
    for s in range(0, a.shape[0], chunk):
        e = min(a.shape[0], s + chunk)
        b = np.array(a[s:e])   # (a writable copy: the source may be a read-only memmap)
        t = torch.from_numpy(b) if fp8 else torch.from_numpy(b.view(np.int16)).view(torch.bfloat16)
        shard.rows[r0 + s:r0 + e].copy_(t.to(shard.device))


def _save_npy(path: str, a: np.ndarray) -> None:
    with open(path, "wb") as f:
        np.save(f, a)
        f.flush()
        os.fsync(f.fileno())


def _rows_to_file(shard: HbmIndexShard, r0: int, r1: int, path: str, chunk: int = 1 << 20) -> int:
    """Rows [r0, r1) straight into the .npy ``path`` (chunked D2H, fsync'd); returns its bytes."""
    fp8 = shard.dtype == "fp8"
    out = np.lib.format.open_memmap(path, mode="w+", dtype=np.uint8 if fp8 else np.uint16,
                                    shape=(r1 - r0, shard.dim))
    for s in range(r0, r1, chunk):
        e = min(r1, s + chunk)
        t = shard.rows[s:e]
        t = t if fp8 else t.view(torch.int16)
        out[s - r0:e - r0] = t.cpu().numpy().view(out.dtype)
    out.flush()
    nbytes = out.nbytes
    del out
    fsync_file(path)
    return nbytes


class SegMerge:
    """A merged segment [row0, n) to stream at write time: the older segments ``sources`` (gen,
    row0, n) covering [row0, p0) read from their files, every older patch (gen, file) applied in
    generation order to the rows of segments older than it, then the overwrites captured at the
    cut (``dirty`` rows / vecs inside [row0, p0)), then the captured new rows [p0, n)."""

    def __init__(self, directory: str, dim: int, dtype, row0: int, p0: int, n: int, sources,
                 patches, dirty, new_rows):
        self.directory, self.dim, self.dtype = directory, dim, dtype
        self.row0, self.p0, self.n = row0, p0, n
        self.sources, self.patches, self.dirty, self.new_rows = sources, patches, dirty, new_rows

    def write(self, path: str, chunk: int = 1 << 20) -> int:
        d, row0 = self.directory, self.row0
        out = np.lib.format.open_memmap(path, mode="w+", dtype=self.dtype,
                                        shape=(self.n - row0, self.dim))
        seg_gen = []   # (start, end, gen) of every source segment
        for gen, s0, m in self.sources:
            src = np.load(os.path.join(d, f"seg.{gen}.npy"), mmap_mode="r")
            for a in range(0, m, chunk):
                b = min(m, a + chunk)
                out[s0 - row0 + a:s0 - row0 + b] = src[a:b]
            del src
            seg_gen.append((s0, s0 + m, gen))
        starts = np.asarray([x[0] for x in seg_gen], np.int64)
        gens = np.asarray([x[2] for x in seg_gen], np.int64)
        for pg in sorted(self.patches):
            rows = np.load(os.path.join(d, f"patch.{pg}.rows.npy"), mmap_mode="r")
            vecs = np.load(os.path.join(d, f"patch.{pg}.vecs.npy"), mmap_mode="r")
            for a in range(0, rows.shape[0], chunk):
                r = np.asarray(rows[a:a + chunk])
                keep = (r >= row0) & (r < self.p0)
                if not keep.any():
                    continue
                # a patch overrides only segments older than itself
                owner = gens[np.searchsorted(starts, r[keep], side="right") - 1]
                sel = np.flatnonzero(keep)[owner < pg]
                if sel.size:
                    out[r[sel] - row0] = np.asarray(vecs[a:a + chunk])[sel]
            del rows, vecs
        if self.dirty is not None:
            rows, vecs = self.dirty
            out[rows - row0] = vecs
        if self.new_rows is not None:
            out[self.p0 - row0:] = self.new_rows
        out.flush()
        nbytes = out.nbytes
        del out
        fsync_file(path)
        return nbytes


class SnapshotJob:
    """Everything one generation writes: captured in host memory at the cut, a ``SegMerge`` to
    stream from the older files, or a segment file the cut already wrote (``seg_file``)."""

    def __init__(self, directory: str, gen: int, manifest: dict, seg, patch, pay, pay_merge,
                 cleanup_wal_upto: int | None):
        self.directory, self.gen, self.manifest = directory, gen, manifest
        self.seg, self.patch, self.pay, self.pay_merge = seg, patch, pay, pay_merge
        self.cleanup_wal_upto = cleanup_wal_upto
        self.bytes_written = 0

    def write(self, _crash_before_commit: bool = False) -> None:
        d, g = self.directory, self.gen
        if self.seg is not None:
            p = os.path.join(d, f"seg.{g}.npy")
            if isinstance(self.seg, SegMerge):
                self.bytes_written += self.seg.write(p)
            elif isinstance(self.seg, str):      # written (and fsync'd) by the cut
                os.replace(self.seg, p)
                self.bytes_written += os.path.getsize(p)
            else:
                _save_npy(p, self.seg)
                self.bytes_written += self.seg.nbytes
        if self.patch is not None:
            rows, vecs = self.patch
            _save_npy(os.path.join(d, f"patch.{g}.rows.npy"), rows)
            _save_npy(os.path.join(d, f"patch.{g}.vecs.npy"), vecs)
            self.bytes_written += rows.nbytes + vecs.nbytes
        if self.pay is not None:
            keys, ents = self.pay
            tmp = os.path.join(d, f"pay.{g}.delta")
            write_payloads(tmp, keys, ents)
            if self.pay_merge:   # fold the older deltas this generation absorbs (from disk)
                merge_payload_files([os.path.join(d, f"pay.{x}.bin") for x in self.pay_merge]
                                    + [tmp], os.path.join(d, f"pay.{g}.bin"))
                os.remove(tmp)
            else:
                os.replace(tmp, os.path.join(d, f"pay.{g}.bin"))
            self.bytes_written += os.path.getsize(os.path.join(d, f"pay.{g}.bin"))
        man = os.path.join(d, f"manifest.{g}.json")
        write_atomic(man, json.dumps(self.manifest).encode())
        if _crash_before_commit:
            return
        write_atomic(os.path.join(d, CURRENT), f"manifest.{g}.json\n".encode())
        self._cleanup()

    def _cleanup(self) -> None:
        """Committed: remove every file the manifest does not reference (older generations,
        leftovers of crashed cuts, the legacy layout) and the WAL files it covers."""
        d, m = self.directory, self.manifest
        keep = {f"manifest.{self.gen}.json", CURRENT, "wal.log"}
        keep |= {f"seg.{s['gen']}.npy" for s in m["segments"]}
        keep |= {f"patch.{p['gen']}.{x}.npy" for p in m["patches"] for x in ("rows", "vecs")}
        keep |= {f"pay.{p['gen']}.bin" for p in m["payloads"]}
        for fn in os.listdir(d):
            path = os.path.join(d, fn)
            if fn in keep:
                continue
            if os.path.isdir(path):
                if fn in ("snapshot", "snapshot.old", "snapshot.tmp") or fn.startswith(_SNAP_PREFIX):
                    _rmtree(path)
                continue
            parts = fn.split(".")
            if parts[0] == "wal" and len(parts) == 3 and parts[1].isdigit():
                if self.cleanup_wal_upto is not None and int(parts[1]) <= self.cleanup_wal_upto:
                    os.remove(path)
                continue
            if parts[0] in ("seg", "patch", "pay", "manifest") and len(parts) >= 3 and parts[1].isdigit():
                os.remove(path)
        fsync_dir(d)


def committed_manifest(directory: str):
    """The committed format-2 manifest dict, or None (no snapshot / legacy layout)."""
    cur = os.path.join(directory, CURRENT)
    if not os.path.exists(cur):
        return None
    with open(cur, encoding="utf-8") as f:
        name = f.read().strip()
    if not name.startswith("manifest."):
        return None
    p = os.path.join(directory, name)
    if not os.path.exists(p):
        raise RuntimeError(f"snapshot pointer {cur} names {name!r}, which is missing")
    with open(p) as f:
        return json.load(f)


def committed_snapshot(directory: str) -> str | None:
    """Path of the committed snapshot: the manifest file (format 2), a legacy ``snapshot.<gen>``
    directory named by CURRENT, or the pre-pointer ``snapshot/`` (``snapshot.old`` when a crash
    hit its two-rename swap).  None when there is none."""
    cur = os.path.join(directory, CURRENT)
    if os.path.exists(cur):
        with open(cur, encoding="utf-8") as f:
            name = f.read().strip()
        p = os.path.join(directory, name)
        if name.startswith("manifest.") and os.path.exists(p):
            return p
        if os.path.exists(os.path.join(p, "meta.json")):
            return p
        raise RuntimeError(f"snapshot pointer {cur} names {name!r}, which is incomplete")
    for legacy in ("snapshot", "snapshot.old"):
        p = os.path.join(directory, legacy)
        if os.path.exists(os.path.join(p, "meta.json")):
            return p
    return None


class ShardPersister:
    """Snapshot state of one shard directory.  The shard records what changed since the last
    cut (``_persisted`` = rows covered, ``_dirty`` = covered rows overwritten since,
    ``payloads.dirty`` = rows whose point / payload changed since); ``_persist_key`` ties that
    record to this directory's committed generation, so a shard that did not come from (or last
    snapshot into) this directory gets a full snapshot."""

    MAX_PATCH_FRAC = 0.25     # patched rows above this share of the shard: full rewrite
    MAX_PATCH_FILES = 32
    # a base snapshot (no committed generation to build on) larger than this streams the rows
    # into its segment file under the lock instead of capturing them in host memory
    FULL_CAPTURE_MAX = 1 << 30

    def __init__(self, directory: str):
        self.directory = directory
        os.makedirs(directory, exist_ok=True)

    def _next_gen(self) -> int:
        g = 0
        for fn in os.listdir(self.directory):
            parts = fn.split(".")
            if len(parts) >= 2 and parts[1].isdigit() and parts[0] in (
                    "seg", "patch", "pay", "manifest", "wal", "snapshot"):
                g = max(g, int(parts[1]))
        return g + 1

    def cut(self, shard: HbmIndexShard, rotate_wal=None, full: bool = False) -> SnapshotJob:
        """Capture the next generation (caller holds the shard's write lock).  ``rotate_wal``:
        callable(seq) the store uses to rotate its WAL at exactly this point."""
        d = self.directory
        man = committed_manifest(d)
        gen = self._next_gen()
        n = shard.count
        incremental = (not full and man is not None
                       and getattr(shard, "_persist_key", None) == (os.path.abspath(d), man["gen"]))
        segs = [dict(s) for s in man["segments"]] if incremental else []
        patches = [dict(p) for p in man["patches"]] if incremental else []
        pays = [dict(p) for p in man["payloads"]] if incremental else []
        p0 = shard._persisted if incremental else 0
        dirty = sorted(r for r in shard._dirty if r < p0) if incremental else []
        # too many patched rows or patch files: one segment rewritten from disk (row0 = 0)
        rewrite = incremental and (
            len(dirty) + sum(p["m"] for p in patches) > self.MAX_PATCH_FRAC * max(n, 1)
            or len(patches) >= self.MAX_PATCH_FILES)
        # new segment = rows [p0, n), merged geometrically with its predecessors; a rewrite for
        # too many patches merges every segment (row0 = 0) the same way, from disk
        row0 = p0
        popped = []
        # (a rewrite merges every segment even when no row was appended since the last cut: a
        # shard that only gets overwrites must still fold its patches back in)
        while segs and (rewrite or (n - row0 > 0 and 2 * (n - row0) >= segs[-1]["n"])):
            popped.insert(0, segs.pop())
            row0 = popped[0]["row0"]
        fp8 = shard.dtype == "fp8"
        host_dt = np.uint8 if fp8 else np.uint16

        def capture(rows_list):
            rows = np.asarray(rows_list, np.int64)
            v = shard.rows.index_select(0, torch.from_numpy(rows).to(shard.device))
            v = v if fp8 else v.view(torch.int16)
            return rows, v.cpu().numpy().view(host_dt)

        seg = None
        if n > row0:
            if incremental:
                # only what is not on disk: the new rows and the overwrites inside the merged range
                in_seg = [r for r in dirty if r >= row0]
                seg = SegMerge(d, shard.dim, host_dt, row0, p0, n,
                               [(x["gen"], x["row0"], x["n"]) for x in popped],
                               [x["gen"] for x in patches] if popped else [],
                               capture(in_seg) if in_seg else None,
                               _rows_to_host(shard, p0, n) if n > p0 else None)
            elif (n - row0) * shard.dim * (1 if fp8 else 2) > self.FULL_CAPTURE_MAX:
                # no committed base: stream the shard into the segment file now (under the lock)
                tmp = os.path.join(d, f"seg.{gen}.npy.tmp")
                _rows_to_file(shard, row0, n, tmp)
                seg = tmp
            else:
                seg = _rows_to_host(shard, row0, n)
            segs.append({"gen": gen, "row0": row0, "n": n - row0})
            # patches wholly inside the rewritten range are superseded by it
            patches = [p for p in patches if p["min_row"] < row0]
        patch = None
        dirty = [r for r in dirty if r < row0]
        if dirty:
            rows, vecs = capture(dirty)
            patch = (rows, vecs)
            patches.append({"gen": gen, "m": len(dirty), "min_row": int(rows.min())})
        # payload delta: every row whose point / payload changed since the last cut (all rows
        # on a full snapshot), merged geometrically with the previous deltas
        ps = shard.payloads
        prows = sorted(r for r in ps.dirty if r < n) if incremental else sorted(
            set(ps.point_ids) | set(ps.fields))
        pay, merge = None, []
        if prows:
            pay = (np.asarray(prows, np.int64), [(ps.point_ids.get(r), ps.fields.get(r)) for r in prows])
            m_new = len(prows)
            while pays and 2 * m_new >= pays[-1]["m"]:
                last = pays.pop()
                merge.insert(0, last["gen"])
                m_new += last["m"]
            pays.append({"gen": gen, "m": m_new})
        manifest = {"format": 2, "gen": gen, "dim": shard.dim, "dtype": shard.dtype, "count": n,
                    "segments": segs, "patches": patches, "payloads": pays}
        if rotate_wal is not None:
            rotate_wal(gen)
        # the shard's change record now starts from this cut
        ps.track = True
        shard._persisted = n
        shard._dirty = set()
        ps.dirty = set()
        shard._persist_key = (os.path.abspath(d), gen)
        return SnapshotJob(d, gen, manifest, seg, patch, pay, merge,
                           cleanup_wal_upto=gen if rotate_wal is not None else None)

    def load(self, shard: HbmIndexShard) -> int:
        man = committed_manifest(self.directory)
        if man is None:
            return 0
        if man["dim"] != shard.dim:
            raise ValueError(f"snapshot dim {man['dim']} != index dim {shard.dim}")
        if man.get("dtype", "bf16") != shard.dtype:
            raise ValueError(f"snapshot dtype {man.get('dtype')} != index dtype {shard.dtype}")
        n = man["count"]
        if shard.count:
            raise RuntimeError("load into a non-empty shard")
        d = self.directory
        shard._reserve(n)
        events = ([(s["gen"], 0, s) for s in man["segments"]]
                  + [(p["gen"], 1, p) for p in man["patches"]])
        for _g, kind, s in sorted(events, key=lambda e: (e[0], e[1])):
            if kind == 0:
                _host_to_rows(shard, s["row0"], np.load(os.path.join(d, f"seg.{s['gen']}.npy"),
                                                         mmap_mode="r"))
            else:
                rows = np.load(os.path.join(d, f"patch.{s['gen']}.rows.npy"))
                vecs = np.load(os.path.join(d, f"patch.{s['gen']}.vecs.npy"))
                t = torch.from_numpy(vecs if shard.dtype == "fp8" else vecs.view(np.int16))
                if shard.dtype != "fp8":
                    t = t.view(torch.bfloat16)
                shard.rows.index_copy_(0, torch.from_numpy(rows).to(shard.device), t.to(shard.device))
        shard.rows_written(0, n)     # int8 / e4m3 images of every row
        for p in man["payloads"]:
            keys, ents = read_payloads(os.path.join(d, f"pay.{p['gen']}.bin"))
            for r, (pid, f) in zip(keys.tolist(), ents):
                if r < n:
                    shard.payloads.set(r, pid, None if f is None else Payload(*f))
        shard.payloads.dirty = set()
        shard.payloads.track = True
        shard.publish()
        shard._persisted = n
        shard._dirty = set()
        shard._persist_key = (os.path.abspath(d), man["gen"])
        return n


def save_snapshot(shard: HbmIndexShard, directory: str, _crash_before_commit: bool = False,
                  full: bool = False) -> SnapshotJob:
    """Synchronous snapshot of ``shard`` into ``directory`` (incremental when the shard's change
    record belongs to this directory's committed generation).  ``_crash_before_commit`` stops
    right before the pointer swap (tests)."""
    job = ShardPersister(directory).cut(shard, full=full)
    job.write(_crash_before_commit=_crash_before_commit)
    return job


def _load_legacy(shard: HbmIndexShard, snap: str, chunk: int = 1 << 20) -> int:
    """Format 1: ``snapshot.<gen>/`` (meta.json, vectors.npy, payloads.jsonl)."""
    with open(os.path.join(snap, "meta.json")) as f:
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
    _host_to_rows(shard, r0, mm, chunk)
    shard.rows_written(r0, n)
    with open(os.path.join(snap, "payloads.jsonl"), encoding="utf-8") as f:
        empty = None
        for r, line in enumerate(f):
            if line == empty:
                continue
            a = json.loads(line)
            if a[0] is None and a[1:] == ["", "", "", 0, "", 0]:
                empty = line
                continue
            shard.payloads.set(r0 + r, a[0], Payload(*a[1:]))
    shard.payloads.dirty = set()
    shard.publish()
    return n


def load_snapshot(shard: HbmIndexShard, directory: str) -> int:
    """Load the committed snapshot of ``directory`` into an empty shard; returns its row count."""
    if committed_manifest(directory) is not None:
        return ShardPersister(directory).load(shard)
    snap = committed_snapshot(directory)
    if snap is None:
        return 0
    return _load_legacy(shard, snap)


def committed_gen(directory: str) -> int:
    """Generation of the committed snapshot (0: none or legacy) -- rotated WAL files above it are
    not covered by it."""
    man = committed_manifest(directory)
    return man["gen"] if man else 0
