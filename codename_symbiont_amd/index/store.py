"""VectorStore: the Qdrant-collection replacement used by vector_memory_service.

One HBM shard (or, with ``group``, the rank-0 view of a multi-GPU IndexGroup) + host payload
store + durability (WAL per upsert batch, periodic snapshots).  API mirrors what the reference
does with qdrant-client (vector_memory_service/src/main.rs): ``upsert`` points with UUID ids
and 6-field payloads (wait=true semantics: durable + searchable on return) and ``search``
(limit=top_k, payload on, vectors off, no filter / threshold), returning cosine scores sorted
descending with fewer than k results when the collection is small.
"""
from __future__ import annotations

import logging
import os
import threading

import numpy as np
import torch

from .persist import ShardPersister, Wal, committed_gen, load_snapshot, wal_files
from .shard import HbmIndexShard, Payload

log = logging.getLogger("symbiont.index")


class DimensionError(ValueError):
    pass


from ..ops._ext import native as _native  # noqa: E402

class _RWLock:
    """Many readers (searches enqueuing their two halves) or one writer (an upsert enqueuing its
    row writes), writer-preferring: once a writer waits, new readers queue behind it, so a steady
    stream of searches cannot starve upserts.  Held while kernels are ENQUEUED; the only device
    sync under the read side is the large-k search's overflow check (k > 16, one ``item()``)."""

    def __init__(self):
        self._cv = threading.Condition()
        self._readers = 0
        self._writer = False
        self._writers_waiting = 0

    def acquire_read(self):
        with self._cv:
            while self._writer or self._writers_waiting:
                self._cv.wait()
            self._readers += 1

    def release_read(self):
        with self._cv:
            self._readers -= 1
            if self._readers == 0:
                self._cv.notify_all()

    def acquire_write(self):
        with self._cv:
            self._writers_waiting += 1
            try:
                while self._writer or self._readers:
                    self._cv.wait()
            finally:
                self._writers_waiting -= 1
            self._writer = True

    def release_write(self):
        with self._cv:
            self._writer = False
            self._cv.notify_all()


class VectorStore:
    def __init__(self, dim: int, capacity: int, device=None, snapshot_dir: str = "",
                 snapshot_every: int = 100_000, group=None, dtype: str = "bf16",
                 prefilter: str | None = None, prune: str | None = None):
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.dim = dim
        self.group = group
        self.shard = group.shard if group is not None else HbmIndexShard(dim, capacity, device,
                                                                            dtype=dtype,
                                                                            prefilter=prefilter,
                                                                            prune=prune)
        self.dir = snapshot_dir
        self.snapshot_every = snapshot_every
        self._since_snapshot = 0
        self._lock = threading.Lock()
        self._frag: dict[int, tuple[bytes, bytes]] = {}
        # SYMB_SEARCH_PIPELINE (default on, single GPU shard): a search's query-side pre-pass
        # (HbmIndexShard.search_begin) runs on one stream and its full-shard scan (search_end) on
        # another, so with the service's two scans in flight the next burst's pre-pass runs
        # under the current burst's scan (the bench's pipelined step, profiles/r3_pipeline/)
        self._streams = None
        if (group is None and self.shard.device.type == "cuda"
                and os.environ.get("SYMB_SEARCH_PIPELINE", "1") not in ("", "0")):
            self._streams = (torch.cuda.Stream(self.shard.device), torch.cuda.Stream(self.shard.device))
        # a pipelined search enqueues its pre-pass (begin) and its scan (end) under the read
        # side, an upsert its row writes under the write side: no write can land between one
        # search's begin and end (the scan would see rows, int8 images and bounds the pre-pass's
        # thresholds never saw), and every write is ordered after both halves (wait_stream)
        self._rw = _RWLock()
        self.wal = None
        self._bg: threading.Thread | None = None   # background snapshot writer
        self.snapshot_error: BaseException | None = None
        self.last_snapshot: dict = {}
        if snapshot_dir:
            import time

            os.makedirs(snapshot_dir, exist_ok=True)
            t0 = time.perf_counter()
            # a group restores every rank's shard collectively, then re-applies the WAL over it
            n = load_snapshot(self.shard, snapshot_dir) if group is None else group.load(snapshot_dir)
            self.shard.payloads.track = True
            t1 = time.perf_counter()
            m = 0
            # every WAL file the committed snapshot does not cover, in order (a crash between a
            # cut and its commit leaves the rotated file of that cut)
            for path in wal_files(snapshot_dir, committed_gen(snapshot_dir) if group is None else 0):
                Wal.repair(path)
                for ids, pls, vecs in Wal.replay(path, dim):
                    self._upsert_nolog(ids, vecs, pls)
                    m += len(ids)
            self.boot_s = {"snapshot_load_s": round(t1 - t0, 3),
                           "wal_replay_s": round(time.perf_counter() - t1, 3)}
            log.info("[INDEX_RESTORE] snapshot rows=%d (%.2fs), WAL replayed=%d (%.2fs)", n,
                     t1 - t0, m, self.boot_s["wal_replay_s"])
            self.wal = Wal(os.path.join(snapshot_dir, "wal.log"), dim)

    @property
    def count(self) -> int:
        return self.group.count if self.group is not None else self.shard.count

    def _upsert_nolog(self, point_ids, vecs, payloads):
        t = torch.as_tensor(np.ascontiguousarray(vecs, dtype=np.float32))
        if self._streams is not None:
            self._rw.acquire_write()
            try:
                # in-place overwrites (rows, int8 image, bounds) must not land under a pipelined
                # search's pre-pass or scan of those rows: order them after both streams' work
                cur = torch.cuda.current_stream(self.shard.device)
                cur.wait_stream(self._streams[0])
                cur.wait_stream(self._streams[1])
                out = self.shard.upsert(point_ids, t, payloads)
            finally:
                self._rw.release_write()
        elif self.group is not None:
            out = self.group.upsert(point_ids, t, payloads)
        else:
            out = self.shard.upsert(point_ids, t, payloads)
        for g in out or ():
            self._frag.pop(int(g), None)   # (re)written rows: their cached result JSON is stale
        return out

    def upsert(self, point_ids: list[str], vecs: np.ndarray, payloads: list[Payload]) -> None:
        vecs = np.asarray(vecs, dtype=np.float32)
        if vecs.ndim != 2 or vecs.shape[1] != self.dim:
            got = vecs.shape[-1] if vecs.ndim else 0
            raise DimensionError(f"Wrong input: Vector dimension error: expected dim: {self.dim}, got {got}")
        with self._lock:
            if self.group is not None:
                self.group.check_alive()    # refuse before logging: a refused upsert never lands
            if self.wal is not None:
                self.wal.append(point_ids, payloads, vecs)
            self._upsert_nolog(point_ids, vecs, payloads)
            if self.shard.device.type == "cuda":
                torch.cuda.synchronize(self.shard.device)  # wait=true: searchable on return
            self._since_snapshot += len(point_ids)
            if (self.wal is not None and self._since_snapshot >= self.snapshot_every
                    and not self.snapshot_running()):
                # cut under the lock (O(rows since the last snapshot)), write in the background
                self._start(self._cut_locked(), background=True)

    def snapshot_running(self) -> bool:
        return self._bg is not None and self._bg.is_alive()

    def flush(self) -> None:
        """Wait for a background snapshot to commit."""
        if self._bg is not None:
            self._bg.join()
            self._bg = None

    def _cut_locked(self):
        """The snapshot cut (caller holds ``_lock``): a group checkpoints collectively and
        synchronously (every rank incremental), then the WAL restarts; a single shard captures its
        changes and rotates the WAL, and returns the job that writes them."""
        self._since_snapshot = 0
        if self.group is not None:
            self.group.snapshot(self.dir)
            if self.wal is not None:
                self.wal.truncate()
            return None
        return ShardPersister(self.dir).cut(
            self.shard, rotate_wal=self.wal.rotate if self.wal is not None else None)

    def _start(self, job, background: bool) -> None:
        if job is None:
            return

        def run():
            import time

            t0 = time.perf_counter()
            try:
                job.write()
                self.last_snapshot = {"gen": job.gen, "bytes": job.bytes_written,
                                      "write_s": round(time.perf_counter() - t0, 3),
                                      "rows": job.manifest["count"]}
            except BaseException as e:  # noqa: BLE001 -- reported; the next snapshot is full
                self.snapshot_error = e
                self.shard._persist_key = None
                log.error("[INDEX_SNAPSHOT] generation %d failed: %s", job.gen, e)
        if background:
            self._bg = threading.Thread(target=run, name="index-snapshot", daemon=True)
            self._bg.start()
        else:
            run()
            if self.snapshot_error is not None:
                e, self.snapshot_error = self.snapshot_error, None
                raise e

    def snapshot(self, wait: bool = True) -> None:
        """Checkpoint now: incremental (rows, overwrites and payloads changed since the previous
        snapshot); ``wait=False`` writes in the background."""
        if not self.dir:
            return
        self.flush()
        with self._lock:
            job = self._cut_locked()
        self._start(job, background=not wait)

    def search(self, queries: np.ndarray, k: int):
        """queries f32 [nq, D] (any norm) -> (scores f32 [nq, k'], rows int64 [nq, k']); -1 = empty."""
        q = np.asarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None]
        if q.shape[1] != self.dim:
            raise DimensionError(f"Wrong input: Vector dimension error: expected dim: {self.dim}, "
                                 f"got {q.shape[1]}")
        k = int(k)
        if k <= 0 or self.count == 0:
            return np.zeros((q.shape[0], 0), np.float32), np.zeros((q.shape[0], 0), np.int64)
        if self._streams is not None:
            return self._search_pipelined(q, k)
        qt = torch.nn.functional.normalize(torch.from_numpy(q).to(self.shard.device), dim=-1)
        qt = qt.to(torch.bfloat16)
        if self.group is not None:
            try:
                s, r = self.group.search(qt, k)
            except Exception as e:
                if hasattr(e, "take"):   # PartialSearchError: hand numpy arrays to the service
                    e.scores, e.ids = e.scores.float().cpu().numpy(), e.ids.long().cpu().numpy()
                raise
        else:
            s, r = self.shard.search(qt, k)
        return s.float().cpu().numpy(), r.long().cpu().numpy()

    def _search_pipelined(self, q: np.ndarray, k: int):
        """search() of a single GPU shard on two streams: pre-pass (begin) on the first, scan
        (end) on the second.  Both order after every write already enqueued on the default
        stream (upserts), and each stream runs its calls in the order they were made, so two
        concurrent callers overlap one's pre-pass with the other's scan."""
        pre, scan = self._streams
        dev = self.shard.device
        qh = torch.from_numpy(q).to(dev, non_blocking=False)   # (before the lock: a host copy)
        self._rw.acquire_read()
        try:
            pre.wait_stream(torch.cuda.default_stream(dev))
            with torch.cuda.stream(pre):
                qt = torch.nn.functional.normalize(qh, dim=-1).to(torch.bfloat16)
                ctx = self.shard.search_begin(qt, k)
                done = torch.cuda.Event()
                done.record(pre)
            scan.wait_event(done)
            with torch.cuda.stream(scan):
                s, r = self.shard.search_end(ctx)
                ev = torch.cuda.Event()
                ev.record(scan)
        finally:
            self._rw.release_read()
        ev.synchronize()
        return s.float().cpu().numpy(), r.long().cpu().numpy()

    def lookup(self, gid: int):
        if self.group is not None:
            return self.group.payload(gid)
        return self.shard.payloads.get(int(gid))

    FRAG_CACHE_MAX = 1 << 20

    def result_fragments(self, gid: int):
        """(prefix, suffix) JSON bytes of this point's SemanticSearchResultItem around its score,
        cached per row (search results are encoded by concatenation, search_result_json);
        None for rows without a point id."""
        gid = int(gid)
        f = self._frag.get(gid)
        if f is None:
            pid, p = self.lookup(gid)
            if pid is None:
                return None
            from ..wire import QdrantPointPayload

            pl = QdrantPointPayload(p.original_document_id, p.source_url, p.sentence_text,
                                    int(p.sentence_order) & 0xFFFFFFFF, p.model_name,
                                    int(p.processed_at_ms)).to_json()
            f = (b'{"qdrant_point_id":' + _native().json_dumps(pid) + b',"score":',
                 b',"payload":' + pl + b'}')
            if len(self._frag) >= self.FRAG_CACHE_MAX:
                self._frag.clear()
            self._frag[gid] = f
        return f

    def close(self) -> None:
        if self.wal is not None:
            self.flush()
            self.snapshot()
            self.wal.close()
