"""vector_memory_service: storage + semantic search over the in-HBM index
(services/vector_memory_service/src/main.rs, with Qdrant replaced by index.store.VectorStore).

* ``data.text.with_embeddings`` -> one point per sentence: fresh UUIDv4 id and the 6-field
  payload {original_document_id, source_url, sentence_text, sentence_order (index within the
  message, + ``sentence_order_offset`` when the producer chunked), model_name, processed_at_ms
  (= message timestamp)} (main.rs:142-177); upsert is durable (WAL) before returning (wait=true).
* ``tasks.search.semantic.request`` request/reply -> SemanticSearchNatsResult; concurrent
  requests are coalesced into one fused MFMA scan by the SearchBatcher.  Error replies keep the
  reference's texts ("Failed to deserialize SemanticSearchNatsTask: ...", request_id "unknown";
  "Qdrant search failed for request_id <id>: <error>").
"""
from __future__ import annotations

import asyncio
import time
import uuid

import numpy as np

from ..utils.trace import stage
from ..index.shard import Payload, resolve_prune
from ..index.store import VectorStore
from ..models.config import get_config
from ..ops._ext import native
from ..utils import log as ulog
from ..wire import (SemanticSearchNatsResult, SemanticSearchNatsTask, TextWithEmbeddingsMessage,
                    WireError, subjects)
from .base import Service
from .batcher import SearchBatcher
from ..parallel.index_group import PartialSearchError


class VectorMemoryService(Service):
    name = "vector_memory_service"

    def __init__(self, *a, store: VectorStore | None = None, **kw):
        super().__init__(*a, **kw)
        dim = self.cfg.index_dim or get_config(self.cfg.model).hidden
        self.store = store or VectorStore(dim, self.cfg.index_capacity,
                                          device="cpu" if self.cfg.force_cpu else None,
                                          snapshot_dir=self.cfg.snapshot_dir,
                                          dtype=self.cfg.index_dtype,
                                          prefilter=self.cfg.index_prefilter or None,
                                          prune=resolve_prune(self.cfg.index_prune,
                                                              self.cfg.index_dtype, dim,
                                                              self.cfg.index_prefilter,
                                                              device=self._index_device()))
        if self.cfg.index_fill_random and self.store.count == 0:
            self.store.shard.fill_random(self.cfg.index_fill_random, seed=17)
        self.store.shard.scan_cus = self.cfg.scan_cus
        self.SEARCH_MAX_BATCH = max(1, self.cfg.search_max_batch)
        self.log.info("[INDEX_SETUP] collection '%s': dim %d, capacity %d, device %s, %d points",
                      self.cfg.collection, dim, self.store.shard.capacity, self.store.shard.device,
                      self.store.count)
        self.searcher = SearchBatcher(self.store.search, metrics=self.metrics)
        self._inflight: asyncio.Semaphore | None = None
        # scans in flight (token -> loop-clock start) and a running mean of the scan's duration:
        # while one runs, the next burst keeps collecting until it is a full 256-query block or
        # the running scan is due to end (_fill_deadline)
        self._scan_starts: dict[int, float] = {}
        self._scan_token = 0
        self._scan_ema: float | None = None

    def _index_device(self) -> str:
        """Where VectorStore(device=None) puts the shard (FORCE_CPU or no GPU: the CPU)."""
        import torch

        return "cpu" if self.cfg.force_cpu or not torch.cuda.is_available() else "cuda"

    async def setup(self) -> None:
        await self.subscribe_loop(subjects.TEXT_WITH_EMBEDDINGS, self.handle_store)
        # searches: whole drained bursts -> one native decode + one index scan + one socket write
        fill = self.cfg.search_align if self.cfg.search_fill else 0
        await self.subscribe_batches(subjects.SEARCH_SEMANTIC_REQUEST, self.handle_search_batch,
                                     max_batch=self.SEARCH_MAX_BATCH, align=self.cfg.search_align,
                                     gate=self._search_slot, fill=fill,
                                     fill_until=self._fill_deadline)

    async def _search_slot(self) -> None:
        """Wait for a free scan slot BEFORE drawing the next burst (requests keep queueing)."""
        if self._inflight is None:
            self._inflight = asyncio.Semaphore(self.SEARCH_MAX_INFLIGHT)
        await self._inflight.acquire()

    def _fill_deadline(self) -> float | None:
        """When the earliest scan in flight is due to end (loop clock), or None when none runs:
        an idle service launches a lone query at once; a busy one collects until the GPU is
        about to free up or the burst fills a 256-query block (a 100M-row scan costs about the
        same for 134 or 256 queries -- profiles/r5_e2e/ launched 134 on average, spending the
        shared GPU's time on partial blocks)."""
        if not self._scan_starts or self._scan_ema is None:
            return None
        return min(self._scan_starts.values()) + self._scan_ema

    # ------------------------------------------------------------------ storage
    async def handle_store(self, nmsg) -> None:
        try:
            msg = TextWithEmbeddingsMessage.from_json(nmsg.data)
        except WireError as e:
            self.log.warning("[TASK_DESERIALIZE_FAIL] Failed to deserialize TextWithEmbeddingsMessage: %s", e)
            return
        offset = 0
        try:  # extra field added by our chunking producer; absent from reference producers
            offset = int(native().json_loads(bytes(nmsg.data), False).get("sentence_order_offset", 0))
        except Exception:
            offset = 0
        self.log.info("[QDRANT_HANDLER] Received TextWithEmbeddingsMessage (original_id: %s), %d "
                      "embeddings from model '%s'.", msg.original_id, len(msg.embeddings_data),
                      msg.model_name)
        if not msg.embeddings_data:
            self.log.warning("[QDRANT_HANDLER] No embeddings data found in message for original_id: %s. "
                             "Skipping.", msg.original_id)
            return
        ids = [str(uuid.uuid4()) for _ in msg.embeddings_data]
        pls = [Payload(msg.original_id, msg.source_url, se.sentence_text, offset + i, msg.model_name,
                       msg.timestamp_ms) for i, se in enumerate(msg.embeddings_data)]
        try:
            vecs = np.stack([np.asarray(se.embedding, np.float32) for se in msg.embeddings_data])
        except ValueError as e:
            self.log.error("[QDRANT_HANDLER_ERROR] ragged embeddings for original_id %s: %s",
                           msg.original_id, e)
            return
        loop = asyncio.get_running_loop()
        try:
            with stage("upsert", self.metrics, trace_id=msg.original_id, n=len(ids)):
                await loop.run_in_executor(None, self.store.upsert, ids, vecs, pls)
        except Exception as e:
            self.log.error("[QDRANT_HANDLER_ERROR] Failed to upsert points for original_id %s: %s",
                           msg.original_id, e)
            self.metrics.inc("upsert_errors")
            return
        self.metrics.inc("points_upserted", len(ids))
        self.log.info("[QDRANT_HANDLER] Successfully upserted %d points for original_id: %s",
                      len(ids), msg.original_id)

    # ------------------------------------------------------------------ search
    async def reply(self, nmsg, res: SemanticSearchNatsResult) -> None:
        if nmsg.reply:
            await self.nc.publish(nmsg.reply, res.to_json())
        else:
            self.log.warning("[SEARCH_HANDLER] No reply subject provided for search task_id %s. "
                             "Results not sent.", res.request_id)

    SEARCH_MAX_BATCH = 512      # queries per fused scan launch (cfg.search_max_batch)
    SEARCH_MAX_INFLIGHT = 2     # scans in flight: batch i+1 decodes/scans while i's replies encode

    async def handle_search_batch(self, msgs) -> None:
        """A burst of SemanticSearchNatsTask requests: the regular ones are decoded natively into
        one [n, D] query matrix and answered from one scan; irregular ones (decode errors, wrong
        dimension, extra keys) take ``handle_search``, which produces the reference's error
        replies.  The scan runs in an executor thread while this loop goes back for the next
        burst (at most SEARCH_MAX_INFLIGHT scans in flight: the subscription's gate,
        ``_search_slot``, took a slot before this burst was drawn; ``_finish_search_batch``
        returns it)."""
        with stage("search_decode", self.metrics, n=len(msgs)):
            ok, ids, topk, q = native().search_tasks_batch([bytes(m.data) for m in msgs],
                                                           self.store.dim)
        good = np.flatnonzero(ok)
        if len(good) < len(msgs):
            for i in np.flatnonzero(~ok):
                self.spawn(self.handle_search(msgs[int(i)]))
        if not len(good):
            self._inflight.release()   # (the scan slot _search_slot took for this burst)
            return
        ks = topk[good]
        loop = asyncio.get_running_loop()
        self._scan_token += 1
        token = self._scan_token
        self._scan_starts[token] = loop.time()
        fut = loop.run_in_executor(None, self._batch_search, q[good], int(ks.max()))
        self.spawn(self._finish_search_batch([msgs[int(i)] for i in good],
                                             [ids[int(i)] for i in good], ks, fut, token))

    def _batch_search(self, qs, k):
        t0 = time.perf_counter()
        with stage("index_search", self.metrics, nq=len(qs), k=k):
            out = self.store.search(qs, k)
        dt = time.perf_counter() - t0
        self._scan_ema = dt if self._scan_ema is None else 0.8 * self._scan_ema + 0.2 * dt
        return out

    async def _finish_search_batch(self, msgs, rids, ks, fut, token=None) -> None:
        try:
            try:
                scores, rows = await fut
                errs = [None] * len(msgs)
            except PartialSearchError as e:
                scores, rows = e.scores, e.ids
                errs = [f"Qdrant search failed for request_id {r}: {e}" for r in rids]
                self.log.error("[SEARCH_HANDLER_QDRANT_FAIL] %s", errs[0])
                self.metrics.inc("search.partial", len(msgs))
            except Exception as e:
                out = []
                for m, r in zip(msgs, rids):
                    err = f"Qdrant search failed for request_id {r}: {e}"
                    self.log.error("[SEARCH_HANDLER_QDRANT_FAIL] %s", err)
                    if m.reply:
                        out.append((m.reply, SemanticSearchNatsResult(r, [], err).to_json()))
                await self.nc.publish_many(out)
                return
        finally:
            self._scan_starts.pop(token, None)
            self._inflight.release()
        self.metrics.inc("search.batched_queries", len(msgs))
        self.metrics.inc("search.launches")
        t_enc = time.perf_counter()
        # every reply of the burst in one native call (cached per-row result fragments around
        # the f32 scores; the same bytes as SemanticSearchNatsResult(...).to_json())
        bodies, skipped = native().search_results_batch(
            rids, np.ascontiguousarray(scores, np.float32), np.ascontiguousarray(rows, np.int64),
            np.asarray(ks, np.int64), self.store._frag, self.store.result_fragments,
            None if all(e is None for e in errs) else errs)
        out, sent = [], 0
        for m, rid, body in zip(msgs, rids, bodies):
            if m.reply:
                out.append((m.reply, body))
                sent += 1
            else:
                self.log.warning("[SEARCH_HANDLER] No reply subject provided for search task_id %s. "
                                 "Results not sent.", rid)
        if skipped:
            self.log.warning("[SEARCH_HANDLER] Found %d point(s) with missing or unexpected ID format. "
                             "Skipping.", skipped)
        self.metrics.observe("search_encode", (time.perf_counter() - t_enc) * 1e3)
        await self.nc.publish_many(out)
        self.log.info("[SEARCH_HANDLER] Sent search results for %d request(s) (one scan, request_ids "
                      "%s..%s)", sent, rids[0], rids[-1])

    async def handle_search(self, nmsg) -> None:
        try:
            task = SemanticSearchNatsTask.from_json(nmsg.data)
        except WireError as e:
            err = f"Failed to deserialize SemanticSearchNatsTask: {e}"
            self.log.error("[SEARCH_HANDLER_DESERIALIZE_FAIL] %s", err)
            await self.reply(nmsg, SemanticSearchNatsResult("unknown", [], err))
            return
        self.log.info("[SEARCH_HANDLER] Processing SemanticSearchNatsTask (request_id: %s, top_k: %d)",
                      task.request_id, task.top_k)
        try:
            q = np.asarray(task.query_embedding, np.float32)
            if q.shape[0] != self.store.dim:
                raise ValueError(f"Wrong input: Vector dimension error: expected dim: {self.store.dim}, "
                                 f"got {q.shape[0]}")
            with stage("search_request", self.metrics, trace_id=task.request_id, k=task.top_k):
                scores, rows = await self.searcher.search(q, task.top_k)
        except PartialSearchError as e:
            # a peer index rank is down: rank 0's own shard still answers (partial results)
            partial = f"Qdrant search failed for request_id {task.request_id}: {e}"
            self.log.error("[SEARCH_HANDLER_QDRANT_FAIL] %s", partial)
            self.metrics.inc("search.partial")
            scores, rows = e.scores, e.ids
        except Exception as e:
            err = f"Qdrant search failed for request_id {task.request_id}: {e}"
            self.log.error("[SEARCH_HANDLER_QDRANT_FAIL] %s", err)
            await self.reply(nmsg, SemanticSearchNatsResult(task.request_id, [], err))
            return
        else:
            partial = None
        # result JSON = per-point cached fragments around f32 scores (native concatenation; the
        # same bytes as SemanticSearchNatsResult(...).to_json())
        frags, keep = [], []
        skipped = 0
        for s, r in zip(scores.tolist(), rows.tolist()):
            if r < 0:
                continue
            f = self.store.result_fragments(r)
            if f is None:
                skipped += 1
                continue
            frags.append(f)
            keep.append(s)
        if skipped:  # one line per request (the reference logs one per point)
            self.log.warning("[SEARCH_HANDLER] Found %d point(s) with missing or unexpected ID format. "
                             "Skipping.", skipped)
        body = native().search_result_json(task.request_id, np.asarray(keep, np.float32), frags,
                                           partial)
        if nmsg.reply:
            await self.nc.publish(nmsg.reply, body)
        else:
            self.log.warning("[SEARCH_HANDLER] No reply subject provided for search task_id %s. "
                             "Results not sent.", task.request_id)
        self.log.info("[SEARCH_HANDLER] Sent %d search results for request_id %s", len(frags),
                      task.request_id)

    async def stop(self) -> None:
        await super().stop()
        self.store.close()


def main() -> None:
    """Single GPU: ``python -m ...vector_memory``.  A node: launch one process per GPU
    (``torch.distributed.run --nproc-per-node N -m codename_symbiont_amd.services.vector_memory``):
    rank 0 serves NATS over an IndexGroup, the other ranks execute its collective ops."""
    import os

    ulog.setup(VectorMemoryService.name, "info")
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        asyncio.run(VectorMemoryService().run_forever())
        return
    from ..parallel import dist as D
    from ..parallel.index_group import IndexGroup

    from ..utils.config import Config

    cfg = Config()
    info = D.init()
    dim = cfg.index_dim or get_config(cfg.model).hidden
    group = IndexGroup(info, dim, cfg.index_capacity // info.world + 1, dtype=cfg.index_dtype,
                       prefilter=cfg.index_prefilter or None,
                       prune=resolve_prune(cfg.index_prune, cfg.index_dtype, dim,
                                           cfg.index_prefilter, device=info.device))
    group.snapshot_root = cfg.snapshot_dir or None
    # liveness: every rank heart-beats on health.index.<rank>; rank 0 refuses ops while a peer is
    # silent (fast error replies instead of a collective blocked until the RCCL timeout)
    from ..parallel.heartbeat import Heartbeat, HeartbeatMonitor

    hb = Heartbeat(cfg.nats_url, info.rank, count_fn=lambda: group.shard.count)
    hb.start()
    if info.is_root:
        group.liveness = HeartbeatMonitor(cfg.nats_url, info.world)
        group.liveness.start()
    try:
        if info.is_root:
            store = VectorStore(dim, 0, snapshot_dir=cfg.snapshot_dir, group=group)
            asyncio.run(VectorMemoryService(cfg, store=store).run_forever())
        else:
            group.serve()
    finally:
        hb.stop()
        if group.liveness is not None:
            group.liveness.stop()
        group.stop()
        D.shutdown(info)


if __name__ == "__main__":
    main()
