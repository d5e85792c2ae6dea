"""Dynamic micro-batchers in front of the GPU.

The reference encodes each message's sentences in fixed chunks of 8 padded to 514 tokens and
handles every query with its own B=1 forward (embedding_generator.rs:146, preprocessing main.rs
:205-246), blocking a tokio worker meanwhile.  Here concurrent requests from
any number of handlers are coalesced (up to a token budget / a short window) into ONE packed
varlen launch executed off the event loop, and the results are scattered back to the callers.
The same pattern batches concurrent semantic searches into one fused index scan.

The collection window only applies under load: a request that finds the batcher idle (no launch
ended within the last window) goes out with whatever is already queued, so an unloaded query pays
no batching delay.  Under load the next batch forms while the previous launch runs anyway.
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..utils.trace import stage


@dataclass
class _Req:
    texts: list
    fut: asyncio.Future
    t0: float = field(default_factory=time.perf_counter)


async def _collect(q: asyncio.Queue, first, window: float, last_end: float, full) -> list:
    """``first`` plus everything already queued; then, if a launch ended less than ``window`` ago
    (the batcher is busy), keep collecting until ``window`` after ``first`` or ``full(batch)``."""
    loop = asyncio.get_running_loop()
    batch = [first]
    while not full(batch) and not q.empty():
        batch.append(q.get_nowait())
    if loop.time() - last_end >= window:
        return batch
    deadline = loop.time() + window
    while not full(batch):
        timeout = deadline - loop.time()
        if timeout <= 0:
            break
        try:
            batch.append(await asyncio.wait_for(q.get(), timeout))
        except asyncio.TimeoutError:
            break
    return batch


class EmbedBatcher:
    """``depth`` launch groups in flight: group i + 1 is collected and tokenized (native, GIL
    released) while group i runs on the GPU, and only the enqueue of a group's kernels is
    serialized (``_gpu_lock``: the encoder's workspaces and captured graphs are shared); each
    group then waits on its OWN completion event, not on the stream (profiles/r5_e2e/: the serial
    loop left the mpnet query hop at 204 ms p50, tokenize + enqueue + a full-stream sync per
    group back to back)."""

    def __init__(self, encoder, tokenizer, token_budget: int = 65536, window_ms: float = 2.0,
                 max_seqs: int = 4096, metrics=None, depth: int = 2):
        import threading

        self.encoder = encoder
        self.tok = tokenizer
        self.token_budget = token_budget
        self.window = window_ms / 1000.0
        self.max_seqs = max_seqs
        self.metrics = metrics
        self.depth = max(1, int(depth))
        self._q: asyncio.Queue = asyncio.Queue()
        self._task: asyncio.Task | None = None
        self._lock = asyncio.Lock()
        self._gpu_lock = threading.Lock()
        self._last_end = float("-inf")   # loop time the last launch finished
        self._inflight = 0
        self._finishing: set = set()

    def start(self) -> None:
        if self._task is None:
            self._task = asyncio.create_task(self._run())

    async def embed(self, texts: list[str]) -> np.ndarray:
        """-> float32 [len(texts), H] pooled embeddings (the wire representation)."""
        if not texts:
            return np.zeros((0, self.encoder.cfg.hidden), np.float32)
        self.start()
        fut = asyncio.get_running_loop().create_future()
        await self._q.put(_Req(list(texts), fut))
        return await fut

    async def _run(self) -> None:
        loop = asyncio.get_running_loop()
        slots = asyncio.Semaphore(self.depth)
        while True:
            await slots.acquire()        # (requests keep queueing while every slot is busy)
            first = await self._q.get()
            # a group in flight counts as busy: collect for the window
            busy_since = loop.time() if self._inflight else self._last_end
            batch = await _collect(self._q, first, self.window, busy_since,
                                   lambda b: sum(len(r.texts) for r in b) >= self.max_seqs)
            texts = [t for r in batch for t in r.texts]
            self._inflight += 1
            fut = loop.run_in_executor(None, self._encode_all, texts)
            t = asyncio.create_task(self._finish(batch, texts, fut, slots))
            self._finishing.add(t)          # (a strong reference until it is done)
            t.add_done_callback(self._finishing.discard)

    async def _finish(self, batch, texts, fut, slots) -> None:
        loop = asyncio.get_running_loop()
        try:
            out = await fut
        except Exception as e:  # propagate to every waiter
            for r in batch:
                if not r.fut.done():
                    r.fut.set_exception(e)
            return
        finally:
            self._inflight -= 1
            self._last_end = loop.time()
            slots.release()
        o = 0
        for r in batch:
            if not r.fut.done():
                r.fut.set_result(out[o:o + len(r.texts)])
            o += len(r.texts)
            if self.metrics is not None:
                self.metrics.observe("embed.request", (time.perf_counter() - r.t0) * 1e3)
        if self.metrics is not None:
            self.metrics.inc("embed.sentences", len(texts))
            self.metrics.inc("embed.launch_groups")

    def _encode_all(self, texts: list[str]) -> np.ndarray:
        """Tokenize (native, GIL released) and run token-budgeted packed forwards."""
        from ..models.encoder import PackedBatch

        cfg = self.encoder.cfg
        with stage("tokenize", self.metrics, n=len(texts)):
            ids, cu = self.tok.encode_packed(texts)
        lens = np.diff(cu)
        dev = getattr(self.encoder, "device", torch.device("cpu"))
        if dev.type == "cuda":
            return self._encode_all_gpu(ids, cu, lens, dev)
        with self._gpu_lock:
            return self._encode_all_cpu(texts, ids, cu, lens, dev)

    def _encode_all_cpu(self, texts, ids, cu, lens, dev) -> np.ndarray:
        from ..models.encoder import PackedBatch

        cfg = self.encoder.cfg
        outs = []
        s = 0
        while s < len(texts):
            e, tok = s, 0
            while e < len(texts) and (e == s or tok + lens[e] <= self.token_budget):
                tok += int(lens[e])
                e += 1
            a, b = int(cu[s]), int(cu[e])
            sub_ids = ids[a:b]
            sub_cu = (cu[s:e + 1] - cu[s]).astype(np.int32)
            pos = np.concatenate([np.arange(cfg.position_offset, cfg.position_offset + int(L),
                                            dtype=np.int32) for L in lens[s:e]])
            pb = PackedBatch(torch.from_numpy(np.ascontiguousarray(sub_ids)), torch.from_numpy(pos),
                             None, torch.from_numpy(sub_cu), int(lens[s:e].max()))
            if dev.type == "cuda":
                pb = pb.to(dev, non_blocking=False)
            pooled, _unit = self.encoder.forward_packed(pb)
            outs.append(pooled.float().cpu().numpy())
            s = e
        return np.concatenate(outs, 0) if outs else np.zeros((0, cfg.hidden), np.float32)


    def _encode_all_gpu(self, ids, cu, lens, dev) -> np.ndarray:
        """K0/K19 pipeline: pinned host staging, H2D of sub-batch i+1 on a copy
        stream while sub-batch i computes, async D2H of every pooled block into one pinned output,
        ONE host sync per group (the reference syncs per chunk of 8, embedding_generator.rs:214)."""
        from ..models.encoder import PackedBatch

        cfg = self.encoder.cfg
        n = len(lens)
        out = torch.empty((n, cfg.hidden), dtype=torch.float32, pin_memory=True)
        keep = []   # host/device tensors that must outlive their async copies
        with self._gpu_lock:
            done = self._enqueue_gpu(ids, cu, lens, dev, cfg, out, keep)
        with stage("encode_d2h_sync", self.metrics):
            done.synchronize()   # this group's copies only, not a later group's kernels
        return out.numpy()

    def _enqueue_gpu(self, ids, cu, lens, dev, cfg, out, keep):
        from ..models.encoder import PackedBatch

        n = len(lens)
        compute = torch.cuda.current_stream(dev)
        copy = self._copy_stream(dev)
        s = 0
        while s < n:
            e, tok = s, 0
            while e < n and (e == s or tok + lens[e] <= self.token_budget):
                tok += int(lens[e])
                e += 1
            a, b = int(cu[s]), int(cu[e])
            sub_cu = (cu[s:e + 1] - cu[s]).astype(np.int32)
            pos = np.concatenate([np.arange(cfg.position_offset, cfg.position_offset + int(L),
                                            dtype=np.int32) for L in lens[s:e]])
            with stage("h2d", self.metrics):
                host = [torch.from_numpy(np.ascontiguousarray(x)).pin_memory()
                        for x in (ids[a:b], pos, sub_cu)]
                with torch.cuda.stream(copy):
                    d = [h.to(dev, non_blocking=True) for h in host]
                    ready = torch.cuda.Event()
                    ready.record(copy)
                compute.wait_event(ready)
                for t in d:
                    t.record_stream(compute)
            pb = PackedBatch(d[0], d[1], None, d[2], int(lens[s:e].max()))
            fwd = getattr(self.encoder, "forward_auto", self.encoder.forward_packed)
            with stage("encode_launch", self.metrics, tokens=b - a):
                pooled, _unit = fwd(pb)   # small groups replay a captured hipGraph
            out[s:e].copy_(pooled.float(), non_blocking=True)
            keep.append((host, pooled))
            s = e
        done = torch.cuda.Event()
        done.record(compute)
        return done

    def _copy_stream(self, dev):
        st = getattr(self, "_cs", None)
        if st is None:
            st = self._cs = torch.cuda.Stream(dev)
        return st


@dataclass
class _SReq:
    q: np.ndarray
    k: int
    fut: asyncio.Future


class SearchBatcher:
    """Coalesce concurrent searches into one fused scan (Q up to ``max_q`` queries per launch)."""

    def __init__(self, search_fn, window_ms: float = 1.0, max_q: int = 256, metrics=None):
        self.search_fn = search_fn  # (np.ndarray [nq, D] f32, k) -> (scores [nq,k], ids [nq,k])
        self.window = window_ms / 1000.0
        self.max_q = max_q
        self.metrics = metrics
        self._q: asyncio.Queue = asyncio.Queue()
        self._task = None
        self._last_end = float("-inf")

    async def search(self, q: np.ndarray, k: int):
        if self._task is None:
            self._task = asyncio.create_task(self._run())
        fut = asyncio.get_running_loop().create_future()
        await self._q.put(_SReq(np.asarray(q, np.float32).reshape(1, -1), int(k), fut))
        return await fut

    def _timed_search(self, qs, k):
        with stage("index_search", self.metrics, nq=len(qs), k=k):
            return self.search_fn(qs, k)

    async def _run(self) -> None:
        loop = asyncio.get_running_loop()
        while True:
            first = await self._q.get()
            batch = await _collect(self._q, first, self.window, self._last_end,
                                   lambda b: len(b) >= self.max_q)
            kmax = max(r.k for r in batch)
            qs = np.concatenate([r.q for r in batch], 0)
            try:
                s, i = await loop.run_in_executor(None, self._timed_search, qs, kmax)
            except Exception as e:
                self._last_end = loop.time()
                for j, r in enumerate(batch):
                    if not r.fut.done():
                        # a partial-result error carries per-query rows: give each its own slice
                        r.fut.set_exception(e.take(j, r.k) if hasattr(e, "take") else e)
                continue
            self._last_end = loop.time()
            for j, r in enumerate(batch):
                if not r.fut.done():
                    r.fut.set_result((s[j, :r.k], i[j, :r.k]))
            if self.metrics is not None:
                self.metrics.inc("search.batched_queries", len(batch))
                self.metrics.inc("search.launches")
