"""Concurrency properties of the micro-batchers (SURVEY.md §5 race detection: hypothesis-driven
concurrency tests).  Any interleaving of concurrent callers with any request sizes must give
every caller exactly the result of processing its own request alone, and an executor failure
must reach every waiter of that launch group instead of hanging it."""
import asyncio

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from codename_symbiont_amd.services.batcher import EmbedBatcher, SearchBatcher


class _ToyEncoder:
    """Deterministic 'encoder': the pooled row of a sentence is a hash of its token ids."""

    class cfg:
        hidden = 8
        position_offset = 0

    import torch as _t
    device = _t.device("cpu")

    def forward_packed(self, b):
        import torch

        cu = b.cu_seqlens.tolist()
        ids = b.ids.tolist()
        rows = []
        for s, e in zip(cu[:-1], cu[1:]):
            seq = ids[s:e]
            rows.append([float((sum(seq) * (j + 1) + len(seq)) % 97) for j in range(8)])
        t = torch.tensor(rows, dtype=torch.float32)
        return t, t.bfloat16()


class _ToyTokenizer:
    def encode_packed(self, texts):
        ids, cu = [], [0]
        for t in texts:
            toks = [len(w) * 31 + ord(w[0]) for w in t.split()] or [1]
            ids += toks
            cu.append(len(ids))
        return np.array(ids, np.int32), np.array(cu, np.int32)


def _expected(texts):
    enc, tok = _ToyEncoder(), _ToyTokenizer()
    import torch

    from codename_symbiont_amd.models.encoder import PackedBatch

    ids, cu = tok.encode_packed(texts)
    b = PackedBatch(torch.from_numpy(ids), torch.zeros(len(ids), dtype=torch.int32), None,
                    torch.from_numpy(cu), 1)
    return enc.forward_packed(b)[0].numpy()


_words = st.text(alphabet="abcdefgh", min_size=1, max_size=6)
_texts = st.lists(st.lists(_words, min_size=1, max_size=5).map(" ".join), min_size=1, max_size=6)


@settings(max_examples=30, deadline=None)
@given(reqs=st.lists(_texts, min_size=1, max_size=12), budget=st.integers(4, 64),
       window_ms=st.sampled_from([0.0, 0.5, 3.0]))
def test_embed_batcher_concurrent_callers_get_their_own_rows(reqs, budget, window_ms):
    async def main():
        b = EmbedBatcher(_ToyEncoder(), _ToyTokenizer(), token_budget=budget, window_ms=window_ms)

        async def call(i, texts):
            await asyncio.sleep((i % 3) * 0.0005)   # interleave arrivals
            return await b.embed(texts)
        outs = await asyncio.gather(*(call(i, t) for i, t in enumerate(reqs)))
        b._task.cancel()
        return outs
    outs = asyncio.run(main())
    for texts, got in zip(reqs, outs):
        np.testing.assert_array_equal(got, _expected(texts))


@settings(max_examples=30, deadline=None)
@given(ks=st.lists(st.integers(1, 7), min_size=1, max_size=20), max_q=st.integers(1, 8))
def test_search_batcher_scatters_per_request_k(ks, max_q):
    rng = np.random.default_rng(len(ks))
    qs = [rng.standard_normal(4).astype(np.float32) for _ in ks]

    def search_fn(q, k):   # score j of query i = i-th query's first coordinate + j, ids = j
        s = np.stack([np.arange(k, dtype=np.float32) + row[0] for row in q])
        return s, np.tile(np.arange(k), (len(q), 1))

    async def main():
        b = SearchBatcher(search_fn, window_ms=1.0, max_q=max_q)
        outs = await asyncio.gather(*(b.search(q, k) for q, k in zip(qs, ks)))
        b._task.cancel()
        return outs
    for q, k, (s, i) in zip(qs, ks, asyncio.run(main())):
        assert s.shape == (k,) and i.tolist() == list(range(k))
        np.testing.assert_allclose(s, np.arange(k) + q[0])


def test_batcher_failure_reaches_every_waiter():
    def boom(q, k):
        raise RuntimeError("scan failed")

    async def main():
        b = SearchBatcher(boom, window_ms=5.0, max_q=64)
        res = await asyncio.gather(*(b.search(np.zeros(4, np.float32), 3) for _ in range(5)),
                                   return_exceptions=True)
        b._task.cancel()
        return res
    res = asyncio.run(asyncio.wait_for(main(), 10))
    assert all(isinstance(r, RuntimeError) and "scan failed" in str(r) for r in res)


def test_embed_batcher_failure_reaches_every_waiter():
    class Broken(_ToyEncoder):
        def forward_packed(self, b):
            raise RuntimeError("encoder failed")

    async def main():
        b = EmbedBatcher(Broken(), _ToyTokenizer(), token_budget=8, window_ms=2.0)
        res = await asyncio.gather(*(b.embed(["ab cd", "ef"]) for _ in range(4)),
                                   return_exceptions=True)
        ok = await asyncio.gather(b.embed([]), return_exceptions=True)   # empty: no launch
        b._task.cancel()
        return res, ok
    res, ok = asyncio.run(asyncio.wait_for(main(), 10))
    assert all(isinstance(r, RuntimeError) and "encoder failed" in str(r) for r in res)
    assert ok[0].shape == (0, 8)


def test_idle_request_skips_window_busy_requests_coalesce():
    """An unloaded request goes out at once (no batching delay); one that arrives while a launch
    just ended waits the window and is coalesced with the requests behind it."""
    import time

    launches = []

    def search_fn(q, k):
        launches.append(len(q))
        return np.zeros((len(q), k), np.float32), np.zeros((len(q), k), np.int64)

    async def main():
        b = SearchBatcher(search_fn, window_ms=300.0, max_q=64)
        t0 = time.perf_counter()
        await b.search(np.ones(4, np.float32), 1)          # idle: no 300 ms wait
        idle_s = time.perf_counter() - t0

        async def late(d):
            await asyncio.sleep(d)
            return await b.search(np.ones(4, np.float32), 1)
        # right after a launch ended: the first waits the window, the later two join it
        await asyncio.gather(late(0.0), late(0.05), late(0.1))
        b._task.cancel()
        return idle_s
    idle_s = asyncio.run(asyncio.wait_for(main(), 10))
    assert idle_s < 0.2
    assert launches == [1, 3]


def test_embed_batcher_overlaps_groups():
    """depth 2: group 2 is collected and tokenized while group 1 is still in its (slow) encode,
    and each caller still gets its own rows."""
    import threading
    import time

    events = []
    lock = threading.Lock()

    class SlowTok(_ToyTokenizer):
        def encode_packed(self, texts):
            with lock:
                events.append(("tok", texts[0].split()[0], time.perf_counter()))
            return super().encode_packed(texts)

    class SlowEnc(_ToyEncoder):
        def forward_packed(self, b):
            time.sleep(0.4)
            return super().forward_packed(b)

    async def main():
        b = EmbedBatcher(SlowEnc(), SlowTok(), token_budget=64, window_ms=0.0, depth=2)
        first = asyncio.create_task(b.embed(["aa bb"]))
        await asyncio.sleep(0.05)              # group 1 is in its encode now
        second = asyncio.create_task(b.embed(["cc dd"]))
        outs = await asyncio.gather(first, second)
        b._task.cancel()
        return outs
    outs = asyncio.run(asyncio.wait_for(main(), 10))
    np.testing.assert_array_equal(outs[0], _expected(["aa bb"]))
    np.testing.assert_array_equal(outs[1], _expected(["cc dd"]))
    t = {name: ts for _, name, ts in events}
    # group 2 tokenized ~50 ms after group 1, i.e. during group 1's 400 ms encode
    assert t["cc"] - t["aa"] < 0.35
