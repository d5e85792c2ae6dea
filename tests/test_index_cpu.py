"""Index shard semantics + checkpoint/resume (snapshot + WAL) on CPU."""
import os

import numpy as np
import pytest
import torch

from codename_symbiont_amd.index.persist import Wal
from codename_symbiont_amd.index.shard import HbmIndexShard, Payload
from codename_symbiont_amd.index.store import DimensionError, VectorStore


def _vecs(n, d, seed=0):
    return np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)


def test_shard_search_exact_and_small():
    sh = HbmIndexShard(16, 100, device="cpu")
    v = _vecs(50, 16)
    sh.append_f32(torch.from_numpy(v))
    q = torch.nn.functional.normalize(torch.from_numpy(v[[3, 7]]), dim=-1).bfloat16()
    s, r = sh.search(q, 3)
    assert r[:, 0].tolist() == [3, 7] and torch.all(s[:, 0] > 0.99)
    s, r = sh.search(q, 80)                     # k > rows: trailing slots empty
    assert (r[:, 50:] == -1).all() and torch.isinf(s[:, 50:]).all()
    with pytest.raises(MemoryError):
        sh.append_f32(torch.zeros(51, 16))


def test_upsert_overwrites_existing_ids():
    st = VectorStore(8, 10, device="cpu")
    v = _vecs(3, 8)
    st.upsert(["a", "b", "c"], v, [Payload("d", "u", t) for t in "abc"])
    st.upsert(["b"], -v[1:2], [Payload("d", "u", "B")])
    assert st.count == 3
    s, r = st.search(-v[1], 1)
    pid, p = st.lookup(r[0, 0])
    assert pid == "b" and p.sentence_text == "B"
    with pytest.raises(DimensionError, match="expected dim: 8, got 5"):
        st.upsert(["x"], _vecs(1, 5), [Payload()])


def _files(d, prefix=("manifest", "seg", "patch", "pay", "wal", "snapshot")):
    return sorted(n for n in os.listdir(d) if n.split(".")[0] in prefix)


def test_snapshot_wal_resume_and_torn_tail(tmp_path):
    d = str(tmp_path / "idx")
    st = VectorStore(8, 1000, device="cpu", snapshot_dir=d, snapshot_every=10)
    v = _vecs(25, 8, 1)
    for i in range(0, 25, 5):   # 25 points: snapshots at 10 and 20, 5 rows left in the WAL
        st.upsert([f"p{j}" for j in range(i, i + 5)], v[i:i + 5],
                  [Payload(f"doc{j}", "u", f"s{j}", j, "m", 100 + j) for j in range(i, i + 5)])
        st.flush()                                    # background snapshots, one at a time
    from codename_symbiont_amd.index.persist import committed_manifest

    man = committed_manifest(d)
    assert man["gen"] == 2 and man["count"] == 20
    # generation 2 absorbed generation 1 (10 new rows >= half of 10): one segment, one delta,
    # the rotated WALs both generations covered are gone
    assert _files(d) == ["manifest.2.json", "pay.2.bin", "seg.2.npy", "wal.log"]
    st.wal.close()  # crash: no close() snapshot
    with open(os.path.join(d, "wal.log"), "ab") as f:   # torn record at the tail
        f.write(b"SYMB\x05\x00\x00\x00garbage")
    st2 = VectorStore(8, 1000, device="cpu", snapshot_dir=d)
    assert st2.count == 25
    s, r = st2.search(v[22], 1)
    pid, p = st2.lookup(r[0, 0])
    assert pid == "p22" and p.sentence_order == 22 and p.processed_at_ms == 122
    # the torn tail was dropped, new writes still append and replay
    st2.upsert(["z"], v[:1] * 3, [Payload("dz")])
    st2.wal.close()
    recs = list(Wal.replay(os.path.join(d, "wal.log"), 8))
    assert sum(len(ids) for ids, _, _ in recs) >= 1
    st3 = VectorStore(8, 1000, device="cpu", snapshot_dir=d)
    assert st3.count == 26


def _store_with(d, n, seed=1, snapshot_every=1 << 30):
    st = VectorStore(8, 1000, device="cpu", snapshot_dir=d, snapshot_every=snapshot_every)
    v = _vecs(n, 8, seed)
    st.upsert([f"p{j}" for j in range(n)], v, [Payload(f"doc{j}", "u", f"s{j}", j) for j in range(n)])
    return st, v


def test_snapshot_crash_before_commit_keeps_previous_generation(tmp_path):
    """A crash after the new generation is written but before CURRENT moves: the boot loads the
    previous committed generation and replays the (untruncated) WAL -- nothing is lost, and the
    next snapshot still succeeds over the leftover files (and removes them)."""
    from codename_symbiont_amd.index import persist

    d = str(tmp_path / "idx")
    st, v = _store_with(d, 10)
    st.snapshot()                                     # gen 1 committed, its WAL deleted
    more = _vecs(5, 8, 9)
    st.upsert([f"q{j}" for j in range(5)], more, [Payload("dq")] * 5)   # in the WAL only
    persist.save_snapshot(st.shard, d, _crash_before_commit=True)       # gen 2 uncommitted
    st.wal.close()                                    # crash
    assert open(os.path.join(d, "CURRENT")).read().strip() == "manifest.1.json"
    st2 = VectorStore(8, 1000, device="cpu", snapshot_dir=d)
    assert st2.count == 15
    s, r = st2.search(more[3], 1)
    assert st2.lookup(r[0, 0])[0] == "q3"
    st2.snapshot()                                    # gen 3 commits; gens 1 and 2 are removed
    assert _files(d) == ["manifest.3.json", "pay.3.bin", "seg.3.npy", "wal.log"]
    st2.wal.close()
    assert VectorStore(8, 1000, device="cpu", snapshot_dir=d).count == 15


def _write_legacy(sh, d, name="snapshot.1"):
    """The round-2 full-rewrite format (meta.json + vectors.npy + payloads.jsonl)."""
    import json

    p = os.path.join(d, name)
    os.makedirs(p)
    with open(os.path.join(p, "meta.json"), "w") as f:
        json.dump({"dim": sh.dim, "count": sh.count, "format": 1, "dtype": "bf16"}, f)
    np.save(os.path.join(p, "vectors.npy"),
            sh.rows[:sh.count].view(torch.int16).numpy().view(np.uint16))
    with open(os.path.join(p, "payloads.jsonl"), "w") as f:
        for r in range(sh.count):
            pid, pl = sh.payloads.get(r)
            f.write(json.dumps([pid, pl.original_document_id, pl.source_url, pl.sentence_text,
                                pl.sentence_order, pl.model_name, pl.processed_at_ms]) + "\n")


def test_snapshot_legacy_layout_and_interrupted_swap(tmp_path):
    """Directories written by the previous formats still load: ``snapshot.<gen>`` named by
    CURRENT, or (pre-pointer) ``snapshot.old`` when a crash hit the old two-rename swap; the
    next snapshot writes the incremental format and removes the legacy directories."""
    from codename_symbiont_amd.index import persist

    d = str(tmp_path / "idx")
    os.makedirs(d)
    sh = HbmIndexShard(8, 100, device="cpu")
    sh.upsert([f"a{i}" for i in range(7)], torch.from_numpy(_vecs(7, 8)),
              [Payload(f"d{i}") for i in range(7)])
    _write_legacy(sh, d)
    with open(os.path.join(d, "CURRENT"), "w") as f:
        f.write("snapshot.1\n")
    sh1 = HbmIndexShard(8, 100, device="cpu")
    assert persist.load_snapshot(sh1, d) == 7 and sh1.payloads.get(3)[0] == "a3"
    os.remove(os.path.join(d, "CURRENT"))
    os.rename(os.path.join(d, "snapshot.1"), os.path.join(d, "snapshot.old"))
    sh2 = HbmIndexShard(8, 100, device="cpu")
    assert persist.load_snapshot(sh2, d) == 7
    assert torch.equal(sh2.rows[:7], sh.rows[:7])
    persist.save_snapshot(sh2, d)                     # stale .old no longer blocks a snapshot
    assert not os.path.exists(os.path.join(d, "snapshot.old"))
    sh3 = HbmIndexShard(8, 100, device="cpu")
    assert persist.load_snapshot(sh3, d) == 7 and sh3.payloads.get(6)[1].original_document_id == "d6"


def test_incremental_snapshot_cost_follows_new_rows(tmp_path):
    """5M-row shard: the first snapshot writes every row; the next one, after 10k new points and
    50 overwrites of old rows, writes only those (one segment, one patch, one payload delta) --
    its bytes and time follow the rows written since, not the shard.  Boot applies segment,
    patch and delta in generation order and reproduces the shard exactly."""
    import time

    from codename_symbiont_amd.index import persist

    D, N, NEW = 64, 5_000_000, 10_000
    d = str(tmp_path / "big")
    sh = HbmIndexShard(D, N + NEW, device="cpu")
    sh.fill_random(N, seed=3)
    t0 = time.perf_counter()
    j1 = persist.save_snapshot(sh, d)
    full_s = time.perf_counter() - t0
    assert j1.bytes_written >= N * D * 2
    rng = np.random.default_rng(0)
    v = rng.standard_normal((NEW, D)).astype(np.float32)
    sh.upsert([f"n{i}" for i in range(NEW)], torch.from_numpy(v),
              [Payload(f"doc{i}", "u", f"t{i}", i) for i in range(NEW)])
    old = rng.choice(N, 50, replace=False)
    sh.write_rows_f32(np.sort(old), torch.from_numpy(rng.standard_normal((50, D)).astype(np.float32)))
    t0 = time.perf_counter()
    j2 = persist.save_snapshot(sh, d)
    inc_s = time.perf_counter() - t0
    man = persist.committed_manifest(d)
    assert [s["n"] for s in man["segments"]] == [N, NEW] and man["patches"][0]["m"] == 50
    assert j2.bytes_written < (NEW + 50) * D * 2 * 2 + 4 * 1024 * 1024   # rows + payload delta
    # bytes (above) are the exact criterion; wall time is noisy on a loaded host (pytest -n)
    assert inc_s < full_s / 3, (inc_s, full_s)
    t0 = time.perf_counter()
    sh2 = HbmIndexShard(D, N + NEW, device="cpu")
    assert persist.load_snapshot(sh2, d) == N + NEW
    boot_s = time.perf_counter() - t0
    assert torch.equal(sh2.rows[:N + NEW], sh.rows[:N + NEW])
    assert sh2.payloads.get(N + 77)[1].sentence_text == "t77" and sh2.payloads.get(5)[0] is None
    print(f"full {full_s:.2f}s, incremental {inc_s:.3f}s, boot {boot_s:.2f}s")


def test_snapshot_merges_stream_from_disk_with_bounded_host_memory(tmp_path):
    """A cut that merges the big segment (here: too many patched rows, so every segment is
    rewritten) holds only the new rows and the overwrites in host memory: the merged segment is
    streamed from the older files at write time.  A base snapshot above
    FULL_CAPTURE_MAX streams the shard into its file under the lock instead of capturing it.
    Both reload exactly, patches of older generations included."""
    import tracemalloc

    from codename_symbiont_amd.index import persist

    D, N = 64, 400_000
    shard_bytes = N * D * 2
    d = str(tmp_path / "s")
    sh = HbmIndexShard(D, N + 5000, device="cpu")
    sh.fill_random(N, seed=11)
    old_cap = persist.ShardPersister.FULL_CAPTURE_MAX
    persist.ShardPersister.FULL_CAPTURE_MAX = shard_bytes // 8
    try:
        tracemalloc.start()
        j1 = persist.ShardPersister(d).cut(sh)      # base snapshot: streamed to its file
        peak1 = tracemalloc.get_traced_memory()[1]
        j1.write()
        tracemalloc.stop()
    finally:
        persist.ShardPersister.FULL_CAPTURE_MAX = old_cap
    assert isinstance(j1.seg, str) and peak1 < shard_bytes / 4, peak1
    rng = np.random.default_rng(5)
    # gen 2: a small patch on old rows; gen 3: > MAX_PATCH_FRAC patched rows -> full merge
    a = np.sort(rng.choice(N, 500, replace=False))
    sh.write_rows_f32(a, torch.from_numpy(rng.standard_normal((500, D)).astype(np.float32)))
    persist.save_snapshot(sh, d)
    assert len(persist.committed_manifest(d)["patches"]) == 1
    b = np.sort(rng.choice(N, int(N * 0.3), replace=False))
    sh.write_rows_f32(b, torch.from_numpy(rng.standard_normal((b.size, D)).astype(np.float32)))
    sh.append_f32(torch.from_numpy(rng.standard_normal((3000, D)).astype(np.float32)))
    tracemalloc.start()
    j3 = persist.ShardPersister(d).cut(sh)
    peak3 = tracemalloc.get_traced_memory()[1]
    tracemalloc.stop()
    assert isinstance(j3.seg, persist.SegMerge) and j3.seg.row0 == 0
    # the overwrites (30 % of the rows) and new rows, not the shard: < 0.45 x its bytes
    assert peak3 < 0.45 * shard_bytes, (peak3, shard_bytes)
    j3.write()
    man = persist.committed_manifest(d)
    assert man["patches"] == [] and [x["n"] for x in man["segments"]] == [N + 3000]
    sh2 = HbmIndexShard(D, N + 5000, device="cpu")
    assert persist.load_snapshot(sh2, d) == N + 3000
    assert torch.equal(sh2.rows[:N + 3000], sh.rows[:N + 3000])


def test_overwrite_only_shard_keeps_patch_files_bounded(tmp_path):
    """A shard that only gets overwrites (no appends between cuts) still folds its patches back
    into one segment once MAX_PATCH_FILES is reached (the rewrite used to need new
    rows), and every generation reloads exactly."""
    from codename_symbiont_amd.index import persist

    D, N = 8, 2000
    d = str(tmp_path / "o")
    sh = HbmIndexShard(D, N, device="cpu")
    sh.fill_random(N, seed=2)
    persist.save_snapshot(sh, d)
    rng = np.random.default_rng(1)
    for _ in range(3 * persist.ShardPersister.MAX_PATCH_FILES):
        rows = np.sort(rng.choice(N, 5, replace=False))
        sh.write_rows_f32(rows, torch.from_numpy(rng.standard_normal((5, D)).astype(np.float32)))
        persist.save_snapshot(sh, d)
        man = persist.committed_manifest(d)
        assert len(man["patches"]) <= persist.ShardPersister.MAX_PATCH_FILES
        assert sum(s["n"] for s in man["segments"]) == N
        n_patch_files = sum(1 for f in os.listdir(d) if f.startswith("patch.") and f.endswith(".rows.npy"))
        assert n_patch_files <= persist.ShardPersister.MAX_PATCH_FILES
    sh2 = HbmIndexShard(D, N, device="cpu")
    assert persist.load_snapshot(sh2, d) == N
    assert torch.equal(sh2.rows[:N], sh.rows[:N])


def test_geometric_merges_bound_the_file_count(tmp_path):
    from codename_symbiont_amd.index import persist

    d = str(tmp_path / "m")
    sh = HbmIndexShard(8, 5000, device="cpu")
    v = _vecs(3000, 8, 4)
    for i in range(0, 3000, 100):
        sh.upsert([f"p{j}" for j in range(i, i + 100)], torch.from_numpy(v[i:i + 100]),
                  [Payload(f"d{j}") for j in range(i, i + 100)])
        persist.save_snapshot(sh, d)
        man = persist.committed_manifest(d)
        assert len(man["segments"]) <= 8 and len(man["payloads"]) <= 8
        assert sum(s["n"] for s in man["segments"]) == sh.count
    sh2 = HbmIndexShard(8, 5000, device="cpu")
    assert persist.load_snapshot(sh2, d) == 3000
    assert torch.equal(sh2.rows[:3000], sh.rows[:3000])
    assert all(sh2.payloads.get(r)[0] == f"p{r}" for r in range(0, 3000, 37))


def test_background_snapshot_does_not_block_upserts(tmp_path, monkeypatch):
    import threading
    import time

    from codename_symbiont_amd.index import persist

    d = str(tmp_path / "bg")
    st, v = _store_with(d, 50)
    release = threading.Event()
    real = persist.SnapshotJob.write

    def slow(self, **kw):
        release.wait(10)
        return real(self, **kw)
    monkeypatch.setattr(persist.SnapshotJob, "write", slow)
    st.snapshot(wait=False)                           # cut taken; the write is held back
    assert st.snapshot_running()
    t0 = time.perf_counter()
    st.upsert(["late"], _vecs(1, 8, 8), [Payload("dl")])   # not blocked by the snapshot
    assert time.perf_counter() - t0 < 1.0 and st.snapshot_running()
    release.set()
    st.flush()
    assert persist.committed_manifest(d)["count"] == 50   # the cut, not the later upsert
    st.wal.close()
    st2 = VectorStore(8, 1000, device="cpu", snapshot_dir=d)
    assert st2.count == 51 and st2.lookup(50)[0] == "late"


def test_upsert_duplicate_ids_in_one_batch_last_wins():
    st = VectorStore(8, 10, device="cpu")
    v = _vecs(3, 8)
    st.upsert(["a", "b", "a"], v, [Payload("d", "u", t) for t in ("a1", "b", "a2")])
    assert st.count == 2
    s, r = st.search(v[2], 2)
    assert st.lookup(r[0, 0])[1].sentence_text == "a2"
    assert st.lookup(r[0, 0])[0] == "a"
    assert len(st.shard.payloads.id_to_row) == 2


def test_fp8_shard_cpu_path_and_snapshot(tmp_path):
    """fp8 storage on CPU (torch float8_e4m3fn == gfx950 OCP e4m3): search ranks like fp32 up to
    e4m3 rounding; snapshots keep the raw bytes and refuse a dtype mismatch."""
    from codename_symbiont_amd.index.persist import load_snapshot, save_snapshot

    D = 256
    v = _vecs(500, D, 3)
    sh = HbmIndexShard(D, 600, device="cpu", dtype="fp8")
    sh.append_f32(torch.from_numpy(v))
    assert sh.rows.dtype == torch.uint8
    q = torch.nn.functional.normalize(torch.from_numpy(v[[5, 77, 300]]), dim=-1)
    s, r = sh.search(q.bfloat16(), 4)
    assert r[:, 0].tolist() == [5, 77, 300]
    assert torch.allclose(s[:, 0], torch.ones(3), atol=0.03)   # self-similarity through e4m3
    save_snapshot(sh, str(tmp_path))
    sh2 = HbmIndexShard(D, 600, device="cpu", dtype="fp8")
    assert load_snapshot(sh2, str(tmp_path)) == 500
    assert torch.equal(sh2.rows[:500], sh.rows[:500])
    with pytest.raises(ValueError, match="dtype"):
        load_snapshot(HbmIndexShard(D, 600, device="cpu"), str(tmp_path))
    with pytest.raises(ValueError, match="fp8 index rows"):
        HbmIndexShard(320, 10, device="cpu", dtype="fp8")


def test_stage_tracing_records_metrics(caplog):
    import logging

    from codename_symbiont_amd.services.base import Metrics
    from codename_symbiont_amd.utils import trace

    m = Metrics()
    trace._ENABLED = True
    try:
        with caplog.at_level(logging.INFO, logger="symbiont.trace"):
            with trace.stage("unit", m, trace_id="req-1", n=3):
                pass
    finally:
        trace._ENABLED = False
    snap = m.snapshot()["latency_ms"]
    assert snap["stage.unit"]["n"] == 1
    assert any("[TRACE] stage=unit id=req-1" in r.message and "n=3" in r.message for r in caplog.records)


def test_search_result_fragments_match_wire_encoding_and_follow_overwrites():
    """vector_memory encodes replies by concatenating per-point cached JSON fragments; the bytes
    must equal SemanticSearchNatsResult.to_json() and an overwrite must refresh the fragment."""
    import numpy as np

    from codename_symbiont_amd.index.shard import Payload
    from codename_symbiont_amd.index.store import VectorStore
    from codename_symbiont_amd.ops._ext import native
    from codename_symbiont_amd.wire import (QdrantPointPayload, SemanticSearchNatsResult,
                                            SemanticSearchResultItem)

    st = VectorStore(8, 64, device="cpu")
    rng = np.random.default_rng(0)
    st.upsert(["a", "b\"ü"], rng.standard_normal((2, 8)).astype(np.float32),
              [Payload("d1", "u1", "first \n one", 0, "m", 5), Payload("d2", "u2", "two", 1, "m", 6)])
    scores, rows = st.search(rng.standard_normal((1, 8)).astype(np.float32), 2)
    frags = [st.result_fragments(r) for r in rows[0]]
    got = native().search_result_json("rid", scores[0], frags)
    items = []
    for s, r in zip(scores[0].tolist(), rows[0].tolist()):
        pid, p = st.lookup(r)
        items.append(SemanticSearchResultItem(pid, s, QdrantPointPayload(
            p.original_document_id, p.source_url, p.sentence_text, p.sentence_order, p.model_name,
            p.processed_at_ms)))
    assert got == SemanticSearchNatsResult("rid", items, None).to_json()
    err = 'index rank 1 unavailable: "x"'          # partial results carry an error_message
    assert (native().search_result_json("rid", scores[0], frags, err)
            == SemanticSearchNatsResult("rid", items, err).to_json())
    row_a = st.shard.payloads.id_to_row["a"]
    assert b'"first \\n one"' in st.result_fragments(row_a)[1]
    st.upsert(["a"], rng.standard_normal((1, 8)).astype(np.float32), [Payload("d1", "u1", "new", 0, "m", 9)])
    row_a = st.shard.payloads.id_to_row["a"]
    assert b'"sentence_text":"new"' in st.result_fragments(row_a)[1]


def test_reserved_rows_stay_invisible_until_published():
    """An upsert in another thread reserves rows before it writes them; a search racing it must
    only scan rows whose writes were already enqueued (``visible``), never reserved garbage."""
    sh = HbmIndexShard(8, 100, device="cpu")
    v = _vecs(10, 8)
    sh.append_f32(torch.from_numpy(v))
    r0 = sh._reserve(5)                       # reserved, not yet written
    sh.rows[r0:r0 + 5] = float("nan")
    assert sh.count == 15 and sh.visible == 10
    q = torch.nn.functional.normalize(torch.from_numpy(v[:3]), dim=-1).bfloat16()
    s, r = sh.search(q, 12)
    assert (r[:, 10:] == -1).all() and int(r.max()) < 10 and torch.isfinite(s[:, :10]).all()
    sh.write_f32(r0, torch.from_numpy(_vecs(5, 8, 4)))
    sh.publish()
    s, r = sh.search(q, 15)
    assert int(r.max()) == 14


def test_prefilter_image_follows_every_write(tmp_path):
    """The e4m3 prefilter image tracks appends, overwrites and snapshot loads (CPU path)."""
    from codename_symbiont_amd.index.persist import load_snapshot, save_snapshot

    D = 384
    sh = HbmIndexShard(D, 64, device="cpu", prefilter="fp8")
    st = VectorStore(D, 64, device="cpu", prefilter="fp8")
    v = _vecs(20, D, 5)
    st.upsert([f"p{i}" for i in range(20)], v, [Payload() for _ in range(20)])
    st.upsert(["p3"], -v[3:4], [Payload()])
    dec = lambda s: s.rows8[:s.count].view(torch.float8_e4m3fn).float() / 256.0  # noqa: E731
    assert torch.allclose(dec(st.shard), st.shard.rows[:20].float(), atol=0.01)
    sh.append_unit(st.shard.rows[:20])
    save_snapshot(sh, str(tmp_path))
    sh2 = HbmIndexShard(D, 64, device="cpu", prefilter="fp8")
    load_snapshot(sh2, str(tmp_path))
    assert torch.equal(sh2.rows8[:20], st.shard.rows8[:20])
    with pytest.raises(ValueError, match="prefilter"):
        HbmIndexShard(D, 8, device="cpu", dtype="fp8", prefilter="fp8")


def test_tile_sample_plan_invariants():
    """The emitting scan's in-place threshold sample (index/shard.py _tile_sample_plan, mirrored
    by index_mq.hip's phys_tile): every sampled tile lies inside the rows and below the exact
    tail, no tile is sampled twice (the sample's k-th best must be a lower bound), the gathered
    sub-sample is a subset of the sample, and the tail holds 4096..8191 rows.  A violation here
    is an out-of-bounds GPU read or an inexact search."""
    import torch

    from codename_symbiont_amd.index.shard import TILE_ROWS, HbmIndexShard

    shard = HbmIndexShard(384, 64, device="cpu")
    assert shard._tile_sample_plan(100_000) is None          # too small: gather-sample path
    for n in (1 << 20, (1 << 20) + 777, (1 << 20) + 4096, 12_500_000, 12_502_048, 50_000_000,
              100_000_000, 100_007_424, 2 ** 31 - 2 ** 20):
        ts, nv, t0, idx = shard._tile_sample_plan(n)
        assert ts == shard.MQ_TILE_SHIFT and nv >= shard.SEED_DIV
        assert shard.MQ_TAIL_ROWS <= n - t0 < shard.MQ_TAIL_ROWS + (TILE_ROWS << ts)
        v = torch.arange(nv, dtype=torch.int64)
        # the kernel's mapping, in 32-bit arithmetic as on the GPU
        h = ((v * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - ts)
        phys = (v << ts) + h
        assert int(phys.min()) >= 0 and int(phys.max() + 1) * TILE_ROWS <= t0
        assert len(torch.unique(phys)) == nv                  # one distinct tile per group
        assert bool(((phys >> ts) == v).all())                # tile v stays in group v
        sub_tiles = torch.unique(idx // TILE_ROWS)
        assert idx.numel() == sub_tiles.numel() * TILE_ROWS
        assert bool(torch.isin(sub_tiles, phys).all())        # sub-sample within the sample
    # the gather index is cached per (nv, shift): appends inside one tile group reuse it, and a
    # new group or another shift (the pruned search samples 1 in 2^5) rebuilds it
    n = 100_000_000
    a = shard._tile_sample_plan(n)[3]
    assert shard._tile_sample_plan(n + 1000)[3] is a
    b = shard._tile_sample_plan(n, shard.PRUNE_TILE_SHIFT)[3]
    assert b is not a and not torch.equal(b[: a.numel()], a[: b.numel()])
    c = shard._tile_sample_plan(n + (TILE_ROWS << shard.PRUNE_TILE_SHIFT), shard.PRUNE_TILE_SHIFT)[3]
    assert c is not b and c.numel() >= b.numel()


@pytest.mark.parametrize("stream,D", [("1", 384), ("0", 384), ("1", 1024)])
def test_int8_pruning_bound_holds_and_image_follows_writes(stream, D, monkeypatch):
    """The exact int8-pruned search (csrc/hip/index_stream.hip, index_i8.hip) relies on
    |q.x - q~.x~| <= |q| E + |q - q~| X with E = max |x - x~|, X = max |x~| over the rows written:
    check it for every (query, row) pair of random and outlier-heavy data, and that the shard's
    int8 image (the stream image, or the row-major one with SYMB_PRUNE_STREAM=0) and its (E, X)
    follow appends, scattered overwrites and snapshot loads (1024: stream scan only)."""
    from codename_symbiont_amd.index.shard import resolve_prune
    from codename_symbiont_amd.ops.reference import (quant_rows_i8_ref, stream_i8_decode,
                                                      stream_i8_tile_codes_ref)

    monkeypatch.setenv("SYMB_PRUNE_STREAM", stream)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3000, D, generator=g)
    x[:100, :4] *= 30.0                     # rows dominated by a few large components
    sh = HbmIndexShard(D, 4000, device="cpu", prune="i8")
    assert sh.stream == (stream == "1")
    sh.append_f32(x[:2000])
    sh.write_f32(5, x[2500:2501])           # an overwrite refreshes that row's image
    sh.write_rows_f32([40, 7, 1999], x[2600:2603])   # scattered overwrites too
    sh.append_f32(x[2000:])
    xb = sh.rows[:sh.count]
    # (the stream image: one scale per 32-row sub-tile; the row-major one: per row)
    x8, sx, err, xtn = (stream_i8_tile_codes_ref if sh.stream else quant_rows_i8_ref)(xb)
    if sh.stream:
        y8, ysx = stream_i8_decode(sh.img_i8[:(sh.count + 31) // 32], sh.count, D)
        assert torch.equal(y8, x8) and torch.allclose(ysx, sx)
        assert sh.rows_i8 is None
    else:
        assert torch.equal(sh.rows_i8[:sh.count], x8) and torch.allclose(sh.sx_i8[:sh.count], sx)
    E, X = float(sh.i8_bounds[0]), float(sh.i8_bounds[1])
    assert E >= float(err.max()) - 1e-7 and X >= float(xtn.max()) - 1e-7
    q = torch.nn.functional.normalize(torch.randn(64, D, generator=g), dim=-1).bfloat16()
    q8, sq, eq, _ = quant_rows_i8_ref(q)
    s = q.float() @ xb.float().t()
    s_i8 = (q8.float() @ x8.float().t()) * sq[:, None] * sx[None, :]
    margin = q.float().norm(dim=1) * E + eq * X
    assert ((s - s_i8).abs() <= margin[:, None] + 1e-6).all()
    assert resolve_prune("auto", "bf16", 384) == "i8"
    assert resolve_prune("auto", "bf16", 384, device="cuda") == "i8"
    # a CPU shard never pays for the int8 image under auto
    assert resolve_prune("auto", "bf16", 384, device="cpu") is None
    assert resolve_prune("auto", "fp8", 1024) is None and resolve_prune("none") is None
    assert resolve_prune("auto", "bf16", 384, prefilter="fp8") is None


def test_split_image_bound_holds_and_prunes_anisotropic_rows():
    """calibrate_prune: on the anisotropic corpus (a shared mean direction, power-law spread) the
    shard switches to the split image -- rows and queries rotated into the principal basis, 64
    leading components fp16, the rest int8 -- whose bound must hold for every (query, row) pair
    and must leave far fewer candidates above the true k-th score than the plain int8 bound; on
    isotropic rows the plain image stays.  Overwrites and appends after the calibration are imaged
    in the same basis."""
    from codename_symbiont_amd.index.synth import CorpusGen

    n, k = 20000, 10
    g = CorpusGen("anisotropic", 384, "cpu")
    sh = HbmIndexShard(384, n + 100, device="cpu", prune="i8")
    sh.append_f32(g.rows(n, seed=1))
    assert sh._i8_heavy == 0                       # below CALIB_MIN_ROWS: not calibrated yet
    q = g.unit(48, seed=99).bfloat16()
    xb = sh.rows[:n].float()
    s = q.float() @ xb.t()
    T = s.topk(k, dim=1).values[:, -1:]
    q8, sq, m_plain = sh.prune_query_image(q)
    est = sh.prune_estimate(q8, sq)
    assert ((s - est).abs() <= m_plain[:, None]).all()
    c_plain = (est + m_plain[:, None] >= T).sum(1).float()

    sh.calibrate_prune()
    assert sh._i8_heavy == 64 and sh.calib_share > 0.6 and sh.rows_i8.shape[1] == 448
    rot = sh._i8_rot
    assert torch.allclose(rot @ rot.t(), torch.eye(384, dtype=torch.float64), atol=1e-10)
    sh.write_f32(7, g.rows(1, seed=3))              # an overwrite, imaged in the new basis
    sh.append_f32(g.rows(50, seed=4))
    xb = sh.rows[:sh.count].float()
    s = q.float() @ xb.t()
    q8, sq, m = sh.prune_query_image(q)
    assert q8.shape == (48, 448)
    est = sh.prune_estimate(q8, sq)
    assert ((s - est).abs() <= m[:, None]).all(), float(((s - est).abs() - m[:, None]).max())
    T = s.topk(k, dim=1).values[:, -1:]
    c_split = (est + m[:, None] >= T).sum(1).float()
    assert (c_split >= k).all()                    # (the true top-k always survive)
    assert float(c_split.mean()) * 8 < float(c_plain.mean()), (c_split.mean(), c_plain.mean())
    assert float(m.mean()) * 3 < float(m_plain.mean())

    # isotropic rows keep the plain image (the split one would only cost bytes there)
    r = HbmIndexShard(384, 5000, device="cpu", prune="i8")
    r.append_f32(torch.randn(5000, 384, generator=torch.Generator().manual_seed(2)))
    r.calibrate_prune()
    assert r._i8_heavy == 0 and r.calib_share < 0.3
    assert (r.img_i8 is not None) if r.stream else r.rows_i8.shape[1] == 384


@pytest.mark.parametrize("stream,D", [("1", 384), ("1", 768), ("1", 1024), ("0", 384)])
def test_mx4_image_follows_writes_and_bounds_every_pair(stream, D, monkeypatch):
    """The MX-fp4 first-tier image (e2m1 nibbles + e8m0 block scales; the stream image at 384 and
    768, the row-major one with SYMB_PRUNE_STREAM=0) follows appends and scattered overwrites, its
    (E4, X4) cover every row written, and |q.x - q~.x~| stays within |q| E4 + |q - q~| X4 for every
    (query, row) pair."""
    from codename_symbiont_amd.ops import reference as R

    monkeypatch.setenv("SYMB_PRUNE_STREAM", stream)
    g = torch.Generator().manual_seed(9)
    sh = HbmIndexShard(D, 3000, device="cpu", prune="i8")
    assert sh.mx4_on
    sh.append_f32(torch.randn(2000, D, generator=g))
    sh.upsert(["a", "b"], torch.randn(2, D, generator=g), [Payload("da"), Payload("db")])
    sh.write_rows_f32([3, 100, 1999], torch.randn(3, D, generator=g))
    n = sh.count
    _, _, xt, nr = R.mx4_codes_ref(sh.rows[:n])
    if sh.stream:
        assert torch.equal(R.stream_mx4_decode(sh.img_mx4[:(n + 31) // 32], n, D), xt)
    else:
        img, sc, xt0, _ = R.quant_rows_mx4_ref(sh.rows[:n])
        assert torch.equal(sh.rows_mx4[:n], img) and torch.equal(sh.sc_mx4[:n], sc)
        assert torch.equal(R.mx4_decode_ref(img, sc), xt) and torch.equal(xt0, xt)
    E4, X4 = sh.mx4_bounds.tolist()
    assert E4 >= float(nr[:, 0].max()) - 1e-7 and X4 >= float(nr[:, 1].max()) - 1e-7
    q = torch.nn.functional.normalize(torch.randn(32, D, generator=g), dim=-1).bfloat16()
    q4, qs4, m4 = sh.mx4_query_image(q)
    qt = (R.stream_mx4_query_decode(q4, qs4) if sh.stream else R.mx4_decode_ref(q4, qs4))
    assert torch.equal(qt, R.mx4_codes_ref(q)[2])
    est = qt @ xt.t()
    s = q.float() @ sh.rows[:n].float().t()
    assert ((s - est).abs() <= m4[:, None]).all()


def test_e2m3_grid_and_codes():
    """The e2m3 value table (OCP MX: bias 1, 3 mantissa bits, max 7.5) and the quantiser's rounding:
    every code decodes back to itself, x / s lands on the nearest grid value."""
    from codename_symbiont_amd.ops import reference as R

    grid = torch.tensor(R.E2M3)
    assert grid[0] == 0 and grid[7] == 0.875 and grid[8] == 1.0 and grid[16] == 2.0
    assert grid[24] == 4.0 and grid[31] == 7.5 and bool((grid[1:] > grid[:-1]).all())
    x = torch.randn(64, 384, generator=torch.Generator().manual_seed(1))
    codes, e, xt, nr = R.mx6_codes_ref(x)
    assert int(codes.max()) < 64 and torch.equal(R._mx6_unpack(R._mx6_pack(codes)), codes.long())
    s = torch.ldexp(torch.ones_like(e, dtype=torch.float32), e).repeat_interleave(32, 1)
    a = (x / s).abs()
    assert float(a.max()) <= 7.5
    near = (a[..., None] - grid).abs().min(-1).values
    assert bool(((xt / s).abs() - a).abs().le(near + 1e-6).all())
    # ~4x finer than MX-fp4, ~4x coarser than per-row int8 on gaussian rows
    e4 = R.mx4_codes_ref(x)[3][:, 0] / nr[:, 2]
    e8 = R.quant_rows_i8_ref(x)[2] / nr[:, 2]
    e6 = nr[:, 0] / nr[:, 2]
    assert 2.5 < float(e4.mean() / e6.mean()) < 6 and 2 < float(e6.mean() / e8.mean()) < 8


@pytest.mark.parametrize("D", [384, 768])
def test_mx6_image_follows_writes_and_bounds_every_pair(D, monkeypatch):
    """The MX-fp6 middle-tier stream image (e2m3 codes in two 768-byte planes per k-step + e8m0
    block scales) follows appends and scattered overwrites, its (E6, X6) cover every row written,
    and |q.x - q~.x~| stays within |q| E6 + |q - q~| X6 for every (query, row) pair."""
    from codename_symbiont_amd.ops import reference as R

    monkeypatch.setenv("SYMB_PRUNE_STREAM", "1")
    monkeypatch.setenv("SYMB_PRUNE_MX6", "1")
    g = torch.Generator().manual_seed(19)
    sh = HbmIndexShard(D, 3000, device="cpu", prune="i8")
    assert sh.mx6_on and sh.img_mx6.shape[1] == sh._stream_rec(2)
    sh.append_f32(torch.randn(2000, D, generator=g))
    sh.upsert(["a", "b"], torch.randn(2, D, generator=g), [Payload("da"), Payload("db")])
    sh.write_rows_f32([3, 100, 1999], torch.randn(3, D, generator=g))
    n = sh.count
    _, _, xt, nr = R.mx6_codes_ref(sh.rows[:n])
    assert torch.equal(R.stream_mx6_decode(sh.img_mx6[:(n + 31) // 32], n, D), xt)
    E6, X6 = sh.mx6_bounds.tolist()
    assert E6 >= float(nr[:, 0].max()) - 1e-7 and X6 >= float(nr[:, 1].max()) - 1e-7
    q = torch.nn.functional.normalize(torch.randn(32, D, generator=g), dim=-1).bfloat16()
    q6, qs6, m6 = sh.mx6_query_image(q)
    qt = R.stream_mx6_query_decode(q6, qs6)
    assert torch.equal(qt, R.mx6_codes_ref(q)[2])
    est = qt @ xt.t()
    s = q.float() @ sh.rows[:n].float().t()
    assert ((s - est).abs() <= m6[:, None]).all()
    # the fp6 margin sits between the int8 and fp4 ones
    _, _, m8 = sh.prune_query_image(q)
    _, _, m4 = sh.mx4_query_image(q)
    assert bool((m8 < m6).all()) and bool((m6 < m4).all())


def test_mx6_tier_defaults(monkeypatch):
    """SYMB_PRUNE_MX6=auto keeps no fp6 image (measured never to apply, profiles/r5_lq/), so a
    100M x 384 shard allocates none; SYMB_PRUNE_MX6=1 keeps it at 384 / 768 for A/B runs."""
    a = HbmIndexShard(384, 256, device="cpu", prune="i8")
    b = HbmIndexShard(768, 256, device="cpu", prune="i8")
    assert not a.mx6_on and a.img_mx6 is None and not b.mx6_on
    monkeypatch.setenv("SYMB_PRUNE_MX6", "1")
    c = HbmIndexShard(384, 256, device="cpu", prune="i8")
    assert c.mx6_on == c.stream


def test_rwlock_prefers_a_waiting_writer():
    """Once a writer waits, new readers queue behind it (a stream of searches could
    starve upserts)."""
    import threading
    import time

    from codename_symbiont_amd.index.store import _RWLock

    lk = _RWLock()
    lk.acquire_read()                       # a search in flight
    order = []

    def writer():
        lk.acquire_write()
        order.append("w")
        lk.release_write()

    def reader():
        lk.acquire_read()
        order.append("r")
        lk.release_read()

    tw = threading.Thread(target=writer)
    tw.start()
    time.sleep(0.05)                        # the writer is now waiting on the first reader
    tr = threading.Thread(target=reader)
    tr.start()
    time.sleep(0.05)
    assert order == []                      # the new reader did not overtake the writer
    lk.release_read()
    tw.join(5)
    tr.join(5)
    assert order == ["w", "r"]
