"""Multi-process (gloo, world_size 2-4) tests of the distributed paths on CPU:
ShardedSearcher (all_gather queries -> local scan -> all_to_all partial top-k -> merge) and the
IndexGroup driven by rank 0 (lockstep broadcast ops, least-loaded owners, global ids)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from codename_symbiont_amd.parallel import dist as D
    return D.init(backend="gloo", device_type="cpu")


def _pipelined_worker(rank, world, port, out):
    """The bench's pipelined order on every rank: begin(i + 1) (query all_gather + pre-pass) is
    issued BEFORE end(i) (the packed all_to_all + merge); results equal plain search(), and each
    search costs exactly two collectives."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.parallel.sharded import ShardedSearcher
    info = _init(rank, world, port)
    D_, n, nq, k, steps = 32, 300, 5, 4, 4
    g = torch.Generator().manual_seed(1)
    all_rows = torch.nn.functional.normalize(torch.randn(world * n, D_, generator=g), dim=-1)
    qs = [torch.nn.functional.normalize(torch.randn(world * nq, D_, generator=g), dim=-1)
          for _ in range(steps)]
    shard = HbmIndexShard(D_, n, device="cpu")
    shard.append_unit(all_rows[rank * n:(rank + 1) * n].bfloat16())
    sr = ShardedSearcher(shard, info)
    mine = [q[rank * nq:(rank + 1) * nq].bfloat16() for q in qs]
    plain = [sr.search(q, k) for q in mine]
    c0 = sr.collectives
    h = {0: sr.begin(mine[0], k)}
    piped = []
    for i in range(steps):
        if i + 1 < steps:
            h[i + 1] = sr.begin(mine[i + 1], k)   # batch i+1's all_gather before batch i's end
        piped.append(sr.end(h.pop(i)))
    out[rank] = (all(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
                     for a, b in zip(plain, piped)), c0, sr.collectives - c0)
    D.barrier(info)
    D.shutdown(info)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_pipelined_order_matches_search(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_pipelined_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        same, c_plain, c_piped = out[r]
        assert same, f"rank {r}: pipelined results differ"
        assert c_plain == 2 * 4 and c_piped == 2 * 4   # all_gather + ONE packed all_to_all each


def _sharded_worker(rank, world, port, out):
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.parallel.sharded import ShardedSearcher
    info = _init(rank, world, port)
    D_, n, nq, k = 64, 500, 7, 5
    g = torch.Generator().manual_seed(0)
    all_rows = torch.nn.functional.normalize(torch.randn(world * n, D_, generator=g), dim=-1)
    all_q = torch.nn.functional.normalize(torch.randn(world * nq, D_, generator=g), dim=-1)
    shard = HbmIndexShard(D_, n, device="cpu")
    shard.append_unit(all_rows[rank * n:(rank + 1) * n].bfloat16())
    s, gid = ShardedSearcher(shard, info).search(all_q[rank * nq:(rank + 1) * nq].bfloat16(), k)
    out[rank] = (s.numpy(), gid.numpy())
    D.barrier(info)
    D.shutdown(info)


@pytest.mark.parametrize("world", [2, 3, 8])   # 8: the driver's N=8 rank count, rehearsed on gloo
def test_sharded_searcher_matches_global_topk(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_sharded_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    D_, n, nq, k = 64, 500, 7, 5
    g = torch.Generator().manual_seed(0)
    all_rows = torch.nn.functional.normalize(torch.randn(world * n, D_, generator=g), dim=-1).bfloat16().float()
    all_q = torch.nn.functional.normalize(torch.randn(world * nq, D_, generator=g), dim=-1).bfloat16().float()
    ref_s, ref_i = torch.topk(all_q @ all_rows.t(), k, dim=1)
    for r in range(world):
        s, gid = out[r]
        rows = (gid >> 40) * n + (gid & ((1 << 40) - 1))
        np.testing.assert_array_equal(rows, ref_i[r * nq:(r + 1) * nq].numpy())
        np.testing.assert_allclose(s, ref_s[r * nq:(r + 1) * nq].numpy(), atol=1e-5)


_EMBED_LENS = [[5, 17, 3, 40, 9, 12, 2, 31, 8, 6], [7, 9]]   # the 2-sentence batch leaves ranks idle


def _embed_batches(cfg):
    from codename_symbiont_amd.models.encoder import pack_token_ids

    rng = np.random.default_rng(4)
    return [pack_token_ids([rng.integers(1000, cfg.vocab_size, size=L).astype(np.int32) for L in lens], cfg)
            for lens in _EMBED_LENS]


def _embed_worker(rank, world, port, out, wire=None):
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import TorchEncoder
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.parallel.embed_group import EmbedGroup, GroupEncoder
    info = _init(rank, world, port)
    cfg = get_config("minilm-l6")
    group = EmbedGroup(info, TorchEncoder(cfg, seed=0),
                       wire_dtype=None if wire is None else getattr(torch, wire))
    if info.is_root:
        enc = GroupEncoder(group)
        out[0] = [enc.forward_packed(b)[0].numpy() for b in _embed_batches(cfg)]
        group.stop()
    else:
        group.serve()
    D.barrier(info)
    D.shutdown(info)


@pytest.mark.parametrize("world", [2, 3, 8])   # 8: the driver's N=8 rank count, on gloo
def test_embed_group_matches_single_process(world):
    """DP embedding over the group (token-balanced slices planned by rank 0 and sent in the
    header, all_gather back to rank 0) returns the same pooled embeddings, in input order, as one
    process encoding the whole batch -- also when ranks get no sentence at all (world 8, a
    2-sentence batch)."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import TorchEncoder
    from codename_symbiont_amd.parallel.embed_group import split_by_tokens

    cu = np.array([0, 5, 22, 25, 65, 74], np.int32)
    r = split_by_tokens(cu, 3)
    assert r[0][0] == 0 and r[-1][1] == 5 and all(a <= b for a, b in r)
    assert split_by_tokens(np.array([0, 7], np.int32), 4) == [(0, 1), (1, 1), (1, 1), (1, 1)]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_embed_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    cfg = get_config("minilm-l6")
    ref = TorchEncoder(cfg, seed=0)
    for got, b in zip(out[0], _embed_batches(cfg)):
        np.testing.assert_allclose(got, ref.forward_packed(b)[0].numpy(), rtol=1e-4, atol=1e-4)


def test_embed_group_bf16_wire():
    """The RCCL default wire (bf16 pooled rows) rounds each value once: every row keeps cosine
    >= 0.99999 to the f32 embedding (run here over gloo when its build has bf16 collectives)."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import TorchEncoder

    mgr = mp.Manager()
    out = mgr.dict()
    try:
        mp.start_processes(_embed_worker, args=(2, _free_port(), out, "bfloat16"), nprocs=2,
                           join=True, start_method="spawn")
    except Exception as e:   # noqa: BLE001 -- a gloo build without bf16 all_gather
        pytest.skip(f"gloo bf16 collectives unavailable: {e}")
    cfg = get_config("minilm-l6")
    ref = TorchEncoder(cfg, seed=0)
    for got, b in zip(out[0], _embed_batches(cfg)):
        want = ref.forward_packed(b)[0]
        cos = torch.nn.functional.cosine_similarity(torch.from_numpy(got), want, dim=-1)
        assert cos.min().item() >= 0.99999, cos
        np.testing.assert_allclose(got, want.numpy(), rtol=2 ** -8, atol=1e-6)


def _group_worker(rank, world, port, out):
    from codename_symbiont_amd.index.shard import Payload
    from codename_symbiont_amd.index.store import VectorStore
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.parallel.index_group import IndexGroup
    info = _init(rank, world, port)
    grp = IndexGroup(info, dim=32, capacity_per_rank=1000)
    if rank != 0:
        grp.serve()
        out[rank] = grp.shard.count
    else:
        store = VectorStore(32, 0, group=grp)
        rng = np.random.default_rng(1)
        vecs = rng.standard_normal((300, 32)).astype(np.float32)
        ids = [f"p{i}" for i in range(300)]
        for s in range(0, 300, 70):
            store.upsert(ids[s:s + 70], vecs[s:s + 70], [Payload(f"d{i}", "u", f"t{i}", i) for i in range(s, min(300, s + 70))])
        vecs[5] = -vecs[5]                                    # overwrite one point in place
        store.upsert(["p5"], vecs[5:6], [Payload("d5", "u", "t5-new", 5)])
        q = vecs[[5, 17, 299]]
        sc, gids = store.search(q, 4)
        unit = vecs / np.linalg.norm(vecs, axis=1, keepdims=True)
        ref = np.argsort(-(q / np.linalg.norm(q, axis=1, keepdims=True)) @ unit.T, axis=1)[:, :4]
        got = [[int(store.lookup(g)[1].sentence_text.split("-")[0][1:]) for g in row] for row in gids]
        out[0] = (got, ref.tolist(), store.count, store.lookup(gids[0][0])[1].sentence_text)
        grp.stop()
    D.shutdown(info)


def test_index_group_upsert_search_overwrite():
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_group_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    got, ref, count, text = out[0]
    assert got == ref
    assert count == 300 and text == "t5-new"
    assert out[1] == 100 and out[2] == 100          # least-loaded placement balances the shards


def _group4_worker(rank, world, port, out):
    """4 ranks: batched upserts (new + overwritten ids in one batch) and searches through the lean
    path (one packed all_gather per search) == one shard holding every point."""
    from codename_symbiont_amd.index.shard import HbmIndexShard, Payload
    from codename_symbiont_amd.index.store import VectorStore
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.parallel.index_group import IndexGroup
    info = _init(rank, world, port)
    grp = IndexGroup(info, dim=48, capacity_per_rank=2000)
    if rank != 0:
        grp.serve()
        out[rank] = grp.shard.count
    else:
        store = VectorStore(48, 0, group=grp)
        ref = HbmIndexShard(48, 8000, device="cpu")
        rng = np.random.default_rng(11)
        vecs = rng.standard_normal((3000, 48)).astype(np.float32)
        ids = [f"p{i}" for i in range(3000)]
        pls = [Payload(f"d{i}", "u", f"t{i}", i) for i in range(3000)]
        for s in range(0, 3000, 500):
            store.upsert(ids[s:s + 500], vecs[s:s + 500], pls[s:s + 500])
            ref.upsert(ids[s:s + 500], torch.from_numpy(vecs[s:s + 500]), pls[s:s + 500])
        # one batch mixing 40 overwrites (scattered over every rank) and 10 new points
        ow = rng.choice(3000, 40, replace=False).tolist()
        new_v = rng.standard_normal((50, 48)).astype(np.float32)
        b_ids = [ids[i] for i in ow] + [f"n{i}" for i in range(10)]
        b_pl = [Payload("x", "u", f"w{i}", i) for i in range(50)]
        store.upsert(b_ids, new_v, b_pl)
        ref.upsert(b_ids, torch.from_numpy(new_v), b_pl)
        q = np.concatenate([rng.standard_normal((20, 48)).astype(np.float32), new_v[:5]])
        grp.comm_stats.clear()
        sc, gids = store.search(q, 7)
        rs, rr = ref.search(torch.nn.functional.normalize(torch.from_numpy(q), dim=-1).bfloat16(), 7)
        got = [[store.lookup(g)[1].sentence_text for g in row] for row in gids]
        want = [[ref.payloads.get(int(r))[1].sentence_text for r in row] for row in rr.tolist()]
        out[0] = (got, want, float(np.abs(sc - rs.numpy()).max()), dict(grp.comm_stats),
                  store.count)
        grp.stop()
    D.shutdown(info)


@pytest.mark.parametrize("world", [4, 8])   # 8: the driver's N=8 rank count, on gloo
def test_index_group_four_ranks_lean_search_matches_single_shard(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_group4_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    got, want, sdiff, stats, count = out[0]
    assert got == want and sdiff < 1e-5
    assert count == 3010 and sum(out[r] for r in range(1, world)) + 0 <= 3010
    ops, colls, nbytes = stats["search"]
    assert ops == 1 and colls == 3                 # header, queries, ONE packed all_gather
    assert nbytes == 32 + 25 * 48 * 4 + world * 25 * 7 * 16   # f32 queries on gloo


def _group_snapshot_worker(rank, world, port, snap, phase, out, crash_mid=False):
    """phase 0: ingest, snapshot, ingest more (WAL only), crash.  phase 1: restore + search."""
    from codename_symbiont_amd.index.shard import Payload
    from codename_symbiont_amd.index.store import VectorStore
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.parallel.index_group import IndexGroup
    info = _init(rank, world, port)
    grp = IndexGroup(info, dim=16, capacity_per_rank=500)
    grp.snapshot_root = snap
    rng = np.random.default_rng(7)
    vecs = rng.standard_normal((200, 16)).astype(np.float32)
    if rank != 0:
        grp.serve()
        out[(phase, rank)] = grp.shard.count
    else:
        store = VectorStore(16, 0, snapshot_dir=snap, snapshot_every=10**9, group=grp)
        if phase == 0:
            ids = [f"p{i}" for i in range(200)]
            pls = [Payload(f"d{i}", "u", f"t{i}", i) for i in range(200)]
            store.upsert(ids[:150], vecs[:150], pls[:150])
            store.snapshot()                                   # collective checkpoint
            store.upsert(ids[150:], vecs[150:], pls[150:])     # only in the WAL
            store.upsert(["p3"], -vecs[3:4], [Payload("d3", "u", "t3-new", 3)])
            out[(0, 0)] = store.count
            if crash_mid:
                # crash INSIDE the next snapshot: every rank saved its shard and rank 0 wrote the
                # new payload table, but group.json was never replaced
                from codename_symbiont_amd.parallel.index_group import OP_SNAPSHOT

                with grp._op_lock:
                    grp._header(OP_SNAPSHOT)
                    grp._do_snapshot(snap)
                    grp._commit_group(snap, _crash_before_commit=True)
            store.wal.close()                                  # crash: no final snapshot
        else:
            out[(1, 0)] = store.count
            q = np.concatenate([vecs[[10, 170]], -vecs[3:4]])
            _, gids = store.search(q, 1)
            out["texts"] = [store.lookup(int(g[0]))[1].sentence_text for g in gids]
        grp.stop()
    D.shutdown(info)


@pytest.mark.parametrize("crash_mid", [False, True], ids=["clean", "crash_mid_snapshot"])
def test_index_group_snapshot_restore(tmp_path, crash_mid):
    from codename_symbiont_amd.index.persist import committed_manifest

    world = 2
    snap = str(tmp_path / "snap")
    mgr = mp.Manager()
    out = mgr.dict()
    for phase in (0, 1):
        mp.start_processes(_group_snapshot_worker,
                           args=(world, _free_port(), snap, phase, out, crash_mid),
                           nprocs=world, join=True, start_method="spawn")
    assert os.path.exists(os.path.join(snap, "group.json"))
    man = committed_manifest(os.path.join(snap, "rank1"))
    assert man is not None and all(os.path.exists(os.path.join(snap, "rank1", f"seg.{s['gen']}.npy"))
                                   for s in man["segments"])
    import json

    meta = json.load(open(os.path.join(snap, "group.json")))
    assert meta["format"] == 3 and all(os.path.exists(os.path.join(snap, f"group_pay.{f['gen']}.bin"))
                                       for f in meta["payload_files"])
    assert out[(0, 0)] == 200 and out[(1, 0)] == 200      # 150 from the snapshot + 50 from the WAL
    assert out[(1, 1)] == 100                             # rank 1's shard restored, then WAL rows
    assert out["texts"] == ["t10", "t170", "t3-new"]


def _dead_rank_worker(rank, world, port, out):
    """Rank 1 dies while rank 0 runs a search: rank 0 must get an error, not hang."""
    os.environ["SYMB_COLLECTIVE_TIMEOUT_S"] = "20"
    import time

    from codename_symbiont_amd.index.store import VectorStore
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.parallel.index_group import IndexGroup
    info = _init(rank, world, port)
    grp = IndexGroup(info, dim=8, capacity_per_rank=100)
    if rank == 1:
        h = grp._header(0).tolist()          # the UPSERT op runs normally ...
        grp._do_upsert(h[1])
        grp._header(0)                       # ... then the SEARCH header arrives and the rank dies
        os._exit(3)
    from codename_symbiont_amd.index.shard import Payload
    store = VectorStore(8, 0, group=grp)
    store.upsert(["a", "b", "c", "d"], np.eye(4, 8, dtype=np.float32), [Payload()] * 4)
    t0 = time.time()
    try:
        store.search(np.ones((1, 8), np.float32), 3)
        out["result"] = "returned"
    except Exception as e:     # noqa: BLE001 - any collective error is the expected outcome
        out["result"] = type(e).__name__
    out["seconds"] = time.time() - t0
    os._exit(0)


def test_dead_index_rank_errors_instead_of_hanging():
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_dead_rank_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert not any(p.is_alive() for p in ps)
    assert out.get("result") not in (None, "returned"), out
    assert out["seconds"] < 60


def _heartbeat_worker(rank, world, port, nats_url, out):
    """Rank 2 stops heart-beating (dies) after an upsert; rank 0 must refuse the next search at
    once instead of entering a collective that would wait for the dead peer."""
    os.environ["SYMB_COLLECTIVE_TIMEOUT_S"] = "15"
    # rank 2 dies after the upsert and one healthy search (SYMB_FAULT hook): heartbeats stop
    os.environ["SYMB_FAULT"] = "kill_rank:2:2"
    import time

    from codename_symbiont_amd.index.shard import Payload
    from codename_symbiont_amd.index.store import VectorStore
    from codename_symbiont_amd.parallel.heartbeat import Heartbeat, HeartbeatMonitor
    from codename_symbiont_amd.parallel.index_group import IndexGroup, RankUnavailableError
    info = _init(rank, world, port)
    grp = IndexGroup(info, dim=8, capacity_per_rank=100)
    hb = Heartbeat(nats_url, rank, interval=0.2)
    hb.start()
    if rank in (1, 2):
        try:
            grp.serve()
        except Exception:  # noqa: BLE001 - the group is torn down under it
            pass
        os._exit(0)
    mon = HeartbeatMonitor(nats_url, world, stale_after=1.0, grace=10.0)
    mon.start()
    grp.liveness = mon
    for _ in range(100):                      # all three ranks heard from
        if len(mon.last_seen) == world:
            break
        time.sleep(0.05)
    store = VectorStore(8, 0, group=grp)
    store.upsert(["a", "b", "c"], np.eye(3, 8, dtype=np.float32), [Payload()] * 3)
    out["healthy_search"] = store.search(np.ones((1, 8), np.float32), 2)[0].shape[1]
    time.sleep(2.0)                           # rank 2 has been silent for > stale_after
    t0 = time.time()
    try:
        store.search(np.ones((1, 8), np.float32), 2)
        out["result"] = "returned"
    except RankUnavailableError as e:
        out["result"] = str(e)
        out["partial_ranks"] = sorted({int(g) >> 40 for g in e.ids.ravel() if g >= 0})
        out["partial_n"] = int((e.ids >= 0).sum())
    out["seconds"] = time.time() - t0
    os._exit(0)


def test_dead_rank_detected_by_heartbeat_fails_fast():
    import asyncio

    from codename_symbiont_amd.bus.broker import NativeBroker

    async def start():
        return await NativeBroker().start()
    b = asyncio.run(start())
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_heartbeat_worker, args=(r, 3, port, b.url, out)) for r in range(3)]
    for p in ps:
        p.start()
    ps[0].join(60)
    for p in ps[1:]:
        p.join(30)
        if p.is_alive():
            p.kill()
    asyncio.run(b.stop())
    assert out.get("healthy_search") == 2, dict(out)
    assert "index rank 2 unavailable: no heartbeat" in out.get("result", ""), dict(out)
    assert "partial results from index rank 0 only" in out["result"]
    assert out["partial_ranks"] == [0] and out["partial_n"] >= 1, dict(out)   # rank 0's shard
    assert out["seconds"] < 1.0


def test_search_batcher_slices_partial_results():
    """Coalesced requests each get their own query's partial rows + the error message."""
    import asyncio

    from codename_symbiont_amd.parallel.index_group import PartialSearchError
    from codename_symbiont_amd.services.batcher import SearchBatcher

    def search_fn(qs, k):
        s = np.arange(len(qs) * k, dtype=np.float32).reshape(len(qs), k)
        raise PartialSearchError("index rank 1 unavailable", s, s.astype(np.int64) + 100)

    async def run():
        b = SearchBatcher(search_fn, window_ms=20)
        qs = [b.search(np.ones(4, np.float32), k) for k in (2, 3)]
        return await asyncio.gather(*qs, return_exceptions=True)
    e2, e3 = asyncio.run(run())
    assert isinstance(e2, PartialSearchError) and isinstance(e3, PartialSearchError)
    assert e2.scores.tolist() == [0, 1] and e3.scores.tolist() == [3, 4, 5]
    assert e3.ids.tolist() == [103, 104, 105] and "rank 1 unavailable" in str(e3)
