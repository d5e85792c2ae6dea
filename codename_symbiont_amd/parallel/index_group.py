"""IndexGroup: one logical vector collection sharded over all GPUs of a node.

Process model (one process per GPU): rank 0 hosts vector_memory_service (NATS, payloads, WAL);
ranks 1..N-1 run ``serve()``, a loop that executes the operations rank 0 broadcasts.  Every op is
a short, fixed sequence of collectives, so all ranks stay in lockstep:

  SEARCH : header -> broadcast queries [nq, D] (bf16 over RCCL) -> every rank: fused MFMA scan
           of ITS shard -> ONE all_gather_into_tensor of the per-rank top-k packed as f64
           (score, global id) pairs -> rank 0 merges on the GPU.  Three collectives per search
           (counted in ``comm_stats``); rank 0's op lock covers only their ENQUEUE, so the
           header / query broadcast / scan of search i+1 queue behind search i's exchange while
           the caller of search i waits for its result outside the lock.
  UPSERT : header -> scatter each owner ITS rows only: the per-rank (count, new-row count,
           overwrite targets) over the control group, the vectors [m, D] f32 (padded to the
           largest share m) over RCCL -> every rank writes its share.  A broadcast of every
           vector to every rank sent N times the bytes, and each rank had to find its rows with
           a device read-back.
  SNAPSHOT / LOAD : header -> every rank saves / loads its own shard under <dir>/rank<r>/
           (index/persist.py: incremental segments of the rows written since the previous
           snapshot); rank 0 adds group.json (world, per-rank counts) and a DELTA of the
           gid -> (point id, payload) table (the gids upserted since, merged geometrically with
           earlier deltas).  A load requires the same world size.
  STOP   : header only.
Control plane: on RCCL the 4-word op header (and an upsert's per-rank plan) travels over a gloo
(host TCP) group of the same ranks, so ranks 1..N-1 learn each op with a host receive that never
synchronises a GPU stream -- they enqueue op i + 1's collectives while op i's still run.
Owner assignment is least-loaded-first, so shards stay balanced (the reference's Qdrant has a
single shard: vector_memory_service/src/main.rs:50).  Global id = rank << 40 | row.
Payloads (and the point-id -> gid map) live on rank 0 only; other ranks hold vectors only.
"""
from __future__ import annotations

import json
import logging
import os
import threading

import numpy as np
import torch
import torch.distributed as dist

from ..index.shard import HbmIndexShard, Payload, PayloadStore, dedupe_last
from .dist import DistInfo
from .sharded import RANK_SHIFT, encode_gid, merge_ranked

log = logging.getLogger("symbiont.index_group")

OP_STOP, OP_SEARCH, OP_UPSERT, OP_SNAPSHOT, OP_LOAD = 0, 1, 2, 3, 4


class RankUnavailableError(RuntimeError):
    """A peer index rank stopped heart-beating: the op is refused before any collective starts."""


class PartialSearchError(RankUnavailableError):
    """A search while a peer is down: carries rank 0's own-shard top-k (``scores``, global
    ``ids``; -1 = empty) so the service can reply with partial results + an error_message."""

    def __init__(self, msg: str, scores, ids):
        super().__init__(msg)
        self.scores, self.ids = scores, ids

    def take(self, j: int, k: int) -> "PartialSearchError":
        """Query ``j``'s slice (1-D, first ``k``) -- for a batch of coalesced requests."""
        return PartialSearchError(str(self), self.scores[j, :k], self.ids[j, :k])


class IndexGroup:
    def __init__(self, info: DistInfo, dim: int, capacity_per_rank: int, group=None,
                 dtype: str = "bf16", prefilter: str | None = None, prune: str | None = None):
        self.info = info
        self.dim = dim
        self.group = group
        dev = info.device
        self.shard = HbmIndexShard(dim, capacity_per_rank, dev, dtype=dtype, prefilter=prefilter,
                                   prune=prune)
        self.comm_device = dev if info.backend == "nccl" else torch.device("cpu")
        # query wire format: bf16 over RCCL (half the bytes), f32 over gloo (no bf16 collectives
        # on every gloo build)
        self.wire_dtype = torch.bfloat16 if info.backend == "nccl" else torch.float32
        # a single-rank process group still runs every collective (RCCL tests on one GPU)
        self.collective = info.world > 1 or info.backend != "none"
        # the op headers' group: gloo beside RCCL (host-only receive), else the data group itself
        self.ctrl = group
        if self.collective and info.backend == "nccl" and group is None:
            self.ctrl = dist.new_group(backend="gloo")
        self.ctrl_device = (torch.device("cpu") if self.ctrl is not group
                            else self.comm_device)
        # per-op collective accounting: {op: [ops, collectives, bytes this rank sent]}
        self.comm_stats: dict[str, list[int]] = {}
        # rank-0 bookkeeping; ops may arrive from several executor threads, but the collective
        # sequence of one op must never interleave with another's
        self._op_lock = threading.Lock()
        self.counts = [0] * info.world
        self.payload_by_gid: dict[int, tuple[str, Payload]] = {}
        self.gid_by_pid: dict[str, int] = {}
        # gids upserted since the last group snapshot, and the (directory, generation) that
        # record is relative to (another directory / generation: the next snapshot is full)
        self._dirty_gids: set[int] = set()
        self._group_key = None
        self.snapshot_root: str | None = None   # shared snapshot directory (all ranks)
        # rank 0: parallel/heartbeat.HeartbeatMonitor -- refuse ops while a peer is down
        self.liveness = None
        # SYMB_FAULT=kill_rank:<r>:<n>: rank r exits after serving n ops (failure tests)
        from ..services.base import FaultInjector

        self._kill_after = FaultInjector(os.environ.get("SYMB_FAULT", "")).kill_rank.get(info.rank)
        self._served = 0

    # ------------------------------------------------------------------ plumbing
    def _bcast(self, t: torch.Tensor) -> torch.Tensor:
        if self.collective:
            dist.broadcast(t, src=0, group=self.group)
        return t

    def _header(self, op: int, a: int = 0, b: int = 0) -> torch.Tensor:
        # (a GPU-resident header -- only when the control group is the data group -- is built
        # pinned + non_blocking: it must not wait for the stream)
        h = torch.tensor([op, a, b, 0], dtype=torch.int64)
        if self.ctrl_device.type == "cuda":
            h = h.pin_memory().to(self.ctrl_device, non_blocking=True)
        if self.collective:
            dist.broadcast(h, src=0, group=self.ctrl)
        return h

    def _scatter(self, out: torch.Tensor, parts, group) -> torch.Tensor:
        """Rank 0's parts[r] -> rank r's ``out`` (``parts`` None on ranks 1..N-1)."""
        if self.collective:
            dist.scatter(out, scatter_list=list(parts) if parts is not None else None, src=0,
                         group=group)
        else:
            out.copy_(parts[0])
        return out

    def _count(self, op: str, collectives: int, nbytes: int) -> None:
        c = self.comm_stats.setdefault(op, [0, 0, 0])
        c[0] += 1
        c[1] += collectives
        c[2] += nbytes

    @property
    def count(self) -> int:
        return sum(self.counts) if self.info.is_root else self.shard.count

    # ------------------------------------------------------------------ ops (collective bodies)
    def _do_search(self, q: torch.Tensor, k: int):
        """Local scan + the packed exchange; returns the merged top-k on the shard's device
        (rank 0's result; other ranks discard it)."""
        info = self.info
        s, r = self.shard.search(q.to(self.shard.device, torch.bfloat16), k)
        gid = encode_gid(info.rank, r.to(torch.int64))
        if not self.collective:
            return s, gid
        # one collective: (score, gid) as f64 pairs -- f32 scores and gids < 2^53 are exact
        packed = torch.stack([s.double(), gid.double()], dim=-1).to(self.comm_device).contiguous()
        nq = packed.shape[0]
        allp = torch.empty((info.world * nq,) + tuple(packed.shape[1:]), dtype=packed.dtype,
                           device=self.comm_device)
        dist.all_gather_into_tensor(allp, packed, group=self.group)
        allp = allp.view(info.world, nq, k, 2).to(self.shard.device, non_blocking=True)
        return merge_ranked(allp[..., 0].float(), allp[..., 1].long(), k)

    def _do_upsert(self, m: int, vparts=None, mparts=None) -> None:
        """Receive and write this rank's share of an upsert: ``m`` = the largest share (rows);
        rank 0 passes the per-rank parts (vectors [W, m, D] f32 on the comm device, plan [W,
        2 + m] int64 on the control device: count, new rows first, then the overwrite targets).
        New rows are appended in one call, overwrites written in one batched scatter
        (HbmIndexShard.write_rows_f32)."""
        plan = self._scatter(torch.empty(2 + m, dtype=torch.int64, device=self.ctrl_device),
                             mparts, self.ctrl)
        v = self._scatter(torch.empty(m, self.dim, dtype=torch.float32, device=self.comm_device),
                          vparts, self.group)
        p = plan.tolist()   # (host-resident over the gloo control group: no device sync)
        cnt, n_new = p[0], p[1]
        if cnt == 0:
            return
        v = v[:cnt].to(self.shard.device)
        if n_new:
            self.shard.append_f32(v[:n_new])
        if cnt > n_new:
            self.shard.write_rows_f32(torch.tensor(p[2 + n_new:2 + cnt], dtype=torch.int64),
                                      v[n_new:cnt])

    def _rank_dir(self, directory: str) -> str:
        return os.path.join(directory, f"rank{self.info.rank}")

    def _do_snapshot(self, directory: str) -> None:
        from ..index.persist import save_snapshot

        d = self._rank_dir(directory)
        os.makedirs(d, exist_ok=True)
        save_snapshot(self.shard, d)
        if self.info.world > 1:
            dist.barrier(group=self.group)   # every shard durable before rank 0 commits group.json

    def _do_load(self, directory: str, counts: torch.Tensor) -> int:
        """Load this rank's shard, cut to the row count group.json committed: a crash between
        the per-rank saves and the group.json commit leaves newer rank snapshots whose extra rows
        the WAL (truncated only after the commit) re-applies."""
        from ..index.persist import load_snapshot

        load_snapshot(self.shard, self._rank_dir(directory))
        self.shard.truncate(min(self.shard.count, int(counts[self.info.rank])))
        if self.info.world > 1:
            dist.barrier(group=self.group)
        return self.shard.count

    def check_alive(self) -> None:
        m = self.liveness
        if m is None:
            return
        dead = m.dead_ranks()
        if dead:
            r, age = dead[0]
            raise RankUnavailableError(f"index rank {r} unavailable: no heartbeat for {age:.1f}s")

    # ------------------------------------------------------------------ rank-0 API
    def snapshot(self, directory: str) -> None:
        """Collective checkpoint of every shard + rank 0's payload table (atomic group.json)."""
        assert self.info.is_root
        self.check_alive()
        with self._op_lock:
            self._header(OP_SNAPSHOT)
            self._do_snapshot(directory)
            self._commit_group(directory)

    def _commit_group(self, directory: str, _crash_before_commit: bool = False) -> None:
        """The payload table's DELTA (gids upserted since the previous group snapshot; every gid
        when that record does not belong to this directory's committed generation) goes to a NEW
        versioned file, folded geometrically with the previous deltas (a delta absorbs its
        predecessor while it holds at least half as many entries, read back from disk).  The
        atomic group.json replace is the one commit point for counts + payload files together,
        so a crash can never pair new payloads with old per-rank counts."""
        from ..index.persist import fsync_dir, merge_payload_files, write_atomic, write_payloads

        prev = self._group_meta(directory)
        gen = (prev or {}).get("gen", 0) + 1
        incremental = (prev is not None and prev.get("format") == 3
                       and self._group_key == (os.path.abspath(directory), prev["gen"]))
        files = [dict(f) for f in prev["payload_files"]] if incremental else []
        gids = sorted(self._dirty_gids) if incremental else sorted(self.payload_by_gid)
        entries = []
        for g in gids:
            pid, p = self.payload_by_gid.get(g, (None, None))
            entries.append((pid, None if p is None else tuple(getattr(p, f)
                                                                for f in PayloadStore.FIELDS)))
        m, merge = len(gids), []
        while files and 2 * m >= files[-1]["m"]:
            last = files.pop()
            merge.insert(0, last["gen"])
            m += last["m"]
        if gids or merge:
            tmp = os.path.join(directory, f"group_pay.{gen}.delta")
            write_payloads(tmp, np.asarray(gids, dtype=np.int64), entries)
            out = os.path.join(directory, f"group_pay.{gen}.bin")
            if merge:
                m = merge_payload_files([os.path.join(directory, f"group_pay.{x}.bin")
                                         for x in merge] + [tmp], out)
                os.remove(tmp)
            else:
                os.replace(tmp, out)
            files.append({"gen": gen, "m": m})
        fsync_dir(directory)
        if _crash_before_commit:
            return
        meta = {"world": self.info.world, "counts": self.counts, "dim": self.dim, "format": 3,
                "gen": gen, "payload_files": files}
        write_atomic(os.path.join(directory, "group.json"), json.dumps(meta).encode())
        self._dirty_gids = set()
        self._group_key = (os.path.abspath(directory), gen)
        keep = {f"group_pay.{f['gen']}.bin" for f in files}
        for fn in os.listdir(directory):   # committed: unreferenced tables are garbage
            if (fn.startswith("group_pay") or fn.startswith("group_payloads")) and fn not in keep:
                os.remove(os.path.join(directory, fn))

    @staticmethod
    def _group_meta(directory: str):
        p = os.path.join(directory, "group.json")
        if not os.path.exists(p):
            return None
        with open(p) as f:
            return json.load(f)

    def load(self, directory: str) -> int:
        """Collective restore written by ``snapshot``; returns the number of points (0 if none)."""
        assert self.info.is_root
        meta = self._group_meta(directory)
        if meta is None:
            return 0
        if meta["world"] != self.info.world or meta["dim"] != self.dim:
            raise ValueError(f"group snapshot is for world={meta['world']} dim={meta['dim']}, "
                             f"this group is world={self.info.world} dim={self.dim}")
        with self._op_lock:
            self._header(OP_LOAD)
            c = self._bcast(torch.tensor(meta["counts"], dtype=torch.int64, device=self.comm_device))
            self._do_load(directory, c)
        self.counts = list(meta["counts"])
        self.payload_by_gid.clear()
        self.gid_by_pid.clear()

        def put(g, pid, p):
            # entries past a rank's committed row count are dropped, so a table newer than the
            # counts cannot leave gids pointing beyond a shard
            if (g & ((1 << RANK_SHIFT) - 1)) >= self.counts[g >> RANK_SHIFT]:
                return
            old = self.payload_by_gid.get(g)
            if old is not None and self.gid_by_pid.get(old[0]) == g:
                del self.gid_by_pid[old[0]]
            if pid is None:
                self.payload_by_gid.pop(g, None)
                return
            self.payload_by_gid[g] = (pid, p)
            self.gid_by_pid[pid] = g

        if meta.get("format") == 3:   # binary deltas, applied in generation order
            from ..index.persist import read_payloads

            for fdesc in meta["payload_files"]:
                keys, ents = read_payloads(os.path.join(directory, f"group_pay.{fdesc['gen']}.bin"))
                for g, (pid, f) in zip(keys.tolist(), ents):
                    put(g, pid, Payload(*f) if f is not None else Payload())
            self._group_key = (os.path.abspath(directory), meta["gen"])
        else:   # formats 1 / 2: one JSON-lines table
            name = meta.get("payloads", "group_payloads.jsonl")
            with open(os.path.join(directory, name), encoding="utf-8") as f:
                for line in f:
                    a = json.loads(line)
                    put(a[0], a[1], Payload(*a[2:]))
        self._dirty_gids = set()
        return sum(self.counts)

    def snapshot_dir_exists(self, directory: str) -> bool:
        return os.path.exists(os.path.join(directory, "group.json"))

    def search(self, q_unit: torch.Tensor, k: int):
        assert self.info.is_root
        nq = q_unit.shape[0]
        try:
            self.check_alive()
        except RankUnavailableError as e:
            # degrade: rank 0 scans its own shard (no collective) -> partial results
            s, r = self.shard.search(q_unit.to(self.shard.device, torch.bfloat16), k)
            raise PartialSearchError(f"{e}; partial results from index rank 0 only", s,
                                     encode_gid(0, r.to(torch.int64))) from None
        with self._op_lock:   # enqueue only: the caller's D2H of the result waits outside it
            self._header(OP_SEARCH, nq, k)
            q = self._bcast(q_unit.to(self.comm_device, self.wire_dtype).contiguous())
            out = self._do_search(q, k)
        W, nc = self.info.world, 3 if self.collective else 0
        nbytes = 32 + q.numel() * q.element_size() + (W * nq * k * 16 if nc else 0)
        self._count("search", nc, nbytes)
        log.debug("[INDEX_GROUP] search nq=%d k=%d: %d collectives, %d bytes", nq, k, nc, nbytes)
        return out

    def upsert(self, point_ids: list[str], vecs: torch.Tensor, payloads: list[Payload]) -> list[int]:
        assert self.info.is_root
        self.check_alive()
        with self._op_lock:
            return self._upsert_locked(point_ids, vecs, payloads)

    def _upsert_locked(self, point_ids, vecs, payloads) -> list[int]:
        # an id repeated inside the batch is ONE point, last occurrence wins (HbmIndexShard.upsert)
        pos = dedupe_last(point_ids)
        if len(pos) != len(point_ids):
            ids_u = [point_ids[i] for i in pos]
            gids_u = self._upsert_locked(ids_u, vecs[pos], [payloads[i] for i in pos])
            by_pid = dict(zip(ids_u, gids_u))
            return [by_pid[pid] for pid in point_ids]
        n = len(point_ids)
        owner = np.empty(n, np.int64)
        target = np.full(n, -1, np.int64)
        gids = []
        counts = list(self.counts)
        for i, pid in enumerate(point_ids):
            g = self.gid_by_pid.get(pid)
            if g is not None:  # overwrite in place
                owner[i], target[i] = g >> RANK_SHIFT, g & ((1 << RANK_SHIFT) - 1)
                gids.append(g)
            else:
                r = int(np.argmin(counts))
                owner[i] = r
                gids.append((r << RANK_SHIFT) | counts[r])
                counts[r] += 1
        # per-owner shares, each ordered new rows first (appended in input order) then overwrites
        W = self.info.world
        share = [np.concatenate([np.nonzero((owner == r) & (target < 0))[0],
                                 np.nonzero((owner == r) & (target >= 0))[0]]) for r in range(W)]
        m = max(1, max(len(x) for x in share))
        plan = np.zeros((W, 2 + m), np.int64)
        vsrc = vecs.to(self.comm_device, torch.float32)
        vparts = torch.zeros(W, m, self.dim, dtype=torch.float32, device=self.comm_device)
        for r, idx in enumerate(share):
            plan[r, 0], plan[r, 1] = len(idx), int((target[idx] < 0).sum())
            plan[r, 2:2 + len(idx)] = target[idx]
            if len(idx):
                vparts[r, :len(idx)] = vsrc[torch.from_numpy(idx).to(vsrc.device)]
        self._header(OP_UPSERT, m)
        self._do_upsert(m, vparts, torch.from_numpy(plan).to(self.ctrl_device))
        self.counts = counts
        for pid, g, p in zip(point_ids, gids, payloads):
            self.payload_by_gid[g] = (pid, p)
            self.gid_by_pid[pid] = g
        if self.snapshot_root is not None or self._group_key is not None:
            self._dirty_gids.update(gids)
        return gids

    def payload(self, gid: int) -> tuple[str | None, Payload]:
        return self.payload_by_gid.get(int(gid), (None, Payload()))

    def stop(self) -> None:
        if self.info.is_root and self.info.world > 1:
            with self._op_lock:
                self._header(OP_STOP)

    # ------------------------------------------------------------------ ranks 1..N-1
    def serve(self) -> None:
        assert not self.info.is_root
        while self.serve_one():
            pass

    def serve_one(self) -> bool:
        """Receive and execute one op from rank 0; False once rank 0 sent OP_STOP."""
        h = self._header(OP_STOP).tolist()
        op, a, b = h[0], h[1], h[2]
        if op == OP_STOP:
            return False
        if op == OP_SEARCH:
            q = self._bcast(torch.empty(a, self.dim, dtype=self.wire_dtype, device=self.comm_device))
            self._do_search(q, b)
        elif op == OP_UPSERT:
            self._do_upsert(a)
        elif op in (OP_SNAPSHOT, OP_LOAD):
            if self.snapshot_root is None:
                raise RuntimeError("index rank has no snapshot directory (SYMB_SNAPSHOT_DIR)")
            if op == OP_SNAPSHOT:
                self._do_snapshot(self.snapshot_root)
            else:
                c = self._bcast(torch.empty(self.info.world, dtype=torch.int64,
                                            device=self.comm_device))
                self._do_load(self.snapshot_root, c)
        else:
            raise RuntimeError(f"unknown index op {op}")
        self._served += 1
        if self._kill_after is not None and self._served >= self._kill_after:
            log.error("[FAULT] kill_rank: index rank %d exits after %d ops", self.info.rank,
                      self._served)
            os._exit(137)
        return True
