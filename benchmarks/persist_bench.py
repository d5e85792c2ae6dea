#!/usr/bin/env python3
"""Snapshot / boot cost of the incremental persistence (index/persist.py) at scale.

  python benchmarks/persist_bench.py [--rows 10000000] [--dim 384] [--payload-rows 1000000]
                                     [--new 100000] [--device cpu|cuda] [--dir /tmp/persist_bench]

Builds a shard of ``rows`` random unit rows (the first ``payload-rows`` with point ids and
payloads), takes the first (full) snapshot, then ``new`` more points + 1000 overwrites and a
second (incremental) snapshot through VectorStore's background writer, then boots a fresh store
from the directory.  Prints one JSON line: full / incremental snapshot seconds and bytes, the
time upserts were blocked by the cut, boot seconds (snapshot load + WAL replay)."""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=384)
    ap.add_argument("--payload-rows", type=int, default=1_000_000)
    ap.add_argument("--new", type=int, default=100_000)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--dir", default="/tmp/persist_bench")
    a = ap.parse_args()
    from codename_symbiont_amd.index import persist
    from codename_symbiont_amd.index.shard import Payload
    from codename_symbiont_amd.index.store import VectorStore

    shutil.rmtree(a.dir, ignore_errors=True)
    cap = a.rows + a.new + 16
    st = VectorStore(a.dim, cap, device=a.device, snapshot_dir=a.dir, snapshot_every=1 << 62)
    rng = np.random.default_rng(0)
    t0 = time.perf_counter()
    st.shard.fill_random(a.rows - a.payload_rows, seed=1)
    for s in range(0, a.payload_rows, 100_000):      # points with payloads (WAL + upsert)
        n = min(100_000, a.payload_rows - s)
        v = rng.standard_normal((n, a.dim)).astype(np.float32)
        st._upsert_nolog([f"p{s + i}" for i in range(n)], v,
                         [Payload(f"doc{(s + i) // 20}", "https://example.org/x", f"sentence {s + i}",
                                  (s + i) % 20, "all-MiniLM-L6-v2", 1_700_000_000_000 + s + i)
                          for i in range(n)])
    fill_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    st.snapshot()
    full_s = time.perf_counter() - t0
    full = dict(st.last_snapshot)
    v = rng.standard_normal((a.new, a.dim)).astype(np.float32)
    ids = [f"n{i}" for i in range(a.new)]
    pls = [Payload(f"new{i}", "u", f"t{i}", i) for i in range(a.new)]
    for s in range(0, a.new, 10_000):
        st.upsert(ids[s:s + 10_000], v[s:s + 10_000], pls[s:s + 10_000])
    ow = [f"p{i}" for i in range(0, min(a.payload_rows, 1000))]
    st.upsert(ow, rng.standard_normal((len(ow), a.dim)).astype(np.float32), [Payload("ow")] * len(ow))
    t0 = time.perf_counter()
    st.snapshot(wait=False)
    cut_s = time.perf_counter() - t0          # what an upsert waiting on the lock would see
    t1 = time.perf_counter()
    st.upsert(["after"], v[:1], [Payload("after")])
    blocked_s = time.perf_counter() - t1
    st.flush()
    inc_s = time.perf_counter() - t0
    inc = dict(st.last_snapshot)
    st.wal.close()
    du = sum(os.path.getsize(os.path.join(a.dir, f)) for f in os.listdir(a.dir))
    del st
    if a.device == "cuda":
        torch.cuda.empty_cache()
    t0 = time.perf_counter()
    st2 = VectorStore(a.dim, cap, device=a.device, snapshot_dir=a.dir)
    boot_s = time.perf_counter() - t0
    assert st2.count == a.rows + a.new + 1, st2.count
    out = {"rows": a.rows, "dim": a.dim, "payload_rows": a.payload_rows, "new": a.new,
           "device": a.device, "fill_s": round(fill_s, 2),
           "full_snapshot_s": round(full_s, 2), "full_bytes": full.get("bytes"),
           "incremental_cut_s": round(cut_s, 3), "upsert_during_snapshot_s": round(blocked_s, 3),
           "incremental_snapshot_s": round(inc_s, 3), "incremental_bytes": inc.get("bytes"),
           "boot_s": round(boot_s, 2), **st2.boot_s, "dir_bytes": du,
           "manifest": {k: v for k, v in persist.committed_manifest(a.dir).items()
                        if k in ("gen", "count", "segments", "patches", "payloads")}}
    print(json.dumps(out), flush=True)
    st2.wal.close()
    shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
