#!/usr/bin/env python3
"""Repeat the int8-pruned search's full-shard scan kernel (index_scan_i8_kernel) on the inputs one
real search prepared -- the target of rocprofv3 --pmc passes (benchmarks/pmc_kernel.py
--match index_scan_i8).

    python benchmarks/scan_one.py [--rows 25000000] [--nq 256] [--corpus random] [--iters 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=25_000_000)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--corpus", default="random")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    gen = CorpusGen(a.corpus, 384, "cuda")
    shard = HbmIndexShard(384, a.rows + 8192, device="cuda", prune="i8")
    fill_corpus(shard, gen, a.rows, seed=1)
    q = gen.unit(a.nq, seed=7).bfloat16()
    shard.mq_stats = True
    shard.search(q, 10)
    torch.cuda.synchronize()
    P, n = shard._pruned_last, shard.visible
    h, st = hip(), stream_handle()
    rsplit = 2 if a.nq < 512 else 1
    heavy = shard._i8_heavy

    def scan():
        h.index_scan_i8(shard.rows_i8.data_ptr(), shard.sx_i8.data_ptr(), n, shard.rows_i8.shape[0],
                        P["rows_per_blk"], P["n_rblk"], P["q8"].data_ptr(), a.nq, P["thr"].data_ptr(),
                        P["cs"].data_ptr(), P["ci"].data_ptr(), P["cnt"].data_ptr(), P["cap"], 1, st,
                        rsplit, heavy=heavy, sq=P["sq"].data_ptr() if heavy else 0)

    scan()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        scan()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.iters
    print(json.dumps({"bench": "scan_one", "rows": n, "nq": a.nq, "corpus": a.corpus,
                      "image": "split" if heavy else "plain", "ms": round(ms, 3),
                      "row_bytes_TBps": round(n * shard.rows_i8.shape[1] / ms / 1e9, 2),
                      "cand_max": int(P["cnt"].max())}))


if __name__ == "__main__":
    main()
