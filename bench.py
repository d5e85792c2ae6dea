#!/usr/bin/env python3
"""Headline benchmark: embeds/sec + top-k QPS, all-MiniLM-L6-v2 / 100M x 384 index, 1..8 MI355X.

One STEP = the system's ingest+search cycle on every rank (one process per GPU):
  1. H2D of the next synthetic tokenized batch on a copy stream (overlaps the previous search)
  2. encode B=256 sentences x S=128 tokens with the HIP MiniLM-L6 encoder (bf16, varlen-packed)
  3. upsert the 256 unit embeddings into this rank's HBM index shard
  4. semantic search: the 256 new embeddings are the queries; all_gather the queries of all
     ranks, EXACT top-10 over the rank's shard of the 100M x 384 bf16 corpus, all_to_all the
     partial top-k back to each query's owner and merge.  The exact top-10 is found by an int8
     MFMA scan of an int8 image of the rows that prunes only rows whose score provably cannot
     reach the query's k-th best (Cauchy-Schwarz bound on the quantisation error, tracked at
     every write), and the survivors are re-scored in bf16 (csrc/hip/index_i8.hip): the same
     rows and scores as scanning every row in bf16 (GPU tests compare them); --index-prune none
     runs that full bf16 scan.
So every step embeds 256*N sentences AND answers 256*N top-10 queries over the full 100M-row
corpus: value = embeds/s = top-k QPS (whole job).  Per-rank work is constant in N ("weak").

Data: synthetic token ids, random-init weights (real MiniLM-L6 architecture), random unit
index rows -- there is no network for checkpoints or datasets.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

The other BASELINE.json configs run through the same step (benchmarks/suite.py drives them):
  --mode embed                                   all-MiniLM-L6-v2 bf16 embedding, batch 256
  --mode search                                  100M x 384 sharded cosine top-k
  --model bge-base --mode embed                  bge-base-en-v1.5 DP embedding
  --model e5-large --index-dtype fp8 --index-rows 1000000000
                                                 e5-large-v2 + 1B-vector fp8 index (1B/N rows
                                                 per rank: needs N >= 4 for 1 TB; smaller N
                                                 takes --index-rows that fit)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("embeds/sec + top-k QPS, all-MiniLM-L6-v2 / 100M×384 index at 1/2/4/8 MI355X")
DERIVED_REF_EMBEDS_PER_SEC = 225.0  # BASELINE.md derived estimate (not a published number)


def log(info, *a):
    if info.rank == 0:
        print(*a, file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--index-rows", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--model", default="minilm-l6")
    ap.add_argument("--mode", choices=["full", "embed", "search"], default="full")
    ap.add_argument("--index-dtype", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--index-prefilter", choices=["none", "fp8"], default="none",
                    help="fp8: search the bf16 index through an e4m3 copy for 3k candidates and "
                         "re-score them exactly in bf16 (Qdrant quantization + rescore); the "
                         "headline default is the exact bf16 scan")
    ap.add_argument("--index-prune", choices=["none", "i8"], default="i8",
                    help="i8: EXACT search through an int8 image of the bf16 rows -- rows whose "
                         "int8 score cannot reach the query's k-th best (a proven error bound) are "
                         "pruned, the rest re-scored in bf16 (csrc/hip/index_i8.hip); same top-k "
                         "as the full bf16 scan")
    ap.add_argument("--i8-tile-rows", type=int, choices=[64, 128], default=64,
                    help="rows per tile of the int8 pruning scan")
    ap.add_argument("--i8-waves", type=int, choices=[4, 8], default=8,
                    help="int8 pruning scan: 8-wave workgroups (one per CU) or 4 (two per CU)")
    ap.add_argument("--encoder-dtype", choices=["bf16", "fp8"], default="bf16",
                    help="fp8: e4m3 projection GEMMs (BASELINE config #5); the headline stays bf16")
    ap.add_argument("--embed-dp", choices=["replica", "group"], default="replica",
                    help="--mode embed, N > 1: independent replicas, or ONE global batch of "
                         "batch*N sentences per step split over the ranks and gathered back to "
                         "rank 0 over RCCL (parallel/embed_group.py; BASELINE config #4 over xGMI)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="--mode full: run encode and search back to back on one stream instead of "
                         "encoding batch i+1 on a second stream while batch i is searched")
    ap.add_argument("--scan-cus", type=int, default=0,
                    help="spread the index scans over this many CUs (0 = all), leaving the rest to "
                         "the encoder running beside them on the second stream")
    ap.add_argument("--search-priority", action="store_true",
                    help="run the search (and the step's bookkeeping) on a high-priority stream so "
                         "its short latency-bound kernels dispatch ahead of the encoder's")
    ap.add_argument("--scan-min-tiles", type=int, default=16,
                    help="smallest row block (64-row tiles) of the small list scans")
    ap.add_argument("--prune-sample-shift", type=int, default=0,
                    help="exact pruned search: threshold sample = 1 tile in 2^shift (0 = the "
                         "shard default, HbmIndexShard.PRUNE_TILE_SHIFT)")
    ap.add_argument("--prepass-min-tiles", type=int, default=0,
                    help="row-block floor of the sampled searches' small pre-pass list scans "
                         "(0 = the shard default, 1 tile per workgroup)")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch the encoder's kernels eagerly every step instead of replaying a "
                         "captured hipGraph of the forward")
    args = ap.parse_args()

    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.parallel.sharded import ShardedSearcher

    info = D.init()
    if info.world != args.gpus:
        log(info, f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={info.world}")
    dev = info.device
    torch.manual_seed(1234 + info.rank)
    cfg = get_config(args.model)
    B, S, K, W = args.batch, args.seq, args.steps, args.warmup

    t0 = time.time()
    enc = HipEncoder(cfg, seed=0, device=dev, precision=args.encoder_dtype)
    rows_per_rank = args.index_rows // info.world
    extra = (K + W + 4) * B
    prefilter = None if args.index_prefilter == "none" else args.index_prefilter
    from codename_symbiont_amd.index.shard import resolve_prune

    # exact either way; i8 applies to 384-wide bf16 shards without a prefilter (else: plain scan)
    prune = resolve_prune("auto" if args.index_prune == "i8" and args.mode != "embed" else "none",
                          args.index_dtype, cfg.hidden, prefilter)   # (embed mode never searches)
    shard = HbmIndexShard(cfg.hidden, rows_per_rank + extra, device=dev, dtype=args.index_dtype,
                          prefilter=prefilter, prune=prune)
    if args.mode != "embed":
        shard.fill_random(rows_per_rank, seed=100 + info.rank)
    searcher = ShardedSearcher(shard, info)
    if prune:
        from codename_symbiont_amd.ops._ext import hip as _hip

        _hip().i8_config(args.i8_tile_rows, args.i8_waves)
    shard.mq_stats = os.environ.get("SYMB_MQ_STATS", "0") not in ("", "0")
    shard.scan_cus = args.scan_cus
    shard.scan_min_tiles = args.scan_min_tiles
    if args.prepass_min_tiles:
        shard.prepass_min_tiles = args.prepass_min_tiles
    if args.prune_sample_shift:
        shard.PRUNE_TILE_SHIFT = args.prune_sample_shift
    torch.cuda.synchronize(dev)
    row_bytes = cfg.hidden * (1 if args.index_dtype == "fp8" else 2)
    log(info, f"[bench] setup {time.time() - t0:.1f}s: {cfg.model_name}, shard {rows_per_rank} "
              f"rows x {cfg.hidden} {args.index_dtype} = {rows_per_rank * row_bytes / 1e9:.1f} GB/rank")

    group_dp = args.mode == "embed" and args.embed_dp == "group" and info.world > 1
    if group_dp:
        from codename_symbiont_amd.parallel.embed_group import EmbedGroup

        egroup = EmbedGroup(info, enc)
    # host batches (pinned) rotated through two device buffers filled on a copy stream
    NB = 4
    NBATCH = B * info.world if group_dp else B   # group mode: rank 0 holds the global batch
    host = [synthetic_batch(cfg, NBATCH, S, seed=1000 * info.rank + i) for i in range(NB)]
    host = [type(h)(h.ids.pin_memory(), h.pos.pin_memory(), None, h.cu_seqlens.pin_memory(),
                    h.max_len) for h in host]
    dbuf = [host[0].to(dev), host[1].to(dev)]
    copy_stream = torch.cuda.Stream(dev)
    compute = torch.cuda.current_stream(dev)
    if args.search_priority:
        torch.cuda.synchronize(dev)
        compute = torch.cuda.Stream(dev, priority=-1)
        torch.cuda.set_stream(compute)
    copy_done = [torch.cuda.Event(), torch.cuda.Event()]
    consumed = [torch.cuda.Event(), torch.cuda.Event()]
    out_f32 = torch.empty(B, cfg.hidden, device=dev)
    out_unit = torch.empty(B, cfg.hidden, dtype=torch.bfloat16, device=dev)
    # --mode full pipelines the two halves of a step across two streams: batch i+1 is encoded
    # on enc_stream while batch i's queries are searched on the compute stream (the scan is
    # power-bound; the encoder's small kernels fill its tail and launch gaps).  Every timed step
    # still encodes one batch and searches one batch.
    overlap = args.mode == "full" and not group_dp and not args.no_overlap
    enc_stream = torch.cuda.Stream(dev)
    outs = [(torch.empty(B, cfg.hidden, device=dev),
             torch.empty(B, cfg.hidden, dtype=torch.bfloat16, device=dev)) for _ in range(2)]
    enc_done = [torch.cuda.Event(), torch.cuda.Event()]
    q_free = [torch.cuda.Event(), torch.cuda.Event()]
    # SYMB_GPU_DEBUG=1: assert the host enqueue order the events above rely on
    from codename_symbiont_amd.utils.gpu_debug import BufferRing

    in_ring, out_ring = BufferRing(2, "bench.dbuf"), BufferRing(2, "bench.outs")
    q_fixed = torch.nn.functional.normalize(torch.randn(B, cfg.hidden, device=dev), dim=-1).bfloat16()

    def prefetch(i: int) -> None:
        slot = i % 2
        with torch.cuda.stream(copy_stream):
            if i >= 2:
                copy_stream.wait_event(consumed[slot])
            h, d = host[i % NB], dbuf[slot]
            if overlap:
                in_ring.fill(slot)
            d.ids.copy_(h.ids, non_blocking=True)
            d.pos.copy_(h.pos, non_blocking=True)
            d.cu_seqlens.copy_(h.cu_seqlens, non_blocking=True)
            d.max_len = h.max_len
            copy_done[slot].record(copy_stream)

    # The encoder forward is ~40 kernel launches; on a busy host their enqueue time (0.9-1.2 ms
    # per step measured) approaches the GPU time (1.5 ms), so each (input slot, output buffers)
    # pair is captured once into a hipGraph and replayed: one launch per forward.  Graphs bake
    # pointers and shapes; every bench batch has the same shape and lives in dbuf[slot].
    from codename_symbiont_amd.utils.gpu_debug import debug_enabled

    # (SYMB_GPU_DEBUG syncs after every launch, which a stream capture forbids: eager there).
    # Only the embed-only step is launch-bound; the headline step is bound by the scan (same
    # 13.2k with or without the graph), so it keeps eager launches.
    use_graph = (not args.no_graph and not group_dp and args.mode == "embed"
                 and not debug_enabled())
    graphs = {}

    def run_encoder(slot: int, o32: torch.Tensor, ou: torch.Tensor) -> None:
        g = graphs.get((slot, o32.data_ptr())) if use_graph else None
        if g is None:
            enc.forward_packed(dbuf[slot], o32, ou)
        else:
            g.replay()

    def capture_encoder(slot: int, o32: torch.Tensor, ou: torch.Tensor) -> None:
        enc.forward_packed(dbuf[slot], o32, ou)   # first call: kernel attributes, workspace
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        # thread_local: other threads' HIP calls (e.g. a process group's watchdog) stay legal
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            enc.forward_packed(dbuf[slot], o32, ou)
        torch.cuda.synchronize(dev)
        graphs[(slot, o32.data_ptr())] = g

    if use_graph:   # before any pipelined work is in flight
        for slot in range(2):
            capture_encoder(slot, *(outs[slot] if overlap else (out_f32, out_unit)))

    def encode_async(i: int, ev=None) -> None:
        """Encode batch i on enc_stream into outs[i % 2] (overlap mode)."""
        slot = i % 2
        with torch.cuda.stream(enc_stream):
            enc_stream.wait_event(copy_done[slot])
            if i >= 2:
                enc_stream.wait_event(q_free[slot])   # batch i-2's queries are searched
            if ev:
                ev[0].record(enc_stream)
            in_ring.consume(slot)
            out_ring.fill(slot)
            run_encoder(slot, *outs[slot])
            if ev:
                ev[1].record(enc_stream)
            consumed[slot].record(enc_stream)
            enc_done[slot].record(enc_stream)
        prefetch(i + 1)

    def step_overlap(i: int, ev=None) -> None:
        """Search batch i (encoded by the previous step) while batch i+1 encodes."""
        slot = i % 2
        encode_async(i + 1, ev)
        compute.wait_event(enc_done[slot])
        if ev:
            ev[2].record(compute)
        q = outs[slot][1]
        shard.append_unit(q)
        searcher.search(q, args.k)
        out_ring.consume(slot)
        q_free[slot].record(compute)
        if ev:
            ev[3].record(compute)

    def step(i: int, ev=None) -> None:
        if overlap:
            return step_overlap(i, ev)
        slot = i % 2
        if ev:
            ev[0].record(compute)
        if group_dp:
            if info.is_root:
                compute.wait_event(copy_done[slot])
                egroup.embed(dbuf[slot])
                consumed[slot].record(compute)
                prefetch(i + 1)
            else:
                egroup.embed(None)
            q = None
        elif args.mode != "search":
            compute.wait_event(copy_done[slot])
            run_encoder(slot, out_f32, out_unit)
            consumed[slot].record(compute)
            prefetch(i + 1)
            shard.append_unit(out_unit)
            q = out_unit
        else:
            q = q_fixed
        if ev:
            ev[1].record(compute)
            ev[2].record(compute)
        if args.mode != "embed":
            searcher.search(q, args.k)
        if ev:
            ev[3].record(compute)

    prefetch(0)
    if overlap:
        encode_async(0)
    for i in range(W):
        step(i)
    torch.cuda.synchronize(dev)
    D.barrier(info)
    torch.cuda.synchronize(dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K)]
    t_start = time.perf_counter()
    for j in range(K):
        step(W + j, evs[j])
    host_ms = (time.perf_counter() - t_start) * 1000.0 / K   # host enqueue time per step
    torch.cuda.synchronize(dev)
    D.barrier(info)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    elapsed = D.allreduce_max(info, elapsed)
    e_ms = sum(a.elapsed_time(b) for a, b, _, _ in evs) / K
    s_ms = sum(c.elapsed_time(d) for _, _, c, d in evs) / K

    ms = elapsed * 1000.0 / K
    total = B * info.world * K / elapsed
    headline = (args.model in ("minilm-l6", "minilm", "all-MiniLM-L6-v2") and args.mode == "full"
                and args.index_rows == 100_000_000 and args.index_dtype == "bf16"
                and args.encoder_dtype == "bf16" and prefilter is None)
    short = cfg.model_name.split("/")[-1]
    rows_txt = f"{args.index_rows / 1e6:g}M" if args.index_rows < 10**9 else f"{args.index_rows / 1e9:g}B"
    metric = METRIC if headline else {
        "full": f"embeds/sec + top-k QPS, {short} / {rows_txt}x{cfg.hidden} {args.index_dtype} index"
                + (" (fp8 prefilter + exact bf16 rescore)" if prefilter else ""),
        "embed": f"embeds/sec, {short} ({cfg.key}) {args.encoder_dtype}, batch {B} x seq {S}",
        "search": f"top-{args.k} QPS, {rows_txt}x{cfg.hidden} {args.index_dtype} index, {B} queries/rank"
                  + (" (fp8 prefilter + exact bf16 rescore)" if prefilter else ""),
    }[args.mode]
    if shard._mq_tot is not None:
        print(f"[bench] rank {info.rank} emitting-scan searches: {int(shard._mq_tot[0].item())} "
              f"overflowed, max {int(shard._mq_tot[1].item())} candidates per query "
              f"(cap {shard.MQ_CAP})", file=sys.stderr, flush=True)
    if info.rank == 0:
        res = {
            "metric": metric,
            "value": round(total, 2),
            "unit": f"embeds/s (whole job; every embedded sentence is also answered as a top-{args.k} "
                    f"query over the {rows_txt} x {cfg.hidden} corpus, so this equals top-k QPS)"
                    if args.mode == "full" else ("embeds/s" if args.mode == "embed" else "queries/s"),
            "n_gpus": info.world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.encoder_dtype,
            "index_dtype": args.index_dtype,
            "index_prefilter": prefilter,
            "index_search": ("exact: int8 bound-pruned scan + bf16 re-score" if prune
                             else ("fp8 prefilter + bf16 re-score" if prefilter else "exact bf16 scan")),
            "data": "synthetic token ids, random-init weights, random unit index rows",
            "config": {
                "model": short, "global_batch": B * info.world, "seq_len": S,
                "parallelism": (f"dp{info.world}-rccl-group" if group_dp
                                else f"dp{info.world}+index_shard{info.world}"),
                "index_rows": args.index_rows, "dim": cfg.hidden, "top_k": args.k,
                "mode": args.mode,
                "encode_search_overlap": overlap,
                # per-rank scan kernel: the emitting MFMA scan (csrc/hip/index_mq.hip) for >= 256
                # seeded queries (512 per workgroup at >= 512), else the 256-query list kernel
                "index_scan": (("int8-pruned-" if prune else "emitting-")
                               + ("512q" if B * info.world >= 512 else "256q"))
                              if (shard.scan_mq and args.index_dtype == "bf16" and cfg.hidden == 384
                                  and B * info.world >= shard.mq_min_nq and args.k <= 16)
                              else "list-256q",
                "encoder_hipgraph": use_graph,
                "search_priority": args.search_priority,
                "scan_min_tiles": args.scan_min_tiles,
                "prepass_min_tiles": shard.prepass_min_tiles,
                "prune_sample_shift": shard.PRUNE_TILE_SHIFT if prune else None,
            },
            "embeds_per_sec": round(total, 2) if args.mode != "search" else 0.0,
            "topk_qps": round(total, 2) if args.mode != "embed" else 0.0,
            "embed_ms_per_step_rank0": round(e_ms, 3),
            "search_ms_per_step_rank0": round(s_ms, 3),
            "host_enqueue_ms_per_step_rank0": round(host_ms, 3),
            "vs_derived_reference_estimate": (round(total / DERIVED_REF_EMBEDS_PER_SEC, 1)
                                              if args.mode != "search" else None),
        }
        print(json.dumps(res), flush=True)
    D.shutdown(info)


if __name__ == "__main__":
    main()
