#!/usr/bin/env python3
"""Headline benchmark: embeds/sec + top-k QPS, all-MiniLM-L6-v2 / 100M x 384 index, 1..8 MI355X.

One STEP = the system's ingest+search cycle on every rank (one process per GPU):
  1. H2D of the next synthetic tokenized batch on a copy stream (overlaps the previous search)
  2. encode B=256 sentences x S=128 tokens with the HIP MiniLM-L6 encoder (bf16, varlen-packed)
  3. upsert the 256 unit embeddings into this rank's HBM index shard
  4. semantic search: the 256 new embeddings are the queries; all_gather the queries of all
     ranks, EXACT top-10 over the rank's shard of the 100M x 384 bf16 corpus, all_to_all the
     partial top-k back to each query's owner and merge.  The exact top-10 is found by a
     streaming MFMA scan of an int8 or MX-fp4 image of the rows (csrc/hip/index_stream.hip) that
     prunes only rows whose score provably cannot reach the query's k-th best (Cauchy-Schwarz
     bound on the quantisation error, tracked at every write); the survivors are re-scored in
     bf16: the same rows and scores as scanning every row in bf16 (GPU tests compare them;
     --opt index_prune=none runs that full bf16 scan).
So every step embeds 256*N sentences AND answers 256*N top-10 queries over the full 100M-row
corpus: value = embeds/s = top-k QPS (whole job).  Per-rank work is constant in N ("weak").
After the timed steps the same line also reports the held-out search rate (heldout_topk_qps:
fresh queries drawn from the corpus distribution, never inserted, on the same shard).

Data: synthetic token ids, random-init weights (real MiniLM-L6 architecture), random unit
index rows -- there is no network for checkpoints or datasets.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--opt KEY=VALUE ...]
       N > 1 either under a launcher (python -m torch.distributed.run --nproc-per-node N ...
       bench.py --gpus N: WORLD_SIZE is set) or plainly: with WORLD_SIZE unset this process
       launches the N ranks itself as fresh child processes BEFORE touching the GPU (one per GPU,
       env:// rendezvous on 127.0.0.1) and exits with the first failing rank's status.  A rank
       whose world differs from --gpus exits non-zero; the JSON carries the backend, the world
       and a startup collective self-check (all_gather of rank ids + device ids, verified).
       --opt device=cpu: the same step on the CPU over gloo (fp32 PyTorch encoder, tiny shapes)
       -- the multi-rank contract rehearsal the CPU tests run; never a performance number.

The other BASELINE.json configs run through the same step (benchmarks/suite.py drives them):
  --mode embed                                   all-MiniLM-L6-v2 bf16 embedding, batch 256
  --mode search                                  100M x 384 sharded cosine top-k
  --model bge-base --mode embed --opt embed_dp=group
                                                 bge-base-en-v1.5 DP embedding over RCCL
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


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n: int, argv: list[str]) -> int:
    """Run this script as ``n`` ranks (fresh child processes, one per GPU) and wait for them.

    Called only when WORLD_SIZE is unset, before anything in this process touches the GPU (no
    HIP call, no torch.cuda query): the children start as new programs, so no GPU state is ever
    inherited or exec'd over.  Rank 0 prints the JSON line (stdout is inherited).  The first rank
    to fail ends the job: the others are terminated and its exit status is returned."""
    import signal
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SYMB_BENCH_LAUNCHED="1")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL on this driver)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc, kill_at = 0, None
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"[bench] rank {procs.index(p)} exited with {code}: stopping the job",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.send_signal(signal.SIGTERM)
                kill_at = time.time() + 20.0   # a rank stuck in a collective ignores nothing else
        if kill_at is not None and time.time() > kill_at:
            for q in live:
                q.kill()
            kill_at = None
        time.sleep(0.05)
    return rc


# Secondary knobs: --opt KEY=VALUE (repeatable).  The defaults are the headline configuration;
# the JSON line's config lists every knob set away from its default.
OPTS = {
    "device": ("auto", str, "auto | cuda | cpu (cpu: the multi-rank contract rehearsal over gloo "
                            "with the fp32 PyTorch encoder and tiny shapes; never a performance "
                            "number)"),
    "clusters": (100_000, int, "--corpus clustered: shared cluster centers"),
    "cluster_spread": (0.6, float, "--corpus clustered: noise norm around a center "
                                   "(cos ~ 1/sqrt(1+s^2))"),
    "embed_dp": ("replica", str, "--mode embed, N > 1: replica (independent ranks) | group (ONE "
                                 "global batch of batch*N sentences split over the ranks and "
                                 "gathered to rank 0 over RCCL, parallel/embed_group.py)"),
    "simulate_world": (0, int, "PROJECTION on one GPU: the per-rank work of the N-GPU step (a "
                               "100M/N shard, 256*N gathered queries); the JSON says SIMULATED"),
    "timeline": ("", str, "write per-step GPU times (+ sampled clock/power) to this JSONL file"),
    "heldout_searches": (20, int, "--mode full: after the timed steps, time this many searches of "
                                  "fresh held-out queries (drawn from the corpus distribution, "
                                  "never inserted) on the same shard: heldout_topk_qps"),
    "index_prefilter": ("none", str, "none | fp8 (e4m3 copy for 3k candidates + exact bf16 "
                                     "rescore; Qdrant quantization + rescore)"),
    "index_prune": ("i8", str, "i8 (EXACT pruned search: int8 / MX-fp4 stream scan of a "
                               "bound-checked image + bf16 re-score) | none (full bf16 scan)"),
    "overlap": (1, int, "--mode full: encode batch i+1 on a second stream while batch i is "
                        "searched (0: back to back on one stream)"),
    "search_pipeline": (1, int, "--mode full: run batch i+1's query-side search work under "
                                "batch i's scan on a third stream"),
    "encode_ahead": (2, int, "pipelined step: batch i + AHEAD is encoded during step i (1 | 2)"),
    "scan_after_encode": (0, int, "pipelined step (AHEAD 2): 1 = batch i's scan waits for batch "
                                  "i + 1's encoder (measured slower: 49.0k vs 50.2k at N = 1, "
                                  "equal at simulate_world=8, profiles/r6_step/)"),
    "graph": (1, int, "--mode embed: replay a captured hipGraph of the encoder forward"),
    "prune_shift_mx4": (0, int, "exact pruned search: the sample density while the MX-fp4 tier "
                                "applies (0 = the shard default, 2^7)"),
    "prune_sample_shift": (0, int, "exact pruned search: threshold sample = 1 tile in 2^shift "
                                   "(0 = the shard default)"),
    "prune_block_frac": (0.0, float, "exact pruned search: route a row block to the bf16 scan "
                                     "above this share of the candidate slots (0 = default)"),
}


def _opts_help() -> str:
    return "secondary knobs, KEY=VALUE (repeatable): " + "; ".join(
        f"{k} (default {d!r}): {h}" for k, (d, _, h) in OPTS.items())


def parse_args(argv=None):
    ap = argparse.ArgumentParser(
        description="Headline benchmark: MiniLM-L6 embeds/s = exact top-10 QPS over 100M x 384",
        epilog="--opt keys: " + ", ".join(OPTS))
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--index-rows", type=int, default=100_000_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--model", default="minilm-l6")
    ap.add_argument("--mode", choices=["full", "embed", "search"], default="full")
    ap.add_argument("--corpus", choices=["random", "clustered", "anisotropic"], default="random",
                    help="synthetic index distribution (codename_symbiont_amd/index/synth.py)")
    ap.add_argument("--queries", choices=["self", "heldout"], default=None,
                    help="full mode: self = the batch is upserted and THEN searched (default), "
                         "heldout = searched before it is upserted.  search mode: heldout = fresh "
                         "draws from the corpus distribution, never inserted (default), self = "
                         "stored rows")
    ap.add_argument("--verify", action="store_true",
                    help="after the timed steps, search one batch both ways (this config and the "
                         "full bf16 scan of every row) and report whether the ids are identical")
    ap.add_argument("--index-dtype", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--encoder-dtype", choices=["bf16", "fp8"], default="bf16",
                    help="fp8: e4m3 projection GEMMs (BASELINE config #5); the headline stays bf16")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE", help=_opts_help())
    args = ap.parse_args(argv)
    opts = {k: d for k, (d, _, _) in OPTS.items()}
    for kv in args.opt:
        key, sep, val = kv.partition("=")
        key = key.strip().replace("-", "_")
        if not sep or key not in OPTS:
            ap.error(f"--opt {kv!r}: expected KEY=VALUE with KEY in {sorted(OPTS)}")
        try:
            opts[key] = OPTS[key][1](val)
        except ValueError:
            ap.error(f"--opt {kv!r}: bad value")
    if opts["device"] not in ("auto", "cuda", "cpu"):
        ap.error("--opt device: auto | cuda | cpu")
    if opts["embed_dp"] not in ("replica", "group"):
        ap.error("--opt embed_dp: replica | group")
    if opts["index_prefilter"] not in ("none", "fp8") or opts["index_prune"] not in ("none", "i8"):
        ap.error("--opt index_prefilter: none | fp8; index_prune: i8 | none")
    if opts["encode_ahead"] not in (1, 2):
        ap.error("--opt encode_ahead: 1 | 2")
    args.opts_changed = {k: v for k, v in opts.items() if v != OPTS[k][0]}
    for k, v in opts.items():
        setattr(args, k, v)
    args.no_overlap = not opts["overlap"]
    args.no_search_pipeline = not opts["search_pipeline"]
    args.no_graph = not opts["graph"]
    if args.simulate_world == 1:
        args.simulate_world = 0
    if args.simulate_world and (args.gpus != 1 or args.mode == "embed"):
        ap.error("--opt simulate_world projects the N-GPU search step on ONE GPU: --gpus 1, "
                 "--mode full or search")
    if args.queries is None:
        args.queries = "heldout" if args.mode == "search" else "self"
    return args


class ClockSampler:
    """Background sampler of the GPU's shader clock and power (rocm-smi, ~1 Hz) for --timeline:
    a sustained run records how the power-bound scan's clock settles, not only its step times."""

    def __init__(self, device_index: int):
        import threading

        self.samples, self.dev = [], device_index
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        import re
        import subprocess

        while not self._stop.is_set():
            try:
                out = subprocess.run(["rocm-smi", "-d", str(self.dev), "--showclocks",
                                      "--showpower"], capture_output=True, text=True,
                                     timeout=5).stdout
                sclk = re.search(r"sclk.*?\((\d+)Mhz\)", out)
                pwr = re.search(r"Power \(W\):\s*([\d.]+)", out)
                self.samples.append((time.time(), int(sclk.group(1)) if sclk else None,
                                     float(pwr.group(1)) if pwr else None))
            except Exception:   # noqa: BLE001 -- sampling is best effort
                pass
            self._stop.wait(1.0)

    def stop(self):
        self._stop.set()
        self._t.join(timeout=6)
        return self.samples


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # plain `python bench.py --gpus N`: launch the N ranks (nothing has touched the GPU yet)
        return self_launch(args.gpus, sys.argv[1:] if argv is None else list(argv))

    _claim_stdout()
    from codename_symbiont_amd.parallel import dist as D

    info = D.init(device_type=None if args.device == "auto" else args.device,
                  single_rank_group=bool(args.simulate_world))
    if info.world != args.gpus:
        print(f"[bench] rank {info.rank}: --gpus {args.gpus} but the job has {info.world} "
              f"rank(s) (WORLD_SIZE={os.environ.get('WORLD_SIZE')}): refusing to report a "
              f"{info.world}-rank number as {args.gpus}", file=sys.stderr, flush=True)
        D.shutdown(info)
        return 3
    comm = D.selfcheck(info)
    if info.device.type == "cpu":
        rc = run_cpu(args, info, comm)
    else:
        rc = run_gpu(args, info, comm)
    D.shutdown(info)
    return rc


# stdout carries exactly one line, rank 0's JSON result: everything else a rank process writes
# to fd 1 -- e.g. the version banner RCCL prints when it creates a communicator ("RCCL version :
# ...", one per rank and group) -- goes to stderr, so the driver's parse of stdout sees only the
# result.  (Set in each rank process before torch.distributed initialises.)
_RESULT_OUT = None


def _claim_stdout() -> None:
    global _RESULT_OUT
    if _RESULT_OUT is not None:
        return
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def _emit_result(line: str) -> None:
    print(line, file=_RESULT_OUT or sys.stdout, flush=True)


def metric_and_config(args, info, cfg, prune, prefilter, extra_cfg: dict):
    vw = args.simulate_world or 0
    headline = (not vw and args.model in ("minilm-l6", "minilm", "all-MiniLM-L6-v2")
                and args.mode == "full"
                and args.index_rows == 100_000_000 and args.index_dtype == "bf16"
                and args.encoder_dtype == "bf16" and prefilter is None and args.corpus == "random"
                and args.queries == "self" and info.device.type == "cuda")
    short = cfg.model_name.split("/")[-1]
    rows_txt = f"{args.index_rows / 1e6:g}M" if args.index_rows < 10**9 else f"{args.index_rows / 1e9:g}B"
    dist_txt = "" if args.corpus == "random" else f", {args.corpus} corpus"
    metric = METRIC if headline else {
        "full": f"embeds/sec + top-k QPS, {short} / {rows_txt}x{cfg.hidden} {args.index_dtype} index"
                + (" (fp8 prefilter + exact bf16 rescore)" if prefilter else "") + dist_txt,
        "embed": f"embeds/sec, {short} ({cfg.key}) {args.encoder_dtype}, batch {args.batch} x seq {args.seq}",
        "search": f"top-{args.k} QPS, {rows_txt}x{cfg.hidden} {args.index_dtype} index, "
                  f"{args.batch} {args.queries} queries/rank"
                  + (" (fp8 prefilter + exact bf16 rescore)" if prefilter else "") + dist_txt,
    }[args.mode]
    if vw:
        metric = (f"SIMULATED {vw}-GPU per-rank step on 1 GPU (projection, not a measurement): "
                  + metric)
    config = {
        "model": short, "global_batch": args.batch * info.world, "seq_len": args.seq,
        "parallelism": (f"dp{info.world}-rccl-group" if extra_cfg.pop("_group_dp", False)
                        else f"dp{info.world}+index_shard{info.world}"),
        "index_rows": args.index_rows, "dim": cfg.hidden, "top_k": args.k, "mode": args.mode,
        "corpus": args.corpus, "queries": args.queries,
    }
    if args.corpus == "clustered":
        config.update(clusters=args.clusters, cluster_spread=args.cluster_spread)
    config.update(extra_cfg)
    if vw:
        config.update(simulated_world=vw, parallelism=f"simulated dp{vw}+index_shard{vw} on 1 GPU",
                      global_batch=args.batch * vw, index_rows_per_rank=args.index_rows // vw)
    unit = (f"embeds/s (whole job; every embedded sentence is also answered as a top-{args.k} "
            f"query over the {rows_txt} x {cfg.hidden} corpus, so this equals top-k QPS)"
            if args.mode == "full" else ("embeds/s" if args.mode == "embed" else "queries/s"))
    return metric, config, unit


def scan_label(args, shard, prune, prefilter, dim: int, nq: int) -> str:
    """What the per-rank search actually runs (the JSON's index_scan): the evidence trail, so it
    names the kernel, the image and the exactness."""
    from codename_symbiont_amd.index.shard import MQ_DIMS

    if args.index_dtype == "fp8":
        return ("fp8 index: the list scan (index_fp8.hip) of the e4m3 rows, exact top-k of the "
                "stored fp8 rows")
    if prefilter:
        return "fp8 prefilter scan + exact bf16 re-score of 3k candidates"
    if args.k > 16:
        return ("bf16 emitting scan + radix select (exact, large k)" if dim in MQ_DIMS
                else "bf16 list scan (exact)")
    if prune:
        if shard.stream and shard.i8_ring and not shard._i8_heavy:
            return ("exact pruned: MX-fp4 stream scan (index_stream.hip) / int8 LDS-ring scan "
                    "(index_i8.hip) of bound-checked images + bf16 re-score")
        if shard.stream and not shard._i8_heavy:
            return ("exact pruned: int8 / MX-fp4 stream scan (index_stream.hip) of bound-checked "
                    "images + bf16 re-score")
        return ("exact pruned: " + ("split" if shard._i8_heavy else "int8") +
                " LDS-ring scan (index_i8.hip) + bf16 re-score")
    if shard.scan_mq and dim in MQ_DIMS and nq >= shard.mq_min_nq:
        return f"bf16 emitting scan (index_mq.hip, {'512' if nq >= 512 else '256'} queries/WG)"
    return "bf16 list scan (index_topk.hip, 256 queries/WG)"


def result_line(args, info, comm, metric, unit, config, total, ms, prune, prefilter, data, extra):
    res = {
        "metric": metric,
        "value": round(total, 2),
        "unit": unit,
        "n_gpus": info.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.encoder_dtype,
        "index_dtype": args.index_dtype,
        "index_prefilter": prefilter,
        "index_search": None if args.mode == "embed" else (
                        "exact: bound-pruned scan + bf16 re-score" if prune
                         else ("fp8 prefilter + bf16 re-score" if prefilter
                               else ("exact scan of the e4m3 rows" if args.index_dtype == "fp8"
                                     else "exact bf16 scan"))),
        "data": data,
        "config": config,
        "backend": comm["backend"],
        "world": comm["world"],
        "comm_check": comm,
        "embeds_per_sec": round(total, 2) if args.mode != "search" else 0.0,
        "topk_qps": round(total, 2) if args.mode != "embed" else 0.0,
        "vs_derived_reference_estimate": (round(total / DERIVED_REF_EMBEDS_PER_SEC, 1)
                                          if args.mode != "search" else None),
    }
    res.update(extra)
    vw = args.simulate_world or 0
    if vw:
        # value = the projected whole-job rate of the N-GPU job (N ranks each running this step);
        # n_gpus stays the GPUs actually used
        res.update(simulated=True, simulated_world=vw, value=round(total * vw, 2),
                   projected_per_rank_ms=round(ms, 3),
                   projected_job_rate=round(total * vw, 2),
                   note="projection: per-rank step of the N-GPU job measured on one GPU; "
                        "excludes xGMI transfer time and waiting for the slowest peer")
        res["embeds_per_sec"] = round(total * vw, 2) if args.mode != "search" else 0.0
        res["topk_qps"] = round(total * vw, 2) if args.mode != "embed" else 0.0
    return json.dumps(res)


def _data_txt(args) -> str:
    rows = {"random": "random unit index rows",
            "clustered": f"clustered unit index rows ({args.clusters} centers, spread "
                         f"{args.cluster_spread})",
            "anisotropic": "anisotropic unit index rows (shared mean direction, power-law spread)"}
    q = ("" if args.mode == "full" else
         f", {'held-out draws from the corpus distribution' if args.queries == 'heldout' else 'stored rows'} as queries")
    return f"synthetic token ids, random-init weights, {rows[args.corpus]}{q}"


def _make_searcher(args, shard, info, embed):
    """The step's sharded searcher; --opt simulate_world=N: the per-rank work of the N-GPU search
    on this one rank, the other ranks' queries stood in for by (N - 1) * batch foreign embeddings
    (``embed(n, seed)``: n fresh sentences through this encoder, never inserted here)."""
    from codename_symbiont_amd.parallel.sharded import ShardedSearcher, SimulatedShardedSearcher

    vw = args.simulate_world or 0
    if not vw:
        return ShardedSearcher(shard, info)
    foreign = [embed((vw - 1) * args.batch, 777_000 + j).bfloat16() for j in range(2)]
    return SimulatedShardedSearcher(shard, info, vw, foreign)


def run_cpu(args, info, comm) -> int:
    """The step on the CPU (gloo): encode -> upsert -> sharded search, timed the same way.  For the
    multi-rank contract tests only (fp32 PyTorch encoder, matmul search)."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import TorchEncoder, synthetic_batch
    from codename_symbiont_amd.parallel import dist as D

    torch.manual_seed(1234 + info.rank)
    cfg = get_config(args.model)
    B, S, K, W = args.batch, args.seq, args.steps, args.warmup
    enc = TorchEncoder(cfg, seed=0)
    vw = args.simulate_world or 0
    rows_per_rank = args.index_rows // (vw or info.world)
    shard = HbmIndexShard(cfg.hidden, rows_per_rank + (K + W + 4) * B, device="cpu")
    gen = CorpusGen(args.corpus, cfg.hidden, "cpu", clusters=args.clusters,
                    spread=args.cluster_spread)
    if args.mode != "embed":
        fill_corpus(shard, gen, rows_per_rank, seed=100 + info.rank)
    searcher = _make_searcher(args, shard, info, lambda n, seed: enc.forward_packed(
        synthetic_batch(cfg, n, S, seed=seed))[1])
    host = [synthetic_batch(cfg, B, S, seed=1000 * info.rank + i) for i in range(4)]
    qsets = [gen.unit(B, 5000 + 10 * info.rank + i).bfloat16() for i in range(4)]

    def step(i):
        q = None
        if args.mode != "search":
            _, q = enc.forward_packed(host[i % 4])
            if args.queries == "self":
                shard.append_unit(q)
        else:
            q = qsets[i % 4] if args.queries == "heldout" else shard.rows[(i * B) % max(1, shard.count - B):][:B]
        if args.mode != "embed":
            searcher.search(q, args.k)
        if args.mode != "search" and args.queries == "heldout":
            shard.append_unit(q)

    for i in range(W):
        step(i)
    D.barrier(info)
    t0 = time.perf_counter()
    for j in range(K):
        step(W + j)
    D.barrier(info)
    elapsed = D.allreduce_max(info, time.perf_counter() - t0)
    ms = elapsed * 1000.0 / K
    total = B * info.world * K / elapsed
    extra = {}
    if args.mode == "full" and args.heldout_searches > 0:   # (the GPU run's held-out phase)
        H = args.heldout_searches
        hq = [gen.unit(B, 9000 + 10 * info.rank + i).bfloat16() for i in range(2)]
        D.barrier(info)
        t_h = time.perf_counter()
        for i in range(H):
            searcher.search(hq[i % 2], args.k)
        D.barrier(info)
        el_h = D.allreduce_max(info, time.perf_counter() - t_h)
        extra = {"heldout_topk_qps": round(B * info.world * H / el_h, 2),
                 "heldout_ms_per_search": round(el_h * 1000.0 / H, 3), "heldout_searches": H}
    metric, config, unit = metric_and_config(args, info, cfg, None, None, {"device": "cpu"})
    if info.rank == 0:
        _emit_result(result_line(args, info, comm, metric, unit, config, total, ms, None, None,
                                 _data_txt(args) + " (CPU rehearsal: not a performance number)",
                                 extra))
    return 0


def _framing(cfg):
    """[CLS] / [SEP] ids of the synthetic batches (encoder.synthetic_batch's framing)."""
    return (101, 102) if cfg.vocab_size > 30000 and cfg.pad_token_id == 0 else (0, 2)


def run_embed(args, info, comm, enc, cfg, t_setup: float) -> int:
    """--mode embed (BASELINE configs #2 / #4, replica DP: every rank embeds its own batch).

    One step = B full-length sentences of S tokens through the HIP encoder.  Every step's token
    ids are NEW: drawn on the GPU by torch.randint inside the replayed hipGraph (the graph-safe
    default generator advances its Philox offset on every replay) and framed with [CLS] / [SEP]
    at the sentence bounds; positions and cu_seqlens keep the fixed full-length layout.  No index
    shard is allocated and nothing is upserted (the reference's batch loop,
    preprocessing_service/src/embedding_generator.rs:146-214, only embeds).  The graph holds the
    token draw and the whole forward, so the host enqueues one replay per step."""
    from codename_symbiont_amd.models.encoder import synthetic_batch
    from codename_symbiont_amd.parallel import dist as D
    from codename_symbiont_amd.utils.gpu_debug import debug_enabled

    dev = info.device
    B, S, K, W = args.batch, args.seq, args.steps, args.warmup
    torch.manual_seed(4321 + info.rank)
    batch = synthetic_batch(cfg, B, S, seed=1000 * info.rank).to(dev)
    T = batch.num_tokens
    cls, sep = _framing(cfg)
    cls_at = batch.cu_seqlens[:-1].long()
    sep_at = (batch.cu_seqlens[1:] - 1).long()
    out32 = torch.empty(B, cfg.hidden, device=dev)
    outu = torch.empty(B, cfg.hidden, dtype=torch.bfloat16, device=dev)

    def draw_and_encode() -> None:
        torch.randint(1000, cfg.vocab_size, (T,), device=dev, dtype=torch.int32, out=batch.ids)
        batch.ids.index_fill_(0, cls_at, cls)
        batch.ids.index_fill_(0, sep_at, sep)
        enc.forward_packed(batch, out32, outu)

    draw_and_encode()   # kernel attributes, workspace
    torch.cuda.synchronize(dev)
    use_graph = not args.no_graph and not debug_enabled()
    run = draw_and_encode
    if use_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            draw_and_encode()
        run = graph.replay
    log(info, f"[bench] setup {time.time() - t_setup:.1f}s: {cfg.model_name} embed, {B} x {S} "
              f"tokens per step, no index shard; graph={use_graph}")
    ids_seen = []
    for i in range(max(W, 2)):
        run()
        if i < 2:
            ids_seen.append(batch.ids.clone())
    fresh = not torch.equal(ids_seen[0], ids_seen[1])
    torch.cuda.synchronize(dev)
    D.barrier(info)
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(K)]
    cur = torch.cuda.current_stream(dev)
    t_start = time.perf_counter()
    for j in range(K):
        evs[j][0].record(cur)
        run()
        evs[j][1].record(cur)
    host_ms = (time.perf_counter() - t_start) * 1000.0 / K
    torch.cuda.synchronize(dev)
    D.barrier(info)
    torch.cuda.synchronize(dev)
    elapsed = D.allreduce_max(info, time.perf_counter() - t_start)
    ms = elapsed * 1000.0 / K
    total = B * info.world * K / elapsed
    extra_out = {
        "embed_ms_per_step_rank0": round(sum(a.elapsed_time(b) for a, b in evs) / K, 3),
        "host_enqueue_ms_per_step_rank0": round(host_ms, 3),
        "token_ids": "drawn on the GPU every step inside the replayed graph",
        "token_ids_fresh_per_step": fresh,
        "index_shard": None,
    }
    cfg_extra = dict(args.opts_changed)
    cfg_extra.pop("timeline", None)
    if use_graph:
        cfg_extra["encoder_hipgraph"] = True
    metric, config, unit = metric_and_config(args, info, cfg, None, None, cfg_extra)
    config["parallelism"] = f"dp{info.world} (replica: one batch per rank)"
    if info.rank == 0:
        data = (f"synthetic token ids (fresh every step, {S}-token sentences), random-init "
                f"weights; no index")
        _emit_result(result_line(args, info, comm, metric, unit, config, total, ms, None, None,
                                 data, extra_out))
    return 0


def run_gpu(args, info, comm) -> int:
    from codename_symbiont_amd.index.shard import MQ_DIMS, HbmIndexShard, resolve_prune
    from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, refill_synthetic, synthetic_batch
    from codename_symbiont_amd.parallel import dist as D

    dev = info.device
    torch.manual_seed(1234 + info.rank)
    cfg = get_config(args.model)
    B, S, K, W = args.batch, args.seq, args.steps, args.warmup

    t0 = time.time()
    enc = HipEncoder(cfg, seed=0, device=dev, precision=args.encoder_dtype)
    vw = args.simulate_world or 0
    rows_per_rank = args.index_rows // (vw or info.world)
    extra = (K + W + 4) * B
    prefilter = None if args.index_prefilter == "none" else args.index_prefilter

    # exact either way; i8 applies to 384-wide bf16 shards without a prefilter (else: plain scan)
    prune = resolve_prune("auto" if args.index_prune == "i8" and args.mode != "embed" else "none",
                          args.index_dtype, cfg.hidden, prefilter, device=dev)
    group_dp = args.mode == "embed" and args.embed_dp == "group" and info.world > 1
    if args.mode == "embed" and not group_dp:
        # config #2 / #4: the encoder alone -- no index shard, no upserts, token ids drawn on
        # the GPU inside the replayed graph (run_embed)
        return run_embed(args, info, comm, enc, cfg, t0)
    gen = CorpusGen(args.corpus, cfg.hidden, dev, clusters=args.clusters,
                    spread=args.cluster_spread)
    shard = searcher = None
    if args.mode != "embed":
        shard = HbmIndexShard(cfg.hidden, rows_per_rank + extra, device=dev,
                              dtype=args.index_dtype, prefilter=prefilter, prune=prune)
        fill_corpus(shard, gen, rows_per_rank, seed=100 + info.rank)
        searcher = _make_searcher(args, shard, info, lambda n, seed: enc.forward_packed(
            synthetic_batch(cfg, n, S, seed=seed).to(dev))[1].clone())
        shard.mq_stats = (os.environ.get("SYMB_MQ_STATS", "0") not in ("", "0")
                          or args.mode == "search")
        if args.prune_shift_mx4:
            shard.PRUNE_TILE_SHIFT_MX4 = args.prune_shift_mx4
        if args.prune_sample_shift:
            shard.PRUNE_TILE_SHIFT = shard.PRUNE_TILE_SHIFT_SPLIT = args.prune_sample_shift
            shard.PRUNE_TILE_SHIFT_MX4 = args.prune_sample_shift
        if args.prune_block_frac:
            shard.PRUNE_BLOCK_FRAC = args.prune_block_frac
    torch.cuda.synchronize(dev)
    row_bytes = cfg.hidden * (1 if args.index_dtype == "fp8" else 2)
    log(info, f"[bench] setup {time.time() - t0:.1f}s: {cfg.model_name}, "
              + (f"shard {rows_per_rank} rows x {cfg.hidden} {args.index_dtype} ({args.corpus}) = "
                 f"{rows_per_rank * row_bytes / 1e9:.1f} GB/rank" if shard is not None
                 else "no index shard (embed mode)") + f"; comm {comm}")
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
    copy_done = [torch.cuda.Event(), torch.cuda.Event()]
    consumed = [torch.cuda.Event(), torch.cuda.Event()]
    host_free = [torch.cuda.Event() for _ in range(NB)]   # host slot's H2D copy has finished
    out_f32 = torch.empty(B, cfg.hidden, device=dev)
    out_unit = torch.empty(B, cfg.hidden, dtype=torch.bfloat16, device=dev)
    # --mode full pipelines the two halves of a step across two streams: batch i+1 is encoded
    # on enc_stream while batch i's queries are searched on the compute stream (the scan is
    # power-bound; the encoder's small kernels fill its tail and launch gaps).  Every timed step
    # still encodes one batch and searches one batch.
    overlap = args.mode == "full" and not group_dp and not args.no_overlap
    enc_stream = torch.cuda.Stream(dev)
    # output slots: batch i's embeddings live in outs[i % NO] from its encode to its search's end
    pipeline = overlap and args.queries == "self" and not args.no_search_pipeline
    AHEAD = args.encode_ahead if pipeline else 1
    NO = AHEAD + 1
    outs = [(torch.empty(B, cfg.hidden, device=dev),
             torch.empty(B, cfg.hidden, dtype=torch.bfloat16, device=dev)) for _ in range(NO)]
    enc_done = [torch.cuda.Event() for _ in range(NO)]
    q_free = [torch.cuda.Event() for _ in range(NO)]
    # SYMB_GPU_DEBUG=1: assert the host enqueue order the events above rely on
    from codename_symbiont_amd.utils.gpu_debug import BufferRing

    in_ring, out_ring = BufferRing(2, "bench.dbuf"), BufferRing(NO, "bench.outs")
    # search mode: held-out queries are fresh draws from the corpus distribution (never
    # inserted); self queries are stored rows (each query's best match is itself)
    if args.queries == "heldout":
        qsets = [gen.unit(B, 5000 + 10 * info.rank + i).bfloat16() for i in range(NB)]
    elif shard is not None:
        stride = max(1, rows_per_rank // (NB * B))
        qsets = [shard.rows[torch.arange(B, device=dev) * stride + i].clone() for i in range(NB)]

    # host time per phase of the timed steps (reported as host_phase_ms_per_step): waits on the
    # copy ring, synthetic token generation, and the enqueue of the encoder / search halves
    hph = {"wait_copy_slot": 0.0, "synth_tokens": 0.0, "enc_enqueue": 0.0,
           "search_begin_enqueue": 0.0, "search_end_enqueue": 0.0}

    def prefetch(i: int) -> None:
        """H2D of batch i on the copy stream.  Every step gets NEVER-SEEN token ids: host slot
        i % NB is refilled in place once its previous copy has finished (the host runs at most
        NB batches ahead of the copy stream)."""
        slot, hs = i % 2, i % NB
        t0 = time.perf_counter()
        if i >= NB:
            host_free[hs].synchronize()
        t1 = time.perf_counter()
        refill_synthetic(host[hs], cfg, seed=(info.rank << 32) + i)
        hph["wait_copy_slot"] += t1 - t0
        hph["synth_tokens"] += time.perf_counter() - t1
        with torch.cuda.stream(copy_stream):
            if i >= 2:
                copy_stream.wait_event(consumed[slot])
            h, d = host[hs], dbuf[slot]
            if overlap:
                in_ring.fill(slot)
            d.ids.copy_(h.ids, non_blocking=True)
            d.pos.copy_(h.pos, non_blocking=True)
            d.cu_seqlens.copy_(h.cu_seqlens, non_blocking=True)
            d.max_len = h.max_len
            copy_done[slot].record(copy_stream)
            host_free[hs].record(copy_stream)

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
        """Encode batch i (input slot i % 2) on enc_stream into outs[i % NO] (overlap mode)."""
        slot, o = i % 2, i % NO
        with torch.cuda.stream(enc_stream):
            enc_stream.wait_event(copy_done[slot])
            if i >= NO:
                enc_stream.wait_event(q_free[o])   # batch i - NO's queries are searched
            if ev:
                ev[0].record(enc_stream)
            in_ring.consume(slot)
            out_ring.fill(o)
            run_encoder(slot, *outs[o])
            if ev:
                ev[1].record(enc_stream)
            consumed[slot].record(enc_stream)
            enc_done[o].record(enc_stream)
        prefetch(i + 1)

    # --mode full, self queries: the search is pipelined too.  Batch i+1's query-side search
    # work (upsert, int8 queries, the exact threshold sample, route) runs on pre_stream as soon
    # as it is encoded, under batch i's full-shard scan; the compute stream only runs the scans
    # back to back (ShardedSearcher.begin / end, HbmIndexShard.search_begin / search_end).
    pre_stream = torch.cuda.Stream(dev)
    pre_done = [torch.cuda.Event() for _ in range(NO)]
    handles: dict = {}

    def begin_search(i: int) -> None:
        slot = i % NO
        with torch.cuda.stream(pre_stream):
            pre_stream.wait_event(enc_done[slot])
            q = outs[slot][1]
            shard.append_unit(q)
            handles[i] = searcher.begin(q, args.k)
            pre_done[slot].record(pre_stream)

    def step_pipelined(i: int, ev=None) -> None:
        slot = i % NO
        # with AHEAD = 2, batch i + 2's encoder is enqueued now: it runs once batch i's scan
        # releases the CUs, beside batch i + 1's pre-pass, instead of between them
        t0 = time.perf_counter()
        encode_async(i + AHEAD, ev)
        t1 = time.perf_counter()
        begin_search(i + 1)
        t2 = time.perf_counter()
        compute.wait_event(pre_done[slot])
        if AHEAD == 2 and args.scan_after_encode:
            # (A/B) batch i + 1's encoder finishes before batch i's scan holds every SIMD; measured
            # slower than letting the scan start first (profiles/r6_step/)
            compute.wait_event(enc_done[(i + 1) % NO])
        if ev:
            ev[2].record(compute)
        searcher.end(handles.pop(i))
        hph["enc_enqueue"] += t1 - t0      # (includes prefetch: its waits / tokens counted too)
        hph["search_begin_enqueue"] += t2 - t1
        hph["search_end_enqueue"] += time.perf_counter() - t2
        out_ring.consume(slot)
        q_free[slot].record(compute)
        if ev:
            ev[3].record(compute)

    def step_overlap(i: int, ev=None) -> None:
        """Search batch i (encoded by the previous step) while batch i+1 encodes."""
        if pipeline:
            return step_pipelined(i, ev)
        slot = i % NO
        encode_async(i + 1, ev)
        compute.wait_event(enc_done[slot])
        if ev:
            ev[2].record(compute)
        q = outs[slot][1]
        if args.queries == "self":
            shard.append_unit(q)
        searcher.search(q, args.k)
        if args.queries == "heldout":
            shard.append_unit(q)
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
                egroup.embed(dbuf[slot], cu_host=host[i % NB].cu_seqlens)
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
            if args.queries == "self" and shard is not None:
                shard.append_unit(out_unit)
            q = out_unit
        else:
            q = qsets[i % NB]
        if ev:
            ev[1].record(compute)
            ev[2].record(compute)
        if args.mode != "embed":
            searcher.search(q, args.k)
        if args.mode == "full" and args.queries == "heldout":
            shard.append_unit(q)
        if ev:
            ev[3].record(compute)

    prefetch(0)
    if overlap:
        for j in range(AHEAD):
            encode_async(j)
        if pipeline:
            begin_search(0)
    for i in range(W):
        step(i)
    torch.cuda.synchronize(dev)
    D.barrier(info)
    torch.cuda.synchronize(dev)
    if shard is not None and shard._mq_tot is not None:   # overflows of the timed steps only
        for t in shard._mq_tot:
            t.zero_()
    if shard is not None and shard._mx4_tot is not None:
        shard._mx4_tot.zero_()
    for kph in hph:
        hph[kph] = 0.0
    sampler = ClockSampler(dev.index) if (args.timeline and info.is_root) else None
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
    e_each = [a.elapsed_time(b) for a, b, _, _ in evs]
    s_each = [c.elapsed_time(d) for _, _, c, d in evs]
    e_ms, s_ms = sum(e_each) / K, sum(s_each) / K

    ms = elapsed * 1000.0 / K
    total = B * info.world * K / elapsed
    extra_out = {
        "embed_ms_per_step_rank0": round(e_ms, 3),
        "search_ms_per_step_rank0": round(s_ms, 3),
        "host_enqueue_ms_per_step_rank0": round(host_ms, 3),
        "host_phase_ms_per_step_rank0": {kph: round(v * 1000.0 / K, 3) for kph, v in hph.items()},
    }
    if group_dp:   # ranks 1..N-1's pooled rows cross the wire in this dtype
        extra_out["embed_wire"] = egroup.wire
    if sampler is not None:
        clocks = sampler.stop()
        # step boundaries: the search-end events, relative to the first step's start
        ends = [evs[0][0].elapsed_time(e[3]) for e in evs]
        with open(args.timeline, "w") as f:
            for j in range(K):
                f.write(json.dumps({"step": j, "end_ms": round(ends[j], 3),
                                    "embed_ms": round(e_each[j], 3),
                                    "search_ms": round(s_each[j], 3)}) + "\n")
            for t, sclk, pw in clocks:
                f.write(json.dumps({"t": round(t - clocks[0][0], 2) if clocks else 0,
                                    "sclk_mhz": sclk, "power_w": pw}) + "\n")
        q = max(1, K // 10)
        extra_out["step_ms_first_decile"] = round((ends[q - 1]) / q, 3)
        extra_out["step_ms_last_decile"] = round((ends[-1] - ends[-q - 1]) / q, 3) if K > q else None
        if clocks:
            extra_out["sclk_mhz_samples"] = [c[1] for c in clocks][:: max(1, len(clocks) // 20)]
    if shard is not None and shard._mx4_tot is not None:   # batches the MX-fp4 tier served
        extra_out["search_mx4_tier_batches"] = int(shard._mx4_tot.item())
    if shard is not None and shard._mq_tot is not None:
        ovf = int(shard._mq_tot[0].item())
        extra_out["search_overflow_batches"] = ovf
        extra_out["search_max_candidates"] = int(shard._mq_tot[1].item())
        extra_out["search_dense_route_batches"] = int(shard._mq_tot[2].item()) if len(shard._mq_tot) > 2 else None
        if len(shard._mq_tot) > 4:   # searches that sent only some row blocks to the bf16 scan
            extra_out["search_block_route_batches"] = int(shard._mq_tot[3].item())
            extra_out["search_block_routed_blocks"] = int(shard._mq_tot[4].item())
        if shard.prune_on:   # the pruning image's form (HbmIndexShard.calibrate_prune)
            extra_out["i8_image"] = "split" if shard._i8_heavy else "plain"
            extra_out["i8_calib_share"] = (None if shard.calib_share is None
                                           else round(shard.calib_share, 3))
        print(f"[bench] rank {info.rank} searches: {ovf} overflowed, max "
              f"{int(shard._mq_tot[1].item())} candidates per query", file=sys.stderr, flush=True)
    if args.mode == "full" and args.heldout_searches > 0:
        # the realistic search rate beside the headline: fresh held-out queries (drawn from the
        # corpus distribution, never inserted -- the reference serves arbitrary user text,
        # api_service/src/main.rs:272-512) searched on the same shard after the timed steps
        H = args.heldout_searches
        hq = [gen.unit(B, 9000 + 10 * info.rank + i).bfloat16() for i in range(4)]
        for i in range(2):   # (the sample density adapts to the tier the last searches took)
            searcher.search(hq[i % 4], args.k)
        torch.cuda.synchronize(dev)
        D.barrier(info)
        torch.cuda.synchronize(dev)
        mx_before = int(shard._mx4_tot.item()) if shard._mx4_tot is not None else None
        t_h = time.perf_counter()
        for i in range(H):
            searcher.search(hq[i % 4], args.k)
        torch.cuda.synchronize(dev)
        D.barrier(info)
        torch.cuda.synchronize(dev)
        el_h = D.allreduce_max(info, time.perf_counter() - t_h)
        extra_out["heldout_topk_qps"] = round(B * info.world * H / el_h, 2)
        extra_out["heldout_ms_per_search"] = round(el_h * 1000.0 / H, 3)
        extra_out["heldout_searches"] = H
        if mx_before is not None:
            extra_out["heldout_mx4_tier_batches"] = int(shard._mx4_tot.item()) - mx_before
    if args.verify and args.mode != "embed":
        q = qsets[0] if args.mode == "search" else outs[0][1] if overlap else out_unit
        s1, i1 = searcher.search(q, args.k)
        prune_saved, shard.prune = shard.prune, None
        mq_saved, shard.scan_mq = shard.scan_mq, False
        s2, i2 = searcher.search(q, args.k)          # the seeded full bf16 list scan
        shard.prune, shard.scan_mq = prune_saved, mq_saved
        torch.cuda.synchronize(dev)
        # exact = the same scores (up to fp32 summation order) and the same ids, except where two
        # rows tie at the cut (their exact fp32 scores within 2e-6): tied rows may swap
        d_s = float((s1 - s2).abs().max().item())
        gid1, gid2 = i1.long(), i2.long()
        mism = gid1 != gid2
        n_mism = int(mism.sum().item())
        ties_only = True
        if n_mism and info.world == 1:
            qf = q.float()
            def true_scores(g):
                rows = shard.rows[g.clamp_min(0)].float()
                return torch.einsum("qkd,qd->qk", rows, qf)
            t1, t2 = true_scores(gid1), true_scores(gid2)
            ties_only = bool(((t1 - t2).abs()[mism] <= 2e-6).all().item())
        ok = d_s <= 1e-5 and ties_only
        extra_out["verify_exact"] = D.allreduce_max(info, 0.0 if ok else 1.0) == 0.0
        extra_out["verify_ids_identical"] = n_mism == 0
        extra_out["verify_id_mismatches_all_ties"] = ties_only
        extra_out["verify_max_score_diff"] = d_s
    cfg_extra = dict(args.opts_changed)
    cfg_extra.pop("timeline", None)
    if args.mode != "embed":
        cfg_extra["index_scan"] = scan_label(args, shard, prune, prefilter, cfg.hidden,
                                             B * (vw or info.world))
    if use_graph:
        cfg_extra["encoder_hipgraph"] = True
    metric, config, unit = metric_and_config(args, info, cfg, prune, prefilter,
                                             dict(cfg_extra, _group_dp=group_dp))
    if info.rank == 0:
        _emit_result(result_line(args, info, comm, metric, unit, config, total, ms, prune,
                                 prefilter, _data_txt(args), extra_out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
