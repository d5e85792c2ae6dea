#!/usr/bin/env python3
"""Run every BASELINE.json config on this node and collect one JSON line per config.

  python benchmarks/suite.py [--gpus N] [--out profiles/suite.jsonl] [--fp8-rows 200000000]

Configs (BASELINE.md "Measured" table):
  1 markov          Markov text generation over NATS (CPU)         benchmarks/markov_nats.py
  2 minilm-embed    all-MiniLM-L6-v2 bf16 embedding, batch 256      bench.py --mode embed
  3 index-100m      100M x 384 sharded cosine top-10                bench.py --mode search
  4 bge-dp          bge-base-en-v1.5 DP embedding over RCCL         bench.py --model bge-base --mode embed --opt embed_dp=group
  5 e5-fp8          e5-large-v2 + fp8 index (1B rows at N >= 4)     bench.py --model e5-large --index-dtype fp8
  + headline        MiniLM embed + top-10 over 100M x 384           bench.py
  + mpnet-embed     the reference's own model (paraphrase-multilingual-mpnet-base-v2, 768-d)
                    bf16 embedding, batch 256                       bench.py --model mpnet-multi --mode embed
  + mpnet-full      the reference's default deployment: mpnet embed + top-10 over a
                    100M x 768 collection (vector_memory_service/src/main.rs:22)
                                                                    bench.py --model mpnet-multi
  + e5-embed        e5-large-v2 bf16 embedding (every projection on our kernels)
Each config runs as a CHILD process (torch.distributed.run for N > 1) under its own timeout.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(cmd: list[str], timeout: int) -> dict | None:
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    print("[suite] " + " ".join(cmd), file=sys.stderr, flush=True)
    try:
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        print(f"[suite] timeout after {timeout}s", file=sys.stderr, flush=True)
        return {"error": "timeout", "cmd": cmd}
    sys.stderr.write(p.stderr[-2000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"rc={p.returncode}", "cmd": cmd, "stderr_tail": p.stderr[-800:]}
    return json.loads(lines[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--fp8-rows", type=int, default=0,
                    help="e5 fp8 index rows (default: 1B if N >= 4 else 200M per GPU)")
    ap.add_argument("--only", default="", help="comma list of config names")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    py = sys.executable
    if a.gpus > 1:
        launch = [py, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
                  "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py"]
    else:
        launch = [py, "bench.py"]
    common = ["--gpus", str(a.gpus), "--steps", str(a.steps), "--warmup", str(a.warmup)]
    fp8_rows = a.fp8_rows or (1_000_000_000 if a.gpus >= 4 else 200_000_000 * a.gpus)
    configs = [
        ("markov", [py, "benchmarks/markov_nats.py"], 300),
        ("minilm-embed", launch + common + ["--mode", "embed"], 600),
        ("index-100m", launch + common + ["--mode", "search"], 900),
        # N > 1: one global batch per step split over the GPUs and gathered back over RCCL
        ("bge-dp", launch + common + ["--model", "bge-base", "--mode", "embed",
                                      "--opt", "embed_dp=group"], 600),
        ("e5-fp8", launch + common + ["--model", "e5-large", "--index-dtype", "fp8",
                                      "--encoder-dtype", "fp8", "--index-rows", str(fp8_rows)], 1200),
        ("headline", launch + common, 900),
        ("mpnet-embed", launch + common + ["--model", "mpnet-multi", "--mode", "embed"], 600),
        ("mpnet-full", launch + common + ["--model", "mpnet-multi"], 1200),
        ("e5-embed", launch + common + ["--model", "e5-large", "--mode", "embed"], 600),
    ]
    only = set(filter(None, a.only.split(",")))
    results = []
    for name, cmd, to in configs:
        if only and name not in only:
            continue
        r = run(cmd, to) or {}
        r["suite_config"] = name
        results.append(r)
        print(json.dumps(r), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(r) + "\n")
        if r.get("error") == "timeout":
            break  # a hung GPU step: start nothing more on the GPU


if __name__ == "__main__":
    main()
