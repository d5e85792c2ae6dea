"""bench.py's driver contract on the CPU (gloo): a plain ``python bench.py --gpus N`` launches the
N ranks itself and rank 0 reports the whole job; a job whose world differs from --gpus fails
loudly; the synthetic corpora (index/synth.py) have the shapes the realistic search benchmarks
rely on."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--opt", "device=cpu", "--steps", "2", "--warmup", "1", "--index-rows", "6000", "--batch",
        "4", "--seq", "12", "--opt", "heldout_searches=3"]


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(OMP_NUM_THREADS="2", **(env_extra or {}))
    p = subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=400)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, [json.loads(ln) for ln in lines]


def test_bench_self_launches_n_ranks():
    p, out = _run(["--gpus", "2"] + TINY)
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(out) == 1, p.stdout          # exactly one JSON line, from rank 0 ...
    assert p.stdout.strip().splitlines() == [json.dumps(out[0])], p.stdout   # ... and nothing else
    r = out[0]
    assert r["n_gpus"] == 2 and r["world"] == 2 and r["backend"] == "gloo"
    assert r["comm_check"]["collective"].startswith("all_gather ok")
    assert r["config"]["global_batch"] == 8 and r["config"]["parallelism"] == "dp2+index_shard2"
    assert r["value"] > 0 and r["steps"] == 2 and r["warmup"] == 1
    # the realistic (held-out query) search rate rides in the same line
    assert r["heldout_searches"] == 3 and r["heldout_topk_qps"] > 0 and r["heldout_ms_per_search"] > 0


def test_bench_world_mismatch_fails():
    # a launcher-provided world of 1 with --gpus 2 must not report a 1-rank number as 2 GPUs
    p, out = _run(["--gpus", "2"] + TINY, env_extra={"WORLD_SIZE": "1", "RANK": "0",
                                                     "LOCAL_RANK": "0"}, drop=())
    assert p.returncode != 0 and not out
    assert "refusing" in p.stderr


def test_bench_simulated_world_is_labelled_a_projection():
    """--simulate-world N runs the per-rank work of the N-GPU step on ONE rank (a 1/N shard,
    N x batch gathered queries, the result exchange through a single-rank group): its JSON can
    never pass for an N-GPU measurement -- the metric says SIMULATED, n_gpus and world stay 1,
    and the N-GPU numbers sit in the simulated_* / projected_* fields only."""
    p, out = _run(["--opt", "simulate_world=4"] + TINY)
    assert p.returncode == 0, p.stderr[-2000:]
    r = out[0]
    assert r["metric"].startswith("SIMULATED 4-GPU") and "projection" in r["metric"]
    assert r["n_gpus"] == 1 and r["world"] == 1 and r["simulated"] is True
    assert r["simulated_world"] == 4 and r["config"]["simulated_world"] == 4
    assert r["config"]["index_rows_per_rank"] == 1500 and r["config"]["global_batch"] == 16
    assert "simulated" in r["config"]["parallelism"]
    assert r["value"] == r["projected_job_rate"] > 0
    # and it refuses to pose as a multi-rank run
    p2, out2 = _run(["--opt", "simulate_world=4", "--gpus", "2"] + TINY)
    assert p2.returncode != 0 and not out2


def test_bench_search_clustered_heldout_two_ranks():
    p, out = _run(["--gpus", "2", "--mode", "search", "--corpus", "clustered", "--opt",
                   "clusters=50", "--queries", "heldout"] + TINY)
    assert p.returncode == 0, p.stderr[-2000:]
    r = out[0]
    assert r["n_gpus"] == 2 and r["config"]["corpus"] == "clustered"
    assert r["config"]["queries"] == "heldout" and "held-out" in r["data"]


def test_bench_help_lists_at_most_15_options():
    """The headline's knobs stay few (VERDICT r4 housekeeping): the secondary ones live under
    --opt KEY=VALUE and an unknown key fails loudly."""
    p = subprocess.run([sys.executable, "bench.py", "--help"], cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0
    opts = {ln.split()[0].rstrip(",") for ln in p.stdout.splitlines()
            if ln.startswith("  -") and not ln.startswith("  -h")}
    assert len(opts) <= 15, sorted(opts)
    bad = subprocess.run([sys.executable, "bench.py", "--opt", "nope=1"], cwd=ROOT,
                         capture_output=True, text=True, timeout=120)
    assert bad.returncode != 0 and "expected KEY=VALUE" in bad.stderr


def test_synthetic_corpora_shapes():
    from codename_symbiont_amd.index.synth import CorpusGen

    g = CorpusGen("clustered", 384, "cpu", clusters=20, spread=0.6)
    x = g.unit(2000, seed=3)
    # every row sits near one of the shared centers: cos ~ 1/sqrt(1 + 0.36) = 0.857
    best = (x @ g.centers.t()).max(dim=1).values
    assert float(best.mean()) == pytest.approx(0.857, abs=0.03)
    assert torch.equal(g.rows(100, 9), g.rows(100, 9))          # reproducible per seed
    a = CorpusGen("anisotropic", 384, "cpu").unit(1000, seed=1)
    c = a @ a.t()
    off = c[~torch.eye(1000, dtype=torch.bool)]
    assert float(off.mean()) == pytest.approx(0.3, abs=0.05)
    r = CorpusGen("random", 384, "cpu").unit(1000, seed=1)
    assert abs(float((r @ r.t())[~torch.eye(1000, dtype=torch.bool)].mean())) < 0.01
