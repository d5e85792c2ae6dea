"""Supervisor: the docker-compose.yml replacement (no docker on MI355X boxes).

    python -m codename_symbiont_amd.launch [--gpus N] [--only api,preprocessing,...]
           [--broker-port 4222] [--api-port 8080] [--no-broker] [--env-file .env]

Starts the in-repo NATS broker and every service as child processes with the reference's env
plumbing (NATS_URL, API_SERVER_*, NEO4J_*, ...).  GPU services scale with ``--gpus``:
* preprocessing: N independent processes (one per GPU, HIP_VISIBLE_DEVICES pinned) in the NATS
  queue group "preprocessing" -> data-parallel ingest, each message handled exactly once; or, with
  ``--embed-dp rccl``, ONE service over N ranks whose batches are split across the GPUs and
  gathered back over RCCL (parallel/embed_group.py);
* vector_memory: ONE logical index over N ranks (torch.distributed.run, RCCL), rank 0 on NATS.
Unlike the reference compose file (no restart policies) crashed children are
restarted with exponential backoff.  Children are started as subprocesses, never exec'd.

Like ``docker compose``, a ``.env`` file in the working directory (or ``--env-file``) supplies
variables (the reference's keys: NATS_URL, NEO4J_*, API_SERVER_PORT, ...; .env.example:1-12);
variables already set in the launching shell take precedence over the file.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time

SERVICES = ("text_generator", "perception", "preprocessing", "vector_memory", "knowledge_graph", "api")


class Child:
    def __init__(self, name: str, argv: list[str], env: dict):
        self.name, self.argv, self.env = name, argv, env
        self.proc: subprocess.Popen | None = None
        self.restarts = 0
        self.backoff = 0.5
        self.next_start = 0.0

    def start(self) -> None:
        self.proc = subprocess.Popen(self.argv, env=self.env, start_new_session=True)
        print(f"[launch] started {self.name} pid={self.proc.pid}", file=sys.stderr, flush=True)

    def poll(self) -> None:
        if self.proc is None:
            if time.time() >= self.next_start:
                self.start()
            return
        rc = self.proc.poll()
        if rc is not None:
            print(f"[launch] {self.name} exited rc={rc}; restarting in {self.backoff:.1f}s",
                  file=sys.stderr, flush=True)
            self.proc = None
            self.restarts += 1
            self.next_start = time.time() + self.backoff
            self.backoff = min(30.0, self.backoff * 2)

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            os.killpg(self.proc.pid, signal.SIGTERM)
            try:
                self.proc.wait(10)
            except subprocess.TimeoutExpired:
                os.killpg(self.proc.pid, signal.SIGKILL)


def build_children(a) -> list[Child]:
    from .utils.config import read_env_file
    from .utils.gpu_debug import debug_env

    py = sys.executable
    env_file = getattr(a, "env_file", None)
    if env_file is None and os.path.exists(".env"):
        env_file = ".env"
    # compose semantics: the shell's own variables win over the .env file
    file_env = read_env_file(env_file) if env_file else {}
    base = debug_env(dict(file_env, **os.environ))   # + AMD_SERIALIZE_KERNEL / HIP_LAUNCH_BLOCKING
    base.setdefault("NATS_URL", f"nats://127.0.0.1:{a.broker_port}")
    if a.api_port is not None:
        base["API_SERVER_PORT"] = str(a.api_port)
    base.setdefault("API_SERVER_PORT", "8080")
    only = set(a.only.split(",")) if a.only else set(SERVICES)
    kids = []
    if not a.no_broker:
        kids.append(Child("broker", [py, "-m", "codename_symbiont_amd.bus.broker", "--port",
                                     str(a.broker_port)], base))
    mod = "codename_symbiont_amd.services."
    for s in SERVICES:
        if s not in only:
            continue
        if s == "preprocessing" and a.gpus > 1 and a.embed_dp == "rccl":
            kids.append(Child("preprocessing", [py, "-m", "torch.distributed.run", "--nnodes=1",
                                                f"--nproc-per-node={a.gpus}", "--master-addr",
                                                "127.0.0.1", "--master-port", str(a.dist_port + 1),
                                                "-m", mod + s], base))
        elif s == "preprocessing" and a.gpus > 1:
            for g in range(a.gpus):
                env = dict(base, HIP_VISIBLE_DEVICES=str(g), SYMB_QUEUE_GROUP="preprocessing")
                kids.append(Child(f"preprocessing[{g}]", [py, "-m", mod + s], env))
        elif s == "vector_memory" and a.gpus > 1:
            kids.append(Child("vector_memory", [py, "-m", "torch.distributed.run", "--nnodes=1",
                                                f"--nproc-per-node={a.gpus}", "--master-addr",
                                                "127.0.0.1", "--master-port", str(a.dist_port),
                                                "-m", mod + s], base))
        else:
            kids.append(Child(s, [py, "-m", mod + s], base))
    return kids


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--only", default="")
    ap.add_argument("--broker-port", type=int, default=4222)
    ap.add_argument("--api-port", type=int, default=None,
                    help="gateway port (default: API_SERVER_PORT from the env / .env, else 8080)")
    ap.add_argument("--env-file", default=None, help="compose-style KEY=VALUE file (default .env)")
    ap.add_argument("--dist-port", type=int, default=29600)
    ap.add_argument("--no-broker", action="store_true")
    ap.add_argument("--embed-dp", choices=["queue", "rccl"], default="queue",
                    help="multi-GPU embedding: NATS queue-group replicas or one RCCL group")
    a = ap.parse_args()
    kids = build_children(a)
    stop = {"flag": False}

    def on_sig(*_):
        stop["flag"] = True
    signal.signal(signal.SIGINT, on_sig)
    signal.signal(signal.SIGTERM, on_sig)
    for k in kids:
        k.start()
        if k.name == "broker":
            time.sleep(0.5)
    try:
        while not stop["flag"]:
            for k in kids:
                k.poll()
            time.sleep(0.2)
    finally:
        for k in reversed(kids):
            k.stop()


if __name__ == "__main__":
    main()
