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

Health checks (the compose ``healthcheck`` the reference's CHANGELOG.md:92 mentions but its
compose file lacks): a child that is alive but stuck is killed and restarted.
- Every Python service publishes ``metrics.<service>`` every ``--health-interval`` seconds from
  its event loop (services/base.py). A loop that stops publishing for ``--health-retries``
  intervals is unhealthy.
- The gateway is probed with ``GET /api/health``, and the broker with a NATS PING.
- Probes start after ``--health-grace`` seconds. A service is only judged by its metrics once it
  has reported at least once, because a long index restore must not count as a hang.
- ``--health-interval 0`` turns the checks off.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import threading
import time

SERVICES = ("text_generator", "perception", "preprocessing", "vector_memory", "knowledge_graph", "api")


class Child:
    def __init__(self, name: str, argv: list[str], env: dict, probe: tuple | None = None):
        self.name, self.argv, self.env = name, argv, env
        # ("metrics", service, replica) | ("http", url) | ("nats", url) | None
        self.probe = probe
        self.proc: subprocess.Popen | None = None
        self.restarts = 0
        self.backoff = 0.5
        self.next_start = 0.0
        self.started_at = 0.0
        self.failures = 0

    def start(self) -> None:
        self.proc = subprocess.Popen(self.argv, env=self.env, start_new_session=True)
        self.started_at = time.monotonic()
        self.failures = 0
        print(f"[launch] started {self.name} pid={self.proc.pid}", file=sys.stderr, flush=True)

    def kill_unhealthy(self, why: str) -> None:
        """Take a stuck child down hard; ``poll`` then restarts it with backoff."""
        if self.proc is not None and self.proc.poll() is None:
            print(f"[launch] {self.name} unhealthy ({why}); restarting", file=sys.stderr,
                  flush=True)
            try:
                os.killpg(self.proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass

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


class HealthMonitor(threading.Thread):
    """Last time a ``metrics.<service>`` message arrived per (service, replica), from a daemon
    thread with its own plain-socket NATS subscription (parallel/heartbeat.py's connection)."""

    def __init__(self, nats_url: str):
        super().__init__(daemon=True, name="launch-health")
        self.url = nats_url
        self.last_seen: dict[tuple[str, str], float] = {}
        self._stop = threading.Event()

    def run(self) -> None:
        from .parallel.heartbeat import _Conn

        conn = None
        while not self._stop.is_set():
            try:
                if conn is None:
                    conn = _Conn(self.url)
                    conn.send(b"SUB metrics.> 1\r\nPING\r\n")
                for ev in conn.events(0.5):
                    if ev[0] == "MSG":
                        try:
                            body = json.loads(bytes(ev[-1]))
                            key = (body.get("service", ""), str(body.get("replica", "")))
                        except (ValueError, AttributeError, TypeError):
                            continue
                        self.last_seen[key] = time.monotonic()
                    elif ev[0] == "PING":
                        conn.send(b"PONG\r\n")
            except (OSError, ConnectionError, ValueError):
                if conn is not None:
                    conn.close()
                conn = None
                self._stop.wait(0.5)
        if conn is not None:
            conn.close()

    def stop(self) -> None:
        self._stop.set()


def probe_ok(child: Child, monitor: HealthMonitor | None, stale_s: float) -> tuple[bool, str]:
    """(healthy, reason) for one child's probe."""
    kind = child.probe[0]
    if kind == "metrics":
        seen = monitor.last_seen.get((child.probe[1], child.probe[2])) if monitor else None
        if seen is None or seen < child.started_at:
            # not reporting yet: still initialising (a snapshot restore of a 100M-row index can
            # outlast any fixed grace), so only a child that HAS reported can go stale
            return True, ""
        age = time.monotonic() - seen
        return age <= stale_s, f"no metrics.{child.probe[1]} for {age:.1f}s"
    if kind == "http":
        import urllib.request

        try:
            with urllib.request.urlopen(child.probe[1], timeout=2.0) as r:
                return r.status == 200, f"HTTP {r.status}"
        except Exception as e:   # noqa: BLE001 - any failure is unhealthy
            return False, f"health probe failed: {e}"
    if kind == "nats":
        from .parallel.heartbeat import _Conn

        try:
            conn = _Conn(child.probe[1])
            try:
                conn.send(b"PING\r\n")
                t0 = time.monotonic()
                while time.monotonic() - t0 < 2.0:
                    if any(ev[0] == "PONG" for ev in conn.events(0.5)):
                        return True, ""
            finally:
                conn.close()
        except (OSError, ConnectionError, ValueError) as e:
            return False, f"NATS probe failed: {e}"
        return False, "no PONG within 2s"
    return True, ""


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
    interval = getattr(a, "health_interval", 0) or 0
    if interval:
        base["SYMB_METRICS_INTERVAL"] = str(interval)
    svc = lambda s, r="": ("metrics", f"{s}_service", r) if interval else None  # noqa: E731
    only = set(a.only.split(",")) if a.only else set(SERVICES)
    kids = []
    if not a.no_broker:
        kids.append(Child("broker", [py, "-m", "codename_symbiont_amd.bus.broker", "--port",
                                     str(a.broker_port)], base,
                          ("nats", f"nats://127.0.0.1:{a.broker_port}") if interval else None))
    mod = "codename_symbiont_amd.services."
    for s in SERVICES:
        if s not in only:
            continue
        if s == "preprocessing" and a.gpus > 1 and a.embed_dp == "rccl":
            kids.append(Child("preprocessing", [py, "-m", "torch.distributed.run", "--nnodes=1",
                                                f"--nproc-per-node={a.gpus}", "--master-addr",
                                                "127.0.0.1", "--master-port", str(a.dist_port + 1),
                                                "-m", mod + s], base, svc(s)))
        elif s == "preprocessing" and a.gpus > 1:
            for g in range(a.gpus):
                env = dict(base, HIP_VISIBLE_DEVICES=str(g), SYMB_QUEUE_GROUP="preprocessing",
                           SYMB_REPLICA=str(g))
                kids.append(Child(f"preprocessing[{g}]", [py, "-m", mod + s], env, svc(s, str(g))))
        elif s == "vector_memory" and a.gpus > 1:
            kids.append(Child("vector_memory", [py, "-m", "torch.distributed.run", "--nnodes=1",
                                                f"--nproc-per-node={a.gpus}", "--master-addr",
                                                "127.0.0.1", "--master-port", str(a.dist_port),
                                                "-m", mod + s], base, svc(s)))
        elif s == "api":
            url = f"http://127.0.0.1:{base['API_SERVER_PORT']}/api/health"
            kids.append(Child(s, [py, "-m", mod + s], base, ("http", url) if interval else None))
        else:
            kids.append(Child(s, [py, "-m", mod + s], base, svc(s)))
    return kids


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--only", default="")
    ap.add_argument("--broker-port", type=int, default=4222)
    ap.add_argument("--api-port", type=int, default=None,
                    help="gateway port (default: API_SERVER_PORT from the env / .env, else 8080)")
    ap.add_argument("--env-file", default=None, help="compose-style KEY=VALUE file (default .env)")
    ap.add_argument("--health-interval", type=float, default=10.0,
                    help="seconds between health checks / service metrics reports (0: off)")
    ap.add_argument("--health-retries", type=int, default=3,
                    help="consecutive failed checks before a child is killed and restarted")
    ap.add_argument("--health-grace", type=float, default=120.0,
                    help="seconds after a (re)start before a child is probed (model/index load)")
    ap.add_argument("--dist-port", type=int, default=29600)
    ap.add_argument("--no-broker", action="store_true")
    ap.add_argument("--embed-dp", choices=["queue", "rccl"], default="queue",
                    help="multi-GPU embedding: NATS queue-group replicas or one RCCL group")
    a = ap.parse_args()
    kids = build_children(a)
    stop = {"flag": False}
    monitor = None
    if a.health_interval > 0:
        nats_url = kids[0].env.get("NATS_URL", f"nats://127.0.0.1:{a.broker_port}") if kids else ""
        monitor = HealthMonitor(nats_url)
        monitor.start()
    next_check = time.monotonic() + a.health_interval

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
            if monitor is not None and time.monotonic() >= next_check:
                next_check = time.monotonic() + a.health_interval
                for k in kids:
                    if (k.probe is None or k.proc is None or k.proc.poll() is not None
                            or time.monotonic() - k.started_at < a.health_grace):
                        continue
                    ok, why = probe_ok(k, monitor, a.health_interval * a.health_retries)
                    k.failures = 0 if ok else k.failures + 1
                    # a metrics probe already measures staleness over `retries` intervals
                    if not ok and (k.failures >= a.health_retries or k.probe[0] == "metrics"):
                        k.kill_unhealthy(why)
            time.sleep(0.2)
    finally:
        if monitor is not None:
            monitor.stop()
        for k in reversed(kids):
            k.stop()


if __name__ == "__main__":
    main()
