"""Supervisor (C10, ``codename_symbiont_amd/launch.py``): the docker-compose replacement must bring
the broker + services up as child processes, serve the Markov flow end to end, restart a child
that dies (the reference's compose file has no restart policy) and take every
child down with it on SIGTERM."""
import json
import os
import re
import signal
import socket
import subprocess
import sys
import threading
import time

import httpx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    return True


def _generate(url: str, task_id: str, wait_s: float = 5.0):
    """POST /api/generate-text (from a timer thread: the SSE response head may only arrive with
    the first event) and return the matching SSE event, or None if none came within ``wait_s``."""
    def post():
        try:
            httpx.post(url + "/api/generate-text",
                       json={"task_id": task_id, "prompt": "hi", "max_length": 8}, timeout=10)
        except httpx.HTTPError:
            pass
    threading.Timer(0.5, post).start()
    deadline = time.time() + wait_s
    try:
        with httpx.Client(timeout=wait_s) as c:
            with c.stream("GET", url + "/api/events") as r:
                for line in r.iter_lines():
                    if line.startswith("data: "):
                        ev = json.loads(line[6:])
                        if ev.get("original_task_id") == task_id:
                            return ev
                    if time.time() > deadline:
                        return None
    except httpx.HTTPError:
        return None


def _generate_retry(url: str, tag: str, budget_s: float = 60.0) -> dict:
    """A (re)started generator may not have subscribed yet: core NATS drops the task then."""
    t0 = time.time()
    while time.time() - t0 < budget_s:
        ev = _generate(url, f"{tag}-{int(time.time() * 1e3)}")
        if ev:
            return ev
    raise AssertionError(f"no generated text for {tag} within {budget_s}s")


def test_supervisor_serves_restarts_and_stops():
    bport, aport = _port(), _port()
    env = dict(os.environ, SYMB_LOG="warning", SYMB_FORCE_CPU="1", API_SERVER_HOST="127.0.0.1",
               NATS_URL=f"nats://127.0.0.1:{bport}", SYMB_API_WORKERS="1")
    sup = subprocess.Popen([sys.executable, "-m", "codename_symbiont_amd.launch", "--only",
                            "text_generator,api", "--broker-port", str(bport), "--api-port",
                            str(aport)], cwd=ROOT, env=env, stderr=subprocess.PIPE, text=True,
                           start_new_session=True)
    log: list[str] = []
    threading.Thread(target=lambda: [log.append(ln) for ln in sup.stderr], daemon=True).start()

    def pids() -> dict:
        out = {}
        for ln in list(log):
            m = re.search(r"\[launch\] started (\S+) pid=(\d+)", ln)
            if m:
                out[m.group(1)] = int(m.group(2))   # latest start wins
        return out

    url = f"http://127.0.0.1:{aport}"
    try:
        t0 = time.time()
        while True:   # gateway up and the Markov service answering over the broker
            try:
                if httpx.get(url + "/api/health", timeout=2).status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            assert time.time() - t0 < 90, "services did not come up:\n" + "".join(log[-20:])
            time.sleep(0.3)
        assert set(pids()) == {"broker", "text_generator", "api"}
        ev = _generate_retry(url, "sup-1")
        assert ev["generated_text"].split()[0] == "я"

        old = pids()["text_generator"]
        os.killpg(old, signal.SIGKILL)   # crash the child: the supervisor must bring it back
        t0 = time.time()
        while pids()["text_generator"] == old:
            assert time.time() - t0 < 30, "child was not restarted:\n" + "".join(log[-20:])
            time.sleep(0.2)
        assert any("text_generator exited" in ln for ln in log)
        assert _generate_retry(url, "sup-2")["generated_text"]
        live = pids()
    finally:
        os.killpg(sup.pid, signal.SIGTERM)
        try:
            sup.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(sup.pid, signal.SIGKILL)
            sup.wait(5)
    t0 = time.time()
    while any(_alive(p) for p in live.values()) and time.time() - t0 < 15:
        time.sleep(0.2)
    assert not any(_alive(p) for p in live.values()), "supervisor left children behind"


def test_env_file_compose_semantics(tmp_path, monkeypatch):
    """.env like docker compose: comments, export, quotes; the shell's variables win."""
    import argparse

    from codename_symbiont_amd.launch import build_children
    from codename_symbiont_amd.utils.config import read_env_file

    p = tmp_path / ".env"
    p.write_text("# reference .env.example keys\n"
                 "NATS_URL=nats://cs-nats:4222\n"
                 "export NEO4J_USER=neo4j\n"
                 "NEO4J_PASSWORD=\"pa ss\\\"word\"\n"
                 "API_SERVER_PORT=7070   # gateway\n"
                 "FRONTEND_PORT='3000'\n"
                 "\n"
                 "NOT_A_PAIR\n")
    env = read_env_file(str(p))
    assert env == {"NATS_URL": "nats://cs-nats:4222", "NEO4J_USER": "neo4j",
                   "NEO4J_PASSWORD": 'pa ss"word', "API_SERVER_PORT": "7070",
                   "FRONTEND_PORT": "3000"}
    monkeypatch.setenv("NEO4J_USER", "from-shell")
    monkeypatch.delenv("NATS_URL", raising=False)
    monkeypatch.delenv("API_SERVER_PORT", raising=False)
    a = argparse.Namespace(broker_port=4333, api_port=None, env_file=str(p), only="api",
                           no_broker=True, gpus=1, embed_dp="queue", dist_port=29600)
    (kid,) = build_children(a)
    assert kid.env["NATS_URL"] == "nats://cs-nats:4222"       # from the file
    assert kid.env["NEO4J_USER"] == "from-shell"               # shell wins
    assert kid.env["API_SERVER_PORT"] == "7070"
    a.api_port = 9999                                          # the flag wins over both
    assert build_children(a)[0].env["API_SERVER_PORT"] == "9999"


def test_supervisor_health_checks_restart_stuck_children():
    """Compose-style healthchecks: a child that is alive but stuck (SIGSTOP) stops reporting
    metrics.<service> / answering /api/health; the supervisor kills and restarts it."""
    bport, aport = _port(), _port()
    env = dict(os.environ, SYMB_LOG="warning", SYMB_FORCE_CPU="1", API_SERVER_HOST="127.0.0.1",
               NATS_URL=f"nats://127.0.0.1:{bport}", SYMB_API_WORKERS="1")
    sup = subprocess.Popen([sys.executable, "-m", "codename_symbiont_amd.launch", "--only",
                            "text_generator,api", "--broker-port", str(bport), "--api-port",
                            str(aport), "--health-interval", "1", "--health-retries", "2",
                            "--health-grace", "4"], cwd=ROOT, env=env, stderr=subprocess.PIPE,
                           text=True, start_new_session=True)
    log: list[str] = []
    threading.Thread(target=lambda: [log.append(ln) for ln in sup.stderr], daemon=True).start()

    def pids() -> dict:
        out = {}
        for ln in list(log):
            m = re.search(r"\[launch\] started (\S+) pid=(\d+)", ln)
            if m:
                out[m.group(1)] = int(m.group(2))
        return out

    url = f"http://127.0.0.1:{aport}"
    try:
        t0 = time.time()
        while True:
            try:
                if httpx.get(url + "/api/health", timeout=2).status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            assert time.time() - t0 < 90, "services did not come up:\n" + "".join(log[-20:])
            time.sleep(0.3)
        time.sleep(6)                       # past the grace: healthy children are left alone
        assert not any("unhealthy" in ln for ln in log), "".join(log[-20:])
        for name in ("text_generator", "api"):
            old = pids()[name]
            os.killpg(old, signal.SIGSTOP)  # alive but stuck
            t0 = time.time()
            while pids()[name] == old:
                assert time.time() - t0 < 45, f"{name} not restarted:\n" + "".join(log[-20:])
                time.sleep(0.2)
            assert any(f"{name} unhealthy" in ln for ln in log)
            assert not _alive(old) or open(f"/proc/{old}/stat").read().split()[2] == "Z"
        ev = _generate_retry(url, "health")      # the restarted pair serves again
        assert ev["generated_text"].split()[0] == "я"
    finally:
        os.killpg(sup.pid, signal.SIGTERM)
        sup.wait(30)
