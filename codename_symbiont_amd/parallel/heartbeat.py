"""Index-rank liveness over NATS (SURVEY.md §5 "failure detection").

Every rank of an IndexGroup publishes ``health.index.<rank>`` once a second from a daemon thread
with its own plain-socket NATS connection -- the rank's main thread may sit inside a collective,
so the heartbeat must not depend on it.  Rank 0 runs a ``HeartbeatMonitor`` (same kind of thread,
subscribed to ``health.index.*``) and the group refuses to START a collective op while a peer's
heartbeat is stale: the search handler then replies with an error_message at once, instead of
entering a collective that would block until the RCCL/gloo timeout (minutes) because a peer died.
The supervisor restarts the whole rank group (one torch.distributed.run child), which reloads its
shards from the snapshot + WAL.
"""
from __future__ import annotations

import json
import socket
import threading
import time
from urllib.parse import urlparse

from ..ops._ext import native

SUBJECT = "health.index"


def _hostport(url: str) -> tuple[str, int]:
    u = urlparse(url if "://" in url else f"nats://{url}")
    return u.hostname or "127.0.0.1", u.port or 4222


class _Conn:
    """Minimal blocking NATS connection (CONNECT/PUB/SUB/PING) for a background thread."""

    def __init__(self, url: str, timeout: float = 2.0):
        self.sock = socket.create_connection(_hostport(url), timeout=timeout)
        self.parser = native().NatsParser()
        self.sock.sendall(b'CONNECT {"verbose":false,"pedantic":false,"name":"index-heartbeat",'
                          b'"lang":"python","protocol":1}\r\n')

    def send(self, data: bytes) -> None:
        self.sock.sendall(data)

    def events(self, timeout: float):
        self.sock.settimeout(timeout)
        try:
            chunk = self.sock.recv(65536)
        except socket.timeout:
            return []
        if not chunk:
            raise ConnectionError("closed")
        return self.parser.feed(chunk)

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


class Heartbeat(threading.Thread):
    """Publishes {"rank", "count", "ts_ms"} on health.index.<rank> every ``interval`` seconds."""

    def __init__(self, nats_url: str, rank: int, interval: float = 1.0, count_fn=None):
        super().__init__(daemon=True, name=f"heartbeat-{rank}")
        self.url, self.rank, self.interval = nats_url, rank, interval
        self.count_fn = count_fn or (lambda: 0)
        self._stop = threading.Event()

    def run(self) -> None:
        conn = None
        while not self._stop.is_set():
            try:
                if conn is None:
                    conn = _Conn(self.url)
                body = json.dumps({"rank": self.rank, "count": int(self.count_fn()),
                                   "ts_ms": int(time.time() * 1000)}).encode()
                conn.send(native().nats_pub(f"{SUBJECT}.{self.rank}", None, body))
            except (OSError, ConnectionError):
                if conn is not None:
                    conn.close()
                conn = None
            self._stop.wait(self.interval)
        if conn is not None:
            conn.close()

    def stop(self) -> None:
        self._stop.set()


class HeartbeatMonitor(threading.Thread):
    """Rank 0: last-seen time of every rank's heartbeat."""

    def __init__(self, nats_url: str, world: int, stale_after: float = 3.0, grace: float = 15.0):
        super().__init__(daemon=True, name="heartbeat-monitor")
        self.url, self.world = nats_url, world
        self.stale_after, self.grace = stale_after, grace
        self.started = time.monotonic()
        self.last_seen: dict[int, float] = {}
        self._stop = threading.Event()

    def run(self) -> None:
        conn = None
        while not self._stop.is_set():
            try:
                if conn is None:
                    conn = _Conn(self.url)
                    conn.send(f"SUB {SUBJECT}.* 1\r\nPING\r\n".encode())
                for ev in conn.events(0.5):
                    if ev[0] == "MSG":
                        try:
                            r = int(ev[1].rsplit(".", 1)[1])
                        except ValueError:
                            continue
                        self.last_seen[r] = time.monotonic()
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

    def dead_ranks(self) -> list[tuple[int, float]]:
        """[(rank, seconds since its last heartbeat)] for ranks considered down.  A rank never
        heard from only counts after the start-up grace period."""
        now = time.monotonic()
        out = []
        for r in range(self.world):
            t = self.last_seen.get(r)
            if t is None:
                if now - self.started > self.grace:
                    out.append((r, now - self.started))
            elif now - t > self.stale_after:
                out.append((r, now - t))
        return out
