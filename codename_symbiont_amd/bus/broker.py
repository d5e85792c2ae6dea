"""In-repo NATS core broker (the image ships no nats-server; reference runs nats:2.10.7,
docker-compose.yml:27-34).

Implements the parts of the NATS core protocol the system relies on: INFO/CONNECT handshake,
PUB/HPUB, SUB (with queue groups), UNSUB (with auto-unsubscribe counts), MSG/HMSG delivery,
PING/PONG, ``*``/``>`` wildcards, max_payload enforcement (1 MiB default, -ERR + close like
nats-server), and no-responders status messages (``NATS/1.0 503``) for requests with no
subscriber when the client negotiated headers + no_responders.  At-most-once, no persistence --
exactly NATS core semantics (no JetStream in the reference).

Two implementations with the same interface (``await start()``, ``url``, ``port``, ``stats``,
``await stop()``):

* ``NativeBroker`` (default, ``Broker``): the C++ epoll server in ``csrc/native/natsd.cpp``, run on
  its own thread without the GIL -- what ``launch.py`` deploys.
* ``PyBroker``: this asyncio implementation, kept as the executable specification the native
  server is tested against (``tests/test_bus_cpu.py`` runs every bus test on both).

Run standalone: ``python -m codename_symbiont_amd.bus.broker --port 4222 [--impl native|py]``.
"""
from __future__ import annotations

import argparse
import asyncio
import itertools
import json
import logging
import random

from ..ops._ext import native

log = logging.getLogger("symbiont.broker")

VERSION = "2.10.7"


def subject_valid(subject: str, wildcards: bool) -> bool:
    if not subject or subject.startswith(".") or subject.endswith("."):
        return False
    toks = subject.split(".")
    for i, t in enumerate(toks):
        if not t or any(c in t for c in " \t\r\n"):
            return False
        if ("*" in t or ">" in t):
            if not wildcards or len(t) != 1 or (t == ">" and i != len(toks) - 1):
                return False
    return True


def subject_matches(pattern_toks: list[str], subject_toks: list[str]) -> bool:
    for i, p in enumerate(pattern_toks):
        if p == ">":
            return len(subject_toks) > i
        if i >= len(subject_toks):
            return False
        if p != "*" and p != subject_toks[i]:
            return False
    return len(pattern_toks) == len(subject_toks)


class _Sub:
    __slots__ = ("conn", "sid", "subject", "toks", "queue", "max_msgs", "delivered")

    def __init__(self, conn, sid, subject, queue):
        self.conn = conn
        self.sid = sid
        self.subject = subject
        self.toks = subject.split(".")
        self.queue = queue
        self.max_msgs = None
        self.delivered = 0


class _Conn:
    _ids = itertools.count(1)

    def __init__(self, broker: "PyBroker", reader, writer):
        self.id = next(self._ids)
        self.broker = broker
        self.reader = reader
        self.writer = writer
        self.subs: dict[str, _Sub] = {}
        self.headers = False
        self.no_responders = False
        self.verbose = False
        self.name = ""
        self.closed = False

    def send(self, data: bytes) -> None:
        if not self.closed:
            self.writer.write(data)

    async def err_close(self, msg: str) -> None:
        self.send(f"-ERR '{msg}'\r\n".encode())
        try:
            await self.writer.drain()
        except Exception:
            pass
        self.close()

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        self.broker._remove_conn(self)
        try:
            self.writer.close()
        except Exception:
            pass


class PyBroker:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, max_payload: int = 1 << 20):
        self.host = host
        self.port = port
        self.max_payload = max_payload
        self._server: asyncio.AbstractServer | None = None
        self._conns: set[_Conn] = set()
        self._subs: list[_Sub] = []
        self._qrr: dict[tuple, int] = {}
        self.stats = {"in_msgs": 0, "out_msgs": 0, "in_bytes": 0, "out_bytes": 0}
        self.server_id = "NSYMB" + "".join(random.choice("ABCDEFGHJKLMNPQRSTUVWXYZ234567")
                                           for _ in range(51))

    @property
    def url(self) -> str:
        return f"nats://{self.host}:{self.port}"

    async def start(self) -> "PyBroker":
        self._server = await asyncio.start_server(self._handle, self.host, self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        log.info("[BROKER] listening on %s", self.url)
        return self

    async def stop(self) -> None:
        for c in list(self._conns):
            c.close()
        if self._server:
            self._server.close()
            await self._server.wait_closed()

    async def serve_forever(self) -> None:
        await self.start()
        async with self._server:
            await self._server.serve_forever()

    # ------------------------------------------------------------------ routing
    def _remove_conn(self, c: _Conn) -> None:
        self._conns.discard(c)
        self._subs = [s for s in self._subs if s.conn is not c]

    def _deliver(self, s: _Sub, subject: str, reply, hdr, payload) -> None:
        n = native()
        s.conn.send(n.nats_msg(subject, s.sid, reply, payload, hdr))
        s.delivered += 1
        self.stats["out_msgs"] += 1
        self.stats["out_bytes"] += len(payload)
        if s.max_msgs is not None and s.delivered >= s.max_msgs:
            s.conn.subs.pop(s.sid, None)
            self._subs = [x for x in self._subs if x is not s]

    def route(self, subject: str, reply, hdr, payload, origin: _Conn | None) -> int:
        toks = subject.split(".")
        matched = [s for s in self._subs if subject_matches(s.toks, toks) and not s.conn.closed]
        plain = [s for s in matched if s.queue is None]
        groups: dict[str, list[_Sub]] = {}
        for s in matched:
            if s.queue is not None:
                groups.setdefault(s.queue, []).append(s)
        for s in plain:
            self._deliver(s, subject, reply, hdr, payload)
        for q, members in groups.items():
            k = (q, subject)
            i = self._qrr.get(k, random.randrange(len(members)))
            self._deliver(members[i % len(members)], subject, reply, hdr, payload)
            self._qrr[k] = i + 1
        delivered = len(plain) + len(groups)
        if delivered == 0 and reply and origin is not None and origin.headers and origin.no_responders:
            status = native().nats_headers("503", None, [])
            self.route(reply, None, status, b"", None)
        return delivered

    # ------------------------------------------------------------------ connection handler
    async def _handle(self, reader, writer) -> None:
        c = _Conn(self, reader, writer)
        self._conns.add(c)
        info = {"server_id": self.server_id, "server_name": "symbiont-broker", "version": VERSION,
                "proto": 1, "go": "n/a", "host": self.host, "port": self.port, "headers": True,
                "max_payload": self.max_payload, "client_id": c.id}
        c.send(b"INFO " + json.dumps(info, separators=(",", ":")).encode() + b"\r\n")
        parser = native().NatsParser(4096, self.max_payload)  # size checked on the PUB line
        try:
            while not c.closed:
                chunk = await reader.read(1 << 20)
                if not chunk:
                    break
                try:
                    events = parser.feed(chunk)
                except ValueError as e:
                    await c.err_close(str(e) if "Maximum" in str(e) else "Unknown Protocol Operation")
                    break
                for ev in events:
                    await self._op(c, ev)
                    if c.closed:
                        break
                await writer.drain()
        except (ConnectionError, OSError):
            pass
        finally:
            c.close()

    async def _op(self, c: _Conn, ev) -> None:
        op = ev[0]
        if op == "CONNECT":
            try:
                opts = json.loads(ev[1])
            except ValueError:
                opts = {}
            c.headers = bool(opts.get("headers"))
            c.no_responders = bool(opts.get("no_responders"))
            c.verbose = bool(opts.get("verbose"))
            c.name = opts.get("name", "")
        elif op in ("PUB", "HPUB"):
            subject, reply = ev[1], ev[2]
            hdr = ev[3] if op == "HPUB" else None
            payload = ev[-1]
            size = len(payload) + (len(hdr) if hdr else 0)
            if size > self.max_payload:
                await c.err_close("Maximum Payload Violation")
                return
            if not subject_valid(subject, wildcards=False):
                c.send(b"-ERR 'Invalid Publish Subject'\r\n")
                return
            if c.verbose:
                c.send(b"+OK\r\n")   # nats-server acks a verbose PUB before routing it
            self.stats["in_msgs"] += 1
            self.stats["in_bytes"] += len(payload)
            self.route(subject, reply, hdr, payload, c)
            return
        elif op == "SUB":
            _, subject, queue, sid = ev
            if not subject_valid(subject, wildcards=True):
                c.send(b"-ERR 'Invalid Subject'\r\n")
                return
            if sid not in c.subs:   # nats-server keeps the existing subscription for a live sid
                s = _Sub(c, sid, subject, queue)
                c.subs[sid] = s
                self._subs.append(s)
        elif op == "UNSUB":
            _, sid, max_msgs = ev
            s = c.subs.get(sid)
            if s is not None:
                if max_msgs is not None and s.delivered < max_msgs:
                    s.max_msgs = max_msgs
                else:
                    c.subs.pop(sid, None)
                    self._subs = [x for x in self._subs if x is not s]
        elif op == "PING":
            c.send(b"PONG\r\n")
            return
        elif op in ("PONG",):
            return
        if c.verbose and op != "PING":
            c.send(b"+OK\r\n")


class NativeBroker:
    """The C++ NATS server (``_native.NatsServer``) behind the asyncio broker interface."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, max_payload: int = 1 << 20,
                 max_pending: int = 64 << 20, monitor_port: int = -1):
        """monitor_port >= 0 (0 = ephemeral): nats-server-style HTTP monitoring (GET /varz,
        /connz, /subsz, /healthz) -- the reference compose publishes it on 8222."""
        self.host = host
        self.port = port
        self.max_payload = max_payload
        self._srv = native().NatsServer(host, port, max_payload, max_pending, monitor_port)

    @property
    def monitor_port(self) -> int:
        return self._srv.monitor_port

    @property
    def url(self) -> str:
        return f"nats://{self.host}:{self.port}"

    @property
    def stats(self) -> dict:
        return self._srv.stats()

    async def start(self) -> "NativeBroker":
        self._srv.start()   # binds + listens synchronously (errors raise here), then loops on a thread
        self.port = self._srv.port
        log.info("[BROKER] native server listening on %s", self.url)
        return self

    async def stop(self) -> None:
        self._srv.stop()

    async def serve_forever(self) -> None:
        await self.start()
        try:
            while self._srv.running:
                await asyncio.sleep(3600)
        finally:
            await self.stop()


Broker = NativeBroker
BROKERS = {"native": NativeBroker, "py": PyBroker}


def main() -> None:
    ap = argparse.ArgumentParser(description="symbiont in-repo NATS broker")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=4222)
    ap.add_argument("--max-payload", type=int, default=1 << 20)
    ap.add_argument("--impl", choices=sorted(BROKERS), default="native")
    ap.add_argument("--http-port", type=int, default=-1,
                    help="native server: HTTP monitoring port (nats-server -m; 8222 in the reference)")
    a = ap.parse_args()
    logging.basicConfig(level=logging.INFO)
    if a.impl == "native":
        b = NativeBroker(a.host, a.port, a.max_payload, monitor_port=a.http_port)
    else:
        b = PyBroker(a.host, a.port, a.max_payload)
    asyncio.run(b.serve_forever())


if __name__ == "__main__":
    main()
