"""asyncio NATS client over the native protocol codec (csrc/native/nats_proto.cpp).

Replaces async-nats 0.33 in every reference service (e.g. services/api_service/Cargo.toml:11).
Semantics kept from that client because they are observable:
* request/reply through ONE wildcard inbox subscription (``_INBOX.<nuid>.*``), per-request tokens;
* headers + no_responders negotiated in CONNECT, so a request to a subject nobody serves fails
  fast with ``NoRespondersError`` ("no responders") instead of waiting for the timeout;
* default request timeout 10 s, surfaced as ``RequestTimeoutError`` ("request timed out");
* auto-reconnect with re-subscription of every live subscription (async-nats default behaviour).
Additions: queue-group subscriptions (used for data-parallel ingest over several GPU ranks).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import secrets
import string
from dataclasses import dataclass, field
from urllib.parse import urlparse

from ..ops._ext import native

log = logging.getLogger("symbiont.nats")

_ALPH = string.ascii_letters + string.digits


def nuid(n: int = 22) -> str:
    return "".join(secrets.choice(_ALPH) for _ in range(n))


class NatsError(Exception):
    pass


class NoRespondersError(NatsError):
    def __str__(self):
        return "no responders"


class RequestTimeoutError(NatsError, asyncio.TimeoutError):
    def __str__(self):
        return "request timed out"


class ConnectionClosedError(NatsError):
    def __str__(self):
        return "connection closed"


@dataclass
class Msg:
    subject: str
    reply: str | None
    data: bytes
    headers: list | None = None
    status: str | None = None
    _client: "NatsClient | None" = field(default=None, repr=False)

    @property
    def payload(self) -> bytes:
        return self.data

    async def respond(self, data: bytes, headers: list | None = None) -> None:
        if not self.reply or self._client is None:
            raise NatsError("message has no reply subject")
        await self._client.publish(self.reply, data, headers=headers)


class Subscription:
    def __init__(self, client: "NatsClient", sid: str, subject: str, queue: str | None,
                 pending_limit: int = 65536):
        self._client = client
        self.sid = sid
        self.subject = subject
        self.queue = queue
        self._q: asyncio.Queue = asyncio.Queue(maxsize=pending_limit)
        self._closed = False
        self.dropped = 0

    def _deliver(self, m: Msg) -> None:
        try:
            self._q.put_nowait(m)
        except asyncio.QueueFull:  # slow consumer: drop, as NATS does
            self.dropped += 1

    async def next_msg(self, timeout: float | None = None) -> Msg:
        m = await asyncio.wait_for(self._q.get(), timeout)
        if m is None:
            raise ConnectionClosedError()
        return m

    def __aiter__(self):
        return self

    async def __anext__(self) -> Msg:
        if self._closed and self._q.empty():
            raise StopAsyncIteration
        m = await self._q.get()
        if m is None:
            raise StopAsyncIteration
        return m

    async def next_batch(self, max_n: int = 256, align: int = 0, fill: int = 0,
                         fill_until=None) -> list[Msg] | None:
        """Wait for one message, then take whatever else is already queued (up to ``max_n``);
        None once the subscription has ended.

        ``align`` > 0: when more than ``align`` messages are ready, take a whole multiple of it
        and leave the rest queued for the next call -- a consumer whose unit of work is a block
        of ``align`` items (the index scan's 256-query block) then never pays a whole extra
        block for a few stragglers; a burst of ``align`` or fewer is taken whole (latency).

        ``fill`` > 0 with ``fill_until`` (a callable returning a loop-clock deadline or None):
        after the first message, keep waiting until ``fill`` messages are ready or the deadline
        passes -- a consumer whose device is busy anyway (a scan in flight) collects a full
        block instead of launching a partial one that costs as much."""
        if self._closed and self._q.empty():
            return None
        m = await self._q.get()
        if m is None:
            return None
        batch = [m]
        if fill > 1 and fill_until is not None and 1 + self._q.qsize() < fill:
            deadline = fill_until()
            loop = asyncio.get_running_loop()
            while deadline is not None and 1 + self._q.qsize() < fill:
                left = deadline - loop.time()
                if left <= 0:
                    break
                # (poll: a waiter on the queue would take a message out of order)
                await asyncio.sleep(min(left, 0.0005))
        if align > 0:
            ready = 1 + self._q.qsize()   # (may count an end marker: at worst one short batch)
            if ready > align:
                max_n = min(max_n, ready) // align * align or max_n
        while len(batch) < max_n:
            try:
                x = self._q.get_nowait()
            except asyncio.QueueEmpty:
                break
            if x is None:              # end marker: deliver this batch, end on the next call
                self._q.put_nowait(None)
                break
            batch.append(x)
        return batch

    async def unsubscribe(self) -> None:
        await self._client._unsubscribe(self)

    def _close(self) -> None:
        self._closed = True
        try:
            self._q.put_nowait(None)
        except asyncio.QueueFull:
            pass


class NatsClient:
    def __init__(self):
        self._reader: asyncio.StreamReader | None = None
        self._writer: asyncio.StreamWriter | None = None
        self._subs: dict[str, Subscription] = {}
        self._sid = 0
        self._pongs: list[asyncio.Future] = []
        self._resp_prefix = f"_INBOX.{nuid()}."
        self._resp_sub: Subscription | None = None
        self._resp_map: dict[str, asyncio.Future] = {}
        self._read_task: asyncio.Task | None = None
        self._closed = False
        self._url = None
        self._name = "symbiont"
        self.server_info: dict = {}
        self.max_payload = 1 << 20
        self.reconnect = True
        self.reconnect_wait = 0.5
        self.max_reconnect_attempts = -1
        self.request_timeout = 10.0
        self._connected = asyncio.Event()
        self._wlock = asyncio.Lock()

    # ------------------------------------------------------------------ connection
    @classmethod
    async def connect(cls, url: str | None = None, name: str = "symbiont", reconnect: bool = True,
                      connect_timeout: float = 5.0, request_timeout: float = 10.0,
                      retries: int = 0) -> "NatsClient":
        c = cls()
        c._url = url or os.environ.get("NATS_URL", "nats://localhost:4222")
        c._name = name
        c.reconnect = reconnect
        c.request_timeout = request_timeout
        last = None
        for attempt in range(retries + 1):
            try:
                await asyncio.wait_for(c._open(), connect_timeout)
                break
            except (OSError, asyncio.TimeoutError, NatsError) as e:
                last = e
                if attempt == retries:
                    raise ConnectionError(f"NATS connect error: {e}") from e
                await asyncio.sleep(c.reconnect_wait)
        del last
        c._read_task = asyncio.create_task(c._read_loop())
        return c

    async def _open(self) -> None:
        u = urlparse(self._url if "://" in self._url else "nats://" + self._url)
        host, port = u.hostname or "localhost", u.port or 4222
        self._reader, self._writer = await asyncio.open_connection(host, port)
        self._parser = native().NatsParser(4096, 64 << 20)
        # INFO first
        info = None
        while info is None:
            chunk = await self._reader.read(65536)
            if not chunk:
                raise ConnectionClosedError()
            for ev in self._parser.feed(chunk):
                if ev[0] == "INFO":
                    info = json.loads(ev[1])
        self.server_info = info
        self.max_payload = int(info.get("max_payload", 1 << 20))
        connect = {"verbose": False, "pedantic": False, "lang": "python-symbiont",
                   "version": "0.1.0", "protocol": 1, "headers": True, "no_responders": True,
                   "name": self._name}
        self._writer.write(b"CONNECT " + json.dumps(connect, separators=(",", ":")).encode()
                           + b"\r\nPING\r\n")
        await self._writer.drain()
        # wait for the PONG of the handshake
        while True:
            chunk = await self._reader.read(65536)
            if not chunk:
                raise ConnectionClosedError()
            evs = self._parser.feed(chunk)
            if any(e[0] == "-ERR" for e in evs):
                raise NatsError(next(e[1] for e in evs if e[0] == "-ERR"))
            if any(e[0] == "PONG" for e in evs):
                break
        # (re)subscribe everything that is live
        buf = b""
        for s in self._subs.values():
            buf += self._sub_cmd(s)
        if buf:
            self._writer.write(buf)
            await self._writer.drain()
        self._connected.set()

    @staticmethod
    def _sub_cmd(s: Subscription) -> bytes:
        q = f" {s.queue}" if s.queue else ""
        return f"SUB {s.subject}{q} {s.sid}\r\n".encode()

    async def _read_loop(self) -> None:
        while not self._closed:
            try:
                chunk = await self._reader.read(1 << 20)
                if not chunk:
                    raise ConnectionClosedError()
                for ev in self._parser.feed(chunk):
                    self._dispatch(ev)
            except (ConnectionClosedError, OSError, ValueError) as e:
                if self._closed:
                    return
                self._connected.clear()
                log.warning("[NATS] connection lost: %s", e)
                for f in self._pongs:
                    if not f.done():
                        f.set_exception(ConnectionClosedError())
                self._pongs.clear()
                if not self.reconnect or not await self._reconnect():
                    self._shutdown_subs()
                    return

    async def _reconnect(self) -> bool:
        attempt = 0
        while not self._closed and (self.max_reconnect_attempts < 0
                                    or attempt < self.max_reconnect_attempts):
            attempt += 1
            await asyncio.sleep(self.reconnect_wait)
            try:
                await asyncio.wait_for(self._open(), 5.0)
                log.info("[NATS] reconnected after %d attempt(s)", attempt)
                return True
            except (OSError, asyncio.TimeoutError, NatsError):
                continue
        return False

    def _dispatch(self, ev) -> None:
        op = ev[0]
        if op == "MSG":
            _, subject, sid, reply, data = ev
            self._route(sid, Msg(subject, reply, data, None, None, self))
        elif op == "HMSG":
            _, subject, sid, reply, hdr, data = ev
            status, _desc, kvs = native().nats_parse_headers(hdr)
            self._route(sid, Msg(subject, reply, data, kvs, status, self))
        elif op == "PING":
            asyncio.create_task(self._send(b"PONG\r\n"))
        elif op == "PONG":
            if self._pongs:
                f = self._pongs.pop(0)
                if not f.done():
                    f.set_result(True)
        elif op == "-ERR":
            log.error("[NATS] server error: %s", ev[1])
        elif op == "INFO":
            try:
                self.server_info.update(json.loads(ev[1]))
            except ValueError:
                pass

    def _route(self, sid: str, m: Msg) -> None:
        s = self._subs.get(sid)
        if s is None:
            return
        if s is self._resp_sub:
            token = m.subject[len(self._resp_prefix):]
            fut = self._resp_map.pop(token, None)
            if fut is not None and not fut.done():
                if m.status == "503" and not m.data:
                    fut.set_exception(NoRespondersError())
                else:
                    fut.set_result(m)
            return
        s._deliver(m)

    async def _send(self, data: bytes) -> None:
        if self._closed:
            raise ConnectionClosedError()
        if not self._connected.is_set():
            await asyncio.wait_for(self._connected.wait(), 10.0)
        async with self._wlock:
            self._writer.write(data)
            if self._writer.transport.get_write_buffer_size() > (1 << 20):
                await self._writer.drain()

    # ------------------------------------------------------------------ API
    async def publish(self, subject: str, payload: bytes = b"", reply: str | None = None,
                      headers: list | None = None) -> None:
        payload = bytes(payload)
        if len(payload) > self.max_payload:
            raise NatsError(f"maximum payload exceeded ({len(payload)} > {self.max_payload})")
        hdr = native().nats_headers(None, None, headers) if headers else None
        await self._send(native().nats_pub(subject, reply, payload, hdr))

    async def publish_many(self, msgs: list[tuple[str, bytes]]) -> None:
        """Several PUBs in one socket write (replies to a batch of requests)."""
        out = []
        for subject, payload in msgs:
            payload = bytes(payload)
            if len(payload) > self.max_payload:
                raise NatsError(f"maximum payload exceeded ({len(payload)} > {self.max_payload})")
            out.append(native().nats_pub(subject, None, payload, None))
        if out:
            await self._send(b"".join(out))

    async def subscribe(self, subject: str, queue: str | None = None) -> Subscription:
        self._sid += 1
        s = Subscription(self, str(self._sid), subject, queue)
        self._subs[s.sid] = s
        await self._send(self._sub_cmd(s))
        return s

    async def _unsubscribe(self, s: Subscription) -> None:
        if self._subs.pop(s.sid, None) is not None:
            s._close()
            if not self._closed:
                await self._send(f"UNSUB {s.sid}\r\n".encode())

    async def request(self, subject: str, payload: bytes = b"", timeout: float | None = None,
                      headers: list | None = None) -> Msg:
        if self._resp_sub is None:
            self._resp_sub = await self.subscribe(self._resp_prefix + "*")
        token = nuid(8)
        fut = asyncio.get_running_loop().create_future()
        self._resp_map[token] = fut
        try:
            await self.publish(subject, payload, reply=self._resp_prefix + token, headers=headers)
            return await asyncio.wait_for(fut, timeout if timeout is not None else self.request_timeout)
        except asyncio.TimeoutError:
            raise RequestTimeoutError() from None
        finally:
            self._resp_map.pop(token, None)

    async def flush(self, timeout: float = 5.0) -> None:
        fut = asyncio.get_running_loop().create_future()
        self._pongs.append(fut)
        await self._send(b"PING\r\n")
        async with self._wlock:
            await self._writer.drain()
        await asyncio.wait_for(fut, timeout)

    def _shutdown_subs(self) -> None:
        for s in list(self._subs.values()):
            s._close()
        for f in self._resp_map.values():
            if not f.done():
                f.set_exception(ConnectionClosedError())

    async def close(self) -> None:
        if self._closed:
            return
        try:
            await self.flush(1.0)
        except Exception:
            pass
        self._closed = True
        self._shutdown_subs()
        if self._read_task:
            self._read_task.cancel()
        if self._writer:
            self._writer.close()
            try:
                await self._writer.wait_closed()
            except Exception:
                pass

    @property
    def is_connected(self) -> bool:
        return self._connected.is_set() and not self._closed
