"""Async Bolt (v5.0 / v4.4) client over the native PackStream codec (csrc/native/packstream.cpp).

Replaces neo4rs 0.7.3 in services/knowledge_graph_service.  Messages used: HELLO, BEGIN, RUN,
PULL, COMMIT, ROLLBACK, RESET, GOODBYE; responses SUCCESS / RECORD / IGNORED / FAILURE.
Beyond neo4rs: requests inside a transaction can be PIPELINED -- all RUN+PULL pairs are written
before any response is read -- so the reference's N_sentence + N_token sequential round trips per
document (knowledge_graph_service/src/main.rs:70-125) become one network round trip while the
Cypher text and parameters stay identical.
"""
from __future__ import annotations

import asyncio
import struct
from urllib.parse import urlparse

from ..ops._ext import native

HELLO, GOODBYE, RESET, RUN, BEGIN, COMMIT, ROLLBACK, PULL = 0x01, 0x02, 0x0F, 0x10, 0x11, 0x12, 0x13, 0x3F
SUCCESS, RECORD, IGNORED, FAILURE = 0x70, 0x71, 0x7E, 0x7F
MAGIC = b"\x60\x60\xB0\x17"
# proposals: 5.0, 4.4 (4 bytes each: 0, range, minor, major)
PROPOSALS = bytes([0, 0, 0, 5, 0, 0, 4, 4, 0, 0, 0, 0, 0, 0, 0, 0])


class Structure:
    __slots__ = ("tag", "fields")

    def __init__(self, tag: int, fields: list):
        self.tag = tag
        self.fields = list(fields)

    def __repr__(self):
        return f"Structure(0x{self.tag:02X}, {self.fields!r})"

    def __eq__(self, o):
        return isinstance(o, Structure) and o.tag == self.tag and o.fields == self.fields


def pack(v) -> bytes:
    return native().ps_pack(v)


def unpack(b: bytes):
    return native().ps_unpack(b, Structure)


def message(tag: int, *fields) -> bytes:
    return native().bolt_chunk(pack(Structure(tag, list(fields))))


class BoltError(Exception):
    def __init__(self, code: str, message: str):
        super().__init__(f"{code}: {message}")
        self.code = code
        self.message = message


class BoltConnection:
    def __init__(self, reader, writer, version: tuple[int, int]):
        self.reader = reader
        self.writer = writer
        self.version = version
        self._dechunk = native().BoltDechunker()
        self._pending: list = []

    @classmethod
    async def open(cls, uri: str, user: str, password: str, user_agent: str = "symbiont/0.1",
                   timeout: float = 5.0) -> "BoltConnection":
        u = urlparse(uri)
        host, port = u.hostname or "localhost", u.port or 7687
        reader, writer = await asyncio.wait_for(asyncio.open_connection(host, port), timeout)
        writer.write(MAGIC + PROPOSALS)
        await writer.drain()
        v = await asyncio.wait_for(reader.readexactly(4), timeout)
        if v == b"\x00\x00\x00\x00":
            writer.close()
            raise BoltError("Bolt.Handshake", "server supports none of the proposed versions")
        conn = cls(reader, writer, (v[3], v[2]))
        extra = {"user_agent": user_agent, "scheme": "basic", "principal": user,
                 "credentials": password}
        await conn.send(message(HELLO, extra))
        await conn.read_summary()
        return conn

    async def send(self, data: bytes) -> None:
        self.writer.write(data)
        await self.writer.drain()

    async def _next_message(self):
        while True:
            if self._pending:
                return self._pending.pop(0)
            chunk = await self.reader.read(65536)
            if not chunk:
                raise ConnectionError("Bolt connection closed")
            self._pending.extend(unpack(m) for m in self._dechunk.feed(chunk))

    async def read_summary(self) -> tuple[dict, list]:
        """Read RECORDs until the SUCCESS / FAILURE / IGNORED summary."""
        records = []
        while True:
            m = await self._next_message()
            if m.tag == RECORD:
                records.append(m.fields[0])
            elif m.tag == SUCCESS:
                return m.fields[0] if m.fields else {}, records
            elif m.tag == FAILURE:
                meta = m.fields[0] if m.fields else {}
                raise BoltError(meta.get("code", "?"), meta.get("message", ""))
            elif m.tag == IGNORED:
                raise BoltError("Bolt.Ignored", "request ignored after an earlier failure")

    async def reset(self) -> None:
        await self.send(message(RESET))
        # the server answers IGNORED for everything queued after a FAILURE, then RESET's SUCCESS
        while True:
            m = await self._next_message()
            if m.tag == SUCCESS:
                return

    async def close(self) -> None:
        try:
            self.writer.write(message(GOODBYE))
            await self.writer.drain()
        except Exception:
            pass
        self.writer.close()


class Transaction:
    def __init__(self, conn: BoltConnection):
        self.conn = conn
        self._queued: list[tuple[str, dict]] = []

    async def run(self, query: str, params: dict | None = None) -> list[dict]:
        """RUN + PULL(all) -> records as dicts keyed by the RUN's field names."""
        c = self.conn
        await c.send(message(RUN, query, params or {}, {}) + message(PULL, {"n": -1}))
        meta, _ = await c.read_summary()
        fields = meta.get("fields", [])
        _, records = await c.read_summary()
        return [dict(zip(fields, r)) for r in records]

    def queue(self, query: str, params: dict | None = None) -> None:
        """Buffer a statement; all queued statements go out in ONE write by ``flush``."""
        self._queued.append((query, params or {}))

    async def flush(self) -> list[list[dict]]:
        c = self.conn
        if not self._queued:
            return []
        buf = b"".join(message(RUN, q, p, {}) + message(PULL, {"n": -1}) for q, p in self._queued)
        n = len(self._queued)
        self._queued.clear()
        await c.send(buf)
        out, first_err = [], None
        for _ in range(n):
            try:
                meta, _ = await c.read_summary()
                _, recs = await c.read_summary()
                out.append([dict(zip(meta.get("fields", []), r)) for r in recs])
            except BoltError as e:  # keep draining the pipelined responses (IGNORED after a FAILURE)
                first_err = first_err or e
                out.append([])
        if first_err is not None:
            raise first_err
        return out

    async def commit(self) -> dict:
        await self.conn.send(message(COMMIT))
        meta, _ = await self.conn.read_summary()
        return meta

    async def rollback(self) -> None:
        await self.conn.send(message(ROLLBACK))
        await self.conn.read_summary()


class Graph:
    """Minimal driver: one connection per concurrent user, pooled (max_connections)."""

    def __init__(self, uri: str, user: str, password: str, db: str = "neo4j",
                 max_connections: int = 10):
        self.uri, self.user, self.password, self.db = uri, user, password, db
        self._pool: asyncio.Queue = asyncio.Queue()
        self._sem = asyncio.Semaphore(max_connections)
        self._all: list[BoltConnection] = []

    async def _acquire(self) -> BoltConnection:
        await self._sem.acquire()
        try:
            return self._pool.get_nowait()
        except asyncio.QueueEmpty:
            try:
                c = await BoltConnection.open(self.uri, self.user, self.password)
            except Exception:
                self._sem.release()
                raise
            self._all.append(c)
            return c

    def _release(self, c: BoltConnection, broken: bool = False) -> None:
        if broken:
            if c in self._all:
                self._all.remove(c)
        else:
            self._pool.put_nowait(c)
        self._sem.release()

    async def run(self, query: str, params: dict | None = None) -> list[dict]:
        c = await self._acquire()
        try:
            await c.send(message(RUN, query, params or {}, {"db": self.db}) + message(PULL, {"n": -1}))
            meta, _ = await c.read_summary()
            _, recs = await c.read_summary()
            self._release(c)
            return [dict(zip(meta.get("fields", []), r)) for r in recs]
        except BoltError:
            try:
                await c.reset()
                self._release(c)
            except Exception:
                self._release(c, broken=True)
            raise
        except Exception:
            self._release(c, broken=True)
            raise

    async def transaction(self, fn):
        """BEGIN -> await fn(tx) -> COMMIT (ROLLBACK + re-raise on error)."""
        c = await self._acquire()
        try:
            await c.send(message(BEGIN, {"db": self.db}))
            await c.read_summary()
            tx = Transaction(c)
            try:
                res = await fn(tx)
                await tx.commit()
            except BoltError:
                await c.reset()
                raise
            self._release(c)
            return res
        except BoltError:
            self._release(c)
            raise
        except Exception:
            self._release(c, broken=True)
            raise

    async def close(self) -> None:
        for c in self._all:
            await c.close()
        self._all.clear()


def u16(n: int) -> bytes:
    return struct.pack(">H", n)
