"""A small Bolt server with an in-memory property graph, for tests (no Neo4j in the image).

It speaks real Bolt 4.4/5.0 framing + PackStream (the same native codec as the client) and
executes the exact Cypher statements the knowledge-graph service issues (the reference's text,
knowledge_graph_service/src/main.rs:37-40, :79-83, :111-115, :159-170) with Neo4j's MERGE /
ON CREATE / ON MATCH semantics, transactions (BEGIN/COMMIT/ROLLBACK) and failure handling
(FAILURE then IGNORED until RESET).  Unknown statements fail with a SyntaxError like Neo4j.
Every executed (query, params) is appended to ``log`` for assertions.
"""
from __future__ import annotations

import asyncio
import copy
import itertools
import re
import time

from ..ops._ext import native
from .bolt import (BEGIN, COMMIT, FAILURE, GOODBYE, HELLO, IGNORED, PULL, RECORD, RESET, ROLLBACK, RUN,
                   SUCCESS, Structure, pack, unpack)


def _norm(q: str) -> str:
    return re.sub(r"\s+", " ", q).strip()


class MemGraph:
    def __init__(self):
        self.nodes: dict[int, dict] = {}      # id -> {"labels": set, "props": dict}
        self.rels: list[dict] = []            # {"type", "start", "end", "props"}
        self.constraints: set[str] = set()
        self.indexes: set[str] = set()
        self._ids = itertools.count(0)

    def clone(self) -> "MemGraph":
        g = MemGraph()
        g.nodes = copy.deepcopy(self.nodes)
        g.rels = copy.deepcopy(self.rels)
        g.constraints = set(self.constraints)
        g.indexes = set(self.indexes)
        g._ids = itertools.count(max(self.nodes, default=-1) + 1)
        return g

    def find(self, label: str, key: str, value):
        for nid, n in self.nodes.items():
            if label in n["labels"] and n["props"].get(key) == value:
                return nid
        return None

    def merge_node(self, label: str, key: str, value) -> tuple[int, bool]:
        nid = self.find(label, key, value)
        if nid is not None:
            return nid, False
        nid = next(self._ids)
        self.nodes[nid] = {"labels": {label}, "props": {key: value}}
        return nid, True

    def merge_rel(self, typ: str, start: int, end: int, props: dict) -> None:
        for r in self.rels:
            if r["type"] == typ and r["start"] == start and r["end"] == end and r["props"] == props:
                return
        self.rels.append({"type": typ, "start": start, "end": end, "props": dict(props)})

    # convenience for assertions
    def by_label(self, label: str) -> list[dict]:
        return [n["props"] for n in self.nodes.values() if label in n["labels"]]

    def rels_of(self, typ: str) -> list[dict]:
        return [r for r in self.rels if r["type"] == typ]


class CypherError(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


Q_DOC = _norm("MERGE (d:Document {original_id: $original_id}) ON CREATE SET d.source_url = $source_url, "
              "d.processed_at_ms = $processed_at, d.created_at_ms = timestamp() ON MATCH SET "
              "d.source_url = $source_url, d.processed_at_ms = $processed_at RETURN id(d) AS doc_node_id")
Q_SENT = _norm("MATCH (d:Document) WHERE id(d) = $doc_node_id MERGE (s:Sentence {text: $text}) ON CREATE "
               "SET s.created_at_ms = timestamp() MERGE (d)-[r:HAS_SENTENCE {order: $order}]->(s) "
               "RETURN id(s) AS sentence_node_id")
Q_TOK = _norm("MATCH (d:Document) WHERE id(d) = $doc_node_id MERGE (t:Token {text_lc: $token_text_lc}) "
              "ON CREATE SET t.text_original_case = $token_text_original, t.created_at_ms = timestamp() "
              "ON MATCH SET t.text_original_case = $token_text_original MERGE (d)-[r_ct:CONTAINS_TOKEN]->(t)")
Q_CONSTRAINT = _norm("CREATE CONSTRAINT IF NOT EXISTS FOR (d:Document) REQUIRE d.original_id IS UNIQUE")
Q_INDEX = _norm("CREATE INDEX token_text_lc_index IF NOT EXISTS FOR (t:Token) ON (t.text_lc)")
Q_UNWIND_SENT = _norm("MATCH (d:Document) WHERE id(d) = $doc_node_id UNWIND $rows AS row MERGE (s:Sentence "
                      "{text: row.text}) ON CREATE SET s.created_at_ms = timestamp() MERGE "
                      "(d)-[r:HAS_SENTENCE {order: row.order}]->(s)")
Q_UNWIND_TOK = _norm("MATCH (d:Document) WHERE id(d) = $doc_node_id UNWIND $rows AS row MERGE (t:Token "
                     "{text_lc: row.lc}) ON CREATE SET t.text_original_case = row.orig, t.created_at_ms = "
                     "timestamp() ON MATCH SET t.text_original_case = row.orig MERGE "
                     "(d)-[r_ct:CONTAINS_TOKEN]->(t)")


def execute(g: MemGraph, query: str, p: dict) -> tuple[list[str], list[list]]:
    q = _norm(query)
    now = int(time.time() * 1000)
    if q == Q_DOC:
        nid, created = g.merge_node("Document", "original_id", p["original_id"])
        props = g.nodes[nid]["props"]
        props["source_url"] = p["source_url"]
        props["processed_at_ms"] = p["processed_at"]
        if created:
            props["created_at_ms"] = now
        return ["doc_node_id"], [[nid]]
    if q in (Q_SENT, Q_UNWIND_SENT):
        d = p["doc_node_id"]
        if d not in g.nodes:
            return (["sentence_node_id"] if q == Q_SENT else []), []
        rows = p["rows"] if q == Q_UNWIND_SENT else [{"text": p["text"], "order": p["order"]}]
        out = []
        for row in rows:
            sid, created = g.merge_node("Sentence", "text", row["text"])
            if created:
                g.nodes[sid]["props"]["created_at_ms"] = now
            g.merge_rel("HAS_SENTENCE", d, sid, {"order": row["order"]})
            out.append([sid])
        return (["sentence_node_id"], out) if q == Q_SENT else ([], [])
    if q in (Q_TOK, Q_UNWIND_TOK):
        d = p["doc_node_id"]
        if d not in g.nodes:
            return [], []
        rows = (p["rows"] if q == Q_UNWIND_TOK else
                [{"lc": p["token_text_lc"], "orig": p["token_text_original"]}])
        for row in rows:
            tid, created = g.merge_node("Token", "text_lc", row["lc"])
            g.nodes[tid]["props"]["text_original_case"] = row["orig"]
            if created:
                g.nodes[tid]["props"]["created_at_ms"] = now
            g.merge_rel("CONTAINS_TOKEN", d, tid, {})
        return [], []
    if q == Q_CONSTRAINT:
        g.constraints.add("Document.original_id")
        return [], []
    if q == Q_INDEX:
        g.indexes.add("token_text_lc_index")
        return [], []
    if q.upper().startswith("RETURN 1"):
        return ["1"], [[1]]
    raise CypherError("Neo.ClientError.Statement.SyntaxError", f"unsupported statement: {q[:80]}")


class FakeBoltServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, version=(4, 4)):
        self.host, self.port = host, port
        self.version = version
        self.graph = MemGraph()
        self.log: list[tuple[str, dict]] = []
        self.connections = 0
        self.fail_next: int = 0  # inject N failing RUNs (for retry tests)
        self._server = None

    @property
    def uri(self) -> str:
        return f"bolt://{self.host}:{self.port}"

    async def start(self) -> "FakeBoltServer":
        self._server = await asyncio.start_server(self._handle, self.host, self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def stop(self) -> None:
        if self._server:
            self._server.close()
            await self._server.wait_closed()

    async def _handle(self, reader, writer) -> None:
        self.connections += 1
        try:
            hs = await reader.readexactly(20)
            if hs[:4] != b"\x60\x60\xB0\x17":
                writer.close()
                return
            major, minor = self.version
            writer.write(bytes([0, 0, minor, major]))
            dech = native().BoltDechunker()
            tx_graph = None       # working copy inside an explicit transaction
            failed = False
            results: list = []    # pending result streams for PULL
            while True:
                chunk = await reader.read(65536)
                if not chunk:
                    break
                for raw in dech.feed(chunk):
                    m = unpack(raw)
                    out = []

                    def send(tag, *fields):
                        out.append(native().bolt_chunk(pack(Structure(tag, list(fields)))))

                    if m.tag == RESET:
                        failed, results, tx_graph = False, [], None
                        send(SUCCESS, {})
                    elif failed:
                        send(IGNORED)
                    elif m.tag == HELLO:
                        send(SUCCESS, {"server": "Neo4j/5.18.0", "connection_id": f"bolt-{self.connections}"})
                    elif m.tag == BEGIN:
                        tx_graph = self.graph.clone()
                        send(SUCCESS, {})
                    elif m.tag == RUN:
                        query, params = m.fields[0], m.fields[1]
                        g = tx_graph if tx_graph is not None else self.graph
                        try:
                            if self.fail_next > 0:
                                self.fail_next -= 1
                                raise CypherError("Neo.TransientError.General.DatabaseUnavailable",
                                                  "injected failure")
                            fields, recs = execute(g, query, params)
                            self.log.append((_norm(query), dict(params)))
                            results.append(recs)
                            send(SUCCESS, {"fields": fields, "t_first": 0})
                        except CypherError as e:
                            failed = True
                            send(FAILURE, {"code": e.code, "message": str(e)})
                    elif m.tag == PULL:
                        recs = results.pop(0) if results else []
                        for r in recs:
                            send(RECORD, r)
                        send(SUCCESS, {"has_more": False})
                    elif m.tag == COMMIT:
                        if tx_graph is not None:
                            self.graph = tx_graph
                        tx_graph = None
                        send(SUCCESS, {"bookmark": f"FB:{len(self.log)}"})
                    elif m.tag == ROLLBACK:
                        tx_graph = None
                        send(SUCCESS, {})
                    elif m.tag == GOODBYE:
                        writer.close()
                        return
                    else:
                        failed = True
                        send(FAILURE, {"code": "Neo.ClientError.Request.Invalid", "message": "unknown message"})
                    if out:
                        writer.write(b"".join(out))
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            try:
                writer.close()
            except Exception:
                pass
