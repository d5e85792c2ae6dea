"""knowledge_graph_service: TokenizedTextMessage -> Neo4j graph (services/knowledge_graph_service).

Graph format kept byte-for-byte in Cypher (src/main.rs):
  (:Document {original_id, source_url, processed_at_ms (a STRING: msg.timestamp_ms.to_string()),
              created_at_ms})                                                       :37-48
  (:Sentence {text, created_at_ms}) <-[:HAS_SENTENCE {order}]- (d)   empty sentences skipped :70-93
  (:Token {text_lc, text_original_case, created_at_ms}) <-[:CONTAINS_TOKEN]- (d)  trimmed, empty
                                                          tokens skipped, text_lc = lowercase :100-125
One transaction per message (:32, :132).  Schema (:158-173) ensured in the background with 5 x 3 s
retries (:253-284).  Connection: db "neo4j", up to 10 connections (:238-246).
Differences: statements of a transaction are pipelined (one round trip instead of N_sent + N_tok);
``SYMB_KG_UNWIND=1`` switches to two UNWIND-batched statements producing the same graph.
"""
from __future__ import annotations

import asyncio
import os

from ..kg.bolt import BoltError, Graph
from ..ops._ext import native
from ..utils import log as ulog
from ..wire import TokenizedTextMessage, WireError, subjects
from .base import Service

DOC_Q = ("MERGE (d:Document {original_id: $original_id}) "
         "ON CREATE SET d.source_url = $source_url, d.processed_at_ms = $processed_at, d.created_at_ms = timestamp() "
         "ON MATCH SET d.source_url = $source_url, d.processed_at_ms = $processed_at "
         "RETURN id(d) AS doc_node_id")
SENT_Q = ("MATCH (d:Document) WHERE id(d) = $doc_node_id "
          "MERGE (s:Sentence {text: $text}) "
          "ON CREATE SET s.created_at_ms = timestamp() "
          "MERGE (d)-[r:HAS_SENTENCE {order: $order}]->(s) "
          "RETURN id(s) AS sentence_node_id")
TOK_Q = ("MATCH (d:Document) WHERE id(d) = $doc_node_id "
         "MERGE (t:Token {text_lc: $token_text_lc}) "
         "ON CREATE SET t.text_original_case = $token_text_original, t.created_at_ms = timestamp() "
         "ON MATCH SET t.text_original_case = $token_text_original "
         "MERGE (d)-[r_ct:CONTAINS_TOKEN]->(t)")
SENT_UNWIND_Q = ("MATCH (d:Document) WHERE id(d) = $doc_node_id UNWIND $rows AS row "
                 "MERGE (s:Sentence {text: row.text}) ON CREATE SET s.created_at_ms = timestamp() "
                 "MERGE (d)-[r:HAS_SENTENCE {order: row.order}]->(s)")
TOK_UNWIND_Q = ("MATCH (d:Document) WHERE id(d) = $doc_node_id UNWIND $rows AS row "
                "MERGE (t:Token {text_lc: row.lc}) ON CREATE SET t.text_original_case = row.orig, "
                "t.created_at_ms = timestamp() ON MATCH SET t.text_original_case = row.orig "
                "MERGE (d)-[r_ct:CONTAINS_TOKEN]->(t)")
SCHEMA_Q = ("CREATE CONSTRAINT IF NOT EXISTS FOR (d:Document) REQUIRE d.original_id IS UNIQUE",
            "CREATE INDEX token_text_lc_index IF NOT EXISTS FOR (t:Token) ON (t.text_lc)")


class KnowledgeGraphService(Service):
    name = "knowledge_graph_service"

    def __init__(self, *a, graph: Graph | None = None, **kw):
        super().__init__(*a, **kw)
        self.graph = graph or Graph(self.cfg.neo4j_uri, self.cfg.neo4j_user, self.cfg.neo4j_password,
                                    self.cfg.neo4j_db, max_connections=10)
        self.unwind = os.environ.get("SYMB_KG_UNWIND", "") == "1"
        self.schema_ready = asyncio.Event()

    async def setup(self) -> None:
        self._loops.append(asyncio.create_task(self.ensure_schema()))
        await self.subscribe_loop(subjects.PROCESSED_TEXT_TOKENIZED, self.handle)

    async def ensure_schema(self, attempts: int = 5, wait_s: float = 3.0) -> bool:
        for i in range(attempts):
            try:
                for q in SCHEMA_Q:
                    await self.graph.run(q)
                self.log.info("[NEO4J_SCHEMA] Database schema ensured.")
                self.schema_ready.set()
                return True
            except (BoltError, OSError, ConnectionError) as e:
                self.log.warning("[NEO4J_SCHEMA] attempt %d/%d failed: %s", i + 1, attempts, e)
                await asyncio.sleep(wait_s)
        self.log.error("[NEO4J_SCHEMA] giving up after %d attempts", attempts)
        return False

    async def save(self, msg: TokenizedTextMessage, order_offset: int = 0) -> int:
        self.log.info("[NEO4J_SAVE] Attempting to save data for original_id: %s", msg.original_id)
        rust_trim = native().rust_trim

        async def body(tx):
            rows = await tx.run(DOC_Q, {"original_id": msg.original_id, "source_url": msg.source_url,
                                        "processed_at": str(msg.timestamp_ms)})
            if not rows:
                raise BoltError("Symbiont.NoDocument", "Document node not created/found after MERGE")
            doc = rows[0]["doc_node_id"]
            sents = [(order_offset + i, s) for i, s in enumerate(msg.sentences) if rust_trim(s)]
            toks = [t for t in (rust_trim(x) for x in msg.tokens) if t]
            if self.unwind:
                if sents:
                    tx.queue(SENT_UNWIND_Q, {"doc_node_id": doc,
                                             "rows": [{"text": s, "order": o} for o, s in sents]})
                if toks:
                    tx.queue(TOK_UNWIND_Q, {"doc_node_id": doc,
                                            "rows": [{"lc": t.lower(), "orig": t} for t in toks]})
            else:
                for o, s in sents:
                    tx.queue(SENT_Q, {"doc_node_id": doc, "text": s, "order": o})
                for t in toks:
                    tx.queue(TOK_Q, {"doc_node_id": doc, "token_text_lc": t.lower(),
                                     "token_text_original": t})
            await tx.flush()
            return doc

        doc = await self.graph.transaction(body)
        self.log.info("[NEO4J_SAVE] Successfully committed transaction for original_id: %s",
                      msg.original_id)
        self.metrics.inc("documents_saved")
        return doc

    async def handle(self, nmsg) -> None:
        try:
            msg = TokenizedTextMessage.from_json(nmsg.data)
        except WireError as e:
            self.log.warning("[TASK_DESERIALIZE_FAIL] Failed to deserialize TokenizedTextMessage: %s", e)
            return
        try:
            offset = int(native().json_loads(bytes(nmsg.data), False).get("sentence_order_offset", 0))
        except Exception:
            offset = 0
        self.log.info("[KG_HANDLER] Received TokenizedTextMessage (original_id: %s), %d tokens, %d sentences.",
                      msg.original_id, len(msg.tokens), len(msg.sentences))
        try:
            await self.save(msg, offset)
        except Exception as e:
            self.log.error("[KG_HANDLER_ERROR] Failed to save data to Neo4j for original_id %s: %s",
                           msg.original_id, e)
            self.metrics.inc("save_errors")

    async def stop(self) -> None:
        await super().stop()
        await self.graph.close()


def main() -> None:
    ulog.setup(KnowledgeGraphService.name, "info")
    asyncio.run(KnowledgeGraphService().run_forever())


if __name__ == "__main__":
    main()
