"""preprocessing_service: sentence split + HIP sentence-transformer embeddings
(services/preprocessing_service/src/main.rs, embedding_generator.rs).

* ``data.raw_text.discovered`` (RawTextMessage) -> whitespace-normalise, split on . ? !
  (byte-exact with main.rs:28-62) -> embed every sentence -> ``data.text.with_embeddings``
  (TextWithEmbeddingsMessage).  Messages that would exceed the broker's max_payload (1 MiB:
  ~110 sentences at 768-d) are split; each chunk carries an extra
  ``sentence_order_offset`` field (ignored by serde consumers) so global sentence order survives.
* ``tasks.embedding.for_query`` request/reply -> QueryEmbeddingResult (error replies keep the
  reference's texts, including request_id "unknown" on undecodable tasks, main.rs:178-198).
* Restores the v0.1 feed of the knowledge graph: TokenizedTextMessage on
  ``data.processed_text.tokenized`` (orphaned in v0.3.0; SYMB_PUBLISH_TOKENIZED).
GPU work goes through the EmbedBatcher (packed varlen, token-budgeted, off the event loop).
"""
from __future__ import annotations

import asyncio

from ..models.config import get_config
from ..models.encoder import make_encoder
from ..ops._ext import native
from ..text import normalize_whitespace, split_sentences, whitespace_pretokenize
from ..text.tokenizer import Tokenizer
from ..utils import log as ulog
from ..wire import (QueryEmbeddingResult, QueryForEmbeddingTask, RawTextMessage, SentenceEmbedding,
                    TextWithEmbeddingsMessage, TokenizedTextMessage, WireError,
                    current_timestamp_ms, subjects)
from .base import Service
from .batcher import EmbedBatcher


class PreprocessingService(Service):
    name = "preprocessing_service"

    def __init__(self, *a, encoder=None, **kw):
        super().__init__(*a, **kw)
        self.model_cfg = get_config(self.cfg.model)
        self.log.info("[EMBED_INIT] Initializing encoder %s (force_cpu: %s)", self.model_cfg.model_name,
                      self.cfg.force_cpu)
        self.encoder = encoder or make_encoder(self.model_cfg, force_cpu=self.cfg.force_cpu,
                                               seed=self.cfg.model_seed,
                                               precision=self.cfg.encoder_dtype)
        self.tokenizer = Tokenizer(self.model_cfg, self.cfg.vocab_file or None)
        self.batcher = EmbedBatcher(self.encoder, self.tokenizer, self.cfg.batch_tokens,
                                    self.cfg.batch_window_ms, metrics=self.metrics)
        self.log.info("[EMBED_INIT_SUCCESS] encoder backend=%s hidden=%d", self.encoder.backend,
                      self.model_cfg.hidden)

    @property
    def model_name(self) -> str:
        return self.model_cfg.model_name

    async def setup(self) -> None:
        await self.subscribe_loop(subjects.RAW_TEXT_DISCOVERED, self.handle_raw_text)
        # query embeddings: whole drained bursts -> one EmbedBatcher request + one socket write
        await self.subscribe_batches(subjects.EMBEDDING_FOR_QUERY, self.handle_query_batch)

    # ------------------------------------------------------------------ ingest
    async def process_text_and_embed(self, raw: RawTextMessage):
        cleaned = normalize_whitespace(raw.raw_text)
        if not cleaned:
            raise ValueError(f"Cleaned text is empty for id: {raw.id}")
        sentences = split_sentences(cleaned)
        if not sentences:
            raise ValueError(f"No sentences extracted for id: {raw.id}")
        self.log.info("[TEXT_PROCESSOR_EMBED] Extracted %d sentences for id: %s", len(sentences), raw.id)
        emb = await self.batcher.embed(sentences)
        if emb.shape[0] != len(sentences):
            raise ValueError(f"Mismatch between number of sentences ({len(sentences)}) and "
                             f"embeddings ({emb.shape[0]}) for id: {raw.id}")
        msg = TextWithEmbeddingsMessage(
            raw.id, raw.source_url, [SentenceEmbedding(s, emb[i]) for i, s in enumerate(sentences)],
            self.model_name, current_timestamp_ms())
        return cleaned, sentences, msg

    def chunk_payloads(self, msg: TextWithEmbeddingsMessage, limit: int) -> list[bytes]:
        """Split a message into <= limit-byte JSON payloads (sentence order preserved)."""
        whole = msg.to_json()
        if len(whole) <= limit:
            return [whole]
        n = native()
        head = {"original_id": msg.original_id, "source_url": msg.source_url}
        out, cur, cur_size, offset = [], [], 0, 0
        base = len(n.json_dumps({**head, "embeddings_data": [], "model_name": msg.model_name,
                                 "timestamp_ms": msg.timestamp_ms, "sentence_order_offset": 0}))
        for i, se in enumerate(msg.embeddings_data):
            item = se.to_obj()
            sz = len(n.json_dumps(item)) + 1
            if cur and base + cur_size + sz + 16 > limit:
                out.append((offset, cur))
                offset, cur, cur_size = i, [], 0
            cur.append(item)
            cur_size += sz
        if cur:
            out.append((offset, cur))
        return [n.json_dumps({**head, "embeddings_data": items, "model_name": msg.model_name,
                              "timestamp_ms": msg.timestamp_ms, "sentence_order_offset": off})
                for off, items in out]

    async def handle_raw_text(self, nmsg) -> None:
        try:
            raw = RawTextMessage.from_json(nmsg.data)
        except WireError as e:
            self.log.warning("[TASK_DESERIALIZE_FAIL_RAW_TEXT] Failed to deserialize RawTextMessage: %s", e)
            return
        self.log.info("[TASK_DESERIALIZED_RAW_TEXT] Deserialized RawTextMessage (id: %s, url: %s)",
                      raw.id, raw.source_url)
        try:
            cleaned, sentences, msg = await self.process_text_and_embed(raw)
        except Exception as e:
            self.log.error("[PROCESS_TEXT_FAIL] Failed to process text with embeddings for id %s: %s",
                           raw.id, e)
            return
        limit = getattr(self.nc, "max_payload", 1 << 20)
        payloads = self.chunk_payloads(msg, limit)
        for p in payloads:
            await self.publish(subjects.TEXT_WITH_EMBEDDINGS, p)
        self.log.info("[NATS_PUB_SUCCESS] Successfully published TextWithEmbeddingsMessage "
                      "(original_id: %s) with %d embeddings in %d message(s).", raw.id,
                      len(sentences), len(payloads))
        if self.cfg.publish_tokenized:
            tm = TokenizedTextMessage(raw.id, raw.source_url, whitespace_pretokenize(cleaned),
                                      sentences, msg.timestamp_ms)
            data = tm.to_json()
            if len(data) <= limit:
                await self.publish(subjects.PROCESSED_TEXT_TOKENIZED, data)
            else:  # split tokens/sentences proportionally, keep global order via offsets
                n = native()
                parts = max(2, len(data) // (limit // 2) + 1)
                st = max(1, len(sentences) // parts + 1)
                tt = max(1, len(tm.tokens) // parts + 1)
                for j in range(parts):
                    obj = {"original_id": raw.id, "source_url": raw.source_url,
                           "tokens": tm.tokens[j * tt:(j + 1) * tt],
                           "sentences": sentences[j * st:(j + 1) * st],
                           "timestamp_ms": tm.timestamp_ms, "sentence_order_offset": j * st}
                    await self.publish(subjects.PROCESSED_TEXT_TOKENIZED, n.json_dumps(obj))

    # ------------------------------------------------------------------ query embedding
    async def handle_query_batch(self, msgs) -> None:
        """A burst of QueryForEmbeddingTask requests -> one packed encode (through the
        EmbedBatcher, so it also coalesces with ingest work) -> replies in one write.  Undecodable
        messages get handle_query's error reply."""
        tasks, good = [], []
        for m in msgs:
            try:
                tasks.append(QueryForEmbeddingTask.from_json(m.data))
                good.append(m)
            except WireError:
                self.spawn(self.handle_query(m))
        if tasks:
            self.log.info("[QUERY_EMBED_HANDLER] Processing %d QueryForEmbeddingTask(s) "
                          "(request_ids %s..%s)", len(tasks), tasks[0].request_id,
                          tasks[-1].request_id)
            self.spawn(self._finish_query_batch(good, tasks))

    async def _finish_query_batch(self, msgs, tasks) -> None:
        try:
            out = await self.batcher.embed([t.text_to_embed for t in tasks])
            errs = [None] * len(tasks)
        except Exception as e:
            out = None
            errs = [f"Failed to generate embedding for request_id {t.request_id}: {e}" for t in tasks]
            self.log.error("[QUERY_EMBED_HANDLER_GENERATION_FAIL] %s", errs[0])
        replies = []
        for j, (m, t) in enumerate(zip(msgs, tasks)):
            res = QueryEmbeddingResult(t.request_id, None if out is None else out[j],
                                       self.model_name, errs[j])
            if m.reply:
                replies.append((m.reply, res.to_json()))
            else:
                self.log.warning("[QUERY_EMBED_HANDLER] No reply subject provided for query "
                                 "embedding task_id %s. Result not sent.", t.request_id)
        await self.nc.publish_many(replies)

    async def handle_query(self, nmsg) -> None:
        try:
            task = QueryForEmbeddingTask.from_json(nmsg.data)
        except WireError as e:
            err = f"Failed to deserialize QueryForEmbeddingTask: {e}"
            self.log.error("[QUERY_EMBED_HANDLER_DESERIALIZE_FAIL] %s", err)
            if nmsg.reply:
                await self.nc.publish(nmsg.reply, QueryEmbeddingResult("unknown", None, None, err).to_json())
            return
        self.log.info("[QUERY_EMBED_HANDLER] Processing QueryForEmbeddingTask (request_id: %s), "
                      "text: '%s'", task.request_id, task.text_to_embed)
        emb, err = None, None
        try:
            out = await self.batcher.embed([task.text_to_embed])
            if out.shape[0] == 1:
                emb = out[0]
            else:
                err = (f"Embedding generation for a single sentence returned {out.shape[0]} "
                       f"embeddings for request_id {task.request_id}")
        except Exception as e:
            err = f"Failed to generate embedding for request_id {task.request_id}: {e}"
            self.log.error("[QUERY_EMBED_HANDLER_GENERATION_FAIL] %s", err)
        res = QueryEmbeddingResult(task.request_id, emb, self.model_name, err)
        if nmsg.reply:
            await self.nc.publish(nmsg.reply, res.to_json())
        else:
            self.log.warning("[QUERY_EMBED_HANDLER] No reply subject provided for query embedding "
                             "task_id %s. Result not sent.", task.request_id)


def main() -> None:
    """One GPU: ``python -m ...preprocessing``.  A node with RCCL data parallelism:
    ``torch.distributed.run --nproc-per-node N -m codename_symbiont_amd.services.preprocessing``
    -- rank 0 serves NATS and spreads every packed batch over all ranks (parallel/embed_group.py);
    the other ranks execute its collective ops.  (launch.py's default is N independent replicas in
    a NATS queue group; ``--embed-dp rccl`` selects this mode.)"""
    import os

    ulog.setup(PreprocessingService.name, "info,preprocessing_service=debug")
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        asyncio.run(PreprocessingService().run_forever())
        return
    from ..models import get_config
    from ..parallel import dist as D
    from ..parallel.embed_group import EmbedGroup, GroupEncoder
    from ..utils.config import Config

    cfg = Config()
    info = D.init()
    enc = make_encoder(get_config(cfg.model), force_cpu=cfg.force_cpu, device=info.device,
                       precision=cfg.encoder_dtype)
    group = EmbedGroup(info, enc)
    try:
        if info.is_root:
            asyncio.run(PreprocessingService(cfg, encoder=GroupEncoder(group)).run_forever())
        else:
            group.serve()
    finally:
        group.stop()
        D.shutdown(info)


if __name__ == "__main__":
    main()
