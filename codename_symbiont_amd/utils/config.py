"""Typed configuration: the reference's env-var surface plus the knobs it hard-codes.

Compatible names: NATS_URL, API_SERVER_HOST, API_SERVER_PORT, NEO4J_URI, NEO4J_USER,
NEO4J_PASSWORD, FORCE_CPU, RUST_LOG.  New (SYMB_*): model family, batch token budget, index
dimension/capacity, snapshot dir, timeouts, world size...  Qdrant's QDRANT_URI is accepted and
ignored (the vector store is the in-HBM index now).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field


def _env(name: str, default: str) -> str:
    v = os.environ.get(name)
    return default if v is None or v == "" else v


def _int(name: str, default: int) -> int:
    try:
        return int(_env(name, str(default)))
    except ValueError:
        return default


def _float(name: str, default: float) -> float:
    try:
        return float(_env(name, str(default)))
    except ValueError:
        return default


def _bool(name: str, default: bool) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v == "1" or v.lower() == "true"


@dataclass
class Config:
    # --- reference-compatible ---
    nats_url: str = field(default_factory=lambda: _env("NATS_URL", "nats://localhost:4222"))
    api_host: str = field(default_factory=lambda: _env("API_SERVER_HOST", "0.0.0.0"))
    api_port: int = field(default_factory=lambda: _int("API_SERVER_PORT", 8080))  # parse fail -> 8080
    # gateway worker processes sharing the port (SO_REUSEPORT); each has its own NATS connection
    # and SSE hub, and every worker receives every events.text.generated message
    api_workers: int = field(default_factory=lambda: _int("SYMB_API_WORKERS", 1))
    neo4j_uri: str = field(default_factory=lambda: _env("NEO4J_URI", "bolt://localhost:7687"))
    neo4j_user: str = field(default_factory=lambda: _env("NEO4J_USER", "neo4j"))
    neo4j_password: str = field(default_factory=lambda: _env("NEO4J_PASSWORD", ""))
    neo4j_db: str = "neo4j"
    force_cpu: bool = field(default_factory=lambda: _bool("FORCE_CPU", False))
    # --- hard-coded in the reference, configurable here ---
    model: str = field(default_factory=lambda: _env("SYMB_MODEL", "mpnet-multi"))
    model_seed: int = field(default_factory=lambda: _int("SYMB_MODEL_SEED", 0))
    vocab_file: str = field(default_factory=lambda: _env("SYMB_VOCAB", ""))
    batch_tokens: int = field(default_factory=lambda: _int("SYMB_BATCH_TOKENS", 65536))
    batch_window_ms: float = field(default_factory=lambda: _float("SYMB_BATCH_WINDOW_MS", 2.0))
    index_dim: int = field(default_factory=lambda: _int("SYMB_INDEX_DIM", 0))  # 0 -> model hidden
    index_capacity: int = field(default_factory=lambda: _int("SYMB_INDEX_CAPACITY", 1 << 22))
    # benchmarking only: pre-fill the index with N random unit rows (no payloads) at startup
    index_fill_random: int = field(default_factory=lambda: _int("SYMB_INDEX_FILL_RANDOM", 0))
    # encoder projection GEMMs: "bf16" (default) or "fp8" (e4m3, per-channel/per-token scales)
    encoder_dtype: str = field(default_factory=lambda: os.environ.get("SYMB_ENCODER_DTYPE", "bf16"))
    # "bf16" (default) or "fp8" (OCP e4m3 rows; needs a dim that is a multiple of 256)
    index_dtype: str = field(default_factory=lambda: os.environ.get("SYMB_INDEX_DTYPE", "bf16"))
    # "fp8": bf16 index searched through an e4m3 prefilter + exact bf16 re-score (Qdrant's
    # quantization + rescore); "" = exact bf16 scan
    index_prefilter: str = field(default_factory=lambda: os.environ.get("SYMB_INDEX_PREFILTER", ""))
    # "auto" (default): EXACT search through an int8 image of the bf16 rows where it applies
    # (384-wide bf16 shards): rows whose int8 score provably cannot reach a query's k-th best are
    # pruned, the rest re-scored in bf16 (csrc/hip/index_i8.hip); "none": scan every row in bf16
    index_prune: str = field(default_factory=lambda: os.environ.get("SYMB_INDEX_PRUNE", "auto"))
    snapshot_dir: str = field(default_factory=lambda: _env("SYMB_SNAPSHOT_DIR", ""))
    # queries per fused scan launch of the search service (a 100M-row scan costs about the same
    # for 16 or 256 queries, so bigger bursts buy throughput at the price of latency); 512 = two
    # of the int8 scan's 256-query blocks, taken whole under load (search_align below;
    # profiles/r3_e2e/: 16.1k req/s at 2048 in flight)
    search_max_batch: int = field(default_factory=lambda: _int("SYMB_SEARCH_MAX_BATCH", 512))
    # bursts larger than this take a whole multiple of it (the int8 scan's 256-query block: a
    # 369-query burst would cost two full scans of the shard; 0 = take whatever is queued)
    search_align: int = field(default_factory=lambda: _int("SYMB_SEARCH_ALIGN", 256))
    # while a scan runs, the next burst collects until it fills a search_align block or the
    # running scan is due to end (services/vector_memory.py _fill_deadline); 0 = launch at once
    search_fill: int = field(default_factory=lambda: _int("SYMB_SEARCH_FILL", 1))
    # CUs the index scans may occupy (0 = all): leave some to an encoder sharing the GPU
    scan_cus: int = field(default_factory=lambda: _int("SYMB_SCAN_CUS", 0))
    collection: str = "symbiont_document_embeddings"
    embed_timeout_s: float = field(default_factory=lambda: _float("SYMB_EMBED_TIMEOUT_S", 15.0))
    search_timeout_s: float = field(default_factory=lambda: _float("SYMB_SEARCH_TIMEOUT_S", 20.0))
    nats_request_timeout_s: float = field(default_factory=lambda: _float("SYMB_NATS_REQUEST_TIMEOUT_S", 10.0))
    sse_capacity: int = field(default_factory=lambda: _int("SYMB_SSE_CAPACITY", 32))
    sse_keepalive_s: float = field(default_factory=lambda: _float("SYMB_SSE_KEEPALIVE_S", 15.0))
    max_length_limit: int = 1000
    markov_corpus: str = field(default_factory=lambda: _env(
        "SYMB_MARKOV_CORPUS",
        "я пошел гулять в парк и увидел там собаку собака была очень веселая и я решил с ней поиграть"))
    scrape_timeout_s: float = field(default_factory=lambda: _float("SYMB_SCRAPE_TIMEOUT_S", 15.0))
    user_agent: str = "CodenameSymbiontBot/0.1 (+https://makkenzo.com)"
    publish_tokenized: bool = field(default_factory=lambda: _bool("SYMB_PUBLISH_TOKENIZED", True))
    queue_group: str = field(default_factory=lambda: _env("SYMB_QUEUE_GROUP", ""))
    fault_spec: str = field(default_factory=lambda: _env("SYMB_FAULT", ""))


def read_env_file(path: str) -> dict[str, str]:
    """docker-compose ``.env`` syntax: KEY=VALUE per line, ``#`` comments and blank lines skipped,
    an optional ``export`` prefix, single or double quotes around the value stripped (escapes in
    double quotes: \\n, \\", \\\\), an unquoted value's trailing `` # comment`` dropped."""
    out: dict[str, str] = {}
    with open(path, encoding="utf-8") as f:
        for raw in f:
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            if line.startswith("export "):
                line = line[len("export "):].lstrip()
            key, sep, val = line.partition("=")
            key = key.strip()
            if not sep or not key:
                continue
            val = val.strip()
            if len(val) >= 2 and val[0] == val[-1] and val[0] in "'\"":
                q, val = val[0], val[1:-1]
                if q == '"':
                    val = (val.replace("\\\\", "\0").replace("\\n", "\n").replace('\\"', '"')
                           .replace("\0", "\\"))
            else:
                val = val.split(" #", 1)[0].rstrip()
            out[key] = val
    return out
