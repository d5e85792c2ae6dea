"""The 15 wire contracts of the reference (libs/shared_models/src/lib.rs:3-110), byte-compatible.

Encoding reproduces ``serde_json::to_vec`` of the Rust structs (field order, compact layout,
``Option::None`` -> ``null``, f32 shortest formatting) through the native codec
(csrc/native/json.cpp).  Decoding follows serde's derive semantics: unknown fields are ignored,
a missing non-Option field or a wrongly typed value is an error whose text mimics serde's
("missing field `url` ...", "invalid type: ..., expected u32"), a missing/null Option is None.
Embedding vectors (Vec<f32>) are carried as float32 numpy arrays end to end.
"""
from __future__ import annotations

import time
import uuid
from dataclasses import dataclass, field, fields
from typing import Any, ClassVar

import numpy as np

from ..ops._ext import native

U32_MAX = (1 << 32) - 1
U64_MAX = (1 << 64) - 1


class WireError(ValueError):
    pass


def current_timestamp_ms() -> int:
    """lib.rs:112-117 -- milliseconds since the Unix epoch."""
    return time.time_ns() // 1_000_000


def generate_uuid() -> str:
    """lib.rs:119-121 -- UUIDv4 string."""
    return str(uuid.uuid4())


def _desc(v: Any) -> str:
    if v is None:
        return "null"
    if isinstance(v, bool):
        return f"boolean `{str(v).lower()}`"
    if isinstance(v, int):
        return f"integer `{v}`"
    if isinstance(v, float):
        return f"floating point `{v}`"
    if isinstance(v, str):
        return f'string "{v}"'
    if isinstance(v, (list, np.ndarray)):
        return "a sequence"
    if isinstance(v, dict):
        return "a map"
    return type(v).__name__


def _int(v, name, hi):
    if isinstance(v, bool) or not isinstance(v, int):
        raise WireError(f"invalid type: {_desc(v)}, expected {name}")
    if v < 0 or v > hi:
        raise WireError(f"invalid value: integer `{v}`, expected {name}")
    return v


def _str(v):
    if not isinstance(v, str):
        raise WireError(f"invalid type: {_desc(v)}, expected a string")
    return v


def _f32(v):
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise WireError(f"invalid type: {_desc(v)}, expected f32")
    return float(np.float32(v))


def _vec_f32(v):
    if isinstance(v, np.ndarray):
        return v.astype(np.float32, copy=False)
    if not isinstance(v, list):
        raise WireError(f"invalid type: {_desc(v)}, expected a sequence")
    return np.asarray([_f32(x) for x in v], dtype=np.float32)


def _vec_str(v):
    if isinstance(v, np.ndarray) or not isinstance(v, list):
        if isinstance(v, np.ndarray) and v.size:
            raise WireError(f"invalid type: floating point `{float(v.flat[0])}`, expected a string")
        if isinstance(v, np.ndarray):
            return []
        raise WireError(f"invalid type: {_desc(v)}, expected a sequence")
    return [_str(x) for x in v]


def _kinds():
    return {
        "str": _str,
        "u32": lambda v: _int(v, "u32", U32_MAX),
        "u64": lambda v: _int(v, "u64", U64_MAX),
        "f32": _f32,
        "vec_f32": _vec_f32,
        "vec_str": _vec_str,
    }


_KIND = _kinds()


class WireModel:
    """Base for wire structs.  Subclasses are dataclasses with ``__wire__`` = (name, kind, optional)."""

    __wire__: ClassVar[tuple] = ()

    # ------------------------------------------------------------------ encode
    def to_obj(self) -> dict:
        out = {}
        for name, kind, _opt in self.__wire__:
            v = getattr(self, name)
            if v is None:
                out[name] = None
            elif isinstance(kind, type) and issubclass(kind, WireModel):
                out[name] = v.to_obj()
            elif isinstance(kind, tuple):  # ("vec", Model)
                out[name] = [x.to_obj() for x in v]
            elif kind == "vec_f32":
                out[name] = np.asarray(v, dtype=np.float32)
            else:
                out[name] = v
        return out

    def to_json(self) -> bytes:
        return native().json_dumps(self.to_obj())

    # ------------------------------------------------------------------ decode
    @classmethod
    def from_obj(cls, obj: Any):
        if not isinstance(obj, dict):
            raise WireError(f"invalid type: {_desc(obj)}, expected struct {cls.__name__}")
        kw = {}
        for name, kind, opt in cls.__wire__:
            if name not in obj or (opt and obj[name] is None):
                if opt:
                    kw[name] = None
                    continue
                raise WireError(f"missing field `{name}`")
            v = obj[name]
            if isinstance(kind, type) and issubclass(kind, WireModel):
                kw[name] = kind.from_obj(v)
            elif isinstance(kind, tuple):
                if not isinstance(v, list):
                    if isinstance(v, np.ndarray) and v.size == 0:
                        v = []
                    else:
                        raise WireError(f"invalid type: {_desc(v)}, expected a sequence")
                kw[name] = [kind[1].from_obj(x) for x in v]
            else:
                kw[name] = _KIND[kind](v)
        return cls(**kw)

    @classmethod
    def from_json(cls, data: bytes | str):
        if isinstance(data, str):
            data = data.encode()
        try:
            obj = native().json_loads(bytes(data), True)
        except ValueError as e:
            raise WireError(str(e)) from None
        try:
            return cls.from_obj(obj)
        except WireError as e:
            msg = str(e)
            if msg.startswith("missing field"):
                # serde reports the position of the object's closing brace
                msg += f" at line 1 column {len(bytes(data).rstrip())}"
            raise WireError(msg) from None

    def __eq__(self, other):
        if type(self) is not type(other):
            return NotImplemented
        for f in fields(self):
            a, b = getattr(self, f.name), getattr(other, f.name)
            if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
                if a is None or b is None or not np.array_equal(np.asarray(a), np.asarray(b)):
                    return False
            elif a != b:
                return False
        return True


def _wire(*spec):
    def deco(cls):
        cls.__wire__ = tuple((s[0], s[1], len(s) > 2 and s[2]) for s in spec)
        return cls
    return deco


# --------------------------------------------------------------------------- the 15 contracts
@_wire(("url", "str"))
@dataclass(eq=False)
class PerceiveUrlTask(WireModel):
    url: str


@_wire(("id", "str"), ("source_url", "str"), ("raw_text", "str"), ("timestamp_ms", "u64"))
@dataclass(eq=False)
class RawTextMessage(WireModel):
    id: str
    source_url: str
    raw_text: str
    timestamp_ms: int


@_wire(("original_id", "str"), ("source_url", "str"), ("tokens", "vec_str"),
       ("sentences", "vec_str"), ("timestamp_ms", "u64"))
@dataclass(eq=False)
class TokenizedTextMessage(WireModel):
    original_id: str
    source_url: str
    tokens: list
    sentences: list
    timestamp_ms: int


@_wire(("task_id", "str"), ("prompt", "str", True), ("max_length", "u32"))
@dataclass(eq=False)
class GenerateTextTask(WireModel):
    task_id: str
    prompt: str | None
    max_length: int


@_wire(("original_task_id", "str"), ("generated_text", "str"), ("timestamp_ms", "u64"))
@dataclass(eq=False)
class GeneratedTextMessage(WireModel):
    original_task_id: str
    generated_text: str
    timestamp_ms: int


@_wire(("sentence_text", "str"), ("embedding", "vec_f32"))
@dataclass(eq=False)
class SentenceEmbedding(WireModel):
    sentence_text: str
    embedding: np.ndarray


@_wire(("original_id", "str"), ("source_url", "str"),
       ("embeddings_data", ("vec", SentenceEmbedding)), ("model_name", "str"),
       ("timestamp_ms", "u64"))
@dataclass(eq=False)
class TextWithEmbeddingsMessage(WireModel):
    original_id: str
    source_url: str
    embeddings_data: list
    model_name: str
    timestamp_ms: int


@_wire(("query_text", "str"), ("top_k", "u32"))
@dataclass(eq=False)
class SemanticSearchApiRequest(WireModel):
    query_text: str
    top_k: int


@_wire(("request_id", "str"), ("text_to_embed", "str"))
@dataclass(eq=False)
class QueryForEmbeddingTask(WireModel):
    request_id: str
    text_to_embed: str


@_wire(("request_id", "str"), ("embedding", "vec_f32", True), ("model_name", "str", True),
       ("error_message", "str", True))
@dataclass(eq=False)
class QueryEmbeddingResult(WireModel):
    request_id: str
    embedding: np.ndarray | None = None
    model_name: str | None = None
    error_message: str | None = None


@_wire(("original_document_id", "str"), ("source_url", "str"), ("sentence_text", "str"),
       ("sentence_order", "u32"), ("model_name", "str"), ("processed_at_ms", "u64"))
@dataclass(eq=False)
class QdrantPointPayload(WireModel):
    original_document_id: str
    source_url: str
    sentence_text: str
    sentence_order: int
    model_name: str
    processed_at_ms: int


@_wire(("request_id", "str"), ("query_embedding", "vec_f32"), ("top_k", "u32"))
@dataclass(eq=False)
class SemanticSearchNatsTask(WireModel):
    request_id: str
    query_embedding: np.ndarray
    top_k: int


@_wire(("qdrant_point_id", "str"), ("score", "f32"), ("payload", QdrantPointPayload))
@dataclass(eq=False)
class SemanticSearchResultItem(WireModel):
    qdrant_point_id: str
    score: float
    payload: QdrantPointPayload


@_wire(("request_id", "str"), ("results", ("vec", SemanticSearchResultItem)),
       ("error_message", "str", True))
@dataclass(eq=False)
class SemanticSearchNatsResult(WireModel):
    request_id: str
    results: list = field(default_factory=list)
    error_message: str | None = None


@_wire(("search_request_id", "str"), ("results", ("vec", SemanticSearchResultItem)),
       ("error_message", "str", True))
@dataclass(eq=False)
class SemanticSearchApiResponse(WireModel):
    search_request_id: str
    results: list = field(default_factory=list)
    error_message: str | None = None


# api_service-local types (services/api_service/src/main.rs:26-35)
@_wire(("message", "str"), ("task_id", "str", True))
@dataclass(eq=False)
class ApiResponse(WireModel):
    message: str
    task_id: str | None = None


@_wire(("url", "str"))
@dataclass(eq=False)
class SubmitUrlApiPayload(WireModel):
    url: str


ALL_CONTRACTS = (PerceiveUrlTask, RawTextMessage, TokenizedTextMessage, GenerateTextTask,
                 GeneratedTextMessage, SentenceEmbedding, TextWithEmbeddingsMessage,
                 SemanticSearchApiRequest, QueryForEmbeddingTask, QueryEmbeddingResult,
                 QdrantPointPayload, SemanticSearchNatsTask, SemanticSearchResultItem,
                 SemanticSearchNatsResult, SemanticSearchApiResponse)
