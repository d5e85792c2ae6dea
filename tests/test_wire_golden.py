"""Golden-JSON tests of the 15 wire contracts (stricter than the reference's round-trip-only tests,
libs/shared_models/src/lib.rs:123-537): exact bytes of serde_json::to_vec for every struct."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from codename_symbiont_amd.ops._ext import native
from codename_symbiont_amd.wire import (ALL_CONTRACTS, GeneratedTextMessage, GenerateTextTask,
                                        PerceiveUrlTask, QdrantPointPayload, QueryEmbeddingResult,
                                        QueryForEmbeddingTask, RawTextMessage,
                                        SemanticSearchApiRequest, SemanticSearchApiResponse,
                                        SemanticSearchNatsResult, SemanticSearchNatsTask,
                                        SemanticSearchResultItem, SentenceEmbedding,
                                        TextWithEmbeddingsMessage, TokenizedTextMessage, WireError)

F = lambda *v: np.array(v, dtype=np.float32)  # noqa: E731
PAY = QdrantPointPayload("doc", "http://u", "Text é", 3, "m", 1717000000000)

GOLDEN = [
    (PerceiveUrlTask("https://example.com"), b'{"url":"https://example.com"}'),
    (RawTextMessage("id1", "u", "line1\nline2 \"q\"", 1716500000000),
     b'{"id":"id1","source_url":"u","raw_text":"line1\\nline2 \\"q\\"","timestamp_ms":1716500000000}'),
    (TokenizedTextMessage("o", "u", ["a", "b"], ["s."], 7),
     b'{"original_id":"o","source_url":"u","tokens":["a","b"],"sentences":["s."],"timestamp_ms":7}'),
    (GenerateTextTask("t", None, 50), b'{"task_id":"t","prompt":null,"max_length":50}'),
    (GenerateTextTask("t", "p", 1), b'{"task_id":"t","prompt":"p","max_length":1}'),
    (GeneratedTextMessage("t", "я пошел", 9), '{"original_task_id":"t","generated_text":"я пошел","timestamp_ms":9}'.encode()),
    (SentenceEmbedding("s", F(0.1, -0.5, 1.0)), b'{"sentence_text":"s","embedding":[0.1,-0.5,1.0]}'),
    (TextWithEmbeddingsMessage("o", "u", [SentenceEmbedding("a", F(1e-7)), SentenceEmbedding("b", F())], "m", 1),
     b'{"original_id":"o","source_url":"u","embeddings_data":[{"sentence_text":"a","embedding":[1e-7]},'
     b'{"sentence_text":"b","embedding":[]}],"model_name":"m","timestamp_ms":1}'),
    (SemanticSearchApiRequest("q", 5), b'{"query_text":"q","top_k":5}'),
    (QueryForEmbeddingTask("r", "x"), b'{"request_id":"r","text_to_embed":"x"}'),
    (QueryEmbeddingResult("r", F(0.25, 3.0), "m", None),
     b'{"request_id":"r","embedding":[0.25,3.0],"model_name":"m","error_message":null}'),
    (QueryEmbeddingResult("unknown", None, None, "bad"),
     b'{"request_id":"unknown","embedding":null,"model_name":null,"error_message":"bad"}'),
    (PAY, '{"original_document_id":"doc","source_url":"http://u","sentence_text":"Text é","sentence_order":3,'
          '"model_name":"m","processed_at_ms":1717000000000}'.encode()),
    (SemanticSearchNatsTask("r", F(0.5), 10), b'{"request_id":"r","query_embedding":[0.5],"top_k":10}'),
    (SemanticSearchResultItem("pid", 0.87654321, PAY),
     b'{"qdrant_point_id":"pid","score":0.8765432,"payload":' + PAY.to_json() + b"}"),
    (SemanticSearchNatsResult("r", [], None), b'{"request_id":"r","results":[],"error_message":null}'),
    (SemanticSearchApiResponse("r", [SemanticSearchResultItem("p", 1.0, PAY)], "e"),
     b'{"search_request_id":"r","results":[{"qdrant_point_id":"p","score":1.0,"payload":' + PAY.to_json()
     + b'}],"error_message":"e"}'),
]


@pytest.mark.parametrize("obj,golden", GOLDEN, ids=[type(o).__name__ for o, _ in GOLDEN])
def test_golden_bytes(obj, golden):
    assert obj.to_json() == golden
    back = type(obj).from_json(golden)
    assert back == obj or isinstance(obj, SemanticSearchResultItem)


def test_all_contracts_covered():
    assert {type(o) for o, _ in GOLDEN} == set(ALL_CONTRACTS)


@pytest.mark.parametrize("v,s", [
    (0.1, "0.1"), (1.0, "1.0"), (-0.0, "-0.0"), (0.0, "0.0"), (1e-7, "1e-7"), (1.5e20, "1.5e20"),
    (123456789.0, "123456790.0"), (0.001234, "0.001234"), (1e-6, "0.000001"), (1e13, "1e13"),
    (1e12, "1000000000000.0"), (3.4028235e38, "3.4028235e38"), (1e-45, "1e-45"), (-2.5e-10, "-2.5e-10"),
    (float("nan"), "null"), (float("inf"), "null"), (16777216.0, "16777216.0"), (0.3, "0.3"),
])
def test_f32_ryu_layout(v, s):
    assert native().format_f32(v) == s


@settings(max_examples=2000, deadline=None)
@given(st.floats(width=32, allow_nan=False, allow_infinity=False))
def test_f32_shortest_roundtrips(v):
    s = native().format_f32(v)
    assert np.float32(float(s)) == np.float32(v)

    def sig_digits(txt):
        mant = txt.lstrip("-").split("e")[0].replace(".", "").lstrip("0").rstrip("0")
        return len(mant) or 1
    # same number of significant digits as numpy's shortest (Dragon4 unique) f32 repr
    ref = np.format_float_scientific(np.float32(v), unique=True)
    assert sig_digits(s) == sig_digits(ref)


def test_string_escapes():
    assert native().json_dumps("\x00\x1f\x7f é\\/\t") == b'"\\u0000\\u001f\x7f\xe2\x80\xa8\xc3\xa9\\\\/\\t"'


def test_serde_like_errors():
    with pytest.raises(WireError, match=r"missing field `url` at line 1 column 2"):
        PerceiveUrlTask.from_json(b"{}")
    with pytest.raises(WireError, match=r"invalid type: string \"5\", expected u32"):
        SemanticSearchApiRequest.from_json(b'{"query_text":"q","top_k":"5"}')
    with pytest.raises(WireError, match=r"invalid value: integer `4294967296`, expected u32"):
        SemanticSearchApiRequest.from_json(b'{"query_text":"q","top_k":4294967296}')
    with pytest.raises(WireError, match=r"invalid type: floating point"):
        SemanticSearchApiRequest.from_json(b'{"query_text":"q","top_k":1.5}')
    with pytest.raises(WireError, match=r"invalid type: null, expected a string"):
        PerceiveUrlTask.from_json(b'{"url":null}')
    with pytest.raises(WireError, match="trailing characters"):
        PerceiveUrlTask.from_json(b'{"url":"a"} x')
    with pytest.raises(WireError, match="EOF while parsing"):
        PerceiveUrlTask.from_json(b'{"url":"a"')
    # unknown fields ignored, Option missing -> None, integers accepted for f32
    r = QueryEmbeddingResult.from_json(b'{"request_id":"x","extra":[1,{"a":2}],"embedding":[1,2]}')
    assert r.model_name is None and list(r.embedding) == [1.0, 2.0]


@settings(max_examples=200, deadline=None)
@given(st.text(), st.text(), st.lists(st.text(max_size=20), max_size=10),
       st.integers(0, 2**64 - 1))
def test_roundtrip_tokenized(a, b, toks, ts):
    m = TokenizedTextMessage(a, b, toks, toks[::-1], ts)
    assert TokenizedTextMessage.from_json(m.to_json()) == m


@settings(max_examples=100, deadline=None)
@given(st.lists(st.floats(width=32, allow_nan=False, allow_infinity=False), max_size=64))
def test_roundtrip_embeddings_exact(vals):
    v = np.array(vals, dtype=np.float32)
    m = SemanticSearchNatsTask("r", v, 3)
    back = SemanticSearchNatsTask.from_json(m.to_json())
    assert np.array_equal(back.query_embedding, v)
