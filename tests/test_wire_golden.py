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


_NUM_TEXT = st.one_of(
    st.floats(allow_nan=False, allow_infinity=False, width=32).map(lambda v: str(np.float32(v))),
    st.floats(allow_nan=False, allow_infinity=False).map(repr),
    st.tuples(st.floats(allow_nan=False, allow_infinity=False, min_value=-1e30, max_value=1e30),
              st.integers(0, 20)).map(lambda t: f"{t[0]:.{t[1]}e}"),
    st.tuples(st.floats(allow_nan=False, allow_infinity=False, min_value=-1e6, max_value=1e6),
              st.integers(0, 12)).map(lambda t: f"{t[0]:.{t[1]}f}"),
    st.integers(-(1 << 60), 1 << 60).map(str),
    st.sampled_from(["0", "-0", "-0.0", "0e5", "16777217", "16777219", "33554434.0", "1e22",
                     "1e23", "1e-22", "1e-23", "123456789012345", "1234567890123456",
                     "0.000000000000000000001", "3.4028235e38", "3.4028236e38", "1E+2", "5e-324"]))


@settings(max_examples=300, deadline=None)
@given(st.lists(_NUM_TEXT, min_size=1, max_size=40))
def test_number_parsing_matches_serde_semantics(texts):
    """Floats parse to strtod's double (Python's float()); f32 arrays are that double cast to f32
    (serde_json's f32 = f64-then-cast), including the fast decimal path's edge cases."""
    doc = ("[" + ",".join(texts) + "]").encode()
    got32 = native().json_loads(doc, True)
    want64 = np.array([float(t) for t in texts], np.float64)
    with np.errstate(over="ignore"):
        want32 = want64.astype(np.float32)
    assert got32.dtype == np.float32
    assert got32.tobytes() == want32.tobytes(), (texts, got32, want32)
    got64 = native().json_loads(doc, False)
    for t, g in zip(texts, got64):
        v = float(t)
        if isinstance(g, float):
            assert g == v and np.signbit(g) == np.signbit(v), (t, g)
        else:
            assert g == int(t), (t, g)


@settings(max_examples=200, deadline=None)
@given(st.lists(_NUM_TEXT, min_size=4, max_size=4), st.integers(0, (1 << 32) + 5),
       st.text(max_size=8))
def test_search_tasks_batch_matches_wire_model(texts, k, rid):
    """vector_memory's batch decoder: regular messages decode exactly as SemanticSearchNatsTask
    (same f32 bits), everything irregular is flagged for the wire-model path."""
    import json

    from codename_symbiont_amd.wire import SemanticSearchNatsTask, WireError
    emb = "[" + ",".join(texts) + "]"
    rid_j = json.dumps(rid)
    msgs = [
        f'{{"request_id":{rid_j},"query_embedding":{emb},"top_k":{k}}}',
        f'{{ "top_k" : {k} , "query_embedding" : {emb}, "request_id" : {rid_j} }}',
        f'{{"request_id":{rid_j},"query_embedding":{emb},"top_k":{k},"x":1}}',   # extra key
        f'{{"request_id":{rid_j},"query_embedding":{emb}}}',                     # missing top_k
        f'{{"request_id":{rid_j},"query_embedding":[1,2,3],"top_k":{k}}}',       # other dim
        f'{{"request_id":{rid_j},"query_embedding":{emb},"top_k":{k}',           # truncated
        f'{{"request_id":{rid_j},"query_embedding":{emb},"top_k":-1}}',
    ]
    raw = [m.encode() for m in msgs]
    ok, ids, topk, q = native().search_tasks_batch(raw, 4)
    for i, m in enumerate(raw):
        try:
            t = SemanticSearchNatsTask.from_json(m)
        except WireError:
            assert not ok[i], msgs[i]
            continue
        if len(t.query_embedding) != 4:
            assert not ok[i]
            continue
        if i >= 2:   # irregular shape: left to the wire model even when it parses
            assert not ok[i], msgs[i]
            continue
        assert ok[i], msgs[i]
        assert ids[i] == t.request_id and topk[i] == t.top_k
        assert q[i].tobytes() == np.asarray(t.query_embedding, np.float32).tobytes()
