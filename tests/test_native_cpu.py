"""Host C++ cores: sentence splitter / whitespace (byte parity with the reference rules), Markov chain
(training + generation rules), NATS stream parser (fuzzed chunking), HTML extractor fixtures."""
import random

import pytest
from hypothesis import given, settings, strategies as st

from codename_symbiont_amd.ops._ext import native
from codename_symbiont_amd.text import (extract_html_text, normalize_whitespace, split_sentences,
                                        whitespace_pretokenize)

N = native()


def ref_split(text: str) -> list[str]:
    """Python transliteration of preprocessing_service/src/main.rs:28-62 (oracle)."""
    cleaned = " ".join(text.split())  # Rust split_whitespace ~ Python str.split() for these inputs
    out, start = [], 0
    b = cleaned.encode()
    for i, ch in enumerate(b):
        if ch in b".?!":
            out.append(b[start:i + 1].decode().strip())
            start = i + 1
    if start < len(b):
        rem = b[start:].decode().strip()
        if rem:
            out.append(rem)
    if not out and cleaned:
        out.append(cleaned)
    return out


@pytest.mark.parametrize("text,expected", [
    ("Hello world. How are you?Fine!  tail ", ["Hello world.", "How are you?", "Fine!", "tail"]),
    ("a.b", ["a.", "b"]),
    ("...", [".", ".", "."]),
    ("Hi!!", ["Hi!", "!"]),
    ("no punctuation here", ["no punctuation here"]),
    ("Привет, мир! Как дела?  Хорошо", ["Привет, мир!", "Как дела?", "Хорошо"]),
    ("  x　y. ", ["x y."]),
    ("", []),
])
def test_sentence_split_cases(text, expected):
    assert split_sentences(normalize_whitespace(text)) == expected


@settings(max_examples=500, deadline=None)
@given(st.text(alphabet=st.sampled_from(list("ab. ?!\n\tыё,") + ["é", "x"]), max_size=80))
def test_sentence_split_matches_oracle(text):
    assert split_sentences(normalize_whitespace(text)) == ref_split(text)


def test_whitespace_pretokenize_matches_hf():
    from tokenizers.pre_tokenizers import Whitespace

    s = "Hello, world!! It's 3.14 — ok? Привет: мир..."
    assert whitespace_pretokenize(s) == [t for t, _ in Whitespace().pre_tokenize_str(s)]


CORPUS = "я пошел гулять в парк и увидел там собаку собака была очень веселая и я решил с ней поиграть"


def test_markov_rules():
    m = N.MarkovModel(7)
    assert m.generate(5) == "Model not trained."
    assert m.train(CORPUS)
    assert m.starters() == ["я"]                      # only the first word (reference quirk)
    words = CORPUS.split()
    pairs = set(zip(words, words[1:]))
    for _ in range(200):
        n = random.randint(1, 60)
        out = m.generate(n).split()
        assert out[0] == "я" and 1 <= len(out) <= n
        assert all(p in pairs for p in zip(out, out[1:]))
        if len(out) < n:                              # stopped early only at a dead end
            assert out[-1] == "поиграть"
    assert m.generate(1) == "я"
    assert sorted(m.successors("и")) == ["увидел", "я"]
    m2 = N.MarkovModel(1)
    assert not m2.train("single") and m2.starters() == ["single"]


def _stream():
    msgs = [b"INFO {\"max_payload\":1048576}\r\n", b"PING\r\n", b"PONG\r\n", b"+OK\r\n",
            b"-ERR 'Unknown Subject'\r\n"]
    for i in range(30):
        pay = bytes(random.getrandbits(8) for _ in range(random.randint(0, 300)))
        msgs.append(b"MSG subj.%d %d %s%d\r\n" % (i, i, b"reply.x " if i % 2 else b"", len(pay)) + pay + b"\r\n")
        hdr = b"NATS/1.0\r\nK: v\r\n\r\n"
        msgs.append(b"HMSG h.%d 9 %d %d\r\n" % (i, len(hdr), len(hdr) + len(pay)) + hdr + pay + b"\r\n")
        msgs.append(b"PUB p.%d %d\r\n" % (i, len(pay)) + pay + b"\r\n")
        msgs.append(b"SUB foo.* q%d %d\r\nUNSUB %d 5\r\n" % (i, i, i))
    return b"".join(msgs)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.integers(1, 400), min_size=1, max_size=200))
def test_nats_parser_any_chunking(cuts):
    random.seed(1)
    data = _stream()
    whole = N.NatsParser().feed(data)
    p = N.NatsParser()
    got, pos, i = [], 0, 0
    while pos < len(data):
        step = cuts[i % len(cuts)]
        got += p.feed(data[pos:pos + step])
        pos += step
        i += 1
    assert got == whole
    assert len(whole) == 5 + 30 * 5


def test_nats_parser_errors_and_headers():
    with pytest.raises(ValueError, match="Maximum Payload"):
        N.NatsParser(4096, 10).feed(b"PUB a 11\r\n")
    with pytest.raises(ValueError, match="Unknown Protocol"):
        N.NatsParser().feed(b"BOGUS x\r\n")
    assert N.nats_parse_headers(b"NATS/1.0 503\r\n\r\n") == ("503", None, [])
    h = N.nats_headers(None, None, [("A", "1"), ("B", "x y")])
    assert h == b"NATS/1.0\r\nA: 1\r\nB: x y\r\n\r\n"
    assert N.nats_parse_headers(h)[2] == [("A", "1"), ("B", "x y")]


HTML = """<!DOCTYPE html><html><head><title>T</title><script>var x = "<p>no</p>";</script>
<style>p{}</style></head><body><div class="nav"><p>menu</p></div>
<div class="post-content extra"><h1>Main &amp; Title</h1><p>First <b>bold</b> para.<p>Second para
<li>Item &#x41;</li><span>  spaced   text  </span><!-- <p>comment</p> --></div></body></html>"""


def test_html_container_and_selector_order():
    text, container = extract_html_text(HTML)
    assert container == "div.post-content"
    # grouped by selector type (h1, ..., p, li, span), NOT document order (reference quirk);
    # each text node is trimmed but keeps its internal spacing; <li> closes the open <p>
    assert text.split("\n") == ["Main & Title", "First bold para.", "Second para", "Item A",
                                "spaced   text"]
    assert "menu" not in text and "comment" not in text and "var x" not in text


def test_html_priority_and_body_fallback():
    t, c = extract_html_text("<main><p>in main</p></main><article><p>in article</p></article>")
    assert c == "article" and t == "in article"
    t, c = extract_html_text("plain text only, no tags")
    assert c == "body" and t == ""
    t, c = extract_html_text("<body><p>Привет</p><p> </p><h2>Заголовок</h2></body>")
    assert t == "Заголовок\nПривет"
    t, _ = extract_html_text("<div role='main'><ul><li>a<li>b</ul><p>x <span>y</span></p></div>")
    assert t.split("\n") == ["x y", "a", "b", "y"]


def test_http_load_generator_frames_keepalive_responses():
    """csrc/native/loadgen.cpp (the e2e benchmark's client): every pre-built request is answered
    over keep-alive connections, responses are framed by Content-Length (bodies split across
    reads), non-200 replies are counted, not timed."""
    import asyncio
    import threading

    from codename_symbiont_amd.ops._ext import native

    ready = threading.Event()
    port_box = {}

    async def handle(reader, writer):
        try:
            while True:
                head = await reader.readuntil(b"\r\n\r\n")
                status = b"404 Not Found" if b"/missing" in head else b"200 OK"
                body = b'{"pad":"' + b"x" * 70000 + b'"}'   # larger than one 64 KiB read
                writer.write(b"HTTP/1.1 " + status + b"\r\nContent-Length: "
                             + str(len(body)).encode() + b"\r\n\r\n" + body[:1000])
                await writer.drain()
                writer.write(body[1000:])
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            writer.close()

    def serve():
        loop = asyncio.new_event_loop()
        srv = loop.run_until_complete(asyncio.start_server(handle, "127.0.0.1", 0))
        port_box["port"] = srv.sockets[0].getsockname()[1]
        port_box["loop"] = loop
        ready.set()
        loop.run_forever()

    threading.Thread(target=serve, daemon=True).start()
    assert ready.wait(10)
    reqs = [b"GET /ok HTTP/1.1\r\nHost: t\r\n\r\n"] * 300 + [b"GET /missing HTTP/1.1\r\nHost: t\r\n\r\n"] * 5
    r = native().http_load("127.0.0.1", port_box["port"], reqs, 7, 30.0)
    port_box["loop"].call_soon_threadsafe(port_box["loop"].stop)
    assert r["errors"] == 0 and r["non200"] == 5
    assert len(r["latency_s"]) == 300 and min(r["latency_s"]) > 0
    assert r["t_end"] >= r["t_start"]


def test_http_load_generator_stops_when_every_connection_breaks():
    """Connections the server closes are dropped and their requests counted as errors; once no
    connection is left the client returns at once instead of spinning until its timeout."""
    import asyncio
    import threading
    import time

    from codename_symbiont_amd.ops._ext import native

    ready = threading.Event()
    box = {}

    async def handle(reader, writer):
        for _ in range(2):   # two answers, then hang up
            try:
                await reader.readuntil(b"\r\n\r\n")
            except (asyncio.IncompleteReadError, ConnectionError):
                break
            writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\n{}")
            await writer.drain()
        writer.close()

    def serve():
        loop = asyncio.new_event_loop()
        srv = loop.run_until_complete(asyncio.start_server(handle, "127.0.0.1", 0))
        box["port"] = srv.sockets[0].getsockname()[1]
        box["loop"] = loop
        ready.set()
        loop.run_forever()

    threading.Thread(target=serve, daemon=True).start()
    assert ready.wait(10)
    reqs = [b"GET /ok HTTP/1.1\r\nHost: t\r\n\r\n"] * 100
    t0 = time.time()
    r = native().http_load("127.0.0.1", box["port"], reqs, 4, 30.0)
    box["loop"].call_soon_threadsafe(box["loop"].stop)
    assert time.time() - t0 < 10.0
    # 2 answers per connection; under load a hang-up can overtake the 2nd answer (a request the
    # client already sent to the closing socket draws a reset that drops unread bytes)
    assert 4 <= len(r["latency_s"]) <= 8 and len(r["latency_s"]) + r["errors"] == 100, r


def test_search_results_batch_matches_per_request_encoding():
    """vector_memory's one-call burst encoder == search_result_json per request (cached
    fragments, misses through the callback, skipped rows, -1 slots, per-query k, errors)."""
    import numpy as np

    from codename_symbiont_amd.ops._ext import native

    frag = {r: (b'{"qdrant_point_id":"p%d","score":' % r, b',"payload":{"x":%d}}' % r)
            for r in range(0, 40, 2)}
    cache = dict(list(frag.items())[:5])
    calls = []

    def miss(r):
        calls.append(r)
        f = frag.get(r)
        if f is not None:
            cache[r] = f
        return f

    rng = np.random.default_rng(0)
    n, kmax = 6, 5
    scores = rng.standard_normal((n, kmax)).astype(np.float32)
    rows = rng.integers(-1, 40, (n, kmax)).astype(np.int64)
    ks = np.array([5, 3, 0, 5, 1, 4])
    rids = [f"req-{j}" for j in range(n)]
    errs = [None, "boom", None, None, None, "x\"y"]
    bodies, skipped = native().search_results_batch(rids, scores, rows, ks, cache, miss, errs)
    want_skip = 0
    for j in range(n):
        keep, fr = [], []
        for s, r in zip(scores[j, :ks[j]], rows[j, :ks[j]]):
            if r < 0:
                continue
            if int(r) not in frag:
                want_skip += 1
                continue
            keep.append(s)
            fr.append(frag[int(r)])
        want = native().search_result_json(rids[j], np.asarray(keep, np.float32), fr, errs[j])
        assert bodies[j] == want, j
    assert skipped == want_skip and calls
