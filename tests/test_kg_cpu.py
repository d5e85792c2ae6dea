"""Knowledge-graph path: PackStream codec, Bolt client vs the fake Bolt server, the service's graph
format (reference Cypher) end to end from a TokenizedTextMessage on NATS."""
import asyncio
import math

import pytest
from hypothesis import given, settings, strategies as st

from codename_symbiont_amd.kg.bolt import Graph, Structure, pack, unpack
from codename_symbiont_amd.kg.fake_server import FakeBoltServer
from codename_symbiont_amd.services.knowledge_graph import KnowledgeGraphService
from codename_symbiont_amd.wire import TokenizedTextMessage, subjects

from helpers import broker, cpu_config

values = st.recursive(
    st.none() | st.booleans() | st.integers(-2**63, 2**63 - 1) |
    st.floats(allow_nan=False) | st.text(max_size=300) | st.binary(max_size=300),
    lambda ch: st.lists(ch, max_size=20) | st.dictionaries(st.text(max_size=20), ch, max_size=20),
    max_leaves=40)


@settings(max_examples=300, deadline=None)
@given(values)
def test_packstream_roundtrip(v):
    assert unpack(pack(v)) == v


def test_packstream_markers():
    assert pack(None) == b"\xC0" and pack(True) == b"\xC3" and pack(False) == b"\xC2"
    assert pack(1) == b"\x01" and pack(-16) == b"\xF0" and pack(-17) == b"\xC8\xEF"
    assert pack(128) == b"\xC9\x00\x80" and pack(2**31) == b"\xCB\x00\x00\x00\x00\x80\x00\x00\x00"
    assert pack("a") == b"\x81a" and pack([]) == b"\x90" and pack({}) == b"\xA0"
    assert pack(1.0) == b"\xC1\x3F\xF0\x00\x00\x00\x00\x00\x00"
    assert pack("x" * 16)[:2] == b"\xD0\x10"
    s = Structure(0x4E, [1, ["L"], {}])
    assert unpack(pack(s)) == s


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


def test_bolt_client_tx_and_failure_recovery():
    async def main():
        srv = await FakeBoltServer().start()
        g = Graph(srv.uri, "neo4j", "pw")
        assert await g.run("RETURN 1") == [{"1": 1}]
        from codename_symbiont_amd.kg.bolt import BoltError
        with pytest.raises(BoltError):
            await g.run("MATCH (n) RETURN n")          # unsupported -> FAILURE
        assert await g.run("RETURN 1") == [{"1": 1}]    # RESET recovered the connection
        await g.close()
        await srv.stop()
    run(main())


def test_kg_service_graph_format_over_nats():
    async def main():
        srv = await FakeBoltServer().start()
        async with broker() as b:
            cfg = cpu_config(b.url, neo4j_uri=srv.uri)
            kg = await KnowledgeGraphService(cfg).start()
            await asyncio.wait_for(kg.schema_ready.wait(), 10)
            msg = TokenizedTextMessage("doc-9", "http://s/1", ["Hello", " ", "world", "HELLO", "!"],
                                       ["Hello world.", "  ", "Second one!"], 1700000000123)
            await kg.nc.publish(subjects.PROCESSED_TEXT_TOKENIZED, msg.to_json())
            for _ in range(100):
                if srv.graph.by_label("Document"):
                    break
                await asyncio.sleep(0.05)
            await asyncio.sleep(0.1)
            g = srv.graph
            docs = g.by_label("Document")
            assert len(docs) == 1
            d = docs[0]
            assert d["original_id"] == "doc-9" and d["source_url"] == "http://s/1"
            assert d["processed_at_ms"] == "1700000000123"          # stored as a string
            assert isinstance(d["created_at_ms"], int)
            sents = {s["text"] for s in g.by_label("Sentence")}
            assert sents == {"Hello world.", "Second one!"}          # empty sentence skipped
            orders = sorted(r["props"]["order"] for r in g.rels_of("HAS_SENTENCE"))
            assert orders == [0, 2]                                  # index kept across the skip
            toks = {t["text_lc"]: t["text_original_case"] for t in g.by_label("Token")}
            assert toks == {"hello": "HELLO", "world": "world", "!": "!"}   # last write wins
            assert len(g.rels_of("CONTAINS_TOKEN")) == 3
            assert g.constraints == {"Document.original_id"} and g.indexes == {"token_text_lc_index"}
            # idempotent: the same message again creates nothing new
            await kg.nc.publish(subjects.PROCESSED_TEXT_TOKENIZED, msg.to_json())
            await asyncio.sleep(0.3)
            assert len(srv.graph.by_label("Sentence")) == 2 and len(srv.graph.rels_of("CONTAINS_TOKEN")) == 3
            await kg.stop()
        await srv.stop()
    run(main())


def test_kg_transaction_rolls_back_on_failure():
    async def main():
        srv = await FakeBoltServer().start()
        async with broker() as b:
            cfg = cpu_config(b.url, neo4j_uri=srv.uri)
            kg = KnowledgeGraphService(cfg)
            await kg.connect()
            msg = TokenizedTextMessage("doc-x", "u", ["a", "b"], ["s1.", "s2."], 5)
            # fail the 3rd statement of the transaction: nothing may be committed
            from codename_symbiont_amd.kg import fake_server as fs
            real = fs.execute
            calls = {"n": 0}

            def flaky(g, q, p):
                calls["n"] += 1
                if calls["n"] == 3:
                    raise fs.CypherError("Neo.TransientError.Transaction.Outdated", "boom")
                return real(g, q, p)
            fs.execute = flaky
            try:
                from codename_symbiont_amd.kg.bolt import BoltError
                with pytest.raises(BoltError):
                    await kg.save(msg)
            finally:
                fs.execute = real
            assert srv.graph.by_label("Document") == []              # rolled back
            await kg.save(msg)                                       # connection still usable
            assert len(srv.graph.by_label("Document")) == 1
            await kg.graph.close()
            await kg.nc.close()
        await srv.stop()
    run(main())
