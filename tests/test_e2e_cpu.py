"""End-to-end flows on CPU (gloo-free, no GPU): broker + services + HTTP/SSE gateway.

* Markov over NATS (BASELINE config #1): POST /api/generate-text -> text_generator -> SSE event
* ingest: raw text -> preprocessing (fp32 CPU encoder) -> vector_memory -> POST /api/search/semantic
* gateway error contract: 400s, 503 "no responders", CORS.
"""
import asyncio
import json

import httpx
import numpy as np
import pytest

from codename_symbiont_amd.bus import NatsClient
from codename_symbiont_amd.services.preprocessing import PreprocessingService
from codename_symbiont_amd.services.text_generator import TextGeneratorService
from codename_symbiont_amd.services.vector_memory import VectorMemoryService
from codename_symbiont_amd.wire import RawTextMessage, subjects

from helpers import broker, cpu_config, gateway


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 120))


async def _read_sse_event(client, url, trigger):
    async with client.stream("GET", url + "/api/events") as r:
        assert r.headers["content-type"].startswith("text/event-stream")
        await trigger()
        async for line in r.aiter_lines():
            if line.startswith("data: "):
                return json.loads(line[6:])


@pytest.mark.parametrize("gw", ["py", "native"])
def test_generate_text_to_sse(gw):
    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url)
            gen = await TextGeneratorService(cfg, seed=1).start()
            gwc = gateway(gw, cfg)
            url = await gwc.__aenter__()
            nc = await NatsClient.connect(b.url)
            async with httpx.AsyncClient(timeout=10) as c:
                async def trigger():
                    await asyncio.sleep(0.2)
                    r = await c.post(url + "/api/generate-text",
                                     json={"task_id": "t-1", "prompt": "hi", "max_length": 12})
                    assert r.status_code == 200
                    assert r.json() == {"message": "Text generation task (id: t-1) submitted successfully.",
                                        "task_id": "t-1"}
                ev = await asyncio.wait_for(_read_sse_event(c, url, trigger), 20)
            assert ev["original_task_id"] == "t-1"
            words = ev["generated_text"].split()
            assert 1 <= len(words) <= 12 and words[0] == "я"   # reference starter quirk
            assert set(ev) == {"original_task_id", "generated_text", "timestamp_ms"}
            await gwc.__aexit__(None, None, None)
            await nc.close()
            await gen.stop()
    run(main())


@pytest.mark.parametrize("gw", ["py", "native"])
def test_gateway_serves_ui_page(gw):
    """C9: the gateway serves the single-page client with the reference's three features."""
    async def main():
        async with broker() as b:
            gwc = gateway(gw, cpu_config(b.url))
            url = await gwc.__aenter__()
            nc = await NatsClient.connect(b.url)
            async with httpx.AsyncClient(timeout=10) as c:
                r = await c.get(url + "/")
            assert r.status_code == 200 and r.headers["content-type"].startswith("text/html")
            html = r.text
            for needle in ('id="url-form"', 'id="gen-form"', 'id="search-form"', "/submit-url",
                           "/generate-text", "/search/semantic", "EventSource", "Codename: Symbiont UI"):
                assert needle in html, needle
            await gwc.__aexit__(None, None, None)
            await nc.close()
    run(main())


@pytest.mark.parametrize("gw", ["py", "native"])
def test_gateway_validation_and_no_responders(gw):
    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url)
            gwc = gateway(gw, cfg)
            url = await gwc.__aenter__()
            nc = await NatsClient.connect(b.url)
            async with httpx.AsyncClient(timeout=10) as c:
                r = await c.post(url + "/api/submit-url", json={"url": "   "})
                assert r.status_code == 400 and r.json() == {"message": "URL cannot be empty", "task_id": None}
                r = await c.post(url + "/api/submit-url", json={"url": " http://x.org/a "})
                assert r.status_code == 200
                assert r.json()["message"] == "Task to scrape URL 'http://x.org/a' submitted successfully."
                r = await c.post(url + "/api/generate-text", json={"task_id": " ", "max_length": 5})
                assert r.status_code == 400 and r.json()["message"] == "task_id cannot be empty"
                r = await c.post(url + "/api/generate-text", json={"task_id": "a", "max_length": 0})
                assert r.status_code == 400
                assert r.json() == {"message": "max_length must be between 1 and 1000", "task_id": "a"}
                r = await c.post(url + "/api/generate-text", json={"task_id": "a", "max_length": 1001})
                assert r.status_code == 400
                r = await c.post(url + "/api/generate-text", content=b"{}",
                                 headers={"content-type": "application/json"})
                assert r.status_code == 400 and r.text.startswith("Json deserialize error: missing field")
                r = await c.post(url + "/api/generate-text", content=b"x", headers={"content-type": "text/plain"})
                assert r.status_code == 400 and r.text == "Content type error"
                # nobody serves tasks.embedding.for_query -> fast 503 (no responders)
                r = await c.post(url + "/api/search/semantic", json={"query_text": "q", "top_k": 3})
                assert r.status_code == 503
                body = r.json()
                assert body["results"] == [] and body["error_message"] == \
                    "Failed to get embedding from preprocessing service: no responders"
                assert len(body["search_request_id"]) == 36
                # CORS
                r = await c.options(url + "/api/search/semantic", headers={
                    "origin": "http://localhost:3000", "access-control-request-method": "POST"})
                assert r.status_code == 200
                assert r.headers["access-control-allow-origin"] == "http://localhost:3000"
                assert r.headers["access-control-max-age"] == "3600"
                r = await c.post(url + "/api/submit-url", json={"url": "u"},
                                 headers={"origin": "http://evil.example"})
                assert r.status_code == 400
            await gwc.__aexit__(None, None, None)
            await nc.close()
    run(main())


@pytest.mark.parametrize("gw", ["py", "native"])
def test_ingest_then_semantic_search_cpu(gw):
    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url)
            pre = await PreprocessingService(cfg).start()
            vm = await VectorMemoryService(cfg).start()
            gwc = gateway(gw, cfg)
            url = await gwc.__aenter__()
            nc = await NatsClient.connect(b.url)
            text = ("The GPU index keeps every vector in HBM.   It answers cosine queries! "
                    "Markov chains generate text? Neo4j stores the graph")
            raw = RawTextMessage("doc-1", "http://example.org/p", text, 123)
            await nc.publish(subjects.RAW_TEXT_DISCOVERED, raw.to_json())
            for _ in range(200):
                if vm.store.count >= 4:
                    break
                await asyncio.sleep(0.05)
            assert vm.store.count == 4
            async with httpx.AsyncClient(timeout=30) as c:
                r = await c.post(url + "/api/search/semantic",
                                 json={"query_text": "It answers cosine queries!", "top_k": 3})
            assert r.status_code == 200, r.text
            body = r.json()
            assert body["error_message"] is None and len(body["results"]) == 3
            top = body["results"][0]
            assert top["payload"]["sentence_text"] == "It answers cosine queries!"
            assert top["payload"]["sentence_order"] == 1
            assert top["payload"]["original_document_id"] == "doc-1"
            assert top["payload"]["source_url"] == "http://example.org/p"
            assert top["payload"]["model_name"] == "sentence-transformers/all-MiniLM-L6-v2"
            assert top["score"] > 0.999
            scores = [x["score"] for x in body["results"]]
            assert scores == sorted(scores, reverse=True)
            await gwc.__aexit__(None, None, None)
            await nc.close()
            await pre.stop()
            await vm.stop()
    run(main())


@pytest.mark.parametrize("gw", ["py", "native"])
def test_url_to_search_pipeline_with_fixture_site(gw):
    """POST /api/submit-url -> perception (local fixture site) -> preprocessing -> vector_memory
    -> POST /api/search/semantic, plus the restored tokenized feed."""
    from aiohttp import web

    from codename_symbiont_amd.services.perception import PerceptionService
    from codename_symbiont_amd.wire import TokenizedTextMessage

    page = ("<html><body><nav><p>menu</p></nav><article><h1>Vector search on MI355X</h1>"
            "<p>The fused kernel scans rows in HBM. It keeps the top scores per query.</p>"
            "<li>Queries are batched</li></article></body></html>")

    async def main():
        app = web.Application()
        app.router.add_get("/doc", lambda r: web.Response(text=page, content_type="text/html"))
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        async with broker() as b:
            cfg = cpu_config(b.url)
            per = await PerceptionService(cfg).start()
            pre = await PreprocessingService(cfg).start()
            vm = await VectorMemoryService(cfg).start()
            gwc = gateway(gw, cfg)
            url = await gwc.__aenter__()
            nc = await NatsClient.connect(b.url)
            tok_sub = await nc.subscribe(subjects.PROCESSED_TEXT_TOKENIZED)
            async with httpx.AsyncClient(timeout=30) as c:
                r = await c.post(url + "/api/submit-url", json={"url": f"http://127.0.0.1:{port}/doc"})
                assert r.status_code == 200
                for _ in range(300):
                    if vm.store.count >= 3:
                        break
                    await asyncio.sleep(0.05)
                assert vm.store.count == 3   # "Vector search on MI355X The fused ... HBM." / "It keeps..." / "Queries are batched"
                tm = TokenizedTextMessage.from_json((await tok_sub.next_msg(5)).data)
                assert "MI355X" in tm.tokens and len(tm.sentences) == 3
                r = await c.post(url + "/api/search/semantic",
                                 json={"query_text": "It keeps the top scores per query.", "top_k": 2})
            res = r.json()["results"]
            assert res[0]["payload"]["sentence_text"] == "It keeps the top scores per query."
            assert res[0]["payload"]["source_url"] == f"http://127.0.0.1:{port}/doc"
            await gwc.__aexit__(None, None, None)
            await nc.close()
            for s in (per, pre, vm):
                await s.stop()
        await runner.cleanup()
    run(main())


def test_search_and_query_embedding_bursts_are_answered_per_request():
    """Bursts of concurrent requests are decoded, scanned/encoded and answered as batches
    (vector_memory / preprocessing batch handlers); each reply must still be its own request's,
    with its own top_k, and malformed requests in the same burst get their error replies."""
    from codename_symbiont_amd.wire import (QueryEmbeddingResult, QueryForEmbeddingTask,
                                            SemanticSearchNatsResult, SemanticSearchNatsTask)

    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url)
            pre = await PreprocessingService(cfg).start()
            vm = await VectorMemoryService(cfg).start()
            nc = await NatsClient.connect(b.url)
            sents = ["Alpha beta gamma.", "Delta epsilon zeta!", "Eta theta iota?", "Kappa lambda mu"]
            raw = RawTextMessage("doc-b", "http://example.org/b", " ".join(sents), 1)
            await nc.publish(subjects.RAW_TEXT_DISCOVERED, raw.to_json())
            for _ in range(200):
                if vm.store.count >= 4:
                    break
                await asyncio.sleep(0.05)
            assert vm.store.count == 4

            async def embed(i):
                t = QueryForEmbeddingTask(f"q{i}", sents[i % 4])
                m = await nc.request(subjects.EMBEDDING_FOR_QUERY, t.to_json(), timeout=30)
                return QueryEmbeddingResult.from_json(m.data)
            embs = await asyncio.gather(*[embed(i) for i in range(48)])
            for i, e in enumerate(embs):
                assert e.request_id == f"q{i}" and e.error_message is None
            bad = await nc.request(subjects.EMBEDDING_FOR_QUERY, b'{"request_id": 5}', timeout=30)
            assert "Failed to deserialize QueryForEmbeddingTask" in \
                QueryEmbeddingResult.from_json(bad.data).error_message

            async def search(i):
                if i % 16 == 15:   # wrong dimension inside the burst
                    t = SemanticSearchNatsTask(f"s{i}", np.ones(7, np.float32), 2)
                else:
                    t = SemanticSearchNatsTask(f"s{i}", embs[i].embedding, 1 + i % 4)
                m = await nc.request(subjects.SEARCH_SEMANTIC_REQUEST, t.to_json(), timeout=30)
                return SemanticSearchNatsResult.from_json(m.data)
            res = await asyncio.gather(*[search(i) for i in range(48)])
            for i, r in enumerate(res):
                assert r.request_id == f"s{i}"
                if i % 16 == 15:
                    assert "Vector dimension error" in r.error_message and not r.results
                    continue
                assert r.error_message is None and len(r.results) == 1 + i % 4
                assert r.results[0].payload.sentence_text == sents[i % 4]
            assert vm.metrics.snapshot()["counters"].get("search.launches", 0) >= 1
            await nc.close()
            await pre.stop()
            await vm.stop()
    run(main())
