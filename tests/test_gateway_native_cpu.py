"""The native C++ gateway (csrc/native/gateway.cpp) against the asyncio gateway (services/api.py)
that specifies it: identical status codes, content types and bodies for the reference's request
contract, plus the HTTP mechanics the compiled server implements itself."""
import asyncio
import json
import re

import httpx
import pytest

from codename_symbiont_amd.bus import NatsClient
from codename_symbiont_amd.ops._ext import native

from helpers import broker, cpu_config, gateway


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 120))

# (path, content-type, body): every case runs through both gateways and must answer identically
CASES = [
    ("/api/submit-url", "application/json", b'{"url": "  "}'),
    ("/api/submit-url", "application/json", b'{"url": 5}'),
    ("/api/submit-url", "application/json", b'{"url": null}'),
    ("/api/submit-url", "application/json", b'{}'),
    ("/api/submit-url", "application/json", b'{"url": "a"} x'),
    ("/api/submit-url", "application/json", b'[1, 2]'),
    ("/api/submit-url", "application/json", b'{"url": "\\u00a0 http://x \\u3000"}'),
    ("/api/submit-url", "text/plain", b'{"url": "x"}'),
    ("/api/submit-url", "application/vnd.api+json; charset=utf-8", b'{"url": "x"}'),
    ("/api/submit-url", "application/json", b''),
    ("/api/submit-url", "application/json", b'{"url": "x",}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t", "max_length": -1}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t", "max_length": 4294967296}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t", "max_length": 2.5}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t", "max_length": 1e20}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t", "max_length": true}'),
    ("/api/generate-text", "application/json", b'{"task_id": ["a"], "max_length": 3}'),
    ("/api/generate-text", "application/json", b'{"task_id": {"a": 1}, "max_length": 3}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t", "prompt": 1, "max_length": 3}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t", "prompt": null, "max_length": 3}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t", "max_length": 3, "extra": [1]}'),
    ("/api/generate-text", "application/json", b'{"task_id": "\xd0\xaf", "max_length": 1001}'),
    ("/api/generate-text", "application/json", b'{"task_id": "t"}  \n'),
    ("/api/search/semantic", "application/json", b'{"query_text": "q"}'),
    ("/api/search/semantic", "application/json", b'{"query_text": "q", "top_k": 0.0001}'),
    ("/api/search/semantic", "application/json", b'{"query_text": "q", "top_k": 12345678901234567890}'),
    ("/api/search/semantic", "application/json", b'{"query_text": 1.5e300, "top_k": 3}'),
]


def test_py_float_repr_matches_python():
    N = native()
    for v in (0.0, -0.0, 1.0, 2.5, 0.1, 1e-4, 9.99e-5, 1e-05, 123456789.0, 1e16, 1.5e16, 9999999999999998.0,
              1e20, -3.25e-7, 1.7976931348623157e308, 5e-324, 2.0 ** 60, 0.30000000000000004):
        assert N.py_float_repr(v) == repr(v), v


def test_native_matches_python_gateway_byte_for_byte():
    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url)
            answers = {}
            for impl in ("py", "native"):
                async with gateway(impl, cfg) as url:
                    async with httpx.AsyncClient(timeout=10) as c:
                        got = []
                        for path, ctype, body in CASES:
                            r = await c.post(url + path, content=body, headers={"content-type": ctype})
                            ct = r.headers.get("content-type", "").split(";")[0]
                            text = r.text
                            if r.status_code in (200, 503) and path == "/api/search/semantic":
                                d = r.json()   # the request id is random
                                d["search_request_id"] = len(d["search_request_id"])
                                text = json.dumps(d)
                            got.append((r.status_code, ct, text))
                        answers[impl] = got
            for case, a, n in zip(CASES, answers["py"], answers["native"]):
                assert a == n, (case, a, n)
    run(main())


def test_native_gateway_http_mechanics():
    """keep-alive pipelining, Connection: close, 404/405, health/metrics, CORS preflight."""
    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url)
            async with gateway("native", cfg) as url:
                port = int(url.rsplit(":", 1)[1])
                r, w = await asyncio.open_connection("127.0.0.1", port)
                body = b'{"url": "http://a"}'
                one = (b"POST /api/submit-url HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                       b"Content-Length: %d\r\n\r\n%s" % (len(body), body))
                w.write(one * 3 + b"GET /api/nope HTTP/1.1\r\nHost: x\r\n\r\n"
                        b"GET /api/submit-url HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                data = await asyncio.wait_for(r.read(), 5)      # server closes after the last one
                w.close()
                heads = re.findall(rb"HTTP/1\.1 \d+ [A-Za-z ]+", data)
                assert heads == [b"HTTP/1.1 200 OK"] * 3 + [b"HTTP/1.1 404 Not Found",
                                                             b"HTTP/1.1 405 Method Not Allowed"]
                assert data.count(b"submitted successfully") == 3
                # Expect: 100-continue (curl holds bodies > 1 KiB back until told to send)
                r, w = await asyncio.open_connection("127.0.0.1", port)
                w.write(b"POST /api/submit-url HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                        b"Expect: 100-continue\r\nContent-Length: %d\r\n\r\n" % len(body))
                assert await asyncio.wait_for(r.readline(), 5) == b"HTTP/1.1 100 Continue\r\n"
                assert await r.readline() == b"\r\n"
                w.write(body)
                assert (await asyncio.wait_for(r.readline(), 5)).startswith(b"HTTP/1.1 200")
                w.close()
                async with httpx.AsyncClient(timeout=10) as c:
                    h = (await c.get(url + "/api/health")).json()
                    assert h["status"] == "ok" and h["nats"] is True
                    m = (await c.get(url + "/api/metrics")).json()
                    assert m["api_service"]["counters"]["http.requests"] >= 5
                    r2 = await c.options(url + "/api/generate-text", headers={
                        "origin": "http://127.0.0.1:3000", "access-control-request-method": "DELETE"})
                    assert r2.status_code == 400 and r2.text == "Requested method is not allowed"
                    r3 = await c.post(url + "/api/submit-url", json={"url": "u"},
                                      headers={"origin": "http://marchenzo.dev"})
                    assert r3.status_code == 200
                    assert r3.headers["access-control-allow-origin"] == "http://marchenzo.dev"
    run(main())


def test_native_gateway_sse_broadcast_lag_drop_and_keepalive():
    """Every SSE client gets every event; a client that stops reading keeps only the newest
    `capacity` events (tokio broadcast lag semantics); idle streams carry keep-alive comments."""
    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url, sse_capacity=4, sse_keepalive_s=0.2)
            async with gateway("native", cfg) as url:
                nc = await NatsClient.connect(b.url)
                port = int(url.rsplit(":", 1)[1])
                readers = []
                for _ in range(3):
                    rr, ww = await asyncio.open_connection("127.0.0.1", port)
                    ww.write(b"GET /api/events HTTP/1.1\r\nHost: x\r\n\r\n")
                    readers.append((rr, ww))
                for rr, _ in readers:
                    assert (await rr.readline()).startswith(b"HTTP/1.1 200")
                await asyncio.sleep(0.1)
                N = 20
                for i in range(N):
                    msg = {"original_task_id": f"t{i}", "generated_text": "я тест", "timestamp_ms": i,
                           "ignored": 1}
                    await nc.publish("events.text.generated", json.dumps(msg).encode())
                await nc.publish("events.text.generated", b"not json")    # dropped with a log line
                await nc.flush()

                async def events(rr, want):
                    got = []
                    while len(got) < want:
                        line = await asyncio.wait_for(rr.readline(), 5)
                        if line.startswith(b"data: "):
                            got.append(json.loads(line[6:]))
                    return got
                for rr, _ in readers[:2]:
                    ev = await events(rr, N)
                    assert [e["original_task_id"] for e in ev] == [f"t{i}" for i in range(N)]
                    assert set(ev[0]) == {"original_task_id", "generated_text", "timestamp_ms"}
                    assert ev[0]["generated_text"] == "я тест"
                # keep-alive comment on an idle stream
                rr = readers[0][0]
                while b"keep-alive" not in await asyncio.wait_for(rr.readline(), 5):
                    pass
                for _, ww in readers[:2]:
                    ww.close()
                # reader 2 never read: flood past its socket buffers, then drain it -- it lost
                # events from the middle but still holds the newest `capacity` ones
                big = "x" * 8192
                M = 2000
                for i in range(M):
                    await nc.publish("events.text.generated", json.dumps(
                        {"original_task_id": f"b{i}", "generated_text": big, "timestamp_ms": i}).encode())
                await nc.flush()
                await asyncio.sleep(0.5)
                rr = readers[2][0]
                ids = []
                while not ids or ids[-1] != f"b{M - 1}":   # (keep-alives keep the stream busy)
                    line = await asyncio.wait_for(rr.readline(), 5.0)
                    if line.startswith(b"data: "):
                        ids.append(json.loads(line[6:])["original_task_id"])
                big_ids = [i for i in ids if i.startswith("b")]
                nums = [int(i[1:]) for i in big_ids]
                assert len(nums) < M and nums[-1] == M - 1 and nums == sorted(nums)
                assert nums[0] == 0          # nothing lost before the client lagged
                readers[2][1].close()
                await nc.close()
    run(main())


def test_native_gateway_search_hops_and_timeouts():
    """Two-hop search through fake embedding/index responders: success path, upstream error
    mapping, and the NATS request timeout."""
    async def main():
        async with broker() as b:
            cfg = cpu_config(b.url)
            nc = await NatsClient.connect(b.url)
            mode = {"embed": "ok"}

            async def embedder():
                sub = await nc.subscribe("tasks.embedding.for_query")
                async for m in sub:
                    req = json.loads(m.data)
                    if mode["embed"] == "err":
                        await m.respond(json.dumps({"request_id": req["request_id"], "embedding": None,
                                                    "model_name": None, "error_message": "boom"}).encode())
                    elif mode["embed"] == "garbage":
                        await m.respond(b"{")
                    elif mode["embed"] == "ok":
                        await m.respond(json.dumps({"request_id": req["request_id"],
                                                    "embedding": [0.5, -0.25, 1, 1e-8],
                                                    "model_name": "m"}).encode())

            async def index():
                sub = await nc.subscribe("tasks.search.semantic.request")
                async for m in sub:
                    req = json.loads(m.data)
                    assert req["query_embedding"] == [0.5, -0.25, 1.0, 1e-8] and req["top_k"] == 2
                    item = {"qdrant_point_id": "p1", "score": 0.875, "payload": {
                        "original_document_id": "d", "source_url": "u", "sentence_text": "s",
                        "sentence_order": 3, "model_name": "m", "processed_at_ms": 7}}
                    await m.respond(json.dumps({"request_id": req["request_id"], "results": [item] * 2,
                                                "error_message": None}).encode())
            tasks = [asyncio.create_task(embedder()), asyncio.create_task(index())]
            await nc.flush()
            async with gateway("native", cfg) as url:
                async with httpx.AsyncClient(timeout=20) as c:
                    rs = await asyncio.gather(*[c.post(url + "/api/search/semantic",
                                                       json={"query_text": f"q{i}", "top_k": 2})
                                                for i in range(32)])
                    for r in rs:
                        assert r.status_code == 200, r.text
                        d = r.json()
                        assert d["error_message"] is None and len(d["results"]) == 2
                        assert d["results"][0]["score"] == 0.875
                        assert d["results"][0]["payload"]["sentence_order"] == 3
                    assert len({r.json()["search_request_id"] for r in rs}) == 32
                    mode["embed"] = "err"
                    r = await c.post(url + "/api/search/semantic", json={"query_text": "q", "top_k": 2})
                    assert r.status_code == 500
                    assert r.json()["error_message"] == "Error from preprocessing service: boom"
                    mode["embed"] = "garbage"
                    r = await c.post(url + "/api/search/semantic", json={"query_text": "q", "top_k": 2})
                    assert r.status_code == 500 and r.json()["error_message"] == \
                        "Internal error: Failed to parse embedding service response"
            # a short NATS request timeout: the silent responder times out like async-nats
            from codename_symbiont_amd.services.gateway_native import NativeGateway

            mode["embed"] = "silent"
            gw = NativeGateway(cfg, workers=1, log=False)
            gw._gc.nats_request_timeout_s = 0.3
            await gw.start(host="127.0.0.1", port=0)
            async with httpx.AsyncClient(timeout=20) as c:
                r = await c.post(gw.url + "/api/search/semantic", json={"query_text": "q", "top_k": 2})
            assert r.status_code == 503 and r.json()["error_message"] == \
                "Failed to get embedding from preprocessing service: request timed out"
            await gw.stop()
            for t in tasks:
                t.cancel()
            await nc.close()
    run(main())


def test_native_gateway_reconnects_to_a_restarted_broker():
    async def main():
        from codename_symbiont_amd.bus.broker import NativeBroker
        from codename_symbiont_amd.services.gateway_native import NativeGateway

        b = await NativeBroker().start()
        port = b.port
        gw = await NativeGateway(cpu_config(b.url), workers=1, log=False).start(host="127.0.0.1", port=0)
        await b.stop()
        for _ in range(100):
            if not gw.stats["nats_connected"]:
                break
            await asyncio.sleep(0.02)
        async with httpx.AsyncClient(timeout=10) as c:
            r = await c.get(gw.url + "/api/health")
            assert r.status_code == 503
            r = await c.post(gw.url + "/api/submit-url", json={"url": "x"})
            assert r.status_code == 500
            b2 = await NativeBroker(port=port).start()
            for _ in range(200):
                if gw.stats["nats_connected"]:
                    break
                await asyncio.sleep(0.02)
            r = await c.get(gw.url + "/api/health")
            assert r.status_code == 200
            assert gw.stats["nats_reconnects"] >= 1
        await gw.stop()
        await b2.stop()
    run(main())
