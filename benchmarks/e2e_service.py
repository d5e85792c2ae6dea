#!/usr/bin/env python3
"""End-to-end service benchmark on one GPU: the reference's real usage path, deployed the way
``launch.py`` deploys it (broker, preprocessing, vector_memory and the gateway as separate
processes; the two GPU services share the card) with ``--clients`` client processes.

  ingest : RawTextMessage on data.raw_text.discovered -> preprocessing (native tokenizer + HIP
           encoder, micro-batched) -> data.text.with_embeddings -> vector_memory (HBM index)
           => sentences/s until every point is searchable (polled via /api/metrics counters)
  search : concurrent POST /api/search/semantic -> gateway -> tasks.embedding.for_query (HIP
           encoder) -> tasks.search.semantic.request (fused scan over the pre-filled corpus)
           => requests/s and p50/p99 latency as the clients see them
One JSON line on stdout.

    python benchmarks/e2e_service.py [--docs 200] [--index-rows 10000000] [--requests 4000]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sentences(n: int, seed: int, model: str) -> list[str]:
    import numpy as np

    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.text.tokenizer import Tokenizer

    rng = np.random.default_rng(seed)
    words = [w for w in Tokenizer(get_config(model)).vocab[1000:8000] if w.isalpha()]
    return [" ".join(rng.choice(words, size=int(rng.integers(6, 24)))).capitalize() + "."
            for _ in range(n)]


def _requests(queries: list[str], endpoint: str) -> list[bytes]:
    out = []
    for q in queries:
        if endpoint == "health":
            out.append(b"GET /api/health HTTP/1.1\r\nHost: bench\r\n\r\n")
            continue
        body = json.dumps({"query_text": q, "top_k": 10}).encode()
        out.append(b"POST /api/search/semantic HTTP/1.1\r\nHost: bench\r\n"
                   b"Content-Type: application/json\r\nContent-Length: "
                   + str(len(body)).encode() + b"\r\n\r\n" + body)
    return out


def _client_native(url: str, queries: list[str], conc: int, out, endpoint: str = "search",
                   warmup: int = 0) -> None:
    """C++ epoll client (csrc/native/loadgen.cpp, GIL released): requests pre-built, one in flight
    per keep-alive connection, latency from first byte written to last byte read.  The first
    ``warmup`` requests run untimed (first full-size bursts: allocator growth, cold caches)."""
    try:
        sys.path.insert(0, ROOT)
        from codename_symbiont_amd.ops._ext import native

        host, port = url.split("//")[1].split(":")
        if warmup:
            native().http_load(host, int(port), _requests(queries[:warmup], endpoint), conc, 300.0)
        r = native().http_load(host, int(port), _requests(queries[warmup:], endpoint), conc, 300.0)
        if r["errors"] or r["non200"]:
            raise RuntimeError(f"{r['errors']} transport errors, {r['non200']} non-200 replies")
        out.put((list(r["latency_s"]), r["t_start"], r["t_end"]))
    except BaseException as e:   # never leave the parent waiting on a dead client
        out.put(("error", repr(e)))


def _client(url: str, queries: list[str], conc: int, out, endpoint: str = "search") -> None:
    """Raw asyncio HTTP/1.1 keep-alive client (httpx's per-request cost capped the first version
    of this benchmark at ~420 req/s even on /api/health; one gateway worker serves ~6.5k req/s
    of that endpoint to this client)."""
    host, port = url.split("//")[1].split(":")
    port = int(port)

    async def conn_loop(qs, lat):
        r, w = await asyncio.open_connection(host, port)
        for q in qs:
            if endpoint == "health":
                req = b"GET /api/health HTTP/1.1\r\nHost: bench\r\n\r\n"
            else:
                body = json.dumps({"query_text": q, "top_k": 10}).encode()
                req = (b"POST /api/search/semantic HTTP/1.1\r\nHost: bench\r\n"
                       b"Content-Type: application/json\r\nContent-Length: "
                       + str(len(body)).encode() + b"\r\n\r\n" + body)
            t = time.perf_counter()
            w.write(req)
            await w.drain()
            head = await r.readuntil(b"\r\n\r\n")
            status = int(head.split(b" ", 2)[1])
            n = 0
            for line in head.split(b"\r\n"):
                if line[:15].lower() == b"content-length:":
                    n = int(line[15:])
            await r.readexactly(n)
            if status != 200:
                raise RuntimeError(f"HTTP {status}")
            lat.append(time.perf_counter() - t)
        w.close()

    async def main():
        lat: list[float] = []
        t0 = time.perf_counter()
        await asyncio.gather(*(conn_loop(queries[i::conc], lat) for i in range(conc)))
        return lat, t0, time.perf_counter()

    try:
        out.put(asyncio.run(main()))
    except BaseException as e:   # never leave the parent waiting on a dead client
        out.put(("error", repr(e)))


async def _ingest(nats_url: str, docs: list[str]) -> None:
    from codename_symbiont_amd.bus.client import NatsClient
    from codename_symbiont_amd.wire import RawTextMessage, subjects

    nc = await NatsClient.connect(nats_url, name="bench-ingest")
    for i, d in enumerate(docs):
        await nc.publish(subjects.RAW_TEXT_DISCOVERED,
                         RawTextMessage(f"doc-{i}", f"http://bench/{i}", d, i).to_json())
    await nc.flush()
    await nc.close()


def _metrics(api: str) -> dict:
    import httpx

    return httpx.get(api + "/api/metrics", timeout=10).json()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="minilm-l6")
    ap.add_argument("--docs", type=int, default=200)
    ap.add_argument("--sentences", type=int, default=50)
    ap.add_argument("--index-rows", type=int, default=10_000_000)
    ap.add_argument("--requests", type=int, default=4000)
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--concurrency", type=int, default=64, help="in-flight requests per client")
    ap.add_argument("--api-workers", type=int, default=4)
    ap.add_argument("--api-impl", choices=["native", "py"], default="native",
                    help="native: C++ gateway (worker threads); py: asyncio gateway (worker processes)")
    ap.add_argument("--broker-impl", choices=["native", "py"], default="native")
    ap.add_argument("--endpoint", choices=["search", "health"], default="search")
    ap.add_argument("--client", choices=["native", "py"], default="native",
                    help="load generator: C++ epoll (csrc/native/loadgen.cpp) or asyncio")
    ap.add_argument("--warmup-requests", type=int, default=2000,
                    help="native client: untimed requests first (split over the clients)")
    ap.add_argument("--idle-requests", type=int, default=300,
                    help="after the load phase: this many requests one at a time (unloaded latency)")
    a = ap.parse_args()
    py = sys.executable
    bport, aport = _port(), _port()
    nats = f"nats://127.0.0.1:{bport}"
    api = f"http://127.0.0.1:{aport}"
    env = dict(os.environ, NATS_URL=nats, API_SERVER_HOST="127.0.0.1", API_SERVER_PORT=str(aport),
               SYMB_MODEL=a.model, SYMB_INDEX_FILL_RANDOM=str(a.index_rows),
               SYMB_INDEX_CAPACITY=str(a.index_rows + a.docs * a.sentences + 4096),
               SYMB_LOG="warning", RUST_LOG="warning", SYMB_METRICS_INTERVAL="0.1",
               SYMB_API_WORKERS=str(a.api_workers), SYMB_API_IMPL=a.api_impl,
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    import signal

    signal.signal(signal.SIGTERM, lambda *_: sys.exit(1))   # a timeout still runs the cleanup
    procs = [subprocess.Popen([py, "-m", "codename_symbiont_amd.bus.broker", "--port", str(bport),
                               "--impl", a.broker_impl],
                              env=env, cwd=ROOT, start_new_session=True)]
    time.sleep(0.5)
    for s in ("preprocessing", "vector_memory", "api"):
        procs.append(subprocess.Popen([py, "-m", f"codename_symbiont_amd.services.{s}"], env=env,
                                      cwd=ROOT, start_new_session=True))
    try:
        import httpx
        t_boot = time.time()
        while True:   # ready: the gateway answers and the embedding + index hops respond
            try:
                r = httpx.post(api + "/api/search/semantic", json={"query_text": "warm up", "top_k": 1},
                               timeout=30)
                if r.status_code == 200:
                    break
            except Exception:
                pass
            if time.time() - t_boot > 600:
                raise TimeoutError("services did not come up")
            time.sleep(1.0)
        print(f"[e2e] services up in {time.time() - t_boot:.1f}s", file=sys.stderr, flush=True)
        # ---------------- ingest
        warm = a.warmup_requests if a.client == "native" else 0
        sents = _sentences(a.docs * a.sentences + a.requests + warm, 0, a.model)
        docs = [" ".join(sents[i * a.sentences:(i + 1) * a.sentences]) for i in range(a.docs)]
        queries = sents[a.docs * a.sentences:]
        t0 = time.perf_counter()
        asyncio.run(_ingest(nats, docs))
        target = a.docs * a.sentences
        while True:
            got = (_metrics(api).get("services", {}).get("vector_memory_service", {})
                   .get("counters", {}).get("points_upserted", 0))
            if got >= target:
                break
            if time.perf_counter() - t0 > 600:
                raise TimeoutError(f"ingest stalled at {got}/{target}")
            time.sleep(0.05)
        t_ingest = time.perf_counter() - t0
        # ---------------- search
        q = mp.get_context("spawn").Queue()
        per = [queries[i::a.clients] for i in range(a.clients)]
        if a.client == "native":
            cl = [mp.get_context("spawn").Process(
                target=_client_native, args=(api, p, a.concurrency, q, a.endpoint,
                                             warm // a.clients)) for p in per]
        else:
            cl = [mp.get_context("spawn").Process(target=_client, args=(api, p, a.concurrency, q,
                                                                        a.endpoint))
                  for p in per]
        for p in cl:
            p.start()
        res = []
        while len(res) < len(cl):
            try:
                res.append(q.get(timeout=30))
            except Exception:
                if not any(p.is_alive() for p in cl):
                    raise RuntimeError("search clients died without reporting")
                print(f"[e2e] waiting for clients ({len(res)}/{len(cl)} done)", file=sys.stderr,
                      flush=True)
        for p in cl:
            p.join()
        errs = [r[1] for r in res if r[0] == "error"]
        if errs:
            raise RuntimeError(f"search client failed: {errs[0]}")
        lat = sorted(x for r in res for x in r[0])
        t_search = max(r[2] for r in res) - min(r[1] for r in res)
        m = _metrics(api)
        # ---------------- unloaded latency: one connection, one request in flight
        idle = []
        if a.idle_requests:
            from codename_symbiont_amd.ops._ext import native

            host, port = api.split("//")[1].split(":")
            r = native().http_load(host, int(port),
                                   _requests(queries[:a.idle_requests], a.endpoint), 1, 300.0)
            if r["errors"] or r["non200"]:
                raise RuntimeError(f"idle phase: {r['errors']} errors, {r['non200']} non-200")
            idle = sorted(r["latency_s"])
    finally:   # each service leads its own process group (gateway workers included)
        for p in reversed(procs):
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        for p in procs:
            try:
                p.wait(20)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
    print(json.dumps({
        "metric": "end-to-end service: ingest sentences/s and /api/search/semantic requests/s",
        "value": round(len(lat) / t_search, 1), "unit": "search requests/s", "n_gpus": 1,
        "higher_is_better": True,
        "ingest_sentences_per_s": round(a.docs * a.sentences / t_ingest, 1),
        "search_latency_ms": {"p50": round(1e3 * statistics.median(lat), 2),
                              "p99": round(1e3 * lat[int(0.99 * (len(lat) - 1))], 2)},
        "idle_latency_ms": ({"p50": round(1e3 * statistics.median(idle), 2),
                             "p99": round(1e3 * idle[int(0.99 * (len(idle) - 1))], 2),
                             "n": len(idle)} if idle else None),
        "config": {"model": a.model, "index_rows": a.index_rows + a.docs * a.sentences,
                   "docs": a.docs, "sentences_per_doc": a.sentences, "requests": len(lat),
                   "clients": a.clients, "client_impl": a.client, "warmup_requests": warm,
                   "concurrency_per_client": a.concurrency, "top_k": 10,
                   "deployment": f"{a.broker_impl} broker + preprocessing + vector_memory + "
                                 f"{a.api_impl} gateway x {a.api_workers} workers"},
        "endpoint": a.endpoint,
        "gateway_hops_ms": m.get("api_service", {}).get("latency_ms", {}),
        # per-service stage timers (utils/trace.py) and counters: where each hop's time goes
        "service_stages_ms": {svc: v.get("latency_ms", {})
                              for svc, v in m.get("services", {}).items()},
        "service_counters": {svc: v.get("counters", {})
                             for svc, v in m.get("services", {}).items()},
        "data": "synthetic sentences over the synthetic vocabulary, random-init weights",
    }))


if __name__ == "__main__":
    main()
