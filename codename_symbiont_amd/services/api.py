"""api_service: HTTP gateway + SSE hub (services/api_service/src/main.rs).

Routes (main.rs:575-581), identical paths / status codes / JSON bodies:
  POST /api/submit-url       {"url"}                       -> publish PerceiveUrlTask
  POST /api/generate-text    GenerateTextTask              -> publish on tasks.generation.text
  GET  /api/events           text/event-stream of GeneratedTextMessage JSON (broadcast to all)
  POST /api/search/semantic  SemanticSearchApiRequest      -> 2-hop NATS request/reply
Additions (no effect on the reference contract): GET /api/metrics, GET /api/health, GET / (UI).

Extractor behaviour of actix ``web::Json`` is reproduced: non-JSON content type -> 400
"Content type error"; undecodable body -> 400 "Json deserialize error: <serde message>";
body over 2 MiB -> 413.  CORS (main.rs:555-567): origins starting with http://localhost,
http://marchenzo or http://127.0.0.1; GET/POST/OPTIONS; Authorization/Accept/Content-Type;
max-age 3600.  SSE: one broadcast channel of capacity 32 (a lagging client loses the oldest
messages, main.rs:201-207, :537), keep-alive every 15 s (:212).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time
import uuid

from ..bus.client import NatsError, NoRespondersError, RequestTimeoutError
from ..ops._ext import native
from ..utils import log as ulog
from ..wire import (ApiResponse, GeneratedTextMessage, GenerateTextTask, PerceiveUrlTask,
                    QueryEmbeddingResult, QueryForEmbeddingTask, SemanticSearchApiRequest,
                    SemanticSearchApiResponse, SemanticSearchNatsResult, SemanticSearchNatsTask,
                    SubmitUrlApiPayload, WireError, subjects)
from .base import Service

JSON_LIMIT = 2 * 1024 * 1024
CORS_PREFIXES = (b"http://localhost", b"http://marchenzo", b"http://127.0.0.1")
CORS_METHODS = "GET, OPTIONS, POST"
CORS_HEADERS = "accept, authorization, content-type"


class SseHub:
    """tokio::sync::broadcast(capacity) semantics over asyncio queues."""

    def __init__(self, capacity: int = 32):
        self.capacity = capacity
        self.clients: set[asyncio.Queue] = set()
        self.lagged = 0

    def subscribe(self) -> asyncio.Queue:
        q: asyncio.Queue = asyncio.Queue(maxsize=self.capacity)
        self.clients.add(q)
        return q

    def unsubscribe(self, q: asyncio.Queue) -> None:
        self.clients.discard(q)

    def send(self, payload: str) -> int:
        for q in list(self.clients):
            if q.full():  # receiver lagged: the oldest message is lost
                try:
                    q.get_nowait()
                except asyncio.QueueEmpty:
                    pass
                self.lagged += 1
            q.put_nowait(payload)
        return len(self.clients)


def _json_response(model, status: int = 200):
    from starlette.responses import Response

    return Response(model.to_json(), status_code=status, media_type="application/json")


class ApiService(Service):
    name = "api_service"

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.hub = SseHub(self.cfg.sse_capacity)
        self.service_metrics: dict[str, dict] = {}
        self.server = None

    # ------------------------------------------------------------------ NATS side
    async def setup(self) -> None:
        self.log.info("[NATS_SSE_Bridge] Subscribing to NATS subject: %s", subjects.TEXT_GENERATED)
        await self.subscribe_loop(subjects.TEXT_GENERATED, self._on_generated)
        msub = await self.nc.subscribe("metrics.>")

        async def metrics_loop():
            async for m in msub:
                try:
                    d = json.loads(m.data)
                    self.service_metrics[d.get("service", m.subject)] = d
                except ValueError:
                    pass
        self._loops.append(asyncio.create_task(metrics_loop()))

    async def _on_generated(self, msg) -> None:
        try:
            gm = GeneratedTextMessage.from_json(msg.data)
        except WireError as e:
            self.log.error("[NATS_SSE_Bridge] Failed to deserialize GeneratedTextMessage from NATS: %s", e)
            return
        n = self.hub.send(gm.to_json().decode())
        if n == 0:
            self.log.warning("[NATS_SSE_Bridge] Failed to send message to broadcast channel "
                             "(no active SSE receivers?)")
        else:
            self.log.info("[NATS_SSE_Bridge] Forwarded GeneratedTextMessage (task_id: %s) to SSE "
                          "broadcast channel.", gm.original_task_id)

    # ------------------------------------------------------------------ HTTP side
    async def _read_json(self, request, model):
        """actix web::Json<T> extractor semantics -> (value, None) or (None, error response)."""
        from starlette.responses import PlainTextResponse

        ctype = request.headers.get("content-type", "").split(";")[0].strip().lower()
        if not (ctype == "application/json" or ctype.endswith("+json")):
            return None, PlainTextResponse("Content type error", status_code=400)
        body = await request.body()
        if len(body) > JSON_LIMIT:
            return None, PlainTextResponse(
                f"JSON payload ({len(body)} bytes) is larger than allowed (limit: {JSON_LIMIT} bytes).",
                status_code=413)
        try:
            return model.from_json(body), None
        except WireError as e:
            return None, PlainTextResponse(f"Json deserialize error: {e}", status_code=400)

    async def submit_url(self, request):
        payload, err = await self._read_json(request, SubmitUrlApiPayload)
        if err is not None:
            return err
        url = native().rust_trim(payload.url)
        if not url:
            self.log.warning("[API_SUBMIT_URL] Received empty URL")
            return _json_response(ApiResponse("URL cannot be empty", None), 400)
        self.log.info("[API_SUBMIT_URL] Received request to scrape URL: %s", url)
        try:
            await self.publish(subjects.PERCEIVE_URL, PerceiveUrlTask(url).to_json())
        except (NatsError, OSError) as e:
            self.log.error("[API_SUBMIT_URL] Failed to publish PerceiveUrlTask to NATS: %s", e)
            return _json_response(ApiResponse("Failed to publish task to processing queue", None), 500)
        return _json_response(ApiResponse(f"Task to scrape URL '{url}' submitted successfully.", None))

    async def generate_text(self, request):
        task, err = await self._read_json(request, GenerateTextTask)
        if err is not None:
            return err
        self.log.info("[API] /api/generate-text called with task_id: %s", task.task_id)
        if not native().rust_trim(task.task_id):
            self.log.warning("[API_GENERATE_TEXT] Received task with empty task_id")
            return _json_response(ApiResponse("task_id cannot be empty", None), 400)
        if task.max_length == 0 or task.max_length > self.cfg.max_length_limit:
            self.log.warning("[API_GENERATE_TEXT] Received task with invalid max_length: %d",
                             task.max_length)
            return _json_response(ApiResponse(
                f"max_length must be between 1 and {self.cfg.max_length_limit}", task.task_id), 400)
        try:
            await self.publish(subjects.GENERATE_TEXT, task.to_json())
        except (NatsError, OSError) as e:
            self.log.error("[API_GENERATE_TEXT] Failed to publish GenerateTextTask (id: %s) to NATS: %s",
                           task.task_id, e)
            return _json_response(ApiResponse("Failed to publish generation task to queue",
                                              task.task_id), 500)
        return _json_response(ApiResponse(
            f"Text generation task (id: {task.task_id}) submitted successfully.", task.task_id))

    async def events(self, request):
        from starlette.responses import StreamingResponse

        self.log.info("[API_SSE] New SSE client connected to /api/events")
        q = self.hub.subscribe()
        keepalive = self.cfg.sse_keepalive_s

        async def stream():
            try:
                while True:
                    try:
                        payload = await asyncio.wait_for(q.get(), keepalive)
                        yield f"data: {payload}\n\n".encode()
                    except asyncio.TimeoutError:
                        yield b": keep-alive\n\n"
            finally:
                self.hub.unsubscribe(q)

        return StreamingResponse(stream(), media_type="text/event-stream",
                                 headers={"Cache-Control": "no-cache"})

    async def semantic_search(self, request):
        req, err = await self._read_json(request, SemanticSearchApiRequest)
        if err is not None:
            return err
        rid = str(uuid.uuid4())
        t0 = time.perf_counter()

        def fail(status, msg):
            return _json_response(SemanticSearchApiResponse(rid, [], msg), status)

        self.log.info("[API_SEARCH_HANDLER] Received semantic search request (client_req_id: %s): "
                      "query='%s', top_k=%d", rid, req.query_text, req.top_k)
        task = QueryForEmbeddingTask(rid, req.query_text)
        try:
            resp = await asyncio.wait_for(
                self.nc.request(subjects.EMBEDDING_FOR_QUERY, task.to_json()),
                self.cfg.embed_timeout_s)
        except (NoRespondersError, RequestTimeoutError, NatsError) as e:
            self.log.error("[API_SEARCH_HANDLER] NATS request for embedding failed (client_req_id: %s): %s", rid, e)
            return fail(503, f"Failed to get embedding from preprocessing service: {e}")
        except asyncio.TimeoutError:
            return fail(503, "Timeout: Failed to get embedding from preprocessing service within "
                             f"{int(self.cfg.embed_timeout_s)} seconds")
        try:
            er = QueryEmbeddingResult.from_json(resp.data)
        except WireError:
            return fail(500, "Internal error: Failed to parse embedding service response")
        if er.error_message is not None:
            return fail(500, f"Error from preprocessing service: {er.error_message}")
        if er.embedding is None:
            return fail(500, "Preprocessing service did not return an embedding.")
        t1 = time.perf_counter()
        stask = SemanticSearchNatsTask(rid, er.embedding, req.top_k)
        try:
            resp = await asyncio.wait_for(
                self.nc.request(subjects.SEARCH_SEMANTIC_REQUEST, stask.to_json()),
                self.cfg.search_timeout_s)
        except (NoRespondersError, RequestTimeoutError, NatsError) as e:
            self.log.error("[API_SEARCH_HANDLER] NATS request for search failed (client_req_id: %s): %s", rid, e)
            return fail(503, f"Failed to get search results from vector memory service: {e}")
        except asyncio.TimeoutError:
            return fail(503, "Timeout: Failed to get search results from vector memory service "
                             f"within {int(self.cfg.search_timeout_s)} seconds")
        try:
            sr = SemanticSearchNatsResult.from_json(resp.data)
        except WireError:
            return fail(500, "Internal error: Failed to parse search service response")
        if sr.error_message is not None:
            return fail(500, f"Error from vector memory service: {sr.error_message}")
        t2 = time.perf_counter()
        self.metrics.observe("search.embed_hop", (t1 - t0) * 1e3)
        self.metrics.observe("search.index_hop", (t2 - t1) * 1e3)
        self.metrics.inc("search.requests")
        self.log.info("[API_SEARCH_HANDLER] Successfully received %d search results for client_req_id: %s",
                      len(sr.results), rid)
        resp = _json_response(SemanticSearchApiResponse(rid, sr.results, None))
        self.metrics.observe("search.handler", (time.perf_counter() - t0) * 1e3)
        return resp

    async def metrics_ep(self, request):
        from starlette.responses import JSONResponse

        return JSONResponse({"api_service": self.metrics.snapshot(), "sse_clients": len(self.hub.clients),
                             "sse_lagged": self.hub.lagged, "services": self.service_metrics})

    async def health(self, request):
        from starlette.responses import JSONResponse

        ok = self.nc is not None and self.nc.is_connected
        return JSONResponse({"status": "ok" if ok else "degraded", "nats": ok},
                            status_code=200 if ok else 503)

    async def index_page(self, request):
        from starlette.responses import HTMLResponse, PlainTextResponse

        path = os.path.join(os.path.dirname(__file__), "static", "index.html")
        if not os.path.exists(path):
            return PlainTextResponse("symbiont api", status_code=200)
        with open(path, encoding="utf-8") as f:
            return HTMLResponse(f.read())

    def app(self):
        from starlette.applications import Starlette
        from starlette.routing import Route

        routes = [
            Route("/api/submit-url", self.submit_url, methods=["POST"]),
            Route("/api/generate-text", self.generate_text, methods=["POST"]),
            Route("/api/events", self.events, methods=["GET"]),
            Route("/api/search/semantic", self.semantic_search, methods=["POST"]),
            Route("/api/metrics", self.metrics_ep, methods=["GET"]),
            Route("/api/health", self.health, methods=["GET"]),
            Route("/", self.index_page, methods=["GET"]),
        ]
        return CorsMiddleware(Starlette(routes=routes))

    async def serve(self, host: str | None = None, port: int | None = None):
        import uvicorn

        import socket

        config = uvicorn.Config(self.app(), host=host or self.cfg.api_host,
                                port=self.cfg.api_port if port is None else port,
                                log_level="warning", lifespan="off",
                                # actix keeps connections 5 s like uvicorn; a longer idle keep-alive
                                # avoids close-vs-reuse races with pooled clients under load
                                timeout_keep_alive=75)
        self.server = uvicorn.Server(config)
        self.log.info("[HTTP_SERVER] Starting API HTTP server at http://%s:%s", config.host, config.port)
        if self.cfg.api_workers > 1:   # every worker binds the same port; the kernel balances
            sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
            sock.bind((config.host, config.port))
            sock.listen(2048)
            await self.server.serve(sockets=[sock])
        else:
            await self.server.serve()

    async def run_forever(self) -> None:
        await self.start()
        try:
            await self.serve()
        finally:
            await self.stop()


class CorsMiddleware:
    """actix-cors configuration of the reference as a tiny ASGI middleware."""

    def __init__(self, app):
        self.app = app

    @staticmethod
    def _allowed(origin: bytes) -> bool:
        return any(origin.startswith(p) for p in CORS_PREFIXES)

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        headers = dict(scope.get("headers") or [])
        origin = headers.get(b"origin")
        if origin is None:
            return await self.app(scope, receive, send)
        if not self._allowed(origin):
            await _plain(send, 400, b"Origin is not allowed to make this request")
            return
        if scope["method"] == "OPTIONS" and b"access-control-request-method" in headers:
            req_m = headers[b"access-control-request-method"].decode().upper()
            if req_m not in ("GET", "POST", "OPTIONS"):
                await _plain(send, 400, b"Requested method is not allowed")
                return
            await send({"type": "http.response.start", "status": 200, "headers": [
                (b"access-control-allow-origin", origin),
                (b"access-control-allow-methods", CORS_METHODS.encode()),
                (b"access-control-allow-headers", CORS_HEADERS.encode()),
                (b"access-control-max-age", b"3600"), (b"vary", b"Origin"),
                (b"content-length", b"0")]})
            await send({"type": "http.response.body", "body": b""})
            return

        async def send_with_cors(message):
            if message["type"] == "http.response.start":
                message = dict(message)
                message["headers"] = list(message.get("headers", [])) + [
                    (b"access-control-allow-origin", origin), (b"vary", b"Origin")]
            await send(message)

        await self.app(scope, receive, send_with_cors)


async def _plain(send, status: int, body: bytes) -> None:
    await send({"type": "http.response.start", "status": status,
                "headers": [(b"content-type", b"text/plain; charset=utf-8"),
                            (b"content-length", str(len(body)).encode())]})
    await send({"type": "http.response.body", "body": body})


def main() -> None:
    import subprocess
    import sys

    ulog.setup(ApiService.name, "info")
    cfg = ApiService().cfg
    if "NATS_URL" not in os.environ:
        cfg.nats_url = "nats://cs-nats:4222"  # the reference's api default (main.rs:519-524)
    if os.environ.get("SYMB_API_IMPL", "native") == "native":
        # the compiled gateway (csrc/native/gateway.cpp): api_workers epoll threads in-process
        from .gateway_native import serve_forever

        serve_forever(cfg)
        return
    import signal

    kids = []
    if cfg.api_workers > 1 and not os.environ.get("SYMB_API_CHILD"):
        # extra gateway workers as CHILD processes on the same SO_REUSEPORT port; they die with
        # this process (PR_SET_PDEATHSIG) and SIGTERM unwinds through the cleanup below
        def _die_with_parent():
            import ctypes
            ctypes.CDLL("libc.so.6").prctl(1, signal.SIGTERM)   # PR_SET_PDEATHSIG
        env = dict(os.environ, SYMB_API_CHILD="1", NATS_URL=cfg.nats_url)
        kids = [subprocess.Popen([sys.executable, "-m", "codename_symbiont_amd.services.api"], env=env,
                                 preexec_fn=_die_with_parent)
                for _ in range(cfg.api_workers - 1)]
        signal.signal(signal.SIGTERM, lambda *_: sys.exit(0))
    try:
        asyncio.run(ApiService(cfg).run_forever())
    finally:
        for k in kids:
            k.terminate()
        for k in kids:
            try:
                k.wait(10)
            except subprocess.TimeoutExpired:
                k.kill()


if __name__ == "__main__":
    main()
