"""api_service on the native gateway (csrc/native/gateway.cpp).

The reference's gateway is a compiled actix-web server (services/api_service/src/main.rs); this is
its native counterpart: W epoll worker threads in C++, each with its own SO_REUSEPORT listener
and NATS connection, serving the four reference routes (plus /api/health, /api/metrics and the UI
page) without Python on the request path.  ``services/api.py`` (asyncio/starlette) is the
executable specification both are tested against (tests/test_e2e_cpu.py runs every gateway test
on both implementations).

    python -m codename_symbiont_amd.services.api            # native (SYMB_API_IMPL=native, default)
    SYMB_API_IMPL=py python -m codename_symbiont_amd.services.api
"""
from __future__ import annotations

import asyncio
import os
import signal
import threading
from urllib.parse import urlparse

from ..ops._ext import native
from ..utils.config import Config

STATIC_INDEX = os.path.join(os.path.dirname(__file__), "static", "index.html")


def _nats_hostport(url: str) -> tuple[str, int]:
    u = urlparse(url if "://" in url else f"nats://{url}")
    return u.hostname or "127.0.0.1", u.port or 4222


class NativeGateway:
    def __init__(self, cfg: Config | None = None, workers: int | None = None, log: bool = True):
        self.cfg = cfg or Config()
        N = native()
        gc = N.GatewayConfig()
        gc.host = self.cfg.api_host
        gc.port = self.cfg.api_port
        gc.nats_host, gc.nats_port = _nats_hostport(self.cfg.nats_url)
        gc.workers = max(1, workers if workers is not None else self.cfg.api_workers)
        gc.embed_timeout_s = self.cfg.embed_timeout_s
        gc.search_timeout_s = self.cfg.search_timeout_s
        gc.sse_capacity = self.cfg.sse_capacity
        gc.sse_keepalive_s = self.cfg.sse_keepalive_s
        gc.max_length_limit = self.cfg.max_length_limit
        gc.log = log
        if os.path.exists(STATIC_INDEX):
            with open(STATIC_INDEX, encoding="utf-8") as f:
                gc.index_html = f.read()
        self._gc = gc
        self._gw = None
        self.host = gc.host

    @property
    def port(self) -> int:
        return self._gw.port if self._gw else self._gc.port

    @property
    def url(self) -> str:
        host = "127.0.0.1" if self.host in ("", "0.0.0.0") else self.host
        return f"http://{host}:{self.port}"

    @property
    def stats(self) -> dict:
        return self._gw.stats() if self._gw else {}

    async def start(self, host: str | None = None, port: int | None = None,
                    wait_nats: float = 5.0) -> "NativeGateway":
        if host is not None:
            self._gc.host = self.host = host
        if port is not None:
            self._gc.port = port
        self._gw = native().Gateway(self._gc)
        self._gw.start()
        loop = asyncio.get_running_loop()
        deadline = loop.time() + wait_nats
        while not self._gw.nats_connected and loop.time() < deadline:
            await asyncio.sleep(0.01)
        return self

    async def stop(self) -> None:
        if self._gw is not None:
            self._gw.stop()
            self._gw = None


def serve_forever(cfg: Config) -> None:
    """Run the native gateway in this process until SIGTERM/SIGINT."""
    done = threading.Event()
    for s in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s, lambda *_: done.set())

    async def boot():
        return await NativeGateway(cfg).start(wait_nats=0.0)

    gw = asyncio.run(boot())
    print(f"[HTTP_SERVER] native gateway listening on {gw.url} ({max(1, cfg.api_workers)} workers, "
          f"NATS {cfg.nats_url})", flush=True)
    try:
        done.wait()
    finally:
        asyncio.run(gw.stop())
