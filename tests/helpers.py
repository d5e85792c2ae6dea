"""Shared async harness: in-process broker + services + uvicorn API on ephemeral ports."""
from __future__ import annotations

import asyncio
import contextlib

from codename_symbiont_amd.bus import Broker
from codename_symbiont_amd.utils.config import Config


def cpu_config(broker_url: str, **over) -> Config:
    cfg = Config()
    cfg.nats_url = broker_url
    cfg.force_cpu = True
    cfg.model = "minilm-l6"
    cfg.index_capacity = 4096
    cfg.snapshot_dir = ""
    cfg.fault_spec = ""
    cfg.queue_group = ""
    for k, v in over.items():
        setattr(cfg, k, v)
    return cfg


async def start_api(svc):
    import uvicorn

    await svc.start()
    config = uvicorn.Config(svc.app(), host="127.0.0.1", port=0, log_level="warning", lifespan="off")
    server = uvicorn.Server(config)
    task = asyncio.create_task(server.serve())
    for _ in range(200):
        if server.started:
            break
        await asyncio.sleep(0.02)
    port = server.servers[0].sockets[0].getsockname()[1]
    svc.server = server
    return f"http://127.0.0.1:{port}", task


async def stop_api(svc, task):
    svc.server.should_exit = True
    with contextlib.suppress(Exception):
        await asyncio.wait_for(task, 5)
    await svc.stop()


@contextlib.asynccontextmanager
async def gateway(impl: str, cfg: Config):
    """The api gateway under test: "py" (asyncio/starlette spec) or "native" (C++ epoll)."""
    if impl == "py":
        from codename_symbiont_amd.services.api import ApiService

        api = ApiService(cfg)
        url, task = await start_api(api)
        try:
            yield url
        finally:
            await stop_api(api, task)
    else:
        from codename_symbiont_amd.services.gateway_native import NativeGateway

        gw = await NativeGateway(cfg, workers=2, log=False).start(host="127.0.0.1", port=0)
        assert gw.stats["nats_connected"]
        try:
            yield gw.url
        finally:
            await gw.stop()


@contextlib.asynccontextmanager
async def broker():
    b = await Broker().start()
    try:
        yield b
    finally:
        await b.stop()
