"""Common service runtime: NATS connection, per-message task spawning, metrics, fault injection.

Reference pattern (every services/*/src/main.rs): connect to NATS, subscribe, ``tokio::spawn`` one
task per message, log with bracketed tags; when the subscription stream ends, ``main`` returns.
Here: asyncio tasks per message (bounded by a semaphore so a burst cannot exhaust memory),
a metrics registry (exposed by the api service on ``GET /api/metrics`` and published on
``metrics.<service>``), and ``SYMB_FAULT`` injection for failure tests:

    SYMB_FAULT="drop:<subject>:<prob>,delay:<subject>:<ms>,kill:<service>:<after_n_msgs>,
                kill_rank:<index rank>:<after_n_ops>"
"""
from __future__ import annotations

import asyncio
import gc
import os
import json
import logging
import random
import time
from collections import defaultdict

from ..bus.client import NatsClient
from ..utils.config import Config


class Metrics:
    def __init__(self):
        self.counters: dict[str, float] = defaultdict(float)
        self.hist: dict[str, list[float]] = defaultdict(list)

    def inc(self, name: str, v: float = 1.0) -> None:
        self.counters[name] += v

    def observe(self, name: str, v: float) -> None:
        h = self.hist[name]
        h.append(v)
        if len(h) > 4096:
            del h[:2048]

    def snapshot(self) -> dict:
        out = {"counters": dict(self.counters), "latency_ms": {}}
        for k, v in self.hist.items():
            if v:
                s = sorted(v)
                out["latency_ms"][k] = {"p50": s[len(s) // 2], "p99": s[min(len(s) - 1, int(len(s) * 0.99))],
                                        "n": len(s)}
        return out


class FaultInjector:
    def __init__(self, spec: str):
        self.drop: dict[str, float] = {}
        self.delay: dict[str, float] = {}
        self.kill: dict[str, int] = {}
        self.kill_rank: dict[int, int] = {}   # parallel/index_group.py: serve_one exits the rank
        for part in (p for p in spec.split(",") if p.strip()):
            kind, target, val = (part.split(":") + ["", ""])[:3]
            if kind == "drop":
                self.drop[target] = float(val or 1.0)
            elif kind == "delay":
                self.delay[target] = float(val or 0) / 1000.0
            elif kind == "kill":
                self.kill[target] = int(val or 0)
            elif kind == "kill_rank":
                self.kill_rank[int(target)] = int(val or 0)

    async def on_publish(self, subject: str) -> bool:
        """Returns False when the message must be dropped."""
        if subject in self.delay:
            await asyncio.sleep(self.delay[subject])
        p = self.drop.get(subject)
        return not (p is not None and random.random() < p)


class Service:
    name = "service"

    def __init__(self, cfg: Config | None = None, nc: NatsClient | None = None):
        self.cfg = cfg or Config()
        self.nc = nc
        self._own_nc = nc is None
        self.log = logging.getLogger(self.name)
        self.metrics = Metrics()
        self.faults = FaultInjector(self.cfg.fault_spec)
        self._tasks: set[asyncio.Task] = set()
        self._loops: list[asyncio.Task] = []
        self._sem = asyncio.Semaphore(1024)
        self._stopped = asyncio.Event()
        self._handled = 0

    async def connect(self) -> None:
        if self.nc is None:
            self.log.info("[NATS_CONNECT] Attempting to connect to NATS server at %s...",
                          self.cfg.nats_url)
            self.nc = await NatsClient.connect(self.cfg.nats_url, name=self.name, retries=20,
                                               request_timeout=self.cfg.nats_request_timeout_s)
            self.log.info("[NATS_CONNECT_SUCCESS] %s connected to NATS.", self.name)

    async def publish(self, subject: str, payload: bytes, **kw) -> None:
        if not await self.faults.on_publish(subject):
            self.metrics.inc(f"fault_dropped.{subject}")
            return
        await self.nc.publish(subject, payload, **kw)
        self.metrics.inc(f"published.{subject}")

    def spawn(self, coro) -> asyncio.Task:
        async def guarded():
            async with self._sem:
                try:
                    await coro
                except Exception:  # a failing handler never kills the service (tokio::spawn)
                    self.log.exception("[%s] handler failed", self.name.upper())
                    self.metrics.inc("handler_errors")
        t = asyncio.create_task(guarded())
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)
        return t

    def _count_and_maybe_die(self) -> None:
        self._handled += 1
        n = self.faults.kill.get(self.name)
        if n is not None and self._handled >= n:
            self.log.error("[FAULT] kill injected after %d messages", self._handled)
            asyncio.get_running_loop().call_soon(self._stopped.set)

    async def subscribe_loop(self, subject: str, handler, queue: str | None = None) -> None:
        """Subscribe and spawn ``handler(msg)`` per message until the subscription ends."""
        sub = await self.nc.subscribe(subject, queue=queue or (self.cfg.queue_group or None))
        self.log.info("Subscribed to subject: %s", subject)

        async def loop():
            async for msg in sub:
                self.metrics.inc(f"received.{subject}")
                self._count_and_maybe_die()
                self.spawn(handler(msg))
            self.log.info("[NATS_LOOP_END] subscription to %s ended.", subject)
            self._stopped.set()

        self._loops.append(asyncio.create_task(loop()))

    async def subscribe_batches(self, subject: str, handler, max_batch: int = 256,
                                queue: str | None = None, align: int = 0, gate=None,
                                fill: int = 0, fill_until=None) -> None:
        """Subscribe and call ``await handler(list_of_msgs)`` with everything queued at once (one
        message at least): under load a handler sees whole bursts, so per-message Python costs
        (decode, task, reply write) become per-batch costs.  The handler runs in this loop; it
        may hand work off (spawn) to overlap the next batch with the current one.  ``gate``: an
        async callable awaited before each batch is drawn (a free in-flight slot: messages keep
        queueing meanwhile).  ``align`` / ``fill`` / ``fill_until``: see
        ``Subscription.next_batch``."""
        sub = await self.nc.subscribe(subject, queue=queue or (self.cfg.queue_group or None))
        self.log.info("Subscribed to subject: %s", subject)

        async def loop():
            while True:
                if gate is not None:
                    await gate()
                batch = await sub.next_batch(max_batch, align, fill, fill_until)
                if batch is None:
                    break
                self.metrics.inc(f"received.{subject}", len(batch))
                for _ in batch:
                    self._count_and_maybe_die()
                try:
                    await handler(batch)
                except Exception:
                    self.log.exception("[%s] batch handler failed", self.name.upper())
                    self.metrics.inc("handler_errors")
            self.log.info("[NATS_LOOP_END] subscription to %s ended.", subject)
            self._stopped.set()

        self._loops.append(asyncio.create_task(loop()))

    async def setup(self) -> None:  # pragma: no cover - overridden
        raise NotImplementedError

    async def start(self) -> "Service":
        await self.connect()
        await self.setup()
        self._loops.append(asyncio.create_task(self._metrics_loop()))
        return self

    async def _metrics_loop(self) -> None:
        interval = float(os.environ.get("SYMB_METRICS_INTERVAL", "10"))
        while True:
            await asyncio.sleep(interval)
            try:
                await self.nc.publish(f"metrics.{self.name}", json.dumps(
                    {"service": self.name, "replica": os.environ.get("SYMB_REPLICA", ""),
                     "ts_ms": int(time.time() * 1000), **self.metrics.snapshot()}
                ).encode())
            except Exception:
                pass

    async def wait(self) -> None:
        await self._stopped.wait()

    async def stop(self) -> None:
        for t in self._loops:
            t.cancel()
        for t in list(self._tasks):
            t.cancel()
        if self._own_nc and self.nc is not None:
            await self.nc.close()
        self._stopped.set()

    async def run_forever(self) -> None:
        await self.start()
        # (service processes only) everything allocated while booting -- model weights' Python
        # wrappers, tokenizer tables, the index's host state -- lives as long as the process:
        # move it out of the collector's generations so full collections during serving only
        # walk per-request garbage
        gc.collect()
        gc.freeze()
        try:
            await self.wait()
        finally:
            await self.stop()
