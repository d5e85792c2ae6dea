#!/usr/bin/env python3
"""BASELINE config #1: Markov text generation over NATS (CPU only).

The reference flow (api_service/src/main.rs:113-188 -> text_generator_service/src/main.rs:111-162):
a GenerateTextTask published on ``tasks.generation.text`` is answered by one GeneratedTextMessage
on ``events.text.generated``.  This drives the in-process broker + TextGeneratorService with
``--tasks`` tasks kept ``--inflight`` deep and reports completed tasks/s and the publish->event
latency distribution.  One JSON line on stdout.

    python benchmarks/markov_nats.py [--tasks 20000] [--inflight 64] [--max-length 50]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


async def run(a) -> dict:
    from codename_symbiont_amd.bus.broker import BROKERS
    from codename_symbiont_amd.bus.client import NatsClient
    from codename_symbiont_amd.services.text_generator import TextGeneratorService
    from codename_symbiont_amd.utils.config import Config
    from codename_symbiont_amd.wire import GeneratedTextMessage, GenerateTextTask, subjects

    b = await BROKERS[a.broker]().start()
    cfg = Config()
    cfg.nats_url = b.url
    cfg.fault_spec = ""
    gen = await TextGeneratorService(cfg, seed=1).start()
    nc = await NatsClient.connect(b.url, name="markov-bench")
    sub = await nc.subscribe(subjects.TEXT_GENERATED)
    sent: dict[str, float] = {}
    lat: list[float] = []
    done = asyncio.Event()
    words = 0

    async def reader():
        nonlocal words
        async for m in sub:
            ev = GeneratedTextMessage.from_json(m.payload)
            t0 = sent.pop(ev.original_task_id, None)
            if t0 is not None:
                lat.append(time.perf_counter() - t0)
                words += len(ev.generated_text.split())
            if len(lat) >= a.tasks:
                done.set()
                return

    rt = asyncio.create_task(reader())
    await nc.flush()
    t_start = time.perf_counter()
    for i in range(a.tasks):
        while len(sent) >= a.inflight:
            await asyncio.sleep(0)
        tid = f"bench-{i}"
        sent[tid] = time.perf_counter()
        await nc.publish(subjects.GENERATE_TEXT,
                         GenerateTextTask(tid, None, a.max_length).to_json())
    await asyncio.wait_for(done.wait(), 120)
    elapsed = time.perf_counter() - t_start
    rt.cancel()
    await nc.close()
    await gen.stop()
    await b.stop()
    lat.sort()
    return {
        "metric": "Markov text generation over NATS (tasks/s, publish -> events.text.generated)",
        "value": round(a.tasks / elapsed, 1), "unit": "tasks/s", "higher_is_better": True,
        "n_gpus": 0, "tasks": a.tasks, "inflight": a.inflight, "max_length": a.max_length,
        "words_per_sec": round(words / elapsed, 1),
        "latency_ms": {"p50": round(1e3 * statistics.median(lat), 3),
                       "p99": round(1e3 * lat[int(0.99 * (len(lat) - 1))], 3)},
        "config": {"model": "word-bigram Markov (reference corpus)", "transport": f"in-process {a.broker} NATS broker, TCP loopback"},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tasks", type=int, default=20000)
    ap.add_argument("--broker", choices=["native", "py"], default="native")
    ap.add_argument("--inflight", type=int, default=64)
    ap.add_argument("--max-length", type=int, default=50)
    a = ap.parse_args()
    print(json.dumps(asyncio.run(run(a))))


if __name__ == "__main__":
    main()
