"""NATS client + in-repo broker semantics."""
import asyncio

import pytest

from codename_symbiont_amd.bus import Broker, NatsClient, NoRespondersError, RequestTimeoutError
from codename_symbiont_amd.bus.broker import subject_matches, subject_valid


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


def test_subject_rules():
    m = lambda p, s: subject_matches(p.split("."), s.split("."))  # noqa: E731
    assert m("a.*.c", "a.b.c") and not m("a.*.c", "a.b.d") and not m("a.*", "a.b.c")
    assert m("a.>", "a.b.c") and not m("a.>", "a") and m(">", "x")
    assert subject_valid("a.b", False) and not subject_valid("a.*", False) and subject_valid("a.*", True)
    assert not subject_valid("a..b", True) and not subject_valid("a.>.c", True)


def test_pubsub_queue_groups_request_reply():
    async def main():
        b = await Broker().start()
        a = await NatsClient.connect(b.url)
        c = await NatsClient.connect(b.url)
        wild = await c.subscribe("ev.>")
        g1 = await c.subscribe("work", queue="workers")
        g2 = await a.subscribe("work", queue="workers")
        plain = await c.subscribe("work")
        for i in range(20):
            await a.publish("work", str(i).encode())
        await a.publish("ev.x.y", b"e")
        await a.flush()
        await c.flush()
        await asyncio.sleep(0.1)
        assert g1._q.qsize() + g2._q.qsize() == 20 and g1._q.qsize() > 0 and g2._q.qsize() > 0
        assert plain._q.qsize() == 20                     # plain subscribers get every message
        assert (await wild.next_msg(1)).subject == "ev.x.y"

        async def responder():
            sub = await c.subscribe("svc.echo")
            async for m in sub:
                await m.respond(m.data[::-1])
        t = asyncio.create_task(responder())
        await asyncio.sleep(0.05)
        rs = await asyncio.gather(*[a.request("svc.echo", f"r{i}".encode(), timeout=2) for i in range(50)])
        assert [r.data for r in rs] == [f"r{i}".encode()[::-1] for i in range(50)]
        with pytest.raises(NoRespondersError):
            await a.request("nobody.home", b"", timeout=2)

        async def slow():
            sub = await c.subscribe("svc.slow")
            async for m in sub:
                await asyncio.sleep(1.0)
        t2 = asyncio.create_task(slow())
        await asyncio.sleep(0.05)
        with pytest.raises(RequestTimeoutError) as ei:
            await a.request("svc.slow", b"", timeout=0.2)
        assert str(ei.value) == "request timed out"
        # auto-unsubscribe after N messages
        s = await c.subscribe("once")
        await c._send(f"UNSUB {s.sid} 2\r\n".encode())
        await c.flush()
        for _ in range(5):
            await a.publish("once", b"x")
        await a.flush()
        await asyncio.sleep(0.1)
        assert s._q.qsize() == 2
        t.cancel()
        t2.cancel()
        await a.close()
        await c.close()
        await b.stop()
    run(main())


def test_max_payload_and_reconnect_resubscribe():
    async def main():
        b = await Broker(max_payload=1000).start()
        port = b.port
        a = await NatsClient.connect(b.url)
        assert a.max_payload == 1000
        with pytest.raises(Exception, match="maximum payload"):
            await a.publish("x", b"z" * 1001)
        c = await NatsClient.connect(b.url)
        c.reconnect_wait = 0.1
        a.reconnect_wait = 0.1
        sub = await c.subscribe("after.restart")
        await b.stop()                                    # broker dies
        await asyncio.sleep(0.3)
        b2 = await Broker(port=port).start()              # ... and comes back on the same port
        for _ in range(100):
            if c.is_connected and a.is_connected:
                break
            await asyncio.sleep(0.05)
        await asyncio.sleep(0.2)
        await a.publish("after.restart", b"hello again")
        m = await sub.next_msg(3)                          # subscription was re-established
        assert m.data == b"hello again"
        await a.close()
        await c.close()
        await b2.stop()
    run(main())
