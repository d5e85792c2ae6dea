"""NATS client + in-repo broker semantics."""
import asyncio

import pytest

from codename_symbiont_amd.bus import NatsClient, NoRespondersError, RequestTimeoutError
from codename_symbiont_amd.bus.broker import BROKERS, subject_matches, subject_valid
from codename_symbiont_amd.ops._ext import native


@pytest.fixture(params=sorted(BROKERS))
def Broker(request):
    """Every bus test runs against the native C++ server and the asyncio reference broker."""
    return BROKERS[request.param]


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


def test_subject_rules():
    m = lambda p, s: subject_matches(p.split("."), s.split("."))  # noqa: E731
    assert m("a.*.c", "a.b.c") and not m("a.*.c", "a.b.d") and not m("a.*", "a.b.c")
    assert m("a.>", "a.b.c") and not m("a.>", "a") and m(">", "x")
    assert subject_valid("a.b", False) and not subject_valid("a.*", False) and subject_valid("a.*", True)
    assert not subject_valid("a..b", True) and not subject_valid("a.>.c", True)
    # the native server applies the same rules
    N = native()
    for subj, wild in [("a.b", False), ("a.*", False), ("a.*", True), ("a..b", True),
                       ("a.>.c", True), (">", True), ("a b", False), ("", True), ("a.", True)]:
        assert N.nats_subject_valid(subj, wild) == subject_valid(subj, wild), (subj, wild)
    for pat, subj in [("a.*.c", "a.b.c"), ("a.*.c", "a.b.d"), ("a.*", "a.b.c"), ("a.>", "a.b.c"),
                      ("a.>", "a"), (">", "x"), ("a.b", "a.b"), ("a.b", "a.b.c")]:
        assert N.nats_subject_matches(pat, subj) == subject_matches(pat.split("."), subj.split("."))


def test_pubsub_queue_groups_request_reply(Broker):
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


def test_max_payload_and_reconnect_resubscribe(Broker):
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


async def _raw(port):
    r, w = await asyncio.open_connection("127.0.0.1", port)
    info = await r.readline()
    assert info.startswith(b"INFO {") and b'"headers":true' in info
    return r, w


def test_raw_protocol_semantics(Broker):
    """Wire-level behaviour a NATS client relies on, identical on both brokers."""
    async def main():
        b = await Broker(max_payload=64).start()
        r, w = await _raw(b.port)
        w.write(b'CONNECT {"verbose":true,"headers":true,"no_responders":true,"name":"t",'
                b'"opts":{"x":[1,2,{"y":null}]},"lang":"py"}\r\n')
        assert await r.readline() == b"+OK\r\n"
        w.write(b"PING\r\n")
        assert await r.readline() == b"PONG\r\n"
        w.write(b"SUB in.* 7\r\nPUB in.x rep 5\r\nhello\r\n")
        assert await r.readline() == b"+OK\r\n"
        assert await r.readline() == b"+OK\r\n"
        assert await r.readline() == b"MSG in.x 7 rep 5\r\n"
        assert await r.readline() == b"hello\r\n"
        w.write(b"HPUB in.y 12 14\r\nNATS/1.0\r\n\r\nhi\r\n")
        assert await r.readline() == b"+OK\r\n"
        assert await r.readline() == b"HMSG in.y 7 12 14\r\n"
        assert await r.readexactly(16) == b"NATS/1.0\r\n\r\nhi\r\n"
        # request to nobody -> no-responders status on the reply subject
        w.write(b"SUB _INBOX.q 9\r\nPUB nobody _INBOX.q 0\r\n\r\n")
        assert await r.readline() == b"+OK\r\n"
        assert await r.readline() == b"+OK\r\n"
        assert await r.readline() == b"HMSG _INBOX.q 9 16 16\r\n"
        assert await r.readexactly(18) == b"NATS/1.0 503\r\n\r\n\r\n"
        w.write(b"PUB bad.* 1\r\nx\r\n")
        assert await r.readline() == b"-ERR 'Invalid Publish Subject'\r\n"
        w.write(b"PUB big 65\r\n")
        assert await r.readline() == b"-ERR 'Maximum Payload Violation'\r\n"
        assert await r.read() == b""                       # ... and the connection is closed
        w.close()
        r2, w2 = await _raw(b.port)
        w2.write(b"BOGUS\r\n")
        assert (await r2.readline()).startswith(b"-ERR 'Unknown Protocol Operation'")
        w2.close()
        await b.stop()
    run(main())


def test_native_broker_fanout_and_stats():
    """Many publishers x subscribers through the C++ server: every plain subscriber sees every
    message in publish order per publisher; queue-group members split the stream exactly."""
    async def main():
        b = await BROKERS["native"]().start()
        subs_c = [await NatsClient.connect(b.url) for _ in range(4)]
        pubs_c = [await NatsClient.connect(b.url) for _ in range(3)]
        plain = [await c.subscribe("fan.>") for c in subs_c]
        group = [await c.subscribe("fan.q", queue="g") for c in subs_c]
        await asyncio.gather(*[c.flush() for c in subs_c])
        N = 300
        for i in range(N):
            for j, p in enumerate(pubs_c):
                await p.publish("fan.q", f"{j}:{i}".encode())
        await asyncio.gather(*[p.flush() for p in pubs_c])
        for s in plain:
            got = [(await s.next_msg(5)).data.decode() for _ in range(N * len(pubs_c))]
            for j in range(len(pubs_c)):
                assert [int(x.split(":")[1]) for x in got if x.startswith(f"{j}:")] == list(range(N))
        await asyncio.sleep(0.2)
        assert sum(g._q.qsize() for g in group) == N * len(pubs_c)
        st = b.stats
        assert st["in_msgs"] == N * len(pubs_c)
        assert st["out_msgs"] == N * len(pubs_c) * (len(plain) + 1)
        assert st["connections"] == len(subs_c) + len(pubs_c)
        for c in subs_c + pubs_c:
            await c.close()
        await asyncio.sleep(0.1)
        assert b.stats["connections"] == 0 and b.stats["subscriptions"] == 0
        await b.stop()
    run(main())


# ---------------------------------------------------------------------------------------------
# differential property test: random protocol scripts give byte-identical per-connection output
# on the native server and on the asyncio reference broker
from hypothesis import HealthCheck, example, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

_TOK = st.sampled_from(["a", "b", "c"])
_SUBJ = st.lists(_TOK, min_size=1, max_size=3).map(".".join)
_PAT = st.lists(st.one_of(_TOK, st.just("*")), min_size=1, max_size=3).map(".".join) | \
    st.lists(_TOK, min_size=0, max_size=2).map(lambda t: ".".join(t + [">"]))
_OP = st.one_of(
    st.tuples(st.just("sub"), st.integers(0, 2), _PAT, st.integers(1, 6)),
    st.tuples(st.just("pub"), st.integers(0, 2), _SUBJ, st.binary(max_size=12)),
    st.tuples(st.just("hpub"), st.integers(0, 2), _SUBJ, st.binary(max_size=6)),
    st.tuples(st.just("unsub"), st.integers(0, 2), st.integers(1, 6), st.integers(0, 3)),
    st.tuples(st.just("bad"), st.integers(0, 2), st.sampled_from(["a.*", "a..b", " "]), st.just(b"")),
)


async def _script_output(Broker, script):
    b = await Broker(max_payload=4096).start()
    conns = []
    for _ in range(3):
        r, w = await _raw(b.port)
        w.write(b'CONNECT {"verbose":false,"headers":true,"no_responders":true}\r\nPING\r\n')
        assert await r.readline() == b"PONG\r\n"
        conns.append((r, w))
    outs = [bytearray() for _ in conns]
    closed: set[int] = set()

    async def sync():
        # a PING/PONG round trip on EVERY connection after each op makes the outputs
        # deterministic (the broker handles one connection's bytes in order)
        for i, (r, w) in enumerate(conns):
            if i in closed:
                continue
            w.write(b"PING\r\n")
            while True:
                line = await asyncio.wait_for(r.readline(), 5)
                if line == b"PONG\r\n":
                    break
                outs[i] += line
                if not line:          # the server closed this connection (protocol error)
                    closed.add(i)
                    break
    for op in script:
        kind, c = op[0], op[1]
        if c in closed:
            continue
        w = conns[c][1]
        if kind == "sub":
            w.write(f"SUB {op[2]} {op[3]}\r\n".encode())
        elif kind == "pub":
            w.write(f"PUB {op[2]} _INBOX.r {len(op[3])}\r\n".encode() + op[3] + b"\r\n")
        elif kind == "hpub":
            h = b"NATS/1.0\r\nk: v\r\n\r\n"
            w.write(f"HPUB {op[2]} {len(h)} {len(h) + len(op[3])}\r\n".encode() + h + op[3] + b"\r\n")
        elif kind == "unsub":
            w.write(f"UNSUB {op[2]} {op[3]}\r\n".encode() if op[3] else f"UNSUB {op[2]}\r\n".encode())
        else:
            w.write(f"PUB {op[2]} 0\r\n\r\n".encode())
        await sync()
    for _, w in conns:
        w.close()
    await b.stop()
    return [bytes(o) for o in outs]


@settings(max_examples=100, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(_OP, min_size=1, max_size=25))
# a reused sid re-subscribed after a wildcard sub: delivery follows creation order, not sid order
@example([("sub", 0, "a", 1), ("unsub", 0, 1, 0), ("sub", 0, "*.*.*", 2), ("sub", 1, "*", 1),
          ("sub", 0, "a.b.b", 1), ("pub", 0, "a.b.b", b"")])
def test_native_broker_matches_reference_on_random_scripts(script):
    py = run(_script_output(BROKERS["py"], script))
    nat = run(_script_output(BROKERS["native"], script))
    assert nat == py


def test_native_broker_http_monitoring():
    """nats-server-style monitoring endpoints (the reference publishes :8222)."""
    import httpx

    async def main():
        b = await BROKERS["native"](monitor_port=0).start()
        a = await NatsClient.connect(b.url)
        await a.subscribe("m.*")
        await a.publish("m.x", b"123")
        await a.flush()
        base = f"http://127.0.0.1:{b.monitor_port}"
        async with httpx.AsyncClient(timeout=5) as c:
            v = (await c.get(base + "/varz")).json()
            assert v["version"] == "2.10.7" and v["port"] == b.port and v["connections"] == 1
            assert v["in_msgs"] == 1 and v["out_msgs"] == 1 and v["in_bytes"] == 3
            cz = (await c.get(base + "/connz")).json()
            assert cz["num_connections"] == 1 and cz["connections"][0]["subscriptions"] >= 1
            assert (await c.get(base + "/subsz")).json()["num_wildcard"] >= 1
            assert (await c.get(base + "/healthz")).json() == {"status": "ok"}
            assert (await c.get(base + "/nope")).status_code == 404
        await a.close()
        await b.stop()
    run(main())


def test_next_batch_align():
    """next_batch(align=A): with more than A messages ready it takes a whole multiple of A (the
    rest stays queued, in order); A or fewer ready are taken whole."""
    from codename_symbiont_amd.bus.client import Msg, Subscription

    async def with_timeout():
        sub = Subscription(None, "1", "s", None)
        for i in range(700):
            sub._deliver(Msg("s", None, b"%d" % i))
        a = await sub.next_batch(1024, align=256)
        b = await sub.next_batch(1024, align=256)
        assert (len(a), len(b)) == (512, 188)
        assert [int(m.data) for m in a + b] == list(range(700))
        for _ in range(300):
            sub._deliver(Msg("s", None, b"x"))
        assert len(await sub.next_batch(1024, align=0)) == 300
        for _ in range(300):
            sub._deliver(Msg("s", None, b"x"))
        assert len(await sub.next_batch(200, align=256)) == 200   # max_n < align: plain cap
        assert len(await sub.next_batch(200, align=256)) == 100

    asyncio.run(with_timeout())


def test_next_batch_fill_until_deadline():
    """next_batch(fill=F, fill_until=f): with fewer than F ready it keeps collecting until F are
    ready or f()'s deadline passes; a None deadline (nothing in flight) launches at once."""
    from codename_symbiont_amd.bus.client import Msg, Subscription

    async def main():
        loop = asyncio.get_running_loop()
        sub = Subscription(None, "1", "s", None)
        sub._deliver(Msg("s", None, b"0"))
        t0 = loop.time()
        assert len(await sub.next_batch(512, 256, fill=256, fill_until=lambda: None)) == 1
        assert loop.time() - t0 < 0.1

        async def trickle(n, gap):
            for i in range(n):
                await asyncio.sleep(gap)
                sub._deliver(Msg("s", None, b"%d" % i))
        # the block fills before the deadline: exactly 256 taken, the rest stays queued
        sub._deliver(Msg("s", None, b"x"))
        feed = asyncio.create_task(trickle(300, 0.0))
        b = await sub.next_batch(512, 256, fill=256, fill_until=lambda: loop.time() + 5.0)
        await feed
        assert len(b) == 256
        rest = await sub.next_batch(512, 256)
        assert len(rest) == 301 - 256
        # the deadline passes first: whatever arrived by then
        sub._deliver(Msg("s", None, b"y"))
        feed = asyncio.create_task(trickle(5, 0.01))
        t0 = loop.time()
        b = await sub.next_batch(512, 256, fill=256, fill_until=lambda: loop.time() + 0.2)
        assert 0.15 < loop.time() - t0 < 1.5 and 2 <= len(b) <= 6
        await feed

    asyncio.run(asyncio.wait_for(main(), 10))
