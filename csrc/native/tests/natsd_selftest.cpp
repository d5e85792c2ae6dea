// Sanitizer self-test of the native NATS server (csrc/native/natsd.cpp), built WITHOUT Python
// by tests/test_native_sanitize_cpu.py twice: -fsanitize=address,undefined and -fsanitize=thread.
// Drives the epoll loop thread through real sockets: pub/sub with wildcards, queue groups, UNSUB
// max, no-responders, max_payload violation, a slow consumer being cut off, abrupt disconnects
// and random-garbage connections (SURVEY.md §5 race detection / sanitizers).
#define SYMB_NO_PYTHON 1
#include "../natsd.cpp"

#include <random>

#include "selftest_net.h"

using symbn::natsd::Server;

int main() {
  {
    Server srv("127.0.0.1", 0, 1 << 20, 256 << 10);
    srv.start();
    const int port = srv.port();
    // pub/sub with wildcards
    Client sub(port), pub(port);
    sub.send("SUB foo.* 1\r\nSUB foo.> 2\r\nPING\r\n");
    CHECK(sub.read_until("PONG\r\n").size() > 0);
    pub.send("PUB foo.bar 5\r\nhello\r\nPUB foo.a.b 2\r\nhi\r\nPING\r\n");
    CHECK(pub.read_until("PONG\r\n").size() > 0);
    const std::string got = sub.read_until("MSG foo.a.b 2 2\r\nhi\r\n");
    CHECK(got.find("MSG foo.bar 1 5\r\nhello\r\n") != std::string::npos);
    CHECK(got.find("MSG foo.bar 2 5\r\nhello\r\n") != std::string::npos);

    // queue group: each message to exactly one member
    Client q1(port), q2(port);
    q1.send("SUB work grp 1\r\nPING\r\n");
    q2.send("SUB work grp 7\r\nPING\r\n");
    q1.read_until("PONG\r\n");
    q2.read_until("PONG\r\n");
    std::string burst;
    for (int i = 0; i < 100; ++i) burst += "PUB work 1\r\nx\r\n";
    pub.send(burst + "PING\r\n");
    pub.read_until("PONG\r\n");
    const int n1 = count(q1.drain(), "MSG work"), n2 = count(q2.drain(), "MSG work");
    CHECK(n1 + n2 == 100 && n1 > 0 && n2 > 0);

    // UNSUB max
    Client once(port);
    once.send("SUB once 5\r\nUNSUB 5 2\r\nPING\r\n");
    once.read_until("PONG\r\n");
    pub.send("PUB once 1\r\na\r\nPUB once 1\r\nb\r\nPUB once 1\r\nc\r\nPING\r\n");
    pub.read_until("PONG\r\n");
    CHECK(count(once.drain(), "MSG once") == 2);

    // no responders
    Client req(port, true, "CONNECT {\"headers\":true,\"no_responders\":true,\"opts\":[1,{\"a\":null}]}\r\n");
    req.send("SUB _INBOX.r 9\r\nPUB nobody _INBOX.r 0\r\n\r\n");
    CHECK(req.read_until("NATS/1.0 503").find("HMSG _INBOX.r 9 ") != std::string::npos);

    // max_payload violation closes the connection
    Client big(port);
    big.send("PUB big 2000000\r\n");
    CHECK(big.read_until("\r\n").find("Maximum Payload Violation") != std::string::npos);
    CHECK(big.closed_by_peer());

    // slow consumer: subscribes, never reads; the server cuts it off past max_pending
    {
      Client slow(port);
      timeval tv{0, 1000};
      setsockopt(slow.fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
      int small = 4096;
      setsockopt(slow.fd, SOL_SOCKET, SO_RCVBUF, &small, sizeof small);
      slow.send("SUB flood 1\r\nPING\r\n");
      usleep(50000);
      const std::string payload(16384, 'z');
      std::string chunk;
      for (int i = 0; i < 64; ++i) chunk += "PUB flood 16384\r\n" + payload + "\r\n";
      for (int r = 0; r < 16; ++r) pub.send(chunk);
      pub.send("PING\r\n");
      pub.read_until("PONG\r\n", 100);
      CHECK(srv.counters().slow_consumers >= 1);
    }

    // random garbage and abrupt disconnects on many connections
    std::mt19937_64 rng(7);
    const char* frags[] = {"PUB a 3\r\n", "SUB a.* 1\r\n", "HPUB x 12 14\r\nNATS/1.0\r\n\r\n", "UNSUB 1 0\r\n",
                           "PING\r\n", "\r\n", "PUB a.b 999999999999\r\n", "SUB  \r\n", "CONNECT {\r\n",
                           "msg", "\xff\xfe", "PUB a.b 2\r\nxyz", "SUB > q 3\r\n"};
    for (int c = 0; c < 200; ++c) {
      Client g(port, rng() % 2 == 0);
      std::string s;
      const int parts = (int)(rng() % 12);
      for (int p = 0; p < parts; ++p) {
        if (rng() % 3 == 0) {
          for (int k = 0; k < (int)(rng() % 64); ++k) s.push_back((char)(rng() % 256));
        } else {
          s += frags[rng() % (sizeof(frags) / sizeof(frags[0]))];
        }
      }
      g.send(s);
      if (rng() % 4 == 0) g.drain(1);
    }
    // the server is still healthy
    pub.send("PUB foo.ok 2\r\nok\r\nPING\r\n");
    pub.read_until("PONG\r\n");
    CHECK(sub.read_until("MSG foo.ok 1 2\r\nok\r\n").size() > 0);
    const auto cnt = srv.counters();
    CHECK(cnt.in_msgs >= 106 && cnt.out_msgs >= 104);
    srv.stop();
  }
  {  // start/stop cycles
    for (int i = 0; i < 3; ++i) {
      Server srv("127.0.0.1", 0, 1024, 1 << 20);
      srv.start();
      Client c(srv.port());
      c.send("SUB s 1\r\nPUB s 2\r\nab\r\n");
      CHECK(c.read_until("ab\r\n").size() > 0);
      srv.stop();
    }
  }
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("natsd selftest ok\n");
  return 0;
}
