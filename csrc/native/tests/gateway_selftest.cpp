// Sanitizer self-test of the native gateway (csrc/native/gateway.cpp) with the native NATS server,
// built WITHOUT Python by tests/test_native_sanitize_cpu.py under -fsanitize=address,undefined
// and under -fsanitize=thread.  Two gateway worker threads + the server thread + a raw-socket
// responder serving the embedding and search hops; HTTP clients exercise the two-hop search,
// validation errors, pipelining, SSE fan-out and abrupt disconnects while requests are parked.
#define SYMB_NO_PYTHON 1
#include "../natsd.cpp"
#include "../gateway.cpp"

#include <atomic>
#include <random>
#include <thread>

#include "selftest_net.h"

static std::string http_post(const std::string& path, const std::string& body) {
  return "POST " + path + " HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\nContent-Length: " +
         std::to_string(body.size()) + "\r\n\r\n" + body;
}

// answers tasks.embedding.for_query and tasks.search.semantic.request over a raw NATS socket
static void responder(int nats_port, std::atomic<bool>& stop, std::atomic<int>& served) {
  Client c(nats_port);
  c.send("SUB tasks.embedding.for_query 1\r\nSUB tasks.search.semantic.request 2\r\nPING\r\n");
  c.read_until("PONG\r\n");
  while (!stop) {
    const std::string head = c.read_until("\r\n", 1);
    if (head.empty()) continue;
    if (head.rfind("MSG ", 0) != 0) continue;
    // MSG <subject> <sid> <reply> <n>
    std::string subj, sid, reply;
    size_t n = 0;
    {
      char s1[256], s2[32], s3[256];
      unsigned long nn = 0;
      if (std::sscanf(head.c_str(), "MSG %255s %31s %255s %lu", s1, s2, s3, &nn) != 4) continue;
      subj = s1;
      sid = s2;
      reply = s3;
      n = nn;
    }
    std::string payload = c.read_until("\r\n", 20);
    while (payload.size() < n + 2) payload += c.read_until("\r\n", 20);
    payload.resize(n);
    const size_t rp = payload.find("\"request_id\":\"");
    const std::string rid = rp == std::string::npos ? "x" : payload.substr(rp + 14, 36);
    std::string out;
    if (sid == "1") {
      out = "{\"request_id\":\"" + rid + "\",\"embedding\":[0.5,-0.25,1.0],\"model_name\":\"m\","
            "\"error_message\":null}";
    } else {
      const std::string item = "{\"qdrant_point_id\":\"p\",\"score\":0.75,\"payload\":{"
                               "\"original_document_id\":\"d\",\"source_url\":\"u\",\"sentence_text\":\"s\","
                               "\"sentence_order\":1,\"model_name\":\"m\",\"processed_at_ms\":2}}";
      out = "{\"request_id\":\"" + rid + "\",\"results\":[" + item + "," + item + "],\"error_message\":null}";
      ++served;
    }
    c.send("PUB " + reply + " " + std::to_string(out.size()) + "\r\n" + out + "\r\n");
  }
}

int main() {
  using symbn::gw::Config;
  using symbn::gw::Gateway;
  using symbn::natsd::Server;
  Server bus("127.0.0.1", 0, 1 << 20, 64 << 20);
  bus.start();
  Config cfg;
  cfg.host = "127.0.0.1";
  cfg.port = 0;
  cfg.nats_port = bus.port();
  cfg.workers = 2;
  cfg.sse_keepalive_s = 0.1;
  cfg.log = false;
  Gateway gw(cfg);
  gw.start();
  for (int i = 0; i < 200 && !gw.nats_connected(); ++i) usleep(10000);
  CHECK(gw.nats_connected());
  const int hp = gw.port();

  std::atomic<bool> stop{false};
  std::atomic<int> served{0};
  std::thread resp(responder, bus.port(), std::ref(stop), std::ref(served));
  usleep(100000);

  // SSE listeners
  Client sse1(hp, false), sse2(hp, false);
  sse1.send("GET /api/events HTTP/1.1\r\nHost: t\r\n\r\n");
  sse2.send("GET /api/events HTTP/1.1\r\nHost: t\r\n\r\n");
  CHECK(sse1.read_until("\r\n\r\n").find("text/event-stream") != std::string::npos);
  CHECK(sse2.read_until("\r\n\r\n").find("text/event-stream") != std::string::npos);

  // concurrent searches from several client threads (keep-alive, pipelined pairs)
  std::vector<std::thread> cl;
  std::atomic<int> ok{0};
  for (int t = 0; t < 4; ++t) {
    cl.emplace_back([&, t] {
      Client c(hp, false);
      for (int i = 0; i < 25; ++i) {
        const std::string req = http_post("/api/search/semantic",
                                          "{\"query_text\":\"q" + std::to_string(t * 100 + i) +
                                              "\",\"top_k\":2}");
        c.send(req + req);
        for (int k = 0; k < 2; ++k) {
          const std::string h = c.read_until("\r\n\r\n", 50);
          const size_t cl_at = h.find("content-length: ");
          if (h.find("HTTP/1.1 200") == std::string::npos || cl_at == std::string::npos) continue;
          const size_t len = std::stoul(h.substr(cl_at + 16));
          std::string body = c.buf.substr(0, std::min(len, c.buf.size()));
          while (body.size() < len) {
            c.read_until("}", 50);
            body = c.buf.substr(0, std::min(len, c.buf.size()));
          }
          c.buf.erase(0, len);
          if (body.find("\"score\":0.75") != std::string::npos) ++ok;
        }
      }
    });
  }
  // a client that disconnects while its search is parked, and garbage HTTP
  std::mt19937_64 rng(3);
  for (int i = 0; i < 50; ++i) {
    Client g(hp, false);
    if (i % 2) {
      g.send(http_post("/api/search/semantic", "{\"query_text\":\"bye\",\"top_k\":1}"));
    } else {
      std::string s;
      for (int k = 0; k < (int)(rng() % 300); ++k) s.push_back((char)(rng() % 256));
      g.send(s + "\r\n\r\n");
    }
  }
  for (auto& th : cl) th.join();
  CHECK(ok == 200);

  // validation + publish paths
  Client v(hp, false);
  v.send(http_post("/api/generate-text", "{\"task_id\":\"t\",\"max_length\":0}"));
  CHECK(v.read_until("between 1 and 1000").size() > 0);
  v.send(http_post("/api/submit-url", "{\"url\":5}"));
  CHECK(v.read_until("expected a string").size() > 0);
  v.send("GET /api/metrics HTTP/1.1\r\nHost: t\r\n\r\n");
  CHECK(v.read_until("\"search.requests\"").size() > 0);

  // an event reaches both SSE clients; keep-alives flow
  Client pub(bus.port());
  const std::string ev = "{\"original_task_id\":\"e1\",\"generated_text\":\"x\",\"timestamp_ms\":5}";
  pub.send("PUB events.text.generated " + std::to_string(ev.size()) + "\r\n" + ev + "\r\nPING\r\n");
  CHECK(sse1.read_until("e1").size() > 0);
  CHECK(sse2.read_until("e1").size() > 0);
  CHECK(sse1.read_until("keep-alive").size() > 0);

  stop = true;
  pub.send("PUB tasks.embedding.for_query _INBOX.none 2\r\n{}\r\n");  // wake the responder
  resp.join();
  gw.stop();
  bus.stop();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed (ok=%d served=%d)\n", g_fail, ok.load(), served.load());
    return 1;
  }
  std::printf("gateway selftest ok\n");
  return 0;
}
