// Native HTTP/SSE gateway: the api_service of the reference (services/api_service/src/main.rs,
// actix-web) as a C++ epoll server that speaks NATS itself.
//
// Routes and observable contract (the asyncio gateway services/api.py is the
// executable specification and tests/test_gateway_native_cpu.py runs the same checks on both):
//   POST /api/submit-url       {"url"} -> trim -> PerceiveUrlTask on tasks.perceive.url  (:42-111)
//   POST /api/generate-text    GenerateTextTask -> tasks.generation.text                 (:113-188)
//   GET  /api/events           SSE of GeneratedTextMessage JSON, broadcast, capacity 32 with
//                              lag-drop of the oldest, keep-alive comment every 15 s      (:190-270)
//   POST /api/search/semantic  two NATS request-reply hops: tasks.embedding.for_query ->
//                              tasks.search.semantic.request, 503/500 mapping            (:272-512)
//   GET  /api/health, /api/metrics, /   (additions: health, counters, the UI page)
// actix Json extractor behaviour: non-JSON content type -> 400 "Content type error", bodies over
// 2 MiB -> 413, undecodable -> 400 "Json deserialize error: <serde message>" (messages produced
// by the same serde-compatible parser as the Python side, csrc/native/json.cpp).  CORS as
// main.rs:555-567.
//
// Design: W worker threads, each an independent epoll loop with its own SO_REUSEPORT listener
// and its own NATS connection (INFO/CONNECT with headers + no_responders, one wildcard reply
// inbox `_INBOX.<nuid>.*` per loop, reconnect + resubscribe).  A search request parks its HTTP
// connection, issues the embedding request, and continues from the reply callback -- no thread
// per request, no Python on the request path.  SSE clients get events appended straight into
// their output buffers (bounded per-client backlog = the broadcast capacity).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#ifndef SYMB_NO_PYTHON
#include <pybind11/pybind11.h>
#endif
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "json.h"

#ifndef SYMB_NO_PYTHON
namespace py = pybind11;
#endif

namespace symbn {
namespace gw {

using Clock = std::chrono::steady_clock;
static double now_s() {
  return std::chrono::duration<double>(Clock::now().time_since_epoch()).count();
}

// ============================================================================ JSON DOM
// Mirrors json_py.cpp's Loader with f32_arrays=true (what WireModel.from_json uses), so every
// syntax error carries the same serde-style message and position.
struct JVal {
  enum T { Null, Bool, Int, Float, Str, Arr, Obj } t = Null;
  bool b = false;
  std::string s;                      // string value or number text
  std::vector<JVal> a;
  std::vector<std::pair<std::string, JVal>> o;
  const JVal* get(const std::string& k) const {  // last duplicate wins (Python dict semantics)
    for (auto it = o.rbegin(); it != o.rend(); ++it)
      if (it->first == k) return &it->second;
    return nullptr;
  }
};

struct Loader {
  Parser p;
  Loader(const char* s, size_t n) : p(s, n) {}
  JVal value(int depth) {
    if (depth > 128) p.fail("recursion limit exceeded");
    JVal v;
    const char c = p.peek();
    if (c == '{') {
      p.advance();
      v.t = JVal::Obj;
      if (p.peek() == '}') {
        p.advance();
        return v;
      }
      for (;;) {
        if (p.peek() != '"') p.fail("key must be a string");
        std::string k = p.string();
        if (p.peek() != ':') p.fail("expected `:`");
        p.advance();
        JVal x = value(depth + 1);
        v.o.emplace_back(std::move(k), std::move(x));
        const char t = p.peek();
        if (t == ',') {
          p.advance();
          continue;
        }
        if (t == '}') {
          p.advance();
          return v;
        }
        p.fail("expected `,` or `}`");
      }
    }
    if (c == '[') {
      p.advance();
      v.t = JVal::Arr;
      if (p.peek() == ']') {
        p.advance();
        return v;
      }
      for (;;) {
        v.a.push_back(value(depth + 1));
        const char s = p.peek();
        if (s == ',') {
          p.advance();
          continue;
        }
        if (s == ']') {
          p.advance();
          return v;
        }
        p.fail("expected `,` or `]`");
      }
    }
    if (c == '"') {
      v.t = JVal::Str;
      v.s = p.string();
      return v;
    }
    if (c == 't') {
      p.expect_lit("true");
      v.t = JVal::Bool;
      v.b = true;
      return v;
    }
    if (c == 'f') {
      p.expect_lit("false");
      v.t = JVal::Bool;
      return v;
    }
    if (c == 'n') {
      p.expect_lit("null");
      return v;
    }
    if (c == '-' || (c >= '0' && c <= '9')) {
      Number n = p.number();
      v.t = n.is_float ? JVal::Float : JVal::Int;
      v.s = std::move(n.text);
      return v;
    }
    p.fail("expected value");
  }
};

static JVal parse_json(const std::string& body) {
  Loader L(body.data(), body.size());
  JVal v = L.value(0);
  if (!L.p.at_end()) L.p.fail("trailing characters");
  return v;
}

struct WireErr : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Python repr() of a double (what `f"{v}"` prints in models._desc)
static std::string py_float_repr(double d) {
  if (std::isnan(d)) return "nan";
  if (std::isinf(d)) return d > 0 ? "inf" : "-inf";
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, d, std::chars_format::scientific);
  std::string sci(buf, r.ptr);  // [-]d[.ddd]e(+|-)XX
  const size_t e = sci.find('e');
  std::string mant = sci.substr(0, e);
  const int exp10 = std::stoi(sci.substr(e + 1));
  const bool neg = mant[0] == '-';
  if (neg) mant.erase(0, 1);
  std::string digits;
  for (char ch : mant)
    if (ch != '.') digits += ch;
  std::string out;
  if (exp10 >= -5 + 1 && exp10 < 16) {  // Python: repr uses fixed notation for 1e-4 <= |x| < 1e16
    if (exp10 >= 0) {
      if ((int)digits.size() <= exp10 + 1) {
        out = digits + std::string(exp10 + 1 - digits.size(), '0') + ".0";
      } else {
        out = digits.substr(0, exp10 + 1) + "." + digits.substr(exp10 + 1);
      }
    } else {
      out = "0." + std::string(-exp10 - 1, '0') + digits;
    }
  } else {
    out = digits.substr(0, 1);
    if (digits.size() > 1) out += "." + digits.substr(1);
    char eb[16];
    snprintf(eb, sizeof eb, "e%c%02d", exp10 < 0 ? '-' : '+', std::abs(exp10));
    out += eb;
  }
  return neg ? "-" + out : out;
}

static std::string int_text(const std::string& t) {  // Python str(int(text))
  if (t == "-0") return "0";
  return t;
}

static std::string desc(const JVal& v) {
  switch (v.t) {
    case JVal::Null: return "null";
    case JVal::Bool: return std::string("boolean `") + (v.b ? "true" : "false") + "`";
    case JVal::Int: return "integer `" + int_text(v.s) + "`";
    case JVal::Float: return "floating point `" + py_float_repr(std::strtod(v.s.c_str(), nullptr)) + "`";
    case JVal::Str: return "string \"" + v.s + "\"";
    case JVal::Arr: return "a sequence";
    case JVal::Obj: return "a map";
  }
  return "?";
}

static const std::string& want_str(const JVal& v) {
  if (v.t != JVal::Str) throw WireErr("invalid type: " + desc(v) + ", expected a string");
  return v.s;
}

static unsigned long long want_uint(const JVal& v, const char* name, unsigned long long hi) {
  if (v.t != JVal::Int) throw WireErr("invalid type: " + desc(v) + ", expected " + name);
  const std::string t = int_text(v.s);
  const bool neg = !t.empty() && t[0] == '-';
  unsigned long long x = 0;
  bool over = false;
  for (size_t i = neg ? 1 : 0; i < t.size(); ++i) {
    if (x > (~0ull - 9) / 10) over = true;
    x = x * 10 + (unsigned)(t[i] - '0');
  }
  if (neg || over || x > hi) throw WireErr("invalid value: integer `" + t + "`, expected " + name);
  return x;
}

static float want_f32(const JVal& v) {
  if (v.t != JVal::Int && v.t != JVal::Float)
    throw WireErr("invalid type: " + desc(v) + ", expected f32");
  return (float)parse_f64(v.s.data(), v.s.size());
}

static const JVal& want_obj(const JVal& v, const char* name) {
  if (v.t != JVal::Obj) throw WireErr("invalid type: " + desc(v) + ", expected struct " + name);
  return v;
}

// required field (missing -> serde "missing field" error); `opt` fields return nullptr when
// absent or null
static const JVal* field(const JVal& o, const char* name, bool opt = false) {
  const JVal* f = o.get(name);
  if (!f || (opt && f->t == JVal::Null)) {
    if (opt) return nullptr;
    throw WireErr(std::string("missing field `") + name + "`");
  }
  return f;
}

static size_t rstrip_len(const std::string& s) {
  size_t n = s.size();
  while (n && (s[n - 1] == ' ' || s[n - 1] == '\t' || s[n - 1] == '\n' || s[n - 1] == '\r' ||
               s[n - 1] == '\f' || s[n - 1] == '\v'))
    --n;
  return n;
}

// WireModel.from_json error text: JSON syntax errors verbatim, "missing field" + closing position
template <class F>
static bool decode(const std::string& body, F&& f, std::string& err) {
  try {
    JVal v = parse_json(body);
    f(v);
    return true;
  } catch (const JsonError& e) {
    err = e.what();
  } catch (const WireErr& e) {
    err = e.what();
    if (err.rfind("missing field", 0) == 0)
      err += " at line 1 column " + std::to_string(rstrip_len(body));
  }
  return false;
}

// ---- Rust str::trim (Unicode White_Space) ----
static bool is_ws(uint32_t c) {
  return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F ||
         c == 0x205F || c == 0x3000;
}
static uint32_t cp_at(const std::string& s, size_t i, int& len) {
  const unsigned char c = (unsigned char)s[i];
  len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
  if (i + len > s.size()) len = 1;
  if (len == 1) return c;
  uint32_t v = c & (0x7F >> len);
  for (int k = 1; k < len; ++k) v = (v << 6) | ((unsigned char)s[i + k] & 0x3F);
  return v;
}
static std::string rust_trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e) {
    int L;
    if (!is_ws(cp_at(s, b, L))) break;
    b += L;
  }
  while (e > b) {
    size_t st = e - 1;
    while (st > b && (((unsigned char)s[st]) >> 6) == 2) --st;
    int L;
    if (!is_ws(cp_at(s, st, L))) break;
    e = st;
  }
  return s.substr(b, e - b);
}

static std::string jstr(const std::string& s) {
  std::string o;
  append_json_string(o, s.data(), s.size());
  return o;
}

static std::string uuid4(std::mt19937_64& g) {
  uint64_t a = g(), b = g();
  a = (a & 0xFFFFFFFFFFFF0FFFull) | 0x0000000000004000ull;
  b = (b & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;
  char buf[40];
  snprintf(buf, sizeof buf, "%08x-%04x-%04x-%04x-%012llx", (unsigned)(a >> 32),
           (unsigned)((a >> 16) & 0xFFFF), (unsigned)(a & 0xFFFF), (unsigned)(b >> 48),
           (unsigned long long)(b & 0xFFFFFFFFFFFFull));
  return buf;
}

// ============================================================================ configuration
struct Config {
  std::string host = "0.0.0.0";
  int port = 8080;
  std::string nats_host = "127.0.0.1";
  int nats_port = 4222;
  int workers = 1;
  double embed_timeout_s = 15.0, search_timeout_s = 20.0, nats_request_timeout_s = 10.0;
  int sse_capacity = 32;
  double sse_keepalive_s = 15.0;
  unsigned max_length_limit = 1000;
  std::string index_html;
  bool log = true;
};

static constexpr size_t JSON_LIMIT = 2 * 1024 * 1024;
static constexpr size_t MAX_HEADER = 64 * 1024;
static constexpr size_t MAX_BODY = 64ull * 1024 * 1024;

struct Stats {
  std::atomic<long long> requests{0}, search_ok{0}, search_err{0}, published{0}, sse_events{0},
      sse_lagged{0}, sse_clients{0}, nats_reconnects{0}, bad_requests{0};
  std::mutex mu;  // guards the latency reservoirs and the service-metrics map
  std::vector<double> search_ms, embed_hop_ms, index_hop_ms;
  std::unordered_map<std::string, std::string> service_metrics;
  void observe(std::vector<double>& v, double ms) {
    std::lock_guard<std::mutex> g(mu);
    if (v.size() >= 4096) v.erase(v.begin(), v.begin() + 2048);
    v.push_back(ms);
  }
};

class Gateway;

// ============================================================================ per-thread loop
class Loop {
 public:
  Loop(Gateway* gw, const Config& cfg, Stats& st, int idx)
      : gw_(gw), cfg_(cfg), st_(st), idx_(idx), rng_(std::random_device{}() ^ (uint64_t)idx << 32) {
    const char* al = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
    inbox_ = "_INBOX.";
    for (int i = 0; i < 22; ++i) inbox_ += al[rng_() % 62];
    inbox_ += '.';
  }

  int bind_listener() {
    lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (lfd_ < 0) throw std::runtime_error(std::string("socket: ") + strerror(errno));
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)cfg_.port);
    if (cfg_.host.empty() || cfg_.host == "0.0.0.0") a.sin_addr.s_addr = htonl(INADDR_ANY);
    else if (inet_pton(AF_INET, cfg_.host.c_str(), &a.sin_addr) != 1) resolve(cfg_.host, a.sin_addr);
    if (::bind(lfd_, (sockaddr*)&a, sizeof a) < 0 || ::listen(lfd_, 2048) < 0) {
      const std::string m = strerror(errno);
      ::close(lfd_);
      lfd_ = -1;
      throw std::runtime_error("bind " + cfg_.host + ":" + std::to_string(cfg_.port) + ": " + m);
    }
    socklen_t len = sizeof a;
    getsockname(lfd_, (sockaddr*)&a, &len);
    return ntohs(a.sin_port);
  }

  void start() {
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    wake_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    add(lfd_, EPOLLIN, &listen_tag_);
    add(wake_, EPOLLIN, &wake_tag_);
    running_ = true;
    th_ = std::thread([this] { run(); });
  }

  void stop() {
    if (!th_.joinable()) return;
    running_ = false;
    uint64_t one = 1;
    (void)!::write(wake_, &one, sizeof one);
    th_.join();
    for (auto& kv : conns_) ::close(kv.second->fd);
    conns_.clear();
    if (nfd_ >= 0) ::close(nfd_);
    ::close(lfd_);
    ::close(wake_);
    ::close(ep_);
  }

  bool nats_up() const { return nats_state_ == 2; }

 private:
  // ---------------------------------------------------------------- types
  struct HttpConn {
    int fd = -1;
    uint64_t serial = 0;
    std::string in, out;
    size_t out_pos = 0;
    bool closing = false, close_after = false, busy = false, epollout = false;
    bool sse = false, continued = false;
    std::deque<std::string> sse_backlog;
    double sse_last = 0;
    std::string origin;  // CORS origin of the in-flight request (allowed), echoed on the reply
  };
  struct Req {  // a parked /api/search/semantic request
    int fd;
    uint64_t serial;
    std::string rid;
    unsigned top_k;
    int hop;           // 1 = waiting for the embedding, 2 = waiting for the search results
    double t0, t1;     // handler start, embedding received
    double deadline;   // NATS request timeout of the current hop
    double hop_deadline;  // gateway-level hop timeout (15 s / 20 s)
    bool close_after;
  };

  // ---------------------------------------------------------------- epoll helpers
  void add(int fd, uint32_t ev, void* tag) {
    epoll_event e{};
    e.events = ev;
    e.data.ptr = tag;
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
  }
  void mod(int fd, uint32_t ev, void* tag) {
    epoll_event e{};
    e.events = ev;
    e.data.ptr = tag;
    epoll_ctl(ep_, EPOLL_CTL_MOD, fd, &e);
  }
  static void resolve(const std::string& host, in_addr& out) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
      throw std::runtime_error("cannot resolve " + host);
    out = ((sockaddr_in*)res->ai_addr)->sin_addr;
    freeaddrinfo(res);
  }
  void logf(const char* fmt, const std::string& a = "", const std::string& b = "") {
    if (!cfg_.log) return;
    fprintf(stderr, "[api_service-native:%d] ", idx_);
    fprintf(stderr, fmt, a.c_str(), b.c_str());
    fputc('\n', stderr);
  }

  // ---------------------------------------------------------------- main loop
  void run() {
    std::vector<epoll_event> evs(512);
    double next_tick = 0;
    while (running_) {
      if (nats_state_ == 0 && now_s() >= nats_retry_at_) nats_connect();
      const int n = epoll_wait(ep_, evs.data(), (int)evs.size(), 50);
      for (int i = 0; i < n; ++i) {
        void* tag = evs[i].data.ptr;
        const uint32_t e = evs[i].events;
        if (tag == &wake_tag_) {
          uint64_t v;
          (void)!::read(wake_, &v, sizeof v);
        } else if (tag == &listen_tag_) {
          accept_all();
        } else if (tag == &nats_tag_) {
          nats_event(e);
        } else {
          HttpConn* c = static_cast<HttpConn*>(tag);
          if (c->closing) continue;
          if (e & EPOLLIN) on_http_readable(c);
          else if (e & (EPOLLERR | EPOLLHUP)) c->closing = true;
          if (!c->closing && (e & EPOLLOUT)) flush(c);
        }
      }
      const double t = now_s();
      if (t >= next_tick) {
        next_tick = t + 0.05;
        tick(t);
      }
      nats_flush();
      reap();
    }
  }

  void tick(double t) {
    // request timeouts (NATS request timeout first, like async-nats' 10 s default)
    std::vector<std::string> expired;
    for (auto& kv : reqs_)
      if (t >= kv.second.deadline || t >= kv.second.hop_deadline) expired.push_back(kv.first);
    for (auto& tok : expired) {
      auto it = reqs_.find(tok);
      if (it == reqs_.end()) continue;
      Req r = it->second;
      reqs_.erase(it);
      const bool nats_to = r.deadline <= r.hop_deadline;
      if (r.hop == 1)
        search_fail(r, 503, nats_to ? "Failed to get embedding from preprocessing service: request timed out"
                                    : "Timeout: Failed to get embedding from preprocessing service within " +
                                          std::to_string((int)cfg_.embed_timeout_s) + " seconds");
      else
        search_fail(r, 503, nats_to ? "Failed to get search results from vector memory service: request timed out"
                                    : "Timeout: Failed to get search results from vector memory service "
                                      "within " + std::to_string((int)cfg_.search_timeout_s) + " seconds");
    }
    // SSE keep-alives
    for (auto& kv : conns_) {
      HttpConn* c = kv.second.get();
      if (c->sse && !c->closing && t - c->sse_last >= cfg_.sse_keepalive_s) {
        sse_write(c, ": keep-alive\n\n");
        c->sse_last = t;
      }
    }
  }

  // ---------------------------------------------------------------- HTTP side
  void accept_all() {
    for (;;) {
      const int fd = accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<HttpConn>();
      c->fd = fd;
      c->serial = ++serial_;
      add(fd, EPOLLIN, c.get());
      conns_[fd] = std::move(c);
    }
  }

  void on_http_readable(HttpConn* c) {
    char buf[1 << 16];
    for (;;) {
      const ssize_t r = ::read(c->fd, buf, sizeof buf);
      if (r > 0) {
        if (!c->sse) c->in.append(buf, (size_t)r);  // SSE clients send nothing we need
        if (c->in.size() > MAX_BODY + MAX_HEADER) {
          c->closing = true;
          return;
        }
        continue;
      }
      if (r == 0) {
        c->closing = true;
        return;
      }
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      c->closing = true;
      return;
    }
    process(c);
  }

  static std::string lower(std::string s) {
    for (auto& ch : s) ch = (char)tolower((unsigned char)ch);
    return s;
  }

  void process(HttpConn* c) {
    while (!c->closing && !c->busy && !c->sse) {
      const size_t he = c->in.find("\r\n\r\n");
      if (he == std::string::npos) {
        if (c->in.size() > MAX_HEADER) {
          respond(c, 431, "text/plain; charset=utf-8", "Request Header Fields Too Large", true);
        }
        return;
      }
      // request line + headers
      const std::string head = c->in.substr(0, he);
      size_t le = head.find("\r\n");
      const std::string rl = head.substr(0, le);
      const size_t s1 = rl.find(' '), s2 = rl.rfind(' ');
      if (s1 == std::string::npos || s2 == s1) {
        respond(c, 400, "text/plain; charset=utf-8", "Bad Request", true);
        return;
      }
      const std::string method = rl.substr(0, s1);
      std::string target = rl.substr(s1 + 1, s2 - s1 - 1);
      const std::string version = rl.substr(s2 + 1);
      const size_t qpos = target.find('?');
      if (qpos != std::string::npos) target.resize(qpos);
      std::unordered_map<std::string, std::string> h;
      size_t pos = le == std::string::npos ? head.size() : le + 2;
      while (pos < head.size()) {
        size_t e = head.find("\r\n", pos);
        if (e == std::string::npos) e = head.size();
        const size_t colon = head.find(':', pos);
        if (colon != std::string::npos && colon < e) {
          std::string k = lower(head.substr(pos, colon - pos));
          size_t vb = colon + 1;
          while (vb < e && (head[vb] == ' ' || head[vb] == '\t')) ++vb;
          size_t ve = e;
          while (ve > vb && (head[ve - 1] == ' ' || head[ve - 1] == '\t')) --ve;
          h[k] = head.substr(vb, ve - vb);
        }
        pos = e + 2;
      }
      if (h.count("transfer-encoding") && lower(h["transfer-encoding"]).find("chunked") != std::string::npos) {
        respond(c, 411, "text/plain; charset=utf-8", "Length Required", true);
        return;
      }
      size_t clen = 0;
      if (h.count("content-length")) {
        const std::string& v = h["content-length"];
        auto r = std::from_chars(v.data(), v.data() + v.size(), clen);
        if (r.ec != std::errc() || r.ptr != v.data() + v.size()) {
          respond(c, 400, "text/plain; charset=utf-8", "Bad Request", true);
          return;
        }
      }
      if (clen > MAX_BODY) {
        respond(c, 413, "text/plain; charset=utf-8",
                "JSON payload (" + std::to_string(clen) + " bytes) is larger than allowed (limit: " +
                    std::to_string(JSON_LIMIT) + " bytes).", true);
        return;
      }
      if (c->in.size() < he + 4 + clen) {  // body not complete yet
        // curl & co. hold bodies > 1 KiB back until "100 Continue" (or a 1 s timeout)
        if (!c->continued && h.count("expect") && lower(h["expect"]) == "100-continue") {
          c->out += "HTTP/1.1 100 Continue\r\n\r\n";
          c->continued = true;
          flush(c);
        }
        return;
      }
      c->continued = false;
      std::string body = c->in.substr(he + 4, clen);
      c->in.erase(0, he + 4 + clen);
      const std::string conn_h = lower(h.count("connection") ? h["connection"] : "");
      c->close_after = version == "HTTP/1.0" ? conn_h != "keep-alive" : conn_h == "close";
      ++st_.requests;
      route(c, method, target, h, body);
      if (c->close_after) return;  // nothing after a Connection: close request is served
    }
  }

  void route(HttpConn* c, const std::string& method, const std::string& path,
             std::unordered_map<std::string, std::string>& h, const std::string& body) {
    // CORS (actix-cors of main.rs:555-567)
    c->origin.clear();
    auto oit = h.find("origin");
    if (oit != h.end()) {
      const std::string& o = oit->second;
      const bool ok = o.rfind("http://localhost", 0) == 0 || o.rfind("http://marchenzo", 0) == 0 ||
                      o.rfind("http://127.0.0.1", 0) == 0;
      if (!ok) {
        respond(c, 400, "text/plain; charset=utf-8", "Origin is not allowed to make this request");
        return;
      }
      if (method == "OPTIONS" && h.count("access-control-request-method")) {
        std::string m = h["access-control-request-method"];
        for (auto& ch : m) ch = (char)toupper((unsigned char)ch);
        if (m != "GET" && m != "POST" && m != "OPTIONS") {
          respond(c, 400, "text/plain; charset=utf-8", "Requested method is not allowed");
          return;
        }
        std::string extra = "access-control-allow-origin: " + o +
                            "\r\naccess-control-allow-methods: GET, OPTIONS, POST"
                            "\r\naccess-control-allow-headers: accept, authorization, content-type"
                            "\r\naccess-control-max-age: 3600\r\nvary: Origin\r\n";
        respond(c, 200, "", "", false, extra);
        return;
      }
      c->origin = o;
    }
    const bool get = method == "GET", post = method == "POST";
    if (path == "/api/submit-url") {
      if (!post) return method_not_allowed(c);
      return submit_url(c, h, body);
    }
    if (path == "/api/generate-text") {
      if (!post) return method_not_allowed(c);
      return generate_text(c, h, body);
    }
    if (path == "/api/search/semantic") {
      if (!post) return method_not_allowed(c);
      return semantic_search(c, h, body);
    }
    if (path == "/api/events") {
      if (!get) return method_not_allowed(c);
      return events(c);
    }
    if (path == "/api/health") {
      if (!get) return method_not_allowed(c);
      const bool up = nats_up();
      return respond(c, up ? 200 : 503, "application/json",
                     up ? "{\"status\":\"ok\",\"nats\":true,\"impl\":\"native\"}"
                        : "{\"status\":\"degraded\",\"nats\":false,\"impl\":\"native\"}");
    }
    if (path == "/api/metrics") {
      if (!get) return method_not_allowed(c);
      return respond(c, 200, "application/json", gw_metrics());
    }
    if (path == "/") {
      if (!get) return method_not_allowed(c);
      if (cfg_.index_html.empty()) return respond(c, 200, "text/plain; charset=utf-8", "symbiont api");
      return respond(c, 200, "text/html; charset=utf-8", cfg_.index_html);
    }
    respond(c, 404, "text/plain; charset=utf-8", "Not Found");
  }

  void method_not_allowed(HttpConn* c) {
    respond(c, 405, "text/plain; charset=utf-8", "Method Not Allowed");
  }

  static const char* reason(int s) {
    switch (s) {
      case 200: return "OK";
      case 400: return "Bad Request";
      case 404: return "Not Found";
      case 405: return "Method Not Allowed";
      case 411: return "Length Required";
      case 413: return "Payload Too Large";
      case 431: return "Request Header Fields Too Large";
      case 500: return "Internal Server Error";
      case 503: return "Service Unavailable";
    }
    return "OK";
  }

  void respond(HttpConn* c, int status, const std::string& ctype, const std::string& body,
               bool close = false, const std::string& extra = "") {
    std::string& o = c->out;
    o += "HTTP/1.1 ";
    o += std::to_string(status);
    o += ' ';
    o += reason(status);
    o += "\r\nserver: symbiont-native\r\n";
    if (!ctype.empty()) {
      o += "content-type: ";
      o += ctype;
      o += "\r\n";
    }
    o += "content-length: ";
    o += std::to_string(body.size());
    o += "\r\n";
    if (!c->origin.empty()) {
      o += "access-control-allow-origin: ";
      o += c->origin;
      o += "\r\nvary: Origin\r\n";
    }
    o += extra;
    if (close || c->close_after) {
      o += "connection: close\r\n";
      c->close_after = true;
    }
    o += "\r\n";
    o += body;
    if (status >= 400) ++st_.bad_requests;
    flush(c);
  }

  void flush(HttpConn* c) {
    while (c->out_pos < c->out.size()) {
      const ssize_t w = ::send(c->fd, c->out.data() + c->out_pos, c->out.size() - c->out_pos,
                               MSG_NOSIGNAL);
      if (w > 0) {
        c->out_pos += (size_t)w;
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      c->closing = true;
      return;
    }
    if (c->out_pos == c->out.size()) {
      c->out.clear();
      c->out_pos = 0;
      if (c->sse) {  // refill from the backlog
        while (!c->sse_backlog.empty() && c->out.size() < 65536) {
          c->out += c->sse_backlog.front();
          c->sse_backlog.pop_front();
        }
        if (!c->out.empty()) return flush(c);
      } else if (c->close_after && !c->busy) {
        ::shutdown(c->fd, SHUT_WR);
        c->closing = true;
        return;
      }
    } else if (c->out_pos > (1u << 20)) {
      c->out.erase(0, c->out_pos);
      c->out_pos = 0;
    }
    const bool want = !c->out.empty();
    if (want != c->epollout) {
      mod(c->fd, EPOLLIN | (want ? EPOLLOUT : 0), c);
      c->epollout = want;
    }
  }

  HttpConn* find_conn(int fd, uint64_t serial) {
    auto it = conns_.find(fd);
    if (it == conns_.end() || it->second->serial != serial || it->second->closing) return nullptr;
    return it->second.get();
  }

  void reap() {
    for (auto it = conns_.begin(); it != conns_.end();) {
      if (it->second->closing) {
        if (it->second->sse) --st_.sse_clients;
        epoll_ctl(ep_, EPOLL_CTL_DEL, it->first, nullptr);
        ::close(it->first);
        it = conns_.erase(it);
      } else {
        ++it;
      }
    }
  }

  // actix web::Json<T> extractor: content type, size limit, decode
  bool json_body(HttpConn* c, std::unordered_map<std::string, std::string>& h,
                 const std::string& body) {
    std::string ct = lower(h.count("content-type") ? h["content-type"] : "");
    const size_t semi = ct.find(';');
    if (semi != std::string::npos) ct.resize(semi);
    while (!ct.empty() && (ct.back() == ' ' || ct.back() == '\t')) ct.pop_back();
    while (!ct.empty() && (ct.front() == ' ' || ct.front() == '\t')) ct.erase(0, 1);
    const bool json = ct == "application/json" ||
                      (ct.size() >= 5 && ct.compare(ct.size() - 5, 5, "+json") == 0);
    if (!json) {
      respond(c, 400, "text/plain; charset=utf-8", "Content type error");
      return false;
    }
    if (body.size() > JSON_LIMIT) {
      respond(c, 413, "text/plain; charset=utf-8",
              "JSON payload (" + std::to_string(body.size()) +
                  " bytes) is larger than allowed (limit: " + std::to_string(JSON_LIMIT) + " bytes).");
      return false;
    }
    return true;
  }

  static std::string api_response(const std::string& msg, const std::string* task_id) {
    return "{\"message\":" + jstr(msg) + ",\"task_id\":" + (task_id ? jstr(*task_id) : "null") + "}";
  }

  void submit_url(HttpConn* c, std::unordered_map<std::string, std::string>& h,
                  const std::string& body) {
    if (!json_body(c, h, body)) return;
    std::string url, err;
    if (!decode(body, [&](const JVal& v) {
          url = want_str(*field(want_obj(v, "SubmitUrlApiPayload"), "url"));
        }, err))
      return respond(c, 400, "text/plain; charset=utf-8", "Json deserialize error: " + err);
    url = rust_trim(url);
    if (url.empty()) return respond(c, 400, "application/json", api_response("URL cannot be empty", nullptr));
    if (!nats_publish("tasks.perceive.url", "", "{\"url\":" + jstr(url) + "}"))
      return respond(c, 500, "application/json",
                     api_response("Failed to publish task to processing queue", nullptr));
    respond(c, 200, "application/json",
            api_response("Task to scrape URL '" + url + "' submitted successfully.", nullptr));
  }

  void generate_text(HttpConn* c, std::unordered_map<std::string, std::string>& h,
                     const std::string& body) {
    if (!json_body(c, h, body)) return;
    std::string task_id, err;
    const std::string* prompt = nullptr;
    std::string prompt_s;
    unsigned long long max_len = 0;
    if (!decode(body, [&](const JVal& v) {
          const JVal& o = want_obj(v, "GenerateTextTask");
          task_id = want_str(*field(o, "task_id"));
          if (const JVal* p = field(o, "prompt", true)) {
            prompt_s = want_str(*p);
            prompt = &prompt_s;
          }
          max_len = want_uint(*field(o, "max_length"), "u32", 0xFFFFFFFFull);
        }, err))
      return respond(c, 400, "text/plain; charset=utf-8", "Json deserialize error: " + err);
    if (rust_trim(task_id).empty())
      return respond(c, 400, "application/json", api_response("task_id cannot be empty", nullptr));
    if (max_len == 0 || max_len > cfg_.max_length_limit)
      return respond(c, 400, "application/json",
                     api_response("max_length must be between 1 and " +
                                      std::to_string(cfg_.max_length_limit), &task_id));
    const std::string task = "{\"task_id\":" + jstr(task_id) + ",\"prompt\":" +
                             (prompt ? jstr(*prompt) : "null") + ",\"max_length\":" +
                             std::to_string(max_len) + "}";
    if (!nats_publish("tasks.generation.text", "", task))
      return respond(c, 500, "application/json",
                     api_response("Failed to publish generation task to queue", &task_id));
    respond(c, 200, "application/json",
            api_response("Text generation task (id: " + task_id + ") submitted successfully.", &task_id));
  }

  void events(HttpConn* c) {
    std::string o = "HTTP/1.1 200 OK\r\nserver: symbiont-native\r\n"
                    "content-type: text/event-stream; charset=utf-8\r\ncache-control: no-cache\r\n";
    if (!c->origin.empty()) o += "access-control-allow-origin: " + c->origin + "\r\nvary: Origin\r\n";
    o += "transfer-encoding: chunked\r\n\r\n";
    c->out += o;
    c->sse = true;
    c->sse_last = now_s();
    c->in.clear();
    ++st_.sse_clients;
    flush(c);
  }

  static std::string chunk(const std::string& data) {
    char hex[16];
    snprintf(hex, sizeof hex, "%zx\r\n", data.size());
    return hex + data + "\r\n";
  }

  void sse_write(HttpConn* c, const std::string& data) {
    std::string ch = chunk(data);
    if (c->out.empty()) {
      c->out = std::move(ch);
      flush(c);
      return;
    }
    if ((int)c->sse_backlog.size() >= cfg_.sse_capacity) {  // lagging receiver: drop the oldest
      c->sse_backlog.pop_front();
      ++st_.sse_lagged;
    }
    c->sse_backlog.push_back(std::move(ch));
  }

  void broadcast_generated(const std::string& payload) {
    // decode + re-encode as GeneratedTextMessage (drops unknown fields, canonical layout)
    std::string id, text, err;
    unsigned long long ts = 0;
    if (!decode(payload, [&](const JVal& v) {
          const JVal& o = want_obj(v, "GeneratedTextMessage");
          id = want_str(*field(o, "original_task_id"));
          text = want_str(*field(o, "generated_text"));
          ts = want_uint(*field(o, "timestamp_ms"), "u64", ~0ull);
        }, err)) {
      logf("[NATS_SSE_Bridge] Failed to deserialize GeneratedTextMessage from NATS: %s", err);
      return;
    }
    const std::string ev = "data: {\"original_task_id\":" + jstr(id) + ",\"generated_text\":" +
                           jstr(text) + ",\"timestamp_ms\":" + std::to_string(ts) + "}\n\n";
    const double t = now_s();
    int n = 0;
    for (auto& kv : conns_) {
      HttpConn* c = kv.second.get();
      if (!c->sse || c->closing) continue;
      sse_write(c, ev);
      c->sse_last = t;
      ++n;
    }
    st_.sse_events += n;
  }

  // ---------------------------------------------------------------- semantic search
  void semantic_search(HttpConn* c, std::unordered_map<std::string, std::string>& h,
                       const std::string& body) {
    if (!json_body(c, h, body)) return;
    std::string query, err;
    unsigned long long top_k = 0;
    if (!decode(body, [&](const JVal& v) {
          const JVal& o = want_obj(v, "SemanticSearchApiRequest");
          query = want_str(*field(o, "query_text"));
          top_k = want_uint(*field(o, "top_k"), "u32", 0xFFFFFFFFull);
        }, err))
      return respond(c, 400, "text/plain; charset=utf-8", "Json deserialize error: " + err);
    Req r;
    r.fd = c->fd;
    r.serial = c->serial;
    r.rid = uuid4(rng_);
    r.top_k = (unsigned)top_k;
    r.hop = 1;
    r.t0 = now_s();
    r.t1 = 0;
    r.close_after = c->close_after;
    const std::string task = "{\"request_id\":" + jstr(r.rid) + ",\"text_to_embed\":" + jstr(query) + "}";
    c->busy = true;
    std::string nerr;
    const std::string tok = nats_request("tasks.embedding.for_query", task, nerr);
    if (tok.empty()) {
      c->busy = false;
      return search_fail_conn(c, r.rid, 503, "Failed to get embedding from preprocessing service: " + nerr);
    }
    r.deadline = r.t0 + cfg_.nats_request_timeout_s;
    r.hop_deadline = r.t0 + cfg_.embed_timeout_s;
    reqs_[tok] = r;
  }

  static std::string search_body(const std::string& rid, const std::string& results,
                                 const std::string* err) {
    return "{\"search_request_id\":" + jstr(rid) + ",\"results\":" + results +
           ",\"error_message\":" + (err ? jstr(*err) : "null") + "}";
  }

  void search_fail_conn(HttpConn* c, const std::string& rid, int status, const std::string& msg) {
    ++st_.search_err;
    respond(c, status, "application/json", search_body(rid, "[]", &msg));
  }

  void search_fail(const Req& r, int status, const std::string& msg) {
    HttpConn* c = find_conn(r.fd, r.serial);
    if (!c) return;
    c->busy = false;
    search_fail_conn(c, r.rid, status, msg);
    process(c);  // pipelined requests queued behind this one
  }

  void on_reply(const std::string& token, const char* hdr, size_t hl, const char* pl, size_t pn) {
    auto it = reqs_.find(token);
    if (it == reqs_.end()) return;  // late reply after a timeout
    Req r = it->second;
    reqs_.erase(it);
    const bool no_responders = hl >= 12 && std::string(hdr, std::min<size_t>(hl, 16)).find(" 503") != std::string::npos;
    const std::string payload(pl, pn);
    if (r.hop == 1) {
      if (no_responders)
        return search_fail(r, 503, "Failed to get embedding from preprocessing service: no responders");
      std::string err, emb;
      const std::string* error_message = nullptr;
      std::string em_s;
      bool has_emb = false;
      if (!decode(payload, [&](const JVal& v) {
            const JVal& o = want_obj(v, "QueryEmbeddingResult");
            want_str(*field(o, "request_id"));
            if (const JVal* e = field(o, "embedding", true)) {
              if (e->t != JVal::Arr) throw WireErr("invalid type: " + desc(*e) + ", expected a sequence");
              emb.reserve(e->a.size() * 12 + 2);
              std::vector<float> f(e->a.size());
              for (size_t i = 0; i < f.size(); ++i) f[i] = want_f32(e->a[i]);
              append_f32_array(emb, f.data(), f.size());
              has_emb = true;
            }
            if (const JVal* m = field(o, "model_name", true)) want_str(*m);
            if (const JVal* m = field(o, "error_message", true)) {
              em_s = want_str(*m);
              error_message = &em_s;
            }
          }, err))
        return search_fail(r, 500, "Internal error: Failed to parse embedding service response");
      if (error_message) return search_fail(r, 500, "Error from preprocessing service: " + *error_message);
      if (!has_emb) return search_fail(r, 500, "Preprocessing service did not return an embedding.");
      r.t1 = now_s();
      st_.observe(st_.embed_hop_ms, (r.t1 - r.t0) * 1e3);
      const std::string task = "{\"request_id\":" + jstr(r.rid) + ",\"query_embedding\":" + emb +
                               ",\"top_k\":" + std::to_string(r.top_k) + "}";
      std::string nerr;
      const std::string tok = nats_request("tasks.search.semantic.request", task, nerr);
      if (tok.empty())
        return search_fail(r, 503, "Failed to get search results from vector memory service: " + nerr);
      r.hop = 2;
      r.deadline = r.t1 + cfg_.nats_request_timeout_s;
      r.hop_deadline = r.t1 + cfg_.search_timeout_s;
      reqs_[tok] = r;
      return;
    }
    if (no_responders)
      return search_fail(r, 503, "Failed to get search results from vector memory service: no responders");
    std::string err, results = "[";
    const std::string* error_message = nullptr;
    std::string em_s;
    if (!decode(payload, [&](const JVal& v) {
          const JVal& o = want_obj(v, "SemanticSearchNatsResult");
          want_str(*field(o, "request_id"));
          const JVal* rs = field(o, "results");
          if (rs->t != JVal::Arr) throw WireErr("invalid type: " + desc(*rs) + ", expected a sequence");
          bool first = true;
          for (const JVal& it : rs->a) {
            const JVal& item = want_obj(it, "SemanticSearchResultItem");
            const std::string& pid = want_str(*field(item, "qdrant_point_id"));
            const float score = want_f32(*field(item, "score"));
            const JVal& p = want_obj(*field(item, "payload"), "QdrantPointPayload");
            const std::string& doc = want_str(*field(p, "original_document_id"));
            const std::string& src = want_str(*field(p, "source_url"));
            const std::string& sent = want_str(*field(p, "sentence_text"));
            const unsigned long long order = want_uint(*field(p, "sentence_order"), "u32", 0xFFFFFFFFull);
            const std::string& model = want_str(*field(p, "model_name"));
            const unsigned long long at = want_uint(*field(p, "processed_at_ms"), "u64", ~0ull);
            if (!first) results += ',';
            first = false;
            results += "{\"qdrant_point_id\":" + jstr(pid) + ",\"score\":";
            append_f32(results, score);
            results += ",\"payload\":{\"original_document_id\":" + jstr(doc) + ",\"source_url\":" +
                       jstr(src) + ",\"sentence_text\":" + jstr(sent) + ",\"sentence_order\":" +
                       std::to_string(order) + ",\"model_name\":" + jstr(model) +
                       ",\"processed_at_ms\":" + std::to_string(at) + "}}";
          }
          if (const JVal* m = field(o, "error_message", true)) {
            em_s = want_str(*m);
            error_message = &em_s;
          }
        }, err))
      return search_fail(r, 500, "Internal error: Failed to parse search service response");
    if (error_message) return search_fail(r, 500, "Error from vector memory service: " + *error_message);
    results += ']';
    HttpConn* c = find_conn(r.fd, r.serial);
    const double t2 = now_s();
    st_.observe(st_.index_hop_ms, (t2 - r.t1) * 1e3);
    st_.observe(st_.search_ms, (t2 - r.t0) * 1e3);
    ++st_.search_ok;
    if (!c) return;
    c->busy = false;
    respond(c, 200, "application/json", search_body(r.rid, results, nullptr));
    process(c);
  }

  std::string gw_metrics();

  // ---------------------------------------------------------------- NATS side
  void nats_connect() {
    nfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)cfg_.nats_port);
    try {
      if (inet_pton(AF_INET, cfg_.nats_host.c_str(), &a.sin_addr) != 1) resolve(cfg_.nats_host, a.sin_addr);
    } catch (const std::exception&) {
      ::close(nfd_);
      nfd_ = -1;
      nats_retry_at_ = now_s() + 0.5;
      return;
    }
    int one = 1;
    setsockopt(nfd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    const int r = ::connect(nfd_, (sockaddr*)&a, sizeof a);
    if (r < 0 && errno != EINPROGRESS) {
      ::close(nfd_);
      nfd_ = -1;
      nats_retry_at_ = now_s() + 0.5;
      return;
    }
    nats_state_ = 1;  // connecting: wait for INFO
    nin_.clear();
    nin_pos_ = 0;
    nout_.clear();
    nout_pos_ = 0;
    nneed_ = -1;
    add(nfd_, EPOLLIN, &nats_tag_);  // the server's INFO line doubles as "connected"
    nats_epollout_ = false;
  }

  void nats_down(const char* why) {
    if (nfd_ >= 0) {
      epoll_ctl(ep_, EPOLL_CTL_DEL, nfd_, nullptr);
      ::close(nfd_);
      nfd_ = -1;
    }
    if (nats_state_ == 2) {
      logf("[NATS] connection lost (%s); reconnecting", why);
      ++st_.nats_reconnects;
    }
    nats_state_ = 0;
    nats_retry_at_ = now_s() + 0.25;
    // in-flight requests cannot be answered on a new connection's inbox traffic any more
    std::vector<Req> lost;
    for (auto& kv : reqs_) lost.push_back(kv.second);
    reqs_.clear();
    for (const Req& r : lost)
      search_fail(r, 503, std::string(r.hop == 1 ? "Failed to get embedding from preprocessing service: "
                                                 : "Failed to get search results from vector memory service: ") +
                             "connection closed");
  }

  void nats_event(uint32_t e) {
    if (e & (EPOLLERR | EPOLLHUP)) {
      if (!(e & EPOLLIN)) return nats_down("socket error");
    }
    if (e & EPOLLIN) {
      char buf[1 << 16];
      for (;;) {
        const ssize_t r = ::read(nfd_, buf, sizeof buf);
        if (r > 0) {
          nin_.append(buf, (size_t)r);
          continue;
        }
        if (r == 0) return nats_down("closed by server");
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        return nats_down(strerror(errno));
      }
      nats_parse();
    }
    if (nfd_ >= 0 && (e & EPOLLOUT)) nats_flush();
  }

  void nats_send(const std::string& s) { nout_ += s; }

  void nats_flush() {
    if (nfd_ < 0) return;
    while (nout_pos_ < nout_.size()) {
      const ssize_t w = ::send(nfd_, nout_.data() + nout_pos_, nout_.size() - nout_pos_, MSG_NOSIGNAL);
      if (w > 0) {
        nout_pos_ += (size_t)w;
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == ENOTCONN)) break;
      return nats_down("write failed");
    }
    if (nout_pos_ == nout_.size()) {
      nout_.clear();
      nout_pos_ = 0;
    }
    const bool want = !nout_.empty();
    if (want != nats_epollout_) {
      mod(nfd_, EPOLLIN | (want ? EPOLLOUT : 0), &nats_tag_);
      nats_epollout_ = want;
    }
  }

  bool nats_publish(const std::string& subject, const std::string& reply, const std::string& payload) {
    if (nats_state_ != 2) return false;
    if ((long long)payload.size() > max_payload_) return false;
    std::string o = "PUB " + subject;
    if (!reply.empty()) o += " " + reply;
    o += " " + std::to_string(payload.size()) + "\r\n";
    o += payload;
    o += "\r\n";
    nats_send(o);
    ++st_.published;
    return true;
  }

  // returns the reply token, or "" with err set
  std::string nats_request(const std::string& subject, const std::string& payload, std::string& err) {
    if (nats_state_ != 2) {
      err = "connection closed";
      return "";
    }
    if ((long long)payload.size() > max_payload_) {
      err = "maximum payload exceeded (" + std::to_string(payload.size()) + " > " +
            std::to_string(max_payload_) + ")";
      return "";
    }
    const std::string tok = std::to_string(++tok_seq_);
    nats_publish(subject, inbox_ + tok, payload);
    return tok;
  }

  void nats_parse() {
    std::string& b = nin_;
    while (nfd_ >= 0) {
      const size_t avail = b.size() - nin_pos_;
      if (nneed_ >= 0) {
        if ((long long)avail < nneed_ + 2) break;
        const char* p = b.data() + nin_pos_;
        nats_msg(p, (size_t)nneed_);
        nin_pos_ += (size_t)nneed_ + 2;
        nneed_ = -1;
        continue;
      }
      const char* s = b.data() + nin_pos_;
      const void* nl = memchr(s, '\n', avail);
      if (!nl) break;
      size_t len = (const char*)nl - s;
      nin_pos_ += len + 1;
      if (len && s[len - 1] == '\r') --len;
      nats_control(std::string(s, len));
    }
    if (nin_pos_ == b.size()) {
      b.clear();
      nin_pos_ = 0;
    } else if (nin_pos_ > (1u << 16)) {
      b.erase(0, nin_pos_);
      nin_pos_ = 0;
    }
  }

  static std::vector<std::string> split_ws(const std::string& s) {
    std::vector<std::string> out;
    size_t i = 0;
    while (i < s.size()) {
      while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
      if (i >= s.size()) break;
      size_t j = i;
      while (j < s.size() && s[j] != ' ' && s[j] != '\t') ++j;
      out.emplace_back(s.substr(i, j - i));
      i = j;
    }
    return out;
  }

  void nats_control(const std::string& line) {
    auto a = split_ws(line);
    if (a.empty()) return;
    std::string op = a[0];
    for (auto& ch : op) ch = (char)toupper((unsigned char)ch);
    if (op == "MSG" && (a.size() == 4 || a.size() == 5)) {
      msg_subject_ = a[1];
      msg_sid_ = a[2];
      msg_hdr_ = 0;
      nneed_ = std::stoll(a.back());
    } else if (op == "HMSG" && (a.size() == 5 || a.size() == 6)) {
      msg_subject_ = a[1];
      msg_sid_ = a[2];
      msg_hdr_ = std::stoll(a[a.size() - 2]);
      nneed_ = std::stoll(a.back());
    } else if (op == "PING") {
      nats_send("PONG\r\n");
    } else if (op == "INFO") {
      const size_t mp = line.find("\"max_payload\":");
      if (mp != std::string::npos) max_payload_ = std::atoll(line.c_str() + mp + 14);
      if (nats_state_ == 1) {
        nats_send("CONNECT {\"verbose\":false,\"pedantic\":false,\"tls_required\":false,"
                  "\"name\":\"api_service-native\",\"lang\":\"cpp\",\"version\":\"0.3.0\","
                  "\"protocol\":1,\"headers\":true,\"no_responders\":true}\r\n");
        nats_send("SUB events.text.generated 1\r\nSUB metrics.> 2\r\nSUB " + inbox_ + "* 3\r\nPING\r\n");
        nats_state_ = 2;
        logf("[NATS] connected, reply inbox %s*", inbox_);
      }
    } else if (op == "-ERR") {
      logf("[NATS] server error: %s", line);
    }
  }

  void nats_msg(const char* p, size_t n) {
    const size_t hl = (size_t)std::min<long long>(msg_hdr_, (long long)n);
    if (msg_sid_ == "3") {
      if (msg_subject_.size() > inbox_.size())
        on_reply(msg_subject_.substr(inbox_.size()), p, hl, p + hl, n - hl);
    } else if (msg_sid_ == "1") {
      broadcast_generated(std::string(p + hl, n - hl));
    } else if (msg_sid_ == "2") {
      std::string payload(p + hl, n - hl), name = msg_subject_, err;
      decode(payload, [&](const JVal& v) {
        if (v.t == JVal::Obj)
          if (const JVal* s = v.get("service"))
            if (s->t == JVal::Str) name = s->s;
      }, err);
      std::lock_guard<std::mutex> g(st_.mu);
      st_.service_metrics[name] = payload;
    }
  }

  // ---------------------------------------------------------------- state
  Gateway* gw_;
  const Config& cfg_;
  Stats& st_;
  int idx_;
  std::mt19937_64 rng_;
  std::string inbox_;
  int lfd_ = -1, ep_ = -1, wake_ = -1, nfd_ = -1;
  int listen_tag_ = 0, wake_tag_ = 0, nats_tag_ = 0;
  std::thread th_;
  std::atomic<bool> running_{false};
  uint64_t serial_ = 0;
  std::unordered_map<int, std::unique_ptr<HttpConn>> conns_;
  std::unordered_map<std::string, Req> reqs_;
  uint64_t tok_seq_ = 0;
  // NATS connection
  std::atomic<int> nats_state_{0};  // 0 down, 1 connecting, 2 up
  double nats_retry_at_ = 0;
  std::string nin_, nout_;
  size_t nin_pos_ = 0, nout_pos_ = 0;
  long long nneed_ = -1, msg_hdr_ = 0, max_payload_ = 1 << 20;
  std::string msg_subject_, msg_sid_;
  bool nats_epollout_ = false;
};

// ============================================================================ Gateway
class Gateway {
 public:
  explicit Gateway(Config cfg) : cfg_(std::move(cfg)) {}
  ~Gateway() { stop(); }

  void start() {
    if (!loops_.empty()) throw std::runtime_error("gateway already running");
    const int W = std::max(1, cfg_.workers);
    for (int i = 0; i < W; ++i) {
      loops_.emplace_back(std::make_unique<Loop>(this, cfg_, st_, i));
      const int p = loops_.back()->bind_listener();
      if (i == 0 && cfg_.port == 0) cfg_.port = p;  // the other workers share the picked port
      port_ = p;
    }
    for (auto& l : loops_) l->start();
  }

  void stop() {
    for (auto& l : loops_) l->stop();
    loops_.clear();
  }

  int port() const { return port_; }
  long long search_ok() const { return st_.search_ok.load(); }
  long long sse_events() const { return st_.sse_events.load(); }
  bool nats_connected() const {
    for (auto& l : loops_)
      if (!l->nats_up()) return false;
    return !loops_.empty();
  }

  static std::string pct_json(std::vector<double> v) {
    if (v.empty()) return "null";
    std::sort(v.begin(), v.end());
    char b[160];
    snprintf(b, sizeof b, "{\"p50\":%.3f,\"p99\":%.3f,\"n\":%zu}", v[v.size() / 2],
             v[std::min(v.size() - 1, (size_t)(v.size() * 0.99))], v.size());
    return b;
  }

  std::string metrics_json() {
    std::string o = "{\"api_service\":{\"impl\":\"native\",\"workers\":" + std::to_string(loops_.size()) +
                    ",\"counters\":{\"http.requests\":" + std::to_string(st_.requests.load()) +
                    ",\"search.requests\":" + std::to_string(st_.search_ok.load()) +
                    ",\"search.errors\":" + std::to_string(st_.search_err.load()) +
                    ",\"nats.published\":" + std::to_string(st_.published.load()) +
                    ",\"nats.reconnects\":" + std::to_string(st_.nats_reconnects.load()) +
                    ",\"http.errors\":" + std::to_string(st_.bad_requests.load()) + "},\"latency_ms\":{";
    std::lock_guard<std::mutex> g(st_.mu);
    o += "\"search.handler\":" + pct_json(st_.search_ms) + ",\"search.embed_hop\":" +
         pct_json(st_.embed_hop_ms) + ",\"search.index_hop\":" + pct_json(st_.index_hop_ms) + "}}";
    o += ",\"sse_clients\":" + std::to_string(st_.sse_clients.load()) +
         ",\"sse_lagged\":" + std::to_string(st_.sse_lagged.load()) + ",\"services\":{";
    bool first = true;
    for (auto& kv : st_.service_metrics) {
      if (!first) o += ',';
      first = false;
      o += jstr(kv.first) + ":" + kv.second;
    }
    o += "}}";
    return o;
  }

#ifndef SYMB_NO_PYTHON
  py::dict stats() {
    py::dict d;
    d["requests"] = st_.requests.load();
    d["search_ok"] = st_.search_ok.load();
    d["search_err"] = st_.search_err.load();
    d["published"] = st_.published.load();
    d["sse_clients"] = st_.sse_clients.load();
    d["sse_events"] = st_.sse_events.load();
    d["sse_lagged"] = st_.sse_lagged.load();
    d["nats_reconnects"] = st_.nats_reconnects.load();
    d["nats_connected"] = nats_connected();
    return d;
  }
#endif

 private:
  Config cfg_;
  Stats st_;
  int port_ = 0;
  std::vector<std::unique_ptr<Loop>> loops_;
};

std::string Loop::gw_metrics() { return gw_->metrics_json(); }

}  // namespace gw

#ifndef SYMB_NO_PYTHON
void register_gateway(py::module_& m) {
  using gw::Config;
  using gw::Gateway;
  py::class_<Config>(m, "GatewayConfig")
      .def(py::init<>())
      .def_readwrite("host", &Config::host)
      .def_readwrite("port", &Config::port)
      .def_readwrite("nats_host", &Config::nats_host)
      .def_readwrite("nats_port", &Config::nats_port)
      .def_readwrite("workers", &Config::workers)
      .def_readwrite("embed_timeout_s", &Config::embed_timeout_s)
      .def_readwrite("search_timeout_s", &Config::search_timeout_s)
      .def_readwrite("nats_request_timeout_s", &Config::nats_request_timeout_s)
      .def_readwrite("sse_capacity", &Config::sse_capacity)
      .def_readwrite("sse_keepalive_s", &Config::sse_keepalive_s)
      .def_readwrite("max_length_limit", &Config::max_length_limit)
      .def_readwrite("index_html", &Config::index_html)
      .def_readwrite("log", &Config::log);
  py::class_<Gateway>(m, "Gateway")
      .def(py::init<Config>())
      .def("start", &Gateway::start)
      .def("stop", &Gateway::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &Gateway::port)
      .def_property_readonly("nats_connected", &Gateway::nats_connected)
      .def("stats", &Gateway::stats)
      .def("metrics_json", &Gateway::metrics_json);
  m.def("py_float_repr", &gw::py_float_repr);
}

#endif  // SYMB_NO_PYTHON

}  // namespace symbn
