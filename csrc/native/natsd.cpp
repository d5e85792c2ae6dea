// Native NATS core server: the message bus every service of the system talks through.
//
// The reference deploys nats-server 2.10.7 as its only inter-process transport
// (docker-compose.yml:27-34; every subject in SURVEY.md §2.2).  This image has no nats-server, so
// the framework ships its own: a single-threaded epoll event loop in C++ that speaks the NATS
// core client protocol (INFO/CONNECT, PUB/HPUB, SUB with queue groups, UNSUB with auto-unsubscribe
// counts, MSG/HMSG delivery, PING/PONG, `*`/`>` wildcards, verbose +OK) with nats-server's
// observable behaviour where the services depend on it:
//   * max_payload (1 MiB default) checked on the PUB control line: -ERR + close;
//   * no-responders: a request (PUB with a reply subject) that reaches no subscriber gets an
//     `HMSG <reply> ... NATS/1.0 503` status message when the client negotiated headers and
//     no_responders (async-nats maps it to "no responders" -> the gateway's fast 503);
//   * queue groups deliver each message to exactly one member (round robin per group+subject);
//   * slow consumers (pending output above max_pending) are disconnected instead of growing
//     without bound.
// At-most-once, no persistence: NATS core semantics (the reference uses no JetStream).
//
// Design: non-blocking sockets, level-triggered epoll; every readable connection is drained and
// parsed, deliveries are appended to per-connection output buffers, and all dirty buffers are
// flushed once per loop iteration (one write() per subscriber per batch of messages, not per
// message).  Literal subscriptions are hashed by subject; wildcard ones are matched token-wise;
// match results are cached per subject until the next SUB/UNSUB.  The loop runs on its own
// std::thread and never touches Python, so a Python process (launch.py's broker child, or a test)
// holds it without the GIL in the way.  The Python asyncio broker (bus/broker.py) remains as the
// reference implementation the tests compare against.
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
#include <chrono>
#include <cerrno>
#include <cstring>
#include <memory>
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
namespace natsd {

static constexpr size_t MAX_CONTROL_LINE = 4096;
static constexpr const char* VERSION = "2.10.7";

struct Conn;

struct Sub {
  Conn* conn;
  std::string sid, subject, queue;
  std::vector<std::string> toks;
  bool wild = false;
  long long max_msgs = -1, delivered = 0;
  uint64_t seq = 0;  // creation order: deliveries follow it (as the Python spec broker does)
};

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in;
  size_t in_pos = 0;
  std::string out;
  size_t out_pos = 0;
  bool headers = false, no_responders = false, verbose = false;
  bool closing = false, epollout = false, dirty = false;
  std::unordered_map<std::string, std::unique_ptr<Sub>> subs;
  // payload being received (need >= 0): PUB/HPUB header fields
  long long need = -1, hdr = 0;
  bool has_reply = false, hpub = false;
  std::string subject, reply;
};

static std::vector<std::string> split_ws(const char* p, size_t n) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < n) {
    while (i < n && (p[i] == ' ' || p[i] == '\t')) ++i;
    if (i >= n) break;
    size_t j = i;
    while (j < n && p[j] != ' ' && p[j] != '\t') ++j;
    out.emplace_back(p + i, j - i);
    i = j;
  }
  return out;
}

static std::vector<std::string> split_dots(const std::string& s) {
  std::vector<std::string> t;
  size_t i = 0;
  for (;;) {
    size_t j = s.find('.', i);
    t.emplace_back(s.substr(i, j == std::string::npos ? std::string::npos : j - i));
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return t;
}

// nats-server subject rules: non-empty dot-separated tokens without whitespace; `*` and `>` only
// as whole tokens of subscriptions, `>` only last.
static bool subject_valid(const std::string& s, bool wildcards) {
  if (s.empty() || s.front() == '.' || s.back() == '.') return false;
  const auto toks = split_dots(s);
  for (size_t i = 0; i < toks.size(); ++i) {
    const std::string& t = toks[i];
    if (t.empty()) return false;
    for (char c : t)
      if (c == ' ' || c == '\t' || c == '\r' || c == '\n') return false;
    if (t.find('*') != std::string::npos || t.find('>') != std::string::npos) {
      if (!wildcards || t.size() != 1 || (t == ">" && i + 1 != toks.size())) return false;
    }
  }
  return true;
}

static bool subject_matches(const std::vector<std::string>& pat, const std::vector<std::string>& st) {
  for (size_t i = 0; i < pat.size(); ++i) {
    if (pat[i] == ">") return st.size() > i;
    if (i >= st.size()) return false;
    if (pat[i] != "*" && pat[i] != st[i]) return false;
  }
  return pat.size() == st.size();
}

static bool parse_int(const std::string& s, long long& v) {
  if (s.empty() || s.size() > 18) return false;
  v = 0;
  for (char c : s) {
    if (c < '0' || c > '9') return false;
    v = v * 10 + (c - '0');
  }
  return true;
}

// ---- minimal JSON walk over CONNECT options (only top-level booleans matter) ----
static void skip_value(Parser& p) {
  const char c = p.peek();
  if (c == '"') {
    p.string();
  } else if (c == '{' || c == '[') {
    const char close = c == '{' ? '}' : ']';
    p.advance();
    if (p.peek() == close) {
      p.advance();
      return;
    }
    for (;;) {
      if (close == '}') {
        p.string();
        if (p.peek() != ':') p.fail("expected ':'");
        p.advance();
      }
      skip_value(p);
      const char d = p.peek();
      p.advance();
      if (d == close) return;
      if (d != ',') p.fail("expected ','");
    }
  } else if (c == 't') {
    p.expect_lit("true");
  } else if (c == 'f') {
    p.expect_lit("false");
  } else if (c == 'n') {
    p.expect_lit("null");
  } else {
    p.number();
  }
}

static void parse_connect(Conn& c, const char* s, size_t n) {
  try {
    Parser p(s, n);
    if (p.peek() != '{') return;
    p.advance();
    if (p.peek() == '}') return;
    for (;;) {
      const std::string key = p.string();
      if (p.peek() != ':') return;
      p.advance();
      const char v = p.peek();
      if ((key == "headers" || key == "no_responders" || key == "verbose") && (v == 't' || v == 'f')) {
        const bool b = v == 't';
        p.expect_lit(b ? "true" : "false");
        if (key == "headers") c.headers = b;
        else if (key == "no_responders") c.no_responders = b;
        else c.verbose = b;
      } else {
        skip_value(p);
      }
      const char d = p.peek();
      p.advance();
      if (d != ',') return;
    }
  } catch (const std::exception&) {
    // nats-server rejects malformed CONNECT; a lenient broker keeps defaults
  }
}

class Server {
 public:
  Server(std::string host, int port, long long max_payload, long long max_pending,
         int monitor_port = -1)
      : host_(std::move(host)), port_(port), max_payload_(max_payload), max_pending_(max_pending),
        mon_port_(monitor_port) {
    std::random_device rd;
    std::mt19937 g(rd());
    const char* al = "ABCDEFGHJKLMNPQRSTUVWXYZ234567";
    server_id_ = "NSYMB";
    for (int i = 0; i < 51; ++i) server_id_ += al[g() % 30];
  }
  ~Server() { stop(); }

  void start() {
    if (thread_.joinable()) throw std::runtime_error("server already running");
    listen_fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (listen_fd_ < 0) throw std::runtime_error("socket: " + std::string(strerror(errno)));
    int one = 1;
    setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port_);
    if (host_.empty() || host_ == "0.0.0.0") {
      a.sin_addr.s_addr = htonl(INADDR_ANY);
    } else if (inet_pton(AF_INET, host_.c_str(), &a.sin_addr) != 1) {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      if (getaddrinfo(host_.c_str(), nullptr, &hints, &res) != 0 || !res) {
        fail_close("cannot resolve host " + host_);
      }
      a.sin_addr = ((sockaddr_in*)res->ai_addr)->sin_addr;
      freeaddrinfo(res);
    }
    if (::bind(listen_fd_, (sockaddr*)&a, sizeof a) < 0)
      fail_close("bind " + host_ + ":" + std::to_string(port_) + ": " + strerror(errno));
    if (::listen(listen_fd_, 1024) < 0) fail_close(std::string("listen: ") + strerror(errno));
    socklen_t len = sizeof a;
    getsockname(listen_fd_, (sockaddr*)&a, &len);
    port_ = ntohs(a.sin_port);
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    wake_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    add_fd(listen_fd_, EPOLLIN, nullptr);
    add_fd(wake_, EPOLLIN, &wake_tag_);
    if (mon_port_ >= 0) {  // nats-server's HTTP monitoring port (8222 in the reference compose)
      mon_fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      setsockopt(mon_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
      a.sin_port = htons((uint16_t)mon_port_);
      if (::bind(mon_fd_, (sockaddr*)&a, sizeof a) < 0 || ::listen(mon_fd_, 64) < 0) {
        const std::string m = strerror(errno);
        ::close(mon_fd_);
        mon_fd_ = -1;
        ::close(ep_);
        ::close(wake_);
        fail_close("monitor bind :" + std::to_string(mon_port_) + ": " + m);
      }
      len = sizeof a;
      getsockname(mon_fd_, (sockaddr*)&a, &len);
      mon_port_ = ntohs(a.sin_port);
      add_fd(mon_fd_, EPOLLIN, &mon_tag_);
    }
    start_time_ = std::chrono::steady_clock::now();
    running_ = true;
    thread_ = std::thread([this] { loop(); });
  }

  void stop() {
    if (!thread_.joinable()) return;
    running_ = false;
    uint64_t one = 1;
    (void)!::write(wake_, &one, sizeof one);
    thread_.join();
    for (auto& kv : conns_) ::close(kv.first);
    conns_.clear();
    for (auto& kv : mons_) ::close(kv.second->fd);
    mons_.clear();
    if (mon_fd_ >= 0) ::close(mon_fd_);
    mon_fd_ = -1;
    literal_.clear();
    wild_.clear();
    cache_.clear();
    ::close(listen_fd_);
    ::close(wake_);
    ::close(ep_);
    listen_fd_ = wake_ = ep_ = -1;
  }

  int port() const { return port_; }
  int monitor_port() const { return mon_fd_ >= 0 ? mon_port_ : -1; }
  bool running() const { return running_; }

  struct Counters {
    long long in_msgs, out_msgs, in_bytes, out_bytes, connections, total_connections,
        subscriptions, slow_consumers;
  };
  Counters counters() const {
    return {in_msgs_.load(), out_msgs_.load(), in_bytes_.load(), out_bytes_.load(),
            n_conns_.load(), total_conns_.load(), n_subs_.load(), slow_.load()};
  }
#ifndef SYMB_NO_PYTHON
  py::dict stats() const {
    py::dict d;
    d["in_msgs"] = in_msgs_.load();
    d["out_msgs"] = out_msgs_.load();
    d["in_bytes"] = in_bytes_.load();
    d["out_bytes"] = out_bytes_.load();
    d["connections"] = n_conns_.load();
    d["total_connections"] = total_conns_.load();
    d["subscriptions"] = n_subs_.load();
    d["slow_consumers"] = slow_.load();
    return d;
  }
#endif

 private:
  [[noreturn]] void fail_close(const std::string& m) {
    ::close(listen_fd_);
    listen_fd_ = -1;
    throw std::runtime_error(m);
  }

  void add_fd(int fd, uint32_t ev, void* tag) {
    epoll_event e{};
    e.events = ev;
    e.data.ptr = tag;
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
  }

  void loop() {
    std::vector<epoll_event> evs(256);
    while (running_) {
      const int n = epoll_wait(ep_, evs.data(), (int)evs.size(), 1000);
      if (n < 0) {
        if (errno == EINTR) continue;
        break;
      }
      for (int i = 0; i < n; ++i) {
        void* tag = evs[i].data.ptr;
        if (tag == &wake_tag_) {
          uint64_t v;
          (void)!::read(wake_, &v, sizeof v);
          continue;
        }
        if (tag == nullptr) {
          accept_all();
          continue;
        }
        if (tag == &mon_tag_) {
          accept_monitor();
          continue;
        }
        if (auto m = mons_.find(tag); m != mons_.end()) {
          on_monitor(m->second.get());
          continue;
        }
        Conn* c = static_cast<Conn*>(tag);
        if (c->closing) continue;
        if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
          if (!(evs[i].events & EPOLLIN)) {
            drop(c);
            continue;
          }
        }
        if (evs[i].events & EPOLLIN) on_readable(c);
        if (!c->closing && (evs[i].events & EPOLLOUT)) mark_dirty(c);
      }
      flush_all();
      reap();
    }
  }

  // ---- HTTP monitoring (GET /varz, /connz, /subsz, /healthz; one request per connection) ----
  struct MonConn {
    int fd;
    std::string in;
  };

  void accept_monitor() {
    for (;;) {
      const int fd = accept4(mon_fd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      auto m = std::make_unique<MonConn>();
      m->fd = fd;
      add_fd(fd, EPOLLIN, m.get());
      mons_[m.get()] = std::move(m);
    }
  }

  std::string monitor_body(const std::string& path, int& status) {
    status = 200;
    const auto up = std::chrono::duration<double>(std::chrono::steady_clock::now() - start_time_).count();
    auto num = [](long long v) { return std::to_string(v); };
    if (path == "/varz" || path == "/") {
      return "{\"server_id\":\"" + server_id_ + "\",\"server_name\":\"symbiont-natsd\",\"version\":\"" +
             VERSION + "\",\"host\":\"" + host_ + "\",\"port\":" + num(port_) +
             ",\"max_payload\":" + num(max_payload_) + ",\"uptime_s\":" + num((long long)up) +
             ",\"connections\":" + num(n_conns_) + ",\"total_connections\":" + num(total_conns_) +
             ",\"subscriptions\":" + num(n_subs_) + ",\"slow_consumers\":" + num(slow_) +
             ",\"in_msgs\":" + num(in_msgs_) + ",\"out_msgs\":" + num(out_msgs_) +
             ",\"in_bytes\":" + num(in_bytes_) + ",\"out_bytes\":" + num(out_bytes_) + "}";
    }
    if (path == "/connz") {
      std::string o = "{\"num_connections\":" + num((long long)conns_.size()) + ",\"connections\":[";
      bool first = true;
      for (auto& kv : conns_) {
        const Conn* c = kv.second.get();
        if (!first) o += ',';
        first = false;
        o += "{\"cid\":" + num((long long)c->id) + ",\"subscriptions\":" + num((long long)c->subs.size()) +
             ",\"pending_bytes\":" + num((long long)(c->out.size() - c->out_pos)) + "}";
      }
      return o + "]}";
    }
    if (path == "/subsz") {
      return "{\"num_subscriptions\":" + num(n_subs_) + ",\"num_literal_subjects\":" +
             num((long long)literal_.size()) + ",\"num_wildcard\":" + num((long long)wild_.size()) +
             ",\"num_cache\":" + num((long long)cache_.size()) + "}";
    }
    if (path == "/healthz") return "{\"status\":\"ok\"}";
    status = 404;
    return "{\"error\":\"not found\"}";
  }

  void on_monitor(MonConn* m) {
    char buf[4096];
    bool eof = false;
    for (;;) {
      const ssize_t r = ::read(m->fd, buf, sizeof buf);
      if (r > 0) {
        m->in.append(buf, (size_t)r);
        if (m->in.size() > 16384) eof = true;
        continue;
      }
      if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)) eof = true;
      if (r < 0 && errno == EINTR) continue;
      break;
    }
    if (m->in.find("\r\n\r\n") != std::string::npos) {
      const size_t sp1 = m->in.find(' '), sp2 = m->in.find(' ', sp1 + 1);
      std::string path = sp1 == std::string::npos ? "/" : m->in.substr(sp1 + 1, sp2 - sp1 - 1);
      const size_t q = path.find('?');
      if (q != std::string::npos) path.resize(q);
      int status = 200;
      const std::string body = monitor_body(path, status);
      const std::string resp = std::string("HTTP/1.1 ") + (status == 200 ? "200 OK" : "404 Not Found") +
                               "\r\nContent-Type: application/json\r\nContent-Length: " +
                               std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body;
      (void)!::send(m->fd, resp.data(), resp.size(), MSG_NOSIGNAL);  // small: fits the socket buffer
      eof = true;
    }
    if (eof) {
      epoll_ctl(ep_, EPOLL_CTL_DEL, m->fd, nullptr);
      ::close(m->fd);
      mons_.erase(m);
    }
  }

  void accept_all() {
    for (;;) {
      const int fd = accept4(listen_fd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->id = ++next_id_;
      Conn* cp = c.get();
      conns_[fd] = std::move(c);
      n_conns_ = conns_.size();
      ++total_conns_;
      add_fd(fd, EPOLLIN, cp);
      std::string info = "INFO {\"server_id\":\"" + server_id_ +
                         "\",\"server_name\":\"symbiont-natsd\",\"version\":\"" + VERSION +
                         "\",\"proto\":1,\"go\":\"n/a\",\"host\":\"" + host_ +
                         "\",\"port\":" + std::to_string(port_) +
                         ",\"headers\":true,\"max_payload\":" + std::to_string(max_payload_) +
                         ",\"client_id\":" + std::to_string(cp->id) + "}\r\n";
      send(cp, info.data(), info.size());
    }
  }

  void on_readable(Conn* c) {
    char buf[1 << 16];
    size_t total = 0;
    for (;;) {
      const ssize_t r = ::read(c->fd, buf, sizeof buf);
      if (r > 0) {
        c->in.append(buf, (size_t)r);
        total += (size_t)r;
        if (total >= (4u << 20)) break;  // fairness: let other connections run
        continue;
      }
      if (r == 0) {
        parse(c);
        drop(c);
        return;
      }
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      drop(c);
      return;
    }
    parse(c);
  }

  void parse(Conn* c) {
    std::string& b = c->in;
    while (!c->closing) {
      const size_t avail = b.size() - c->in_pos;
      if (c->need >= 0) {
        if ((long long)avail < c->need + 2) break;
        const char* p = b.data() + c->in_pos;
        if (p[c->need] != '\r' || p[c->need + 1] != '\n') {
          err_close(c, "Unknown Protocol Operation");
          return;
        }
        on_pub(c, p, (size_t)c->need);
        c->in_pos += (size_t)c->need + 2;
        c->need = -1;
        continue;
      }
      const char* s = b.data() + c->in_pos;
      const void* nl = memchr(s, '\n', avail);
      if (!nl) {
        if (avail > MAX_CONTROL_LINE) err_close(c, "Maximum Control Line Exceeded");
        break;
      }
      size_t len = (const char*)nl - s;
      c->in_pos += len + 1;
      if (len && s[len - 1] == '\r') --len;
      control(c, s, len);
    }
    if (c->in_pos == b.size()) {
      b.clear();
      c->in_pos = 0;
    } else if (c->in_pos > (1u << 16)) {
      b.erase(0, c->in_pos);
      c->in_pos = 0;
    }
  }

  static bool op_is(const char* s, size_t n, const char* op) {
    const size_t L = strlen(op);
    if (n != L) return false;
    for (size_t i = 0; i < L; ++i)
      if (toupper((unsigned char)s[i]) != op[i]) return false;
    return true;
  }

  void control(Conn* c, const char* s, size_t n) {
    size_t sp = 0;
    while (sp < n && s[sp] != ' ' && s[sp] != '\t') ++sp;
    const char* rest = s + std::min(n, sp + 1);
    const size_t rn = sp < n ? n - sp - 1 : 0;
    if (op_is(s, sp, "PUB") || op_is(s, sp, "HPUB")) {
      const bool h = sp == 4;
      auto a = split_ws(rest, rn);
      const size_t want = h ? 3 : 2;
      if (a.size() != want && a.size() != want + 1) {
        err_close(c, "Unknown Protocol Operation");
        return;
      }
      long long total = 0, hdr = 0;
      if (!parse_int(a.back(), total) || (h && !parse_int(a[a.size() - 2], hdr)) || hdr > total) {
        err_close(c, "Unknown Protocol Operation");
        return;
      }
      if (total > max_payload_) {
        err_close(c, "Maximum Payload Violation");
        return;
      }
      c->hpub = h;
      c->subject = a[0];
      c->has_reply = a.size() == want + 1;
      c->reply = c->has_reply ? a[1] : std::string();
      c->hdr = hdr;
      c->need = total;
    } else if (op_is(s, sp, "SUB")) {
      auto a = split_ws(rest, rn);
      if (a.size() != 2 && a.size() != 3) {
        err_close(c, "Unknown Protocol Operation");
        return;
      }
      if (!subject_valid(a[0], true)) {
        send_str(c, "-ERR 'Invalid Subject'\r\n");
        return;
      }
      auto sub = std::make_unique<Sub>();
      sub->conn = c;
      sub->subject = a[0];
      sub->queue = a.size() == 3 ? a[1] : std::string();
      sub->sid = a.back();
      sub->toks = split_dots(a[0]);
      sub->wild = std::any_of(sub->toks.begin(), sub->toks.end(),
                              [](const std::string& t) { return t == "*" || t == ">"; });
      // nats-server keeps the existing subscription when a client reuses a live sid
      if (c->subs.find(sub->sid) == c->subs.end()) {
        index(sub.get());
        c->subs[sub->sid] = std::move(sub);
      }
      ok(c);
    } else if (op_is(s, sp, "UNSUB")) {
      auto a = split_ws(rest, rn);
      long long mx = -1;
      if ((a.size() != 1 && a.size() != 2) || (a.size() == 2 && !parse_int(a[1], mx))) {
        err_close(c, "Unknown Protocol Operation");
        return;
      }
      auto it = c->subs.find(a[0]);
      if (it != c->subs.end()) {
        if (mx >= 0 && it->second->delivered < mx) {
          it->second->max_msgs = mx;
        } else {
          unindex(it->second.get());
          c->subs.erase(it);
        }
      }
      ok(c);
    } else if (op_is(s, sp, "PING")) {
      send_str(c, "PONG\r\n");
    } else if (op_is(s, sp, "PONG") || op_is(s, sp, "+OK") || op_is(s, sp, "-ERR") ||
               op_is(s, sp, "INFO") || sp == 0) {
      // client-side acks / keep-alives: nothing to do
    } else if (op_is(s, sp, "CONNECT")) {
      parse_connect(*c, rest, rn);
      ok(c);
    } else {
      err_close(c, "Unknown Protocol Operation");
    }
  }

  void ok(Conn* c) {
    if (c->verbose) send_str(c, "+OK\r\n");
  }

  void on_pub(Conn* c, const char* p, size_t n) {
    if (!subject_valid(c->subject, false)) {
      send_str(c, "-ERR 'Invalid Publish Subject'\r\n");
      return;
    }
    ok(c);  // nats-server acks a verbose PUB before routing it
    ++in_msgs_;
    in_bytes_ += n - (size_t)c->hdr;
    const size_t hl = c->hpub ? (size_t)c->hdr : 0;
    route(c->subject, c->has_reply ? &c->reply : nullptr, p, hl, p + hl, n - hl, c);
  }

  // ---- subscription index ----
  void index(Sub* s) {
    s->seq = ++sub_seq_;
    if (s->wild) wild_.push_back(s);
    else literal_[s->subject].push_back(s);
    cache_.clear();
    n_subs_ = n_subs_ + 1;
  }

  void unindex(Sub* s) {
    if (s->wild) {
      wild_.erase(std::remove(wild_.begin(), wild_.end(), s), wild_.end());
    } else {
      auto it = literal_.find(s->subject);
      if (it != literal_.end()) {
        auto& v = it->second;
        v.erase(std::remove(v.begin(), v.end(), s), v.end());
        if (v.empty()) literal_.erase(it);
      }
    }
    cache_.clear();
    n_subs_ = n_subs_ - 1;
  }

  const std::vector<Sub*>& match(const std::string& subject) {
    auto it = cache_.find(subject);
    if (it != cache_.end()) return it->second;
    if (cache_.size() > 8192) cache_.clear();
    std::vector<Sub*> m;
    auto lit = literal_.find(subject);
    if (lit != literal_.end()) m = lit->second;
    if (!wild_.empty()) {
      const auto toks = split_dots(subject);
      const size_t n_lit = m.size();
      for (Sub* s : wild_)
        if (subject_matches(s->toks, toks)) m.push_back(s);
      // literal and wildcard lists are each in creation order; merge them into one
      if (n_lit && m.size() > n_lit)
        std::inplace_merge(m.begin(), m.begin() + n_lit, m.end(),
                           [](const Sub* a, const Sub* b) { return a->seq < b->seq; });
    }
    return cache_.emplace(subject, std::move(m)).first->second;
  }

  int route(const std::string& subject, const std::string* reply, const char* hdr, size_t hl,
            const char* pl, size_t pn, Conn* origin) {
    // copy: delivery may auto-unsubscribe (which clears the cache)
    const std::vector<Sub*> m = match(subject);
    std::vector<Sub*> expired;
    int delivered = 0;
    std::vector<std::pair<const std::string*, std::vector<Sub*>>> groups;
    for (Sub* s : m) {
      if (s->conn->closing) continue;
      if (s->queue.empty()) {
        deliver(s, subject, reply, hdr, hl, pl, pn, expired);
        ++delivered;
        continue;
      }
      auto g = std::find_if(groups.begin(), groups.end(),
                            [&](const auto& x) { return *x.first == s->queue; });
      if (g == groups.end()) groups.emplace_back(&s->queue, std::vector<Sub*>{s});
      else g->second.push_back(s);
    }
    for (auto& g : groups) {
      const std::string key = *g.first + '\x1f' + subject;
      uint64_t& rr = qrr_[key];
      deliver(g.second[rr++ % g.second.size()], subject, reply, hdr, hl, pl, pn, expired);
      ++delivered;
    }
    if (qrr_.size() > 65536) qrr_.clear();
    for (Sub* s : expired) {
      Conn* c = s->conn;
      unindex(s);
      c->subs.erase(s->sid);  // frees s
    }
    if (delivered == 0 && reply && origin && origin->headers && origin->no_responders) {
      static const std::string status = "NATS/1.0 503\r\n\r\n";
      route(*reply, nullptr, status.data(), status.size(), "", 0, nullptr);
    }
    return delivered;
  }

  void deliver(Sub* s, const std::string& subject, const std::string* reply, const char* hdr,
               size_t hl, const char* pl, size_t pn, std::vector<Sub*>& expired) {
    Conn* c = s->conn;
    std::string& o = c->out;
    o += hl ? "HMSG " : "MSG ";
    o += subject;
    o += ' ';
    o += s->sid;
    if (reply) {
      o += ' ';
      o += *reply;
    }
    o += ' ';
    if (hl) {
      o += std::to_string(hl);
      o += ' ';
    }
    o += std::to_string(hl + pn);
    o += "\r\n";
    o.append(hdr, hl);
    o.append(pl, pn);
    o += "\r\n";
    mark_dirty(c);
    ++out_msgs_;
    out_bytes_ += pn;
    if (++s->delivered == s->max_msgs) expired.push_back(s);  // UNSUB <sid> <max> reached
    if ((long long)(o.size() - c->out_pos) > max_pending_) {
      ++slow_;
      c->closing = true;  // slow consumer: nats-server disconnects it
      c->out.clear();
      c->out_pos = 0;
    }
  }

  void send(Conn* c, const char* p, size_t n) {
    if (c->closing) return;
    c->out.append(p, n);
    mark_dirty(c);
  }
  void send_str(Conn* c, const char* s) { send(c, s, strlen(s)); }

  void mark_dirty(Conn* c) {
    if (!c->dirty) {
      c->dirty = true;
      dirty_.push_back(c);
    }
  }

  void err_close(Conn* c, const char* msg) {
    std::string m = std::string("-ERR '") + msg + "'\r\n";
    send(c, m.data(), m.size());
    flush(c);
    drop(c);
  }

  // returns false when the connection died
  bool flush(Conn* c) {
    while (c->out_pos < c->out.size()) {
      const ssize_t w = ::send(c->fd, c->out.data() + c->out_pos, c->out.size() - c->out_pos,
                               MSG_NOSIGNAL);
      if (w > 0) {
        c->out_pos += (size_t)w;
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      return false;
    }
    if (c->out_pos == c->out.size()) {
      c->out.clear();
      c->out_pos = 0;
    } else if (c->out_pos > (1u << 20)) {
      c->out.erase(0, c->out_pos);
      c->out_pos = 0;
    }
    const bool want = !c->out.empty();
    if (want != c->epollout) {
      epoll_event e{};
      e.events = EPOLLIN | (want ? EPOLLOUT : 0);
      e.data.ptr = c;
      epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &e);
      c->epollout = want;
    }
    return true;
  }

  void flush_all() {
    // index loop: flushing never adds to dirty_, but drop() may not run mid-iteration
    for (size_t i = 0; i < dirty_.size(); ++i) {
      Conn* c = dirty_[i];
      c->dirty = false;
      if (c->closing) continue;
      if (!flush(c)) drop(c);
    }
    dirty_.clear();
  }

  void drop(Conn* c) {
    if (!c->closing) c->closing = true;
    dead_.push_back(c);
  }

  void reap() {
    // connections marked closing (error, EOF, slow consumer) are removed after the loop pass, so
    // no pointer held by route()/dirty_ dangles mid-iteration
    for (auto& kv : conns_)
      if (kv.second->closing) dead_.push_back(kv.second.get());
    if (dead_.empty()) return;
    std::sort(dead_.begin(), dead_.end());
    dead_.erase(std::unique(dead_.begin(), dead_.end()), dead_.end());
    for (Conn* c : dead_) {
      for (auto& kv : c->subs) unindex(kv.second.get());
      c->subs.clear();
      epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
      // FIN after the queued -ERR, and discard unread input first: closing a socket with unread
      // bytes sends RST, which can destroy the -ERR line before the client reads it
      ::shutdown(c->fd, SHUT_WR);
      char sink[4096];
      for (int i = 0; i < 256 && ::recv(c->fd, sink, sizeof sink, MSG_DONTWAIT) > 0; ++i) {
      }
      ::close(c->fd);
      dirty_.erase(std::remove(dirty_.begin(), dirty_.end(), c), dirty_.end());
      conns_.erase(c->fd);
    }
    dead_.clear();
    n_conns_ = conns_.size();
  }

  std::string host_;
  int port_;
  long long max_payload_, max_pending_;
  std::string server_id_;
  int listen_fd_ = -1, ep_ = -1, wake_ = -1;
  int wake_tag_ = 0;
  int mon_port_ = -1, mon_fd_ = -1, mon_tag_ = 0;
  std::unordered_map<void*, std::unique_ptr<MonConn>> mons_;
  std::chrono::steady_clock::time_point start_time_;
  std::thread thread_;
  std::atomic<bool> running_{false};
  uint64_t next_id_ = 0;
  std::unordered_map<int, std::unique_ptr<Conn>> conns_;
  std::unordered_map<std::string, std::vector<Sub*>> literal_;
  std::vector<Sub*> wild_;
  uint64_t sub_seq_ = 0;
  std::unordered_map<std::string, std::vector<Sub*>> cache_;
  std::unordered_map<std::string, uint64_t> qrr_;
  std::vector<Conn*> dirty_, dead_;
  std::atomic<long long> in_msgs_{0}, out_msgs_{0}, in_bytes_{0}, out_bytes_{0};
  std::atomic<long long> n_conns_{0}, total_conns_{0}, n_subs_{0}, slow_{0};
};

}  // namespace natsd

#ifndef SYMB_NO_PYTHON
void register_natsd(py::module_& m) {
  using natsd::Server;
  py::class_<Server>(m, "NatsServer")
      .def(py::init<std::string, int, long long, long long, int>(), py::arg("host") = "127.0.0.1",
           py::arg("port") = 0, py::arg("max_payload") = 1ll << 20,
           py::arg("max_pending") = 64ll << 20, py::arg("monitor_port") = -1)
      .def_property_readonly("monitor_port", &Server::monitor_port)
      .def("start", &Server::start)
      .def("stop", &Server::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &Server::port)
      .def_property_readonly("running", &Server::running)
      .def("stats", &Server::stats);
  m.def("nats_subject_valid", [](const std::string& s, bool wild) {
    return natsd::subject_valid(s, wild);
  });
  m.def("nats_subject_matches", [](const std::string& pat, const std::string& subj) {
    return natsd::subject_matches(natsd::split_dots(pat), natsd::split_dots(subj));
  });
}

#endif  // SYMB_NO_PYTHON

}  // namespace symbn
