// HTTP/1.1 keep-alive load generator for the end-to-end service benchmark
// (benchmarks/e2e_service.py --client native).
//
// The benchmark's asyncio clients spend ~100 us of Python per request (JSON, stream readers,
// coroutine switches); at 8k search req/s their event loops lag, and the client-side p99 (183 ms)
// sat far above the gateway's own two-hop p99 (27 ms, profiles/r2_e2e).  This drives `conns`
// connections from one epoll thread with the GIL released: each idle connection takes the next
// pre-built request, the response is framed by Content-Length, and the latency is taken from the
// first byte written to the last byte read.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace symbn {
namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Conn {
  int fd = -1;
  long req = -1;            // request in flight (-1: idle)
  size_t out_off = 0;       // bytes of it written
  std::string in;           // response bytes so far
  double t0 = 0.0;
  bool want_out = false;    // EPOLLOUT armed (only while a request is partly written)
  bool dead = false;
};

// Content-Length of a complete header block (`hdr` ends at the blank line), -1 if absent.
long content_length(const std::string& in, size_t hdr_end) {
  size_t p = 0;
  while (p < hdr_end) {
    size_t e = in.find("\r\n", p);
    if (e == std::string::npos || e > hdr_end) e = hdr_end;
    if (e - p > 15 && strncasecmp(in.data() + p, "content-length:", 15) == 0)
      return std::strtol(in.data() + p + 15, nullptr, 10);
    p = e + 2;
  }
  return -1;
}

struct Result {
  std::vector<double> latency_s;
  long errors = 0;
  long non200 = 0;
  double t_start = 0.0, t_end = 0.0;
};

Result run(const std::string& host, int port, const std::vector<std::string>& reqs, int conns,
           double timeout_s) {
  Result res;
  if (conns <= 0) throw std::invalid_argument("conns must be > 0");
  const int ep = epoll_create1(0);
  if (ep < 0) throw std::runtime_error("epoll_create1 failed");
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) {
    close(ep);
    throw std::invalid_argument("host must be an IPv4 address");
  }
  std::vector<Conn> cs((size_t)conns);
  for (int i = 0; i < conns; ++i) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0 || connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
      if (fd >= 0) close(fd);
      for (auto& c : cs)
        if (c.fd >= 0) close(c.fd);
      close(ep);
      throw std::runtime_error(std::string("connect failed: ") + strerror(errno));
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
    cs[(size_t)i].fd = fd;
    // level-triggered EPOLLIN only: EPOLLOUT is armed just while a send is blocked, so idle or
    // fully written connections never wake the loop (the client must not spin a core beside
    // the service it measures)
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u32 = (uint32_t)i;
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
  }
  int alive = conns;
  auto arm_out = [&](Conn& c, uint32_t idx, bool on) {
    if (c.want_out == on) return;
    epoll_event ev{};
    ev.events = EPOLLIN | (on ? EPOLLOUT : 0u);
    ev.data.u32 = idx;
    epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &ev);
    c.want_out = on;
  };
  auto kill = [&](Conn& c) {   // broken connection: count its request, stop polling it
    if (c.dead) return;
    epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
    close(c.fd);
    c.dead = true;
    --alive;
  };
  const long total = (long)reqs.size();
  long next = 0, done = 0;
  res.latency_s.reserve(reqs.size());
  res.t_start = now_s();
  const double deadline = res.t_start + timeout_s;
  auto start_req = [&](Conn& c) {
    if (next >= total) return;
    c.req = next++;
    c.out_off = 0;
    c.in.clear();
    c.t0 = now_s();
  };
  auto flush = [&](Conn& c) -> bool {   // false: connection broken
    const std::string& r = reqs[(size_t)c.req];
    while (c.out_off < r.size()) {
      const ssize_t n = send(c.fd, r.data() + c.out_off, r.size() - c.out_off, MSG_NOSIGNAL);
      if (n > 0) {
        c.out_off += (size_t)n;
      } else if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        return true;
      } else {
        return false;
      }
    }
    return true;
  };
  // start (or continue) writing a connection's request; false: the connection broke
  auto send_req = [&](Conn& c, uint32_t idx) -> bool {
    if (!flush(c)) {
      ++res.errors;
      ++done;
      c.req = -1;
      kill(c);
      return false;
    }
    arm_out(c, idx, c.out_off < reqs[(size_t)c.req].size());
    return true;
  };
  for (int i = 0; i < conns; ++i) {
    start_req(cs[(size_t)i]);
    if (cs[(size_t)i].req >= 0) send_req(cs[(size_t)i], (uint32_t)i);
  }
  std::vector<epoll_event> evs(256);
  char buf[65536];
  while (done < total && alive > 0 && now_s() < deadline) {
    const int n = epoll_wait(ep, evs.data(), (int)evs.size(), 100);
    for (int e = 0; e < n; ++e) {
      const uint32_t idx = evs[(size_t)e].data.u32;
      Conn& c = cs[idx];
      if (c.dead) continue;
      if (c.req < 0) {   // idle: only a hang-up can arrive
        if (evs[(size_t)e].events & (EPOLLHUP | EPOLLERR)) kill(c);
        continue;
      }
      if ((evs[(size_t)e].events & EPOLLOUT) && !send_req(c, idx)) continue;
      if (!(evs[(size_t)e].events & (EPOLLIN | EPOLLHUP | EPOLLERR))) continue;
      for (;;) {
        const ssize_t r = recv(c.fd, buf, sizeof(buf), 0);
        if (r > 0) {
          c.in.append(buf, (size_t)r);
          continue;
        }
        if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
        // closed or failed mid-request
        ++res.errors;
        ++done;
        c.req = -1;
        kill(c);
        break;
      }
      if (c.req < 0) continue;
      // one complete response? (no pipelining: at most one request in flight per connection)
      const size_t hdr = c.in.find("\r\n\r\n");
      if (hdr == std::string::npos) continue;
      const long clen = content_length(c.in, hdr);
      const size_t need = hdr + 4 + (size_t)(clen < 0 ? 0 : clen);
      if (c.in.size() < need) continue;
      const double t = now_s();
      // status line: "HTTP/1.1 200 ..."
      const int status = c.in.size() > 12 ? std::atoi(c.in.data() + 9) : 0;
      if (status == 200)
        res.latency_s.push_back(t - c.t0);
      else
        ++res.non200;
      ++done;
      c.req = -1;
      start_req(c);
      if (c.req >= 0) send_req(c, idx);
    }
  }
  res.t_end = now_s();
  res.errors += total - done;   // unanswered at the deadline / never sent (no live connection)
  for (auto& c : cs)
    if (!c.dead) close(c.fd);
  close(ep);
  return res;
}

}  // namespace

void register_loadgen(py::module_& m) {
  m.def(
      "http_load",
      [](const std::string& host, int port, const std::vector<std::string>& requests, int conns,
         double timeout_s) {
        Result r;
        {
          py::gil_scoped_release nogil;
          r = run(host, port, requests, conns, timeout_s);
        }
        py::dict d;
        d["latency_s"] = r.latency_s;
        d["errors"] = r.errors;
        d["non200"] = r.non200;
        d["t_start"] = r.t_start;
        d["t_end"] = r.t_end;
        return d;
      },
      py::arg("host"), py::arg("port"), py::arg("requests"), py::arg("conns"),
      py::arg("timeout_s") = 120.0,
      "Send every pre-built HTTP/1.1 request over `conns` keep-alive connections (one in flight "
      "per connection); returns per-request latencies of the 200 responses, error counts and the "
      "wall-clock span.");
}

}  // namespace symbn
