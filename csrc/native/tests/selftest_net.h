// Blocking loopback socket client + CHECK macro shared by the Python-free server self-tests.
#pragma once
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <string>

static int g_fail = 0;
#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      ++g_fail;                                                                   \
    }                                                                             \
  } while (0)

struct Client {
  int fd = -1;
  std::string buf;
  explicit Client(int port, bool handshake = true, const char* connect = nullptr) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    timeval tv{0, 300000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
    if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
      ::close(fd);
      fd = -1;
      return;
    }
    if (handshake) {
      CHECK(read_until("\r\n").rfind("INFO {", 0) == 0);
      send(connect ? connect : "CONNECT {\"verbose\":false}\r\n");
    }
  }
  ~Client() {
    if (fd >= 0) ::close(fd);
  }
  void send(const std::string& s) {
    size_t o = 0;
    while (o < s.size()) {
      const ssize_t w = ::send(fd, s.data() + o, s.size() - o, MSG_NOSIGNAL);
      if (w <= 0) return;
      o += (size_t)w;
    }
  }
  // reads until `needle` is in the buffer (or timeout); returns and consumes up to its end
  std::string read_until(const std::string& needle, int tries = 20) {
    for (int t = 0; t < tries; ++t) {
      const size_t p = buf.find(needle);
      if (p != std::string::npos) {
        std::string out = buf.substr(0, p + needle.size());
        buf.erase(0, p + needle.size());
        return out;
      }
      char tmp[65536];
      const ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
      if (r == 0) break;
      if (r > 0) buf.append(tmp, (size_t)r);
    }
    return "";
  }
  std::string drain(int rounds = 5) {
    for (int t = 0; t < rounds; ++t) {
      char tmp[65536];
      const ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
      if (r <= 0) break;
      buf.append(tmp, (size_t)r);
    }
    std::string out;
    out.swap(buf);
    return out;
  }
  bool closed_by_peer() {
    char tmp[4096];
    for (int t = 0; t < 20; ++t) {
      const ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
      if (r == 0) return true;
      if (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK) return true;
    }
    return false;
  }
};

static int count(const std::string& s, const std::string& n) {
  int c = 0;
  for (size_t p = s.find(n); p != std::string::npos; p = s.find(n, p + 1)) ++c;
  return c;
}

