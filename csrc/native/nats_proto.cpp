// NATS core protocol codec (client + server side), replacing the async-nats 0.33 protocol layer
// that every reference service links (e.g. services/api_service/Cargo.toml:11) and providing the
// op parser for the in-repo broker (there is no nats-server in this image).
//
// Streaming parser: feed() arbitrary byte chunks, get complete protocol events back.  Handles
// INFO, CONNECT, PUB, HPUB, SUB, UNSUB, MSG, HMSG, PING, PONG, +OK, -ERR (case-insensitive op
// names, space/tab separated args, payload framing by byte counts, \r\n terminators).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cctype>
#include <string>
#include <vector>

namespace py = pybind11;

namespace symbn {

struct NatsProtocolError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

static std::vector<std::string> split_args(const std::string& s) {
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

static long long to_int(const std::string& s) {
  if (s.empty() || s.size() > 18) throw NatsProtocolError("invalid size");
  long long v = 0;
  for (char c : s) {
    if (c < '0' || c > '9') throw NatsProtocolError("invalid size: " + s);
    v = v * 10 + (c - '0');
  }
  return v;
}

class NatsParser {
 public:
  explicit NatsParser(size_t max_control_line = 4096, long long max_payload = 64ll << 20)
      : max_ctl_(max_control_line), max_payload_(max_payload) {}

  py::list feed(py::bytes chunk) {
    char* p;
    Py_ssize_t n;
    PyBytes_AsStringAndSize(chunk.ptr(), &p, &n);
    buf_.append(p, (size_t)n);
    py::list events;
    for (;;) {
      if (need_ >= 0) {  // waiting for a payload of need_ bytes + \r\n
        if ((long long)(buf_.size() - pos_) < need_ + 2) break;
        if (buf_[pos_ + need_] != '\r' || buf_[pos_ + need_ + 1] != '\n')
          throw NatsProtocolError("payload not terminated by CRLF");
        emit_payload(events, buf_.data() + pos_, (size_t)need_);
        pos_ += need_ + 2;
        need_ = -1;
        continue;
      }
      const size_t eol = buf_.find("\r\n", pos_);
      if (eol == std::string::npos) {
        if (buf_.size() - pos_ > max_ctl_) throw NatsProtocolError("Maximum Control Line Exceeded");
        break;
      }
      std::string line = buf_.substr(pos_, eol - pos_);
      pos_ = eol + 2;
      control(events, line);
    }
    if (pos_ > 65536 || pos_ == buf_.size()) {
      buf_.erase(0, pos_);
      pos_ = 0;
    }
    return events;
  }

 private:
  void control(py::list& ev, const std::string& line) {
    size_t sp = line.find_first_of(" \t");
    std::string op = line.substr(0, sp);
    std::transform(op.begin(), op.end(), op.begin(), ::toupper);
    std::string rest = sp == std::string::npos ? "" : line.substr(sp + 1);
    if (op == "MSG") {
      auto a = split_args(rest);  // subject sid [reply] size
      if (a.size() != 3 && a.size() != 4) throw NatsProtocolError("bad MSG: " + line);
      pend_ = {"MSG", a[0], a[1], a.size() == 4 ? a[2] : "", 0};
      has_reply_ = a.size() == 4;
      start_payload(to_int(a.back()), 0);
    } else if (op == "HMSG") {
      auto a = split_args(rest);  // subject sid [reply] hdr total
      if (a.size() != 4 && a.size() != 5) throw NatsProtocolError("bad HMSG: " + line);
      pend_ = {"HMSG", a[0], a[1], a.size() == 5 ? a[2] : "", 0};
      has_reply_ = a.size() == 5;
      start_payload(to_int(a.back()), to_int(a[a.size() - 2]));
    } else if (op == "PUB") {
      auto a = split_args(rest);  // subject [reply] size
      if (a.size() != 2 && a.size() != 3) throw NatsProtocolError("bad PUB: " + line);
      pend_ = {"PUB", a[0], "", a.size() == 3 ? a[1] : "", 0};
      has_reply_ = a.size() == 3;
      start_payload(to_int(a.back()), 0);
    } else if (op == "HPUB") {
      auto a = split_args(rest);  // subject [reply] hdr total
      if (a.size() != 3 && a.size() != 4) throw NatsProtocolError("bad HPUB: " + line);
      pend_ = {"HPUB", a[0], "", a.size() == 4 ? a[1] : "", 0};
      has_reply_ = a.size() == 4;
      start_payload(to_int(a.back()), to_int(a[a.size() - 2]));
    } else if (op == "SUB") {
      auto a = split_args(rest);  // subject [queue] sid
      if (a.size() != 2 && a.size() != 3) throw NatsProtocolError("bad SUB: " + line);
      ev.append(py::make_tuple("SUB", a[0], a.size() == 3 ? py::object(py::str(a[1])) : py::none(),
                               a.back()));
    } else if (op == "UNSUB") {
      auto a = split_args(rest);  // sid [max]
      if (a.size() != 1 && a.size() != 2) throw NatsProtocolError("bad UNSUB: " + line);
      ev.append(py::make_tuple("UNSUB", a[0],
                               a.size() == 2 ? py::object(py::int_(to_int(a[1]))) : py::none()));
    } else if (op == "PING") {
      ev.append(py::make_tuple("PING"));
    } else if (op == "PONG") {
      ev.append(py::make_tuple("PONG"));
    } else if (op == "+OK") {
      ev.append(py::make_tuple("+OK"));
    } else if (op == "-ERR") {
      std::string m = rest;
      if (m.size() >= 2 && m.front() == '\'' && m.back() == '\'') m = m.substr(1, m.size() - 2);
      ev.append(py::make_tuple("-ERR", m));
    } else if (op == "INFO") {
      ev.append(py::make_tuple("INFO", py::bytes(rest)));
    } else if (op == "CONNECT") {
      ev.append(py::make_tuple("CONNECT", py::bytes(rest)));
    } else if (op.empty()) {
      // tolerate empty keep-alive lines
    } else {
      throw NatsProtocolError("Unknown Protocol Operation: " + op);
    }
  }

  void start_payload(long long total, long long hdr) {
    if (total < 0 || hdr < 0 || hdr > total) throw NatsProtocolError("bad payload sizes");
    if (total > max_payload_) throw NatsProtocolError("Maximum Payload Violation");
    need_ = total;
    pend_.hdr = hdr;
  }

  void emit_payload(py::list& ev, const char* p, size_t n) {
    py::object reply = has_reply_ ? py::object(py::str(pend_.reply)) : py::object(py::none());
    const std::string& kind = pend_.kind;
    if (kind == "MSG") {
      ev.append(py::make_tuple("MSG", pend_.subject, pend_.sid, reply, py::bytes(p, n)));
    } else if (kind == "HMSG") {
      ev.append(py::make_tuple("HMSG", pend_.subject, pend_.sid, reply, py::bytes(p, pend_.hdr),
                               py::bytes(p + pend_.hdr, n - pend_.hdr)));
    } else if (kind == "PUB") {
      ev.append(py::make_tuple("PUB", pend_.subject, reply, py::bytes(p, n)));
    } else {
      ev.append(py::make_tuple("HPUB", pend_.subject, reply, py::bytes(p, pend_.hdr),
                               py::bytes(p + pend_.hdr, n - pend_.hdr)));
    }
  }

  struct Pending {
    std::string kind, subject, sid, reply;
    long long hdr;
  } pend_;
  bool has_reply_ = false;
  std::string buf_;
  size_t pos_ = 0;
  long long need_ = -1;
  size_t max_ctl_;
  long long max_payload_;
};

// ---------------------------------------------------------------- encoders
static py::bytes enc_pub(const std::string& op, const std::string& subject, py::object reply,
                         py::bytes payload, py::object headers) {
  char* p;
  Py_ssize_t n;
  PyBytes_AsStringAndSize(payload.ptr(), &p, &n);
  std::string out = op + " " + subject;
  if (!reply.is_none()) out += " " + reply.cast<std::string>();
  if (!headers.is_none()) {
    std::string h = headers.cast<std::string>();
    out += " " + std::to_string(h.size()) + " " + std::to_string(h.size() + (size_t)n) + "\r\n";
    out += h;
  } else {
    out += " " + std::to_string(n) + "\r\n";
  }
  out.append(p, (size_t)n);
  out += "\r\n";
  return py::bytes(out);
}

// Header block "NATS/1.0[ status[ description]]\r\nK: V\r\n...\r\n"
static py::bytes enc_headers(py::object status, py::object description, py::list kvs) {
  std::string h = "NATS/1.0";
  if (!status.is_none()) {
    h += " " + status.cast<std::string>();
    if (!description.is_none()) h += " " + description.cast<std::string>();
  }
  h += "\r\n";
  for (auto item : kvs) {
    auto t = item.cast<py::tuple>();
    h += t[0].cast<std::string>() + ": " + t[1].cast<std::string>() + "\r\n";
  }
  h += "\r\n";
  return py::bytes(h);
}

static py::tuple dec_headers(py::bytes hdr) {
  std::string h = hdr;
  if (h.rfind("NATS/1.0", 0) != 0) throw NatsProtocolError("bad header block");
  size_t eol = h.find("\r\n");
  std::string first = h.substr(8, eol == std::string::npos ? std::string::npos : eol - 8);
  py::object status = py::none(), desc = py::none();
  size_t i = first.find_first_not_of(' ');
  if (i != std::string::npos) {
    first = first.substr(i);
    size_t sp = first.find(' ');
    status = py::str(first.substr(0, sp));
    if (sp != std::string::npos) desc = py::str(first.substr(sp + 1));
  }
  py::list kvs;
  size_t pos = eol == std::string::npos ? h.size() : eol + 2;
  while (pos < h.size()) {
    size_t e = h.find("\r\n", pos);
    if (e == std::string::npos) e = h.size();
    if (e == pos) break;
    std::string line = h.substr(pos, e - pos);
    size_t c = line.find(':');
    if (c != std::string::npos) {
      std::string k = line.substr(0, c), v = line.substr(c + 1);
      size_t a = v.find_first_not_of(' ');
      v = a == std::string::npos ? "" : v.substr(a);
      kvs.append(py::make_tuple(k, v));
    }
    pos = e + 2;
  }
  return py::make_tuple(status, desc, kvs);
}

void register_nats(py::module_& m) {
  py::register_exception<NatsProtocolError>(m, "NatsProtocolError", PyExc_ValueError);
  py::class_<NatsParser>(m, "NatsParser")
      .def(py::init<size_t, long long>(), py::arg("max_control_line") = 4096,
           py::arg("max_payload") = 64ll << 20)
      .def("feed", &NatsParser::feed);
  m.def("nats_pub", [](const std::string& subject, py::object reply, py::bytes payload,
                       py::object headers) {
    return enc_pub(headers.is_none() ? "PUB" : "HPUB", subject, reply, payload, headers);
  }, py::arg("subject"), py::arg("reply") = py::none(), py::arg("payload") = py::bytes(""),
     py::arg("headers") = py::none());
  m.def("nats_msg", [](const std::string& subject, const std::string& sid, py::object reply,
                       py::bytes payload, py::object headers) {
    return enc_pub(headers.is_none() ? "MSG" : "HMSG", subject + " " + sid, reply, payload,
                   headers);
  }, py::arg("subject"), py::arg("sid"), py::arg("reply") = py::none(),
     py::arg("payload") = py::bytes(""), py::arg("headers") = py::none());
  m.def("nats_headers", &enc_headers, py::arg("status") = py::none(),
        py::arg("description") = py::none(), py::arg("kvs") = py::list());
  m.def("nats_parse_headers", &dec_headers);
}

}  // namespace symbn
