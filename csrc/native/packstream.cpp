// PackStream v1 codec + Bolt message chunking for the knowledge-graph service.
//
// Replaces the neo4rs 0.7.3 Bolt driver used by services/knowledge_graph_service/src/main.rs
// (start_txn :32-35, RUN/PULL :50-59, :90-92, :122-124, commit :132-134).  Values map to Python:
// None/bool/int/float/str/bytes/list/dict and Structure(tag, fields) via a factory callable.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <string>

namespace py = pybind11;

namespace symbn {

struct PackStreamError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

static void be(std::string& o, uint64_t v, int bytes) {
  for (int i = bytes - 1; i >= 0; --i) o.push_back((char)((v >> (8 * i)) & 0xFF));
}

static void pack_size(std::string& o, size_t n, uint8_t tiny, uint8_t m8, uint8_t m16,
                      uint8_t m32, bool has8 = true) {
  if (n < 16 && tiny) {
    o.push_back((char)(tiny | n));
  } else if (n < 256 && has8) {
    o.push_back((char)m8);
    be(o, n, 1);
  } else if (n < 65536) {
    o.push_back((char)m16);
    be(o, n, 2);
  } else {
    o.push_back((char)m32);
    be(o, n, 4);
  }
}

static void pack(std::string& o, py::handle v, int depth) {
  if (depth > 64) throw PackStreamError("nesting too deep");
  PyObject* p = v.ptr();
  if (p == Py_None) {
    o.push_back((char)0xC0);
  } else if (p == Py_True) {
    o.push_back((char)0xC3);
  } else if (p == Py_False) {
    o.push_back((char)0xC2);
  } else if (PyLong_Check(p)) {
    const long long x = v.cast<long long>();
    if (x >= -16 && x <= 127) {
      o.push_back((char)(int8_t)x);
    } else if (x >= -128 && x <= 127) {
      o.push_back((char)0xC8);
      be(o, (uint64_t)x, 1);
    } else if (x >= -32768 && x <= 32767) {
      o.push_back((char)0xC9);
      be(o, (uint64_t)x, 2);
    } else if (x >= -2147483648LL && x <= 2147483647LL) {
      o.push_back((char)0xCA);
      be(o, (uint64_t)x, 4);
    } else {
      o.push_back((char)0xCB);
      be(o, (uint64_t)x, 8);
    }
  } else if (PyFloat_Check(p)) {
    const double d = PyFloat_AS_DOUBLE(p);
    uint64_t bits;
    std::memcpy(&bits, &d, 8);
    o.push_back((char)0xC1);
    be(o, bits, 8);
  } else if (PyUnicode_Check(p)) {
    Py_ssize_t n;
    const char* s = PyUnicode_AsUTF8AndSize(p, &n);
    pack_size(o, (size_t)n, 0x80, 0xD0, 0xD1, 0xD2);
    o.append(s, (size_t)n);
  } else if (PyBytes_Check(p) || PyByteArray_Check(p)) {
    PyObject* bo = PyBytes_Check(p) ? (Py_INCREF(p), p) : PyBytes_FromObject(p);
    if (!bo) throw py::error_already_set();
    std::string b(PyBytes_AS_STRING(bo), (size_t)PyBytes_GET_SIZE(bo));
    Py_DECREF(bo);
    pack_size(o, b.size(), 0, 0xCC, 0xCD, 0xCE);
    o += b;
  } else if (PyList_Check(p) || PyTuple_Check(p)) {
    py::sequence seq = py::reinterpret_borrow<py::sequence>(v);
    pack_size(o, seq.size(), 0x90, 0xD4, 0xD5, 0xD6);
    for (auto item : seq) pack(o, item, depth + 1);
  } else if (PyDict_Check(p)) {
    py::dict d = py::reinterpret_borrow<py::dict>(v);
    pack_size(o, d.size(), 0xA0, 0xD8, 0xD9, 0xDA);
    for (auto kv : d) {
      if (!PyUnicode_Check(kv.first.ptr())) throw PackStreamError("map keys must be strings");
      pack(o, kv.first, depth + 1);
      pack(o, kv.second, depth + 1);
    }
  } else if (py::hasattr(v, "tag") && py::hasattr(v, "fields")) {
    const int tag = v.attr("tag").cast<int>();
    py::sequence fields = v.attr("fields");
    if (fields.size() > 15) throw PackStreamError("structure too large");
    o.push_back((char)(0xB0 | fields.size()));
    o.push_back((char)tag);
    for (auto f : fields) pack(o, f, depth + 1);
  } else {
    throw PackStreamError(std::string("cannot pack ") + Py_TYPE(p)->tp_name);
  }
}

struct Unpacker {
  const uint8_t* p;
  size_t n, i = 0;
  py::object factory;
  uint64_t rd(int bytes) {
    if (i + bytes > n) throw PackStreamError("truncated");
    uint64_t v = 0;
    for (int k = 0; k < bytes; ++k) v = (v << 8) | p[i++];
    return v;
  }
  py::object str(size_t len) {
    if (i + len > n) throw PackStreamError("truncated string");
    py::str s(reinterpret_cast<const char*>(p + i), len);
    i += len;
    return std::move(s);
  }
  py::object list(size_t len, int d) {
    py::list l;
    for (size_t k = 0; k < len; ++k) l.append(value(d + 1));
    return std::move(l);
  }
  py::object map(size_t len, int d) {
    py::dict m;
    for (size_t k = 0; k < len; ++k) {
      py::object key = value(d + 1);
      m[key] = value(d + 1);
    }
    return std::move(m);
  }
  py::object value(int d) {
    if (d > 64) throw PackStreamError("nesting too deep");
    const uint8_t m = (uint8_t)rd(1);
    if (m < 0x80) return py::int_(m);
    if (m >= 0xF0) return py::int_((int)(int8_t)m);
    const uint8_t hi = m & 0xF0, lo = m & 0x0F;
    if (hi == 0x80) return str(lo);
    if (hi == 0x90) return list(lo, d);
    if (hi == 0xA0) return map(lo, d);
    if (hi == 0xB0) {
      const int tag = (int)rd(1);
      py::list fields;
      for (int k = 0; k < lo; ++k) fields.append(value(d + 1));
      return factory(tag, fields);
    }
    switch (m) {
      case 0xC0: return py::none();
      case 0xC2: return py::bool_(false);
      case 0xC3: return py::bool_(true);
      case 0xC1: {
        uint64_t bits = rd(8);
        double x;
        std::memcpy(&x, &bits, 8);
        return py::float_(x);
      }
      case 0xC8: return py::int_((long long)(int8_t)rd(1));
      case 0xC9: return py::int_((long long)(int16_t)rd(2));
      case 0xCA: return py::int_((long long)(int32_t)rd(4));
      case 0xCB: return py::int_((long long)rd(8));
      case 0xCC: case 0xCD: case 0xCE: {
        size_t len = rd(m == 0xCC ? 1 : m == 0xCD ? 2 : 4);
        if (i + len > n) throw PackStreamError("truncated bytes");
        py::bytes b(reinterpret_cast<const char*>(p + i), len);
        i += len;
        return std::move(b);
      }
      case 0xD0: return str(rd(1));
      case 0xD1: return str(rd(2));
      case 0xD2: return str(rd(4));
      case 0xD4: return list(rd(1), d);
      case 0xD5: return list(rd(2), d);
      case 0xD6: return list(rd(4), d);
      case 0xD8: return map(rd(1), d);
      case 0xD9: return map(rd(2), d);
      case 0xDA: return map(rd(4), d);
    }
    throw PackStreamError("unknown marker");
  }
};

py::bytes ps_pack(py::handle v) {
  std::string o;
  pack(o, v, 0);
  return py::bytes(o);
}

py::object ps_unpack(py::bytes data, py::object factory) {
  std::string s = data;
  Unpacker u{reinterpret_cast<const uint8_t*>(s.data()), s.size(), 0, factory};
  py::object v = u.value(0);
  if (u.i != u.n) throw PackStreamError("trailing bytes");
  return v;
}

// One Bolt message -> chunks (<= 65535 bytes each) + 0x0000 end marker.
py::bytes bolt_chunk(py::bytes msg, size_t max_chunk) {
  std::string s = msg, o;
  size_t pos = 0;
  while (pos < s.size()) {
    const size_t n = std::min(max_chunk, s.size() - pos);
    be(o, n, 2);
    o.append(s, pos, n);
    pos += n;
  }
  o.push_back(0);
  o.push_back(0);
  return py::bytes(o);
}

class BoltDechunker {
 public:
  py::list feed(py::bytes data) {
    buf_ += std::string(data);
    py::list out;
    for (;;) {
      if (buf_.size() - pos_ < 2) break;
      const size_t n = ((uint8_t)buf_[pos_] << 8) | (uint8_t)buf_[pos_ + 1];
      if (n == 0) {
        pos_ += 2;
        if (!msg_.empty()) out.append(py::bytes(msg_));
        msg_.clear();
        continue;
      }
      if (buf_.size() - pos_ < 2 + n) break;
      msg_.append(buf_, pos_ + 2, n);
      pos_ += 2 + n;
    }
    buf_.erase(0, pos_);
    pos_ = 0;
    return out;
  }

 private:
  std::string buf_, msg_;
  size_t pos_ = 0;
};

void register_packstream(py::module_& m) {
  py::register_exception<PackStreamError>(m, "PackStreamError", PyExc_ValueError);
  m.def("ps_pack", &ps_pack);
  m.def("ps_unpack", &ps_unpack);
  m.def("bolt_chunk", &bolt_chunk, py::arg("msg"), py::arg("max_chunk") = 65535);
  py::class_<BoltDechunker>(m, "BoltDechunker").def(py::init<>()).def("feed", &BoltDechunker::feed);
}

}  // namespace symbn
