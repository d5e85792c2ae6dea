// Python-object side of the JSON codec: dumps(obj) -> bytes and loads(bytes) -> obj.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <charconv>
#include <cstring>
#include <string>
#include <vector>

#include "json.h"

namespace py = pybind11;

namespace symbn {

static void dump_value(std::string& out, PyObject* o, int depth);

static void dump_value(std::string& out, PyObject* o, int depth) {
  if (depth > 128) throw std::runtime_error("recursion limit exceeded");
  if (o == Py_None) {
    out += "null";
  } else if (o == Py_True) {
    out += "true";
  } else if (o == Py_False) {
    out += "false";
  } else if (PyLong_Check(o)) {
    PyObject* s = PyObject_Str(o);
    if (!s) throw py::error_already_set();
    Py_ssize_t n;
    const char* c = PyUnicode_AsUTF8AndSize(s, &n);
    out.append(c, n);
    Py_DECREF(s);
  } else if (PyFloat_Check(o)) {
    append_f32(out, (float)PyFloat_AS_DOUBLE(o));
  } else if (PyUnicode_Check(o)) {
    Py_ssize_t n;
    const char* c = PyUnicode_AsUTF8AndSize(o, &n);
    if (!c) throw py::error_already_set();
    append_json_string(out, c, (size_t)n);
  } else if (PyDict_Check(o)) {
    out.push_back('{');
    PyObject *k, *v;
    Py_ssize_t pos = 0;
    bool first = true;
    while (PyDict_Next(o, &pos, &k, &v)) {
      if (!PyUnicode_Check(k)) throw std::runtime_error("key must be a string");
      if (!first) out.push_back(',');
      first = false;
      Py_ssize_t n;
      const char* c = PyUnicode_AsUTF8AndSize(k, &n);
      append_json_string(out, c, (size_t)n);
      out.push_back(':');
      dump_value(out, v, depth + 1);
    }
    out.push_back('}');
  } else if (PyList_Check(o) || PyTuple_Check(o)) {
    PyObject* seq = o;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    PyObject** items = PySequence_Fast_ITEMS(seq);
    out.push_back('[');
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (i) out.push_back(',');
      dump_value(out, items[i], depth + 1);
    }
    out.push_back(']');
  } else if (py::isinstance<py::array>(py::handle(o))) {
    auto arr = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(py::handle(o));
    if (!arr) throw std::runtime_error("array not convertible to float32");
    if (arr.ndim() != 1) throw std::runtime_error("only 1-d arrays are serialisable");
    append_f32_array(out, arr.data(), (size_t)arr.size());
  } else if (PyObject_HasAttrString(o, "__float__") && !PyObject_HasAttrString(o, "__index__")) {
    const double d = PyFloat_AsDouble(o);
    if (PyErr_Occurred()) throw py::error_already_set();
    append_f32(out, (float)d);
  } else if (PyObject_HasAttrString(o, "__index__")) {
    PyObject* i = PyNumber_Index(o);
    if (!i) throw py::error_already_set();
    dump_value(out, i, depth + 1);
    Py_DECREF(i);
  } else {
    throw std::runtime_error(std::string("unserialisable type: ") + Py_TYPE(o)->tp_name);
  }
}

py::bytes dumps(py::handle obj) {
  std::string out;
  out.reserve(256);
  dump_value(out, obj.ptr(), 0);
  return py::bytes(out);
}

py::bytes dumps_f32_array(py::array_t<float, py::array::c_style | py::array::forcecast> a) {
  std::string out;
  out.reserve((size_t)a.size() * 12 + 2);
  append_f32_array(out, a.data(), (size_t)a.size());
  return py::bytes(out);
}

// --------------------------------------------------------------------------- loads
struct Loader {
  Parser p;
  bool f32_arrays;
  Loader(const char* s, size_t n, bool f32) : p(s, n), f32_arrays(f32) {}

  py::object number_obj(const Number& n) {
    if (!n.is_float) {
      PyObject* o = PyLong_FromString(n.text.c_str(), nullptr, 10);
      if (!o) throw py::error_already_set();
      return py::reinterpret_steal<py::object>(o);
    }
    return py::float_(parse_f64(n.text.data(), n.text.size()));
  }

  py::object value(int depth) {
    if (depth > 128) p.fail("recursion limit exceeded");
    const char c = p.peek();
    if (c == '{') {
      p.advance();
      py::dict d;
      if (p.peek() == '}') {
        p.advance();
        return std::move(d);
      }
      for (;;) {
        if (p.peek() != '"') p.fail("key must be a string");
        std::string k = p.string();
        if (p.peek() != ':') p.fail("expected `:`");
        p.advance();
        py::object v = value(depth + 1);
        d[py::str(k)] = v;
        const char t = p.peek();
        if (t == ',') {
          p.advance();
          continue;
        }
        if (t == '}') {
          p.advance();
          return std::move(d);
        }
        p.fail("expected `,` or `}`");
      }
    }
    if (c == '[') {
      p.advance();
      if (p.peek() == ']') {
        p.advance();
        return py::list();
      }
      // fast path: an all-number array becomes a float32 numpy buffer when requested
      std::vector<py::object> items;
      std::vector<NumSpan> raw;    // numbers seen before the first non-number element
      bool all_num = f32_arrays;
      for (;;) {
        const char t = p.peek();
        if (all_num && (t == '-' || (t >= '0' && t <= '9'))) {
          raw.push_back(p.number_span());
        } else {
          if (all_num) {  // demote: materialise the numbers parsed so far
            for (const NumSpan& n : raw)
              items.push_back(number_obj(Number{n.is_float, std::string(p.data() + n.start, n.len)}));
            raw.clear();
            all_num = false;
          }
          items.push_back(value(depth + 1));
        }
        const char s = p.peek();
        if (s == ',') {
          p.advance();
          continue;
        }
        if (s == ']') {
          p.advance();
          break;
        }
        p.fail("expected `,` or `]`");
      }
      if (all_num) {
        py::array_t<float> arr((py::ssize_t)raw.size());
        float* dst = arr.mutable_data();
        // f64 then cast, as serde_json reads an f32 (fast path: a 384-float query embedding
        // parses in a few us; libstdc++ 11's from_chars<float> goes through strtod)
        for (size_t i = 0; i < raw.size(); ++i)
          dst[i] = (float)parse_f64(p.data() + raw[i].start, raw[i].len);
        return std::move(arr);
      }
      py::list l(items.size());
      for (size_t i = 0; i < items.size(); ++i) l[i] = items[i];
      return std::move(l);
    }
    if (c == '"') return py::str(p.string());
    if (c == 't') {
      p.expect_lit("true");
      return py::bool_(true);
    }
    if (c == 'f') {
      p.expect_lit("false");
      return py::bool_(false);
    }
    if (c == 'n') {
      p.expect_lit("null");
      return py::none();
    }
    if (c == '-' || (c >= '0' && c <= '9')) return number_obj(p.number());
    p.fail("expected value");
  }
};

py::object loads(py::bytes data, bool f32_arrays) {
  char* buf;
  Py_ssize_t n;
  PyBytes_AsStringAndSize(data.ptr(), &buf, &n);
  Loader L(buf, (size_t)n, f32_arrays);
  py::object v = L.value(0);
  if (!L.p.at_end()) L.p.fail("trailing characters");
  return v;
}

std::string format_f32(float f) {
  std::string s;
  append_f32(s, f);
  return s;
}

// SemanticSearchNatsResult bytes from per-point JSON fragments cached by the vector store:
// frags[i] = (b'{"qdrant_point_id":"<id>","score":', b',"payload":{...}}'); scores are f32 and
// formatted like serde_json.  Identical bytes to SemanticSearchNatsResult(...).to_json().
py::bytes search_result_json(const std::string& request_id,
                             py::array_t<float, py::array::c_style | py::array::forcecast> scores,
                             py::list frags, py::object error_message) {
  const size_t n = (size_t)py::len(frags);
  if ((size_t)scores.size() < n) throw std::runtime_error("fewer scores than fragments");
  const float* sc = scores.data();
  std::string out;
  out.reserve(64 + n * 320);
  out += "{\"request_id\":";
  append_json_string(out, request_id.data(), request_id.size());
  out += ",\"results\":[";
  for (size_t i = 0; i < n; ++i) {
    py::tuple t = frags[i].cast<py::tuple>();
    char* a;
    char* b;
    Py_ssize_t na, nb;
    if (PyBytes_AsStringAndSize(t[0].ptr(), &a, &na) || PyBytes_AsStringAndSize(t[1].ptr(), &b, &nb))
      throw py::error_already_set();
    if (i) out.push_back(',');
    out.append(a, (size_t)na);
    append_f32(out, sc[i]);
    out.append(b, (size_t)nb);
  }
  out += "],\"error_message\":";
  if (error_message.is_none()) {
    out += "null";
  } else {
    const std::string e = error_message.cast<std::string>();
    append_json_string(out, e.data(), e.size());
  }
  out += "}";
  return py::bytes(out);
}


// A whole scan's replies in ONE call (vector_memory's per-burst loop): for query j, the first
// ks[j] (score, row) pairs with row >= 0 whose cached result fragments exist become
// SemanticSearchNatsResult JSON -- the same bytes search_result_json builds per request.  The
// fragments come from `cache` (dict row -> (prefix, suffix) bytes, read without Python bytecode);
// a miss calls `miss(row)` (the store's payload lookup, which fills the cache) and a None from it
// skips the row (a point without an id, as the reference skips undecodable ids).  errs: None or
// a list of per-query error_message values (str or None).  Returns (list of bytes, skipped).
static py::tuple search_results_batch(py::list rids,
                                      py::array_t<float, py::array::c_style | py::array::forcecast> scores,
                                      py::array_t<int64_t, py::array::c_style | py::array::forcecast> rows,
                                      py::array_t<int64_t, py::array::c_style | py::array::forcecast> ks,
                                      py::dict cache, py::object miss, py::object errs) {
  const size_t n = (size_t)py::len(rids);
  if (scores.ndim() != 2 || rows.ndim() != 2 || scores.shape(0) != rows.shape(0) ||
      scores.shape(1) != rows.shape(1) || (size_t)scores.shape(0) < n || (size_t)ks.size() < n)
    throw std::runtime_error("search_results_batch: shape mismatch");
  const size_t kmax = (size_t)scores.shape(1);
  const float* sc = scores.data();
  const int64_t* rw = rows.data();
  const int64_t* kp = ks.data();
  const bool have_errs = !errs.is_none();
  py::list out(n);
  long skipped = 0;
  std::string buf;
  for (size_t j = 0; j < n; ++j) {
    buf.clear();
    buf += "{\"request_id\":";
    const std::string rid = rids[j].cast<std::string>();
    append_json_string(buf, rid.data(), rid.size());
    buf += ",\"results\":[";
    const size_t k = std::min(kmax, (size_t)std::max<int64_t>(0, kp[j]));
    bool first = true;
    for (size_t c = 0; c < k; ++c) {
      const int64_t r = rw[j * kmax + c];
      if (r < 0) continue;
      py::object key = py::int_(r);
      PyObject* f = PyDict_GetItem(cache.ptr(), key.ptr());   // borrowed
      py::object hold;
      if (f == nullptr) {
        hold = miss(key);
        if (hold.is_none()) {
          ++skipped;
          continue;
        }
        f = hold.ptr();
      }
      PyObject* a = PyTuple_GetItem(f, 0);
      PyObject* b = PyTuple_GetItem(f, 1);
      char* pa;
      char* pb;
      Py_ssize_t na, nb;
      if (a == nullptr || b == nullptr || PyBytes_AsStringAndSize(a, &pa, &na) ||
          PyBytes_AsStringAndSize(b, &pb, &nb))
        throw py::error_already_set();
      if (!first) buf.push_back(',');
      first = false;
      buf.append(pa, (size_t)na);
      append_f32(buf, sc[j * kmax + c]);
      buf.append(pb, (size_t)nb);
    }
    buf += "],\"error_message\":";
    py::object e = have_errs ? errs.cast<py::list>()[j] : py::object(py::none());
    if (e.is_none()) {
      buf += "null";
    } else {
      const std::string es = e.cast<std::string>();
      append_json_string(buf, es.data(), es.size());
    }
    buf += "}";
    out[j] = py::bytes(buf);
  }
  return py::make_tuple(out, skipped);
}

// A batch of SemanticSearchNatsTask messages -> (ok[n], request_ids[n], top_k[n], queries[n, dim]).
// Only the regular shape {"request_id": str, "query_embedding": [dim numbers], "top_k": int}
// (keys in any order, each once) is decoded here; anything else -- malformed JSON, other keys,
// wrong types, another length -- gets ok = false and the caller decodes that message with the
// wire model, which produces serde's exact error text.  vector_memory answers a whole drained
// batch of search requests with one call and one index scan.
static py::tuple search_tasks_batch(py::list msgs, int dim) {
  const size_t n = (size_t)py::len(msgs);
  py::array_t<bool> ok((py::ssize_t)n);
  py::array_t<int64_t> topk((py::ssize_t)n);
  py::array_t<float> q({(py::ssize_t)n, (py::ssize_t)dim});
  py::list ids(n);
  bool* okp = ok.mutable_data();
  int64_t* kp = topk.mutable_data();
  float* qp = q.mutable_data();
  for (size_t m = 0; m < n; ++m) {
    okp[m] = false;
    kp[m] = 0;
    ids[m] = py::none();
    char* buf;
    Py_ssize_t len;
    if (PyBytes_AsStringAndSize(msgs[m].ptr(), &buf, &len)) {
      PyErr_Clear();
      continue;
    }
    Parser p(buf, (size_t)len);
    float* row = qp + m * (size_t)dim;
    try {
      if (p.peek() != '{') continue;
      p.advance();
      int seen = 0;  // bit 0 request_id, 1 query_embedding, 2 top_k
      bool good = true;
      std::string rid;
      for (;;) {
        if (p.peek() != '"') { good = false; break; }
        const std::string key = p.string();
        if (p.peek() != ':') { good = false; break; }
        p.advance();
        const char c = p.peek();
        if (key == "request_id" && !(seen & 1) && c == '"') {
          rid = p.string();
          seen |= 1;
        } else if (key == "query_embedding" && !(seen & 2) && c == '[') {
          p.advance();
          int cnt = 0;
          if (p.peek() == ']') {
            p.advance();
          } else {
            for (;;) {
              const char t = p.peek();
              if (!(t == '-' || (t >= '0' && t <= '9')) || cnt >= dim) { good = false; break; }
              row[cnt++] = (float)p.number_f64();
              const char sep = p.peek();
              p.advance();
              if (sep == ']') break;
              if (sep != ',') { good = false; break; }
            }
          }
          if (!good || cnt != dim) { good = false; break; }
          seen |= 2;
        } else if (key == "top_k" && !(seen & 4) && c >= '0' && c <= '9') {
          const NumSpan sp = p.number_span();
          if (sp.is_float || sp.len > 10) { good = false; break; }
          int64_t v = 0;
          for (size_t i = 0; i < sp.len; ++i) v = v * 10 + (p.data()[sp.start + i] - '0');
          if (v > 0xFFFFFFFFll) { good = false; break; }  // u32, like the wire model
          kp[m] = v;
          seen |= 4;
        } else {
          good = false;
          break;
        }
        const char sep = p.peek();
        p.advance();
        if (sep == '}') break;
        if (sep != ',') { good = false; break; }
      }
      if (!good || seen != 7 || !p.at_end()) continue;
      ids[m] = py::str(rid);  // same conversion as json_loads
      okp[m] = true;
    } catch (const JsonError&) {
      continue;
    } catch (const py::error_already_set&) {
      continue;
    }
  }
  return py::make_tuple(ok, ids, topk, q);
}

void register_json(py::module_& m) {
  m.def("search_result_json", &search_result_json, py::arg("request_id"), py::arg("scores"),
        py::arg("frags"), py::arg("error_message") = py::none());
  py::register_exception<JsonError>(m, "JsonError", PyExc_ValueError);
  m.def("search_tasks_batch", &search_tasks_batch, py::arg("msgs"), py::arg("dim"));
  m.def("search_results_batch", &search_results_batch, py::arg("request_ids"), py::arg("scores"),
        py::arg("rows"), py::arg("ks"), py::arg("cache"), py::arg("miss"),
        py::arg("errors") = py::none());
  m.def("json_dumps", &dumps, "serde_json-compatible compact encoding (floats as f32)");
  m.def("json_dumps_f32_array", &dumps_f32_array);
  m.def("json_loads", &loads, py::arg("data"), py::arg("f32_arrays") = false);
  m.def("format_f32", &format_f32);
}

}  // namespace symbn
