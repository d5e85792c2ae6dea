// SentencePiece "Precompiled" normalizer (the tokenizer.json normalizer of XLM-R-family models:
// paraphrase-multilingual-mpnet-base-v2 is the reference's model, preprocessing_service/src/
// main.rs:305, whose tokenizer.json the reference fetches in embedding_generator.rs:25-58 and
// runs through the tokenizers crate).
//
// The charsmap blob (base64 in tokenizer.json, ``normalizer_spec.precompiled_charsmap`` in a
// SentencePiece model) is  [u32 trie_bytes][Darts double-array of u32 units][NUL-terminated
// replacement strings].  A key's value is the byte offset of its replacement string.
//
// Normalisation walks the input by EXTENDED GRAPHEME CLUSTERS (UAX #29, unicode_gcb.h) exactly
// as HF tokenizers does: a cluster shorter than 6 bytes is looked up whole, and the SHORTEST
// key that prefixes it replaces the whole cluster (the rest of the cluster is dropped -- a
// SentencePiece quirk HF preserves, e.g. "ä́" -> "ä"); otherwise (or on no hit)
// each code point is looked up on its own and kept when it has no entry.
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "unicode_gcb.h"

namespace py = pybind11;

namespace symbn {

static uint8_t gcb_of(uint32_t cp) {
  int lo = 0, hi = (int)(sizeof(kGcbRanges) / sizeof(kGcbRanges[0])) - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (cp < kGcbRanges[mid].lo) hi = mid - 1;
    else if (cp > kGcbRanges[mid].hi) lo = mid + 1;
    else return kGcbRanges[mid].cls;
  }
  return kGcbOther;
}

// UTF-8 length of the code point starting at s[i] (1 on an invalid lead byte) and its value.
static int u8next(const std::string& s, size_t i, uint32_t& cp) {
  const unsigned char c = (unsigned char)s[i];
  int n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
  if (i + n > s.size()) n = 1;
  if (n == 1) {
    cp = c;
    return 1;
  }
  cp = c & (0x7F >> n);
  for (int k = 1; k < n; ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
  return n;
}

// Is there a grapheme-cluster boundary between a code point of class `a` and one of class `b`?
// `ri_run`: regional indicators already in the cluster; `pict_zwj`: the cluster so far is
// ExtPict Extend* ZWJ (GB11).
static bool gcb_break(uint8_t a, uint8_t b, int ri_run, bool pict_zwj) {
  if (a == kGcbCR && b == kGcbLF) return false;                                  // GB3
  if (a == kGcbControl || a == kGcbCR || a == kGcbLF) return true;              // GB4
  if (b == kGcbControl || b == kGcbCR || b == kGcbLF) return true;              // GB5
  if (a == kGcbL && (b == kGcbL || b == kGcbV || b == kGcbLV || b == kGcbLVT)) return false;  // GB6
  if ((a == kGcbLV || a == kGcbV) && (b == kGcbV || b == kGcbT)) return false;   // GB7
  if ((a == kGcbLVT || a == kGcbT) && b == kGcbT) return false;                  // GB8
  if (b == kGcbExtend || b == kGcbZWJ) return false;                             // GB9
  if (b == kGcbSpacingMark) return false;                                        // GB9a
  if (a == kGcbPrepend) return false;                                            // GB9b
  if (a == kGcbZWJ && b == kGcbExtPict && pict_zwj) return false;                // GB11
  if (a == kGcbRI && b == kGcbRI) return (ri_run % 2) == 0;                      // GB12/13
  return true;                                                                   // GB999
}

class Precompiled {
 public:
  explicit Precompiled(const std::string& blob) {
    if (blob.size() < 4) throw std::invalid_argument("precompiled charsmap: too short");
    uint32_t trie_bytes;
    std::memcpy(&trie_bytes, blob.data(), 4);
    if (trie_bytes % 4 || 4 + (size_t)trie_bytes > blob.size())
      throw std::invalid_argument("precompiled charsmap: bad trie size");
    units_.resize(trie_bytes / 4);
    std::memcpy(units_.data(), blob.data() + 4, trie_bytes);
    normalized_ = blob.substr(4 + trie_bytes);
    if (units_.empty()) throw std::invalid_argument("precompiled charsmap: empty trie");
  }

  // Darts common-prefix search: value of the SHORTEST key prefixing s[pos, pos+len), or -1.
  long lookup(const char* s, size_t len) const {
    size_t node = 0;
    uint32_t unit = units_[0];
    node ^= offset(unit);
    for (size_t i = 0; i < len; ++i) {
      const unsigned char c = (unsigned char)s[i];
      if (c == 0) break;
      node ^= c;
      if (node >= units_.size()) return -1;
      unit = units_[node];
      if (label(unit) != c) return -1;
      node ^= offset(unit);
      if (node >= units_.size()) return -1;
      if ((unit >> 8) & 1) return (long)(units_[node] & 0x7FFFFFFFu);
    }
    return -1;
  }

  bool transform(const std::string& s, size_t pos, size_t len, std::string& out) const {
    const long v = lookup(s.data() + pos, len);
    if (v < 0 || (size_t)v >= normalized_.size()) return false;
    const char* p = normalized_.data() + v;
    out.append(p, strnlen(p, normalized_.size() - (size_t)v));
    return true;
  }

  std::string normalize(const std::string& s) const {
    std::string out;
    out.reserve(s.size() + s.size() / 4);
    size_t i = 0;
    while (i < s.size()) {
      // one extended grapheme cluster [i, j)
      uint32_t cp;
      size_t j = i + u8next(s, i, cp);
      uint8_t prev = gcb_of(cp);
      int ri_run = prev == kGcbRI ? 1 : 0;
      bool pict = prev == kGcbExtPict, pict_zwj = false;
      while (j < s.size()) {
        uint32_t c2;
        const int n = u8next(s, j, c2);
        const uint8_t cls = gcb_of(c2);
        if (gcb_break(prev, cls, ri_run, pict_zwj)) break;
        ri_run = cls == kGcbRI ? ri_run + 1 : 0;
        pict_zwj = pict && cls == kGcbZWJ;
        if (cls != kGcbExtend && cls != kGcbZWJ) pict = cls == kGcbExtPict;
        prev = cls;
        j += n;
      }
      if (j - i < 6 && transform(s, i, j - i, out)) {
        i = j;
        continue;
      }
      while (i < j) {   // code point by code point
        const int n = u8next(s, i, cp);
        if (!transform(s, i, n, out)) out.append(s, i, n);
        i += n;
      }
    }
    return out;
  }

  // the grapheme clusters of s (tests: segmentation parity)
  std::vector<std::string> graphemes(const std::string& s) const {
    std::vector<std::string> g;
    size_t i = 0;
    while (i < s.size()) {
      uint32_t cp;
      size_t j = i + u8next(s, i, cp);
      uint8_t prev = gcb_of(cp);
      int ri_run = prev == kGcbRI ? 1 : 0;
      bool pict = prev == kGcbExtPict, pict_zwj = false;
      while (j < s.size()) {
        uint32_t c2;
        const int n = u8next(s, j, c2);
        const uint8_t cls = gcb_of(c2);
        if (gcb_break(prev, cls, ri_run, pict_zwj)) break;
        ri_run = cls == kGcbRI ? ri_run + 1 : 0;
        pict_zwj = pict && cls == kGcbZWJ;
        if (cls != kGcbExtend && cls != kGcbZWJ) pict = cls == kGcbExtPict;
        prev = cls;
        j += n;
      }
      g.emplace_back(s.substr(i, j - i));
      i = j;
    }
    return g;
  }

 private:
  static uint32_t offset(uint32_t u) { return (u >> 10) << ((u & (1u << 9)) >> 6); }
  static uint32_t label(uint32_t u) { return u & ((1u << 31) | 0xFFu); }
  std::vector<uint32_t> units_;
  std::string normalized_;
};

#ifndef SYMB_NO_PYTHON
void register_spm_norm(py::module_& m) {
  py::class_<Precompiled>(m, "Precompiled")
      .def(py::init([](py::bytes b) { return Precompiled(std::string(b)); }), py::arg("charsmap"))
      .def("normalize", [](const Precompiled& p, const std::string& s) {
        std::string r;
        {
          py::gil_scoped_release nogil;
          r = p.normalize(s);
        }
        return r;
      })
      .def("normalize_many", [](const Precompiled& p, const std::vector<std::string>& v) {
        std::vector<std::string> r;
        {
          py::gil_scoped_release nogil;
          r.reserve(v.size());
          for (const auto& s : v) r.push_back(p.normalize(s));
        }
        return r;
      })
      .def("graphemes", &Precompiled::graphemes);
}
#endif

}  // namespace symbn
