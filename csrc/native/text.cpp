// Host text cores:
//  * normalize_whitespace / split_sentences -- byte-exact with the reference preprocessing
//    (services/preprocessing_service/src/main.rs:28-62: split_whitespace().join(" "), then a
//    char scan cutting after every '.', '?', '!', each piece trimmed, trimmed remainder, whole text
//    as the single sentence when nothing was cut).
//  * MarkovModel -- word-bigram chain with the reference's training and generation rules
//    (services/text_generator_service/src/main.rs:29-108), including its quirks: starters hold
//    only the first word of each training text; generation stops at a word with no successor.
//  * WordPiece -- BERT BasicTokenizer (clean, CJK split, lowercase + accent strip, punctuation
//    split) + greedy longest-match-first WordPiece with "##" continuations, replacing the HF
//    `tokenizers` crate used by embedding_generator.rs:161-164.
#ifndef SYMB_NO_PYTHON
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif

#include <algorithm>
#include <limits>
#include <random>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#ifndef SYMB_NO_PYTHON
namespace py = pybind11;
#endif

namespace symbn {

// ------------------------------------------------------------------------ UTF-8 helpers
static std::u32string utf8_decode(const std::string& s) {
  std::u32string out;
  out.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int len;
    if (c < 0x80) { cp = c; len = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; len = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; len = 3; }
    else if ((c >> 3) == 30) { cp = c & 0x07; len = 4; }
    else { cp = 0xFFFD; len = 1; }
    if (i + len > s.size()) { cp = 0xFFFD; len = 1; }
    for (int k = 1; k < len; ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
    out.push_back(cp);
    i += len;
  }
  return out;
}

static void utf8_put(std::string& s, uint32_t cp) {
  if (cp < 0x80) s.push_back((char)cp);
  else if (cp < 0x800) { s.push_back((char)(0xC0 | (cp >> 6))); s.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) {
    s.push_back((char)(0xE0 | (cp >> 12))); s.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    s.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    s.push_back((char)(0xF0 | (cp >> 18))); s.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    s.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); s.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

static std::string utf8_encode(const std::u32string& u) {
  std::string s;
  s.reserve(u.size());
  for (uint32_t c : u) utf8_put(s, c);
  return s;
}

// Rust char::is_whitespace (Unicode White_Space property)
static bool is_ws(uint32_t c) {
  return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F ||
         c == 0x205F || c == 0x3000;
}

// Decode one UTF-8 char at byte i (returns byte length); invalid bytes count as 1.
static int u8len(const std::string& s, size_t i) {
  const unsigned char c = (unsigned char)s[i];
  if (c < 0x80) return 1;
  if ((c >> 5) == 6) return 2;
  if ((c >> 4) == 14) return 3;
  if ((c >> 3) == 30) return 4;
  return 1;
}

static uint32_t u8cp(const std::string& s, size_t i, int len) {
  const unsigned char c = (unsigned char)s[i];
  uint32_t cp = len == 1 ? c : len == 2 ? (c & 0x1F) : len == 3 ? (c & 0x0F) : (c & 0x07);
  for (int k = 1; k < len && i + k < s.size(); ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
  return cp;
}

std::string normalize_whitespace(const std::string& s) {
  std::string out;
  out.reserve(s.size());
  size_t i = 0;
  bool in_word = false, any = false;
  while (i < s.size()) {
    const int L = u8len(s, i);
    const uint32_t cp = u8cp(s, i, L);
    if (is_ws(cp)) {
      in_word = false;
    } else {
      if (!in_word && any) out.push_back(' ');
      out.append(s, i, L);
      in_word = any = true;
    }
    i += L;
  }
  return out;
}

static std::string rust_trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e) {
    const int L = u8len(s, b);
    if (!is_ws(u8cp(s, b, L))) break;
    b += L;
  }
  while (e > b) {
    size_t st = e - 1;
    while (st > b && (((unsigned char)s[st]) >> 6) == 2) --st;
    if (!is_ws(u8cp(s, st, u8len(s, st)))) break;
    e = st;
  }
  return s.substr(b, e - b);
}

std::vector<std::string> split_sentences(const std::string& cleaned) {
  std::vector<std::string> out;
  size_t start = 0;
  size_t i = 0;
  while (i < cleaned.size()) {
    const int L = u8len(cleaned, i);
    const char c = cleaned[i];
    if (L == 1 && (c == '.' || c == '?' || c == '!')) {
      if (i >= start) {
        out.push_back(rust_trim(cleaned.substr(start, i + 1 - start)));
        start = i + 1;
      }
    }
    i += L;
  }
  if (start < cleaned.size()) {
    std::string rem = rust_trim(cleaned.substr(start));
    if (!rem.empty()) out.push_back(rem);
  }
  if (out.empty() && !cleaned.empty()) out.push_back(cleaned);
  return out;
}

std::vector<std::string> split_whitespace(const std::string& s) {
  std::vector<std::string> out;
  std::string cur;
  size_t i = 0;
  while (i < s.size()) {
    const int L = u8len(s, i);
    if (is_ws(u8cp(s, i, L))) {
      if (!cur.empty()) out.push_back(std::move(cur)), cur.clear();
    } else {
      cur.append(s, i, L);
    }
    i += L;
  }
  if (!cur.empty()) out.push_back(std::move(cur));
  return out;
}

// ------------------------------------------------------------------------ Markov chain
class MarkovModel {
 public:
  explicit MarkovModel(uint64_t seed = 0) : rng_(seed ? seed : std::random_device{}()) {}

  // Returns false (and trains nothing / only a starter) exactly where the reference warns.
  bool train(const std::string& text) {
    if (text.empty()) return false;
    auto words = split_whitespace(text);
    if (words.size() < 2) {
      if (!words.empty()) starters_.push_back(words[0]);
      return false;
    }
    starters_.push_back(words[0]);
    for (size_t i = 0; i + 1 < words.size(); ++i) {
      auto it = index_.find(words[i]);
      if (it == index_.end()) {
        it = index_.emplace(words[i], next_.size()).first;
        next_.emplace_back();
      }
      next_[it->second].push_back(words[i + 1]);
    }
    std::sort(starters_.begin(), starters_.end());
    starters_.erase(std::unique(starters_.begin(), starters_.end()), starters_.end());
    return true;
  }

  std::string generate(uint32_t max_length) {
    if (index_.empty() || starters_.empty()) return "Model not trained.";
    std::string cur = starters_[pick(starters_.size())];
    std::string out = cur;
    for (uint32_t step = 1; step < max_length; ++step) {
      auto it = index_.find(cur);
      if (it == index_.end()) break;
      const auto& nx = next_[it->second];
      if (nx.empty()) break;
      cur = nx[pick(nx.size())];
      out += " ";
      out += cur;
    }
    return out;
  }

  size_t num_states() const { return index_.size(); }
  std::vector<std::string> starters() const { return starters_; }
  std::vector<std::string> successors(const std::string& w) const {
    auto it = index_.find(w);
    return it == index_.end() ? std::vector<std::string>{} : next_[it->second];
  }

 private:
  size_t pick(size_t n) { return std::uniform_int_distribution<size_t>(0, n - 1)(rng_); }
  std::unordered_map<std::string, size_t> index_;
  std::vector<std::vector<std::string>> next_;
  std::vector<std::string> starters_;
  std::mt19937_64 rng_;
};

// ------------------------------------------------------------------------ BERT tokenizer
static bool is_control(uint32_t c) {
  if (c == '\t' || c == '\n' || c == '\r') return false;
  return c < 0x20 || (c >= 0x7F && c < 0xA0) || c == 0xAD || (c >= 0x200B && c <= 0x200F) ||
         (c >= 0x202A && c <= 0x202E) || (c >= 0x2060 && c <= 0x206F) || c == 0xFEFF;
}

static bool is_cjk(uint32_t c) {
  return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) ||
         (c >= 0x20000 && c <= 0x2A6DF) || (c >= 0x2A700 && c <= 0x2B73F) ||
         (c >= 0x2B740 && c <= 0x2B81F) || (c >= 0x2B820 && c <= 0x2CEAF) ||
         (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}

static bool is_punct(uint32_t c) {
  if ((c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) ||
      (c >= 123 && c <= 126))
    return true;
  // Unicode general category P* (common blocks)
  static const uint32_t ranges[][2] = {
      {0xA1, 0xA1}, {0xA7, 0xA7}, {0xAB, 0xAB}, {0xB6, 0xB7}, {0xBB, 0xBB}, {0xBF, 0xBF},
      {0x37E, 0x37E}, {0x387, 0x387}, {0x55A, 0x55F}, {0x589, 0x58A}, {0x5BE, 0x5BE},
      {0x5C0, 0x5C0}, {0x5C3, 0x5C3}, {0x5C6, 0x5C6}, {0x5F3, 0x5F4}, {0x609, 0x60A},
      {0x60C, 0x60D}, {0x61B, 0x61B}, {0x61E, 0x61F}, {0x66A, 0x66D}, {0x6D4, 0x6D4},
      {0x964, 0x965}, {0x970, 0x970}, {0xE4F, 0xE4F}, {0xE5A, 0xE5B}, {0x2010, 0x2027},
      {0x2030, 0x2043}, {0x2045, 0x2051}, {0x2053, 0x205E}, {0x207D, 0x207E}, {0x208D, 0x208E},
      {0x2308, 0x230B}, {0x2329, 0x232A}, {0x2768, 0x2775}, {0x27C5, 0x27C6}, {0x27E6, 0x27EF},
      {0x2983, 0x2998}, {0x29D8, 0x29DB}, {0x29FC, 0x29FD}, {0x2CF9, 0x2CFC}, {0x2CFE, 0x2CFF},
      {0x2E00, 0x2E2E}, {0x2E30, 0x2E4F}, {0x3001, 0x3003}, {0x3008, 0x3011}, {0x3014, 0x301F},
      {0x3030, 0x3030}, {0x303D, 0x303D}, {0x30A0, 0x30A0}, {0x30FB, 0x30FB}, {0xFE10, 0xFE19},
      {0xFE30, 0xFE52}, {0xFE54, 0xFE61}, {0xFE63, 0xFE63}, {0xFE68, 0xFE68}, {0xFE6A, 0xFE6B},
      {0xFF01, 0xFF03}, {0xFF05, 0xFF0A}, {0xFF0C, 0xFF0F}, {0xFF1A, 0xFF1B}, {0xFF1F, 0xFF20},
      {0xFF3B, 0xFF3D}, {0xFF3F, 0xFF3F}, {0xFF5B, 0xFF5B}, {0xFF5D, 0xFF5D}, {0xFF5F, 0xFF65}};
  for (auto& r : ranges)
    if (c >= r[0] && c <= r[1]) return true;
  return false;
}

// Combining marks (category Mn) dropped after NFD by strip_accents.
static bool is_mn(uint32_t c) {
  return (c >= 0x300 && c <= 0x36F) || (c >= 0x483 && c <= 0x489) || (c >= 0x591 && c <= 0x5BD) ||
         (c >= 0x610 && c <= 0x61A) || (c >= 0x64B && c <= 0x65F) || (c >= 0x1AB0 && c <= 0x1AFF) ||
         (c >= 0x1DC0 && c <= 0x1DFF) || (c >= 0x20D0 && c <= 0x20F0) || (c >= 0xFE20 && c <= 0xFE2F);
}

// Base letter of a precomposed char after NFD + Mn removal (Latin-1, Latin Ext-A, Cyrillic й/ё).
// Tables generated from unicodedata (NFD, drop category Mn); '.' = unchanged.
static uint32_t strip_accent(uint32_t c) {
  static const char* latin1 =  // U+00C0..U+00FF ('.' = no decomposition)
      "AAAAAA.CEEEEIIII.NOOOOO..UUUUY..aaaaaa.ceeeeiiii.nooooo..uuuuy.y";
  if (c >= 0xC0 && c <= 0xFF) {
    const char b = latin1[c - 0xC0];
    return b == '.' ? c : (uint32_t)b;
  }
  static const char* extA =  // U+0100..U+017F
      "AaAaAaCcCcCcCcDd..EeEeEeEeEeGgGgGgGgHh..IiIiIiIiI...JjKk.LlLlLl....NnNnNn...OoOoOo..RrRrRrSsSsSsSsTtTt..UuUuUuUuUuUuWwYyYZzZzZz.";
  if (c >= 0x100 && c <= 0x17F) {
    const char b = extA[c - 0x100];
    return b == '.' ? c : (uint32_t)b;
  }
  switch (c) {
    case 0x419: return 0x418;  // Й -> И
    case 0x439: return 0x438;  // й -> и
    case 0x401: return 0x415;  // Ё -> Е
    case 0x451: return 0x435;  // ё -> е
    case 0x407: return 0x406;  // Ї -> І
    case 0x457: return 0x456;  // ї -> і
  }
  return c;
}

static uint32_t to_lower(uint32_t c) {
  if (c >= 'A' && c <= 'Z') return c + 32;
  if (c < 0x80) return c;
  if ((c >= 0xC0 && c <= 0xDE) && c != 0xD7) return c + 32;
  if (c >= 0x100 && c <= 0x137 && !(c & 1)) return c + 1;
  if (c >= 0x139 && c <= 0x148 && (c & 1)) return c + 1;
  if (c >= 0x14A && c <= 0x177 && !(c & 1)) return c + 1;
  if (c == 0x178) return 0xFF;
  if (c >= 0x179 && c <= 0x17E && (c & 1)) return c + 1;
  if (c >= 0x391 && c <= 0x3A9 && c != 0x3A2) return c + 32;
  if (c >= 0x410 && c <= 0x42F) return c + 32;
  if (c >= 0x400 && c <= 0x40F) return c + 80;
  if (c >= 0x460 && c <= 0x4FF && !(c & 1) && !(c >= 0x482 && c <= 0x489)) return c + 1;
  if (c >= 0x531 && c <= 0x556) return c + 48;
  return c;
}

#ifndef SYMB_NO_PYTHON
// Pack per-sequence id lists into (ids int32[T], cu_seqlens int32[B+1]) numpy arrays.
static py::tuple pack_varlen(const std::vector<std::vector<int>>& all) {
  size_t T = 0;
  for (auto& v : all) T += v.size();
  py::array_t<int32_t> ids((py::ssize_t)T), cu((py::ssize_t)all.size() + 1);
  int32_t* pi = ids.mutable_data();
  int32_t* pc = cu.mutable_data();
  pc[0] = 0;
  size_t o = 0;
  for (size_t b = 0; b < all.size(); ++b) {
    std::copy(all[b].begin(), all[b].end(), pi + o);
    o += all[b].size();
    pc[b + 1] = (int32_t)o;
  }
  return py::make_tuple(ids, cu);
}
#endif

class WordPiece {
 public:
  WordPiece(std::vector<std::string> vocab, bool lowercase, std::string unk, std::string cls,
            std::string sep, int max_chars_per_word)
      : vocab_(std::move(vocab)), lower_(lowercase), max_chars_(max_chars_per_word) {
    for (size_t i = 0; i < vocab_.size(); ++i) ids_.emplace(vocab_[i], (int)i);
    unk_ = id_of(unk);
    cls_ = id_of(cls);
    sep_ = id_of(sep);
  }

  int id_of(const std::string& t) const {
    auto it = ids_.find(t);
    return it == ids_.end() ? -1 : it->second;
  }

  // BasicTokenizer: returns the pre-tokenized words
  std::vector<std::string> basic(const std::string& text) const {
    std::u32string u = utf8_decode(text);
    std::u32string norm;
    norm.reserve(u.size() + 8);
    for (uint32_t c : u) {
      if (c == 0 || c == 0xFFFD || is_control(c)) continue;
      if (is_ws(c)) { norm.push_back(' '); continue; }
      if (is_cjk(c)) { norm.push_back(' '); norm.push_back(c); norm.push_back(' '); continue; }
      if (lower_) {
        if (is_mn(c)) continue;
        c = to_lower(strip_accent(c));
      }
      norm.push_back(c);
    }
    std::vector<std::string> words;
    std::u32string cur;
    auto flush = [&]() {
      if (!cur.empty()) { words.push_back(utf8_encode(cur)); cur.clear(); }
    };
    for (uint32_t c : norm) {
      if (c == ' ') { flush(); continue; }
      if (is_punct(c)) { flush(); words.push_back(utf8_encode(std::u32string(1, c))); continue; }
      cur.push_back(c);
    }
    flush();
    return words;
  }

  void wordpiece(const std::string& word, std::vector<int>& out) const {
    std::u32string u = utf8_decode(word);
    if ((int)u.size() > max_chars_) { out.push_back(unk_); return; }
    // byte offsets of char boundaries
    std::vector<size_t> off(u.size() + 1, 0);
    {
      size_t b = 0;
      for (size_t i = 0; i < u.size(); ++i) {
        off[i] = b;
        b += u[i] < 0x80 ? 1 : u[i] < 0x800 ? 2 : u[i] < 0x10000 ? 3 : 4;
      }
      off[u.size()] = b;
    }
    std::vector<int> pieces;
    size_t start = 0;
    while (start < u.size()) {
      size_t end = u.size();
      int found = -1;
      while (start < end) {
        std::string sub = word.substr(off[start], off[end] - off[start]);
        if (start > 0) sub = "##" + sub;
        auto it = ids_.find(sub);
        if (it != ids_.end()) { found = it->second; break; }
        --end;
      }
      if (found < 0) { out.push_back(unk_); return; }
      pieces.push_back(found);
      start = end;
    }
    out.insert(out.end(), pieces.begin(), pieces.end());
  }

  std::vector<int> encode(const std::string& text, int max_len, bool add_special) const {
    std::vector<int> ids;
    if (add_special) ids.push_back(cls_);
    for (const auto& w : basic(text)) wordpiece(w, ids);
    if (add_special) {
      if (max_len > 0 && (int)ids.size() + 1 > max_len) ids.resize(std::max(1, max_len - 1));
      ids.push_back(sep_);
    } else if (max_len > 0 && (int)ids.size() > max_len) {
      ids.resize(max_len);
    }
    return ids;
  }

  // Batch encode straight into a packed varlen layout: (ids int32[T], cu_seqlens int32[B+1]).
#ifndef SYMB_NO_PYTHON
  py::tuple encode_packed(const std::vector<std::string>& texts, int max_len) const {
    std::vector<std::vector<int>> all;
    all.reserve(texts.size());
    {
      py::gil_scoped_release nogil;
      for (const auto& t : texts) all.push_back(encode(t, max_len, true));
    }
    return pack_varlen(all);
  }
#endif

  std::vector<std::string> tokenize(const std::string& text) const {
    std::vector<int> ids;
    for (const auto& w : basic(text)) wordpiece(w, ids);
    std::vector<std::string> out;
    for (int i : ids) out.push_back(vocab_[i]);
    return out;
  }

  size_t size() const { return vocab_.size(); }
  int unk_id() const { return unk_; }
  int cls_id() const { return cls_; }
  int sep_id() const { return sep_; }

 private:
  std::vector<std::string> vocab_;
  std::unordered_map<std::string, int> ids_;
  bool lower_;
  int max_chars_;
  int unk_ = -1, cls_ = -1, sep_ = -1;
};

// SentencePiece-Unigram segmentation (XLM-R family: paraphrase-multilingual-mpnet-base-v2, the
// reference's model, preprocessing_service/src/main.rs:305; its tokenizer.json is fetched from
// the Hub in embedding_generator.rs:25-58).  Input is NFKC-normalised by the caller.  Pipeline, as
// HF tokenizers runs it: strip trailing whitespace, collapse runs of >= 2 spaces, Metaspace
// (' ' -> U+2581, prepend one to the
// text, split before every U+2581), then per piece a Viterbi over the lattice of vocabulary pieces
// maximising the summed log-probabilities.  A character no single-character piece covers becomes
// an <unk> node scored min_score - 10; consecutive <unk>s are fused into one.
class Unigram {
 public:
  Unigram(const std::vector<std::string>& pieces, const std::vector<double>& scores, int unk_id,
          int bos_id, int eos_id)
      : pieces_(pieces), scores_(scores), unk_(unk_id), bos_(bos_id), eos_(eos_id) {
    if (pieces.size() != scores.size()) throw std::invalid_argument("pieces/scores length mismatch");
    double mn = 0.0;
    for (size_t i = 0; i < pieces.size(); ++i) {
      ids_.emplace(pieces[i], (int)i);
      mn = std::min(mn, scores[i]);
      max_chars_ = std::max(max_chars_, (int)utf8_decode(pieces[i]).size());
    }
    unk_score_ = mn - 10.0;
  }

  // Pre-tokeniser of a tokenizer.json: ``builtin_norm`` false = the text arrives normalised by
  // the file's own normalizer pipeline (text/tokenizer.py), so no Strip / space collapsing here;
  // Metaspace with its replacement char, prepend scheme (0 never, 1 always, 2 first = always for
  // a single section) and split flag.
  void set_pretokenizer(bool builtin_norm, const std::string& replacement, int prepend, bool split) {
    const std::u32string r = utf8_decode(replacement);
    if (r.size() != 1) throw std::invalid_argument("Metaspace replacement must be one character");
    builtin_norm_ = builtin_norm;
    meta_ = r[0];
    prepend_ = prepend;
    split_ = split;
  }

  // Metaspace pre-tokenisation of already-normalised text.
  std::vector<std::u32string> pretokenize(const std::string& text) const {
    std::u32string u = utf8_decode(text), m;
    if (builtin_norm_)
      while (!u.empty() && is_ws(u.back())) u.pop_back();  // Strip(right)
    m.reserve(u.size() + 1);
    for (size_t i = 0; i < u.size(); ++i) {
      if (builtin_norm_ && u[i] == U' ' && i + 1 < u.size() && u[i + 1] == U' ')
        continue;  // " {2,}" -> " "
      m.push_back(u[i] == U' ' ? meta_ : u[i]);
    }
    std::vector<std::u32string> words;
    if (m.empty()) return words;
    if (prepend_ != 0 && m[0] != meta_) m.insert(m.begin(), meta_);
    if (!split_) {
      words.push_back(m);
      return words;
    }
    size_t st = 0;
    for (size_t i = 1; i <= m.size(); ++i) {
      if (i == m.size() || m[i] == meta_) {
        words.emplace_back(m.substr(st, i - st));
        st = i;
      }
    }
    return words;
  }

  void segment(const std::u32string& w, std::vector<int>& out) const {
    const int n = (int)w.size();
    std::vector<size_t> boff(n + 1, 0);  // utf-8 byte offset of each char boundary
    std::string u8;
    for (int i = 0; i < n; ++i) {
      boff[i] = u8.size();
      utf8_put(u8, w[i]);
    }
    boff[n] = u8.size();
    std::vector<double> best(n + 1, -std::numeric_limits<double>::infinity());
    std::vector<int> prev(n + 1, -1), pid(n + 1, -1);
    best[0] = 0.0;
    std::string key;
    for (int i = 0; i < n; ++i) {
      if (best[i] == -std::numeric_limits<double>::infinity()) continue;
      bool single = false;
      const int lmax = std::min(max_chars_, n - i);
      for (int l = 1; l <= lmax; ++l) {
        key.assign(u8, boff[i], boff[i + l] - boff[i]);
        auto it = ids_.find(key);
        if (it == ids_.end()) continue;
        if (l == 1) single = true;
        const double c = best[i] + scores_[it->second];
        if (c > best[i + l]) {
          best[i + l] = c;
          prev[i + l] = i;
          pid[i + l] = it->second;
        }
      }
      if (!single) {
        const double c = best[i] + unk_score_;
        if (c > best[i + 1]) {
          best[i + 1] = c;
          prev[i + 1] = i;
          pid[i + 1] = unk_;
        }
      }
    }
    std::vector<int> rev;
    for (int p = n; p > 0; p = prev[p]) rev.push_back(pid[p]);
    bool prev_unk = false;  // fuse runs of <unk> within this piece (HF fuse_unk)
    for (auto it = rev.rbegin(); it != rev.rend(); ++it) {
      const bool u = *it == unk_;
      if (!(u && prev_unk)) out.push_back(*it);
      prev_unk = u;
    }
  }

  std::vector<int> encode(const std::string& text, int max_len, bool add_special) const {
    std::vector<int> ids;
    if (add_special) ids.push_back(bos_);
    for (const auto& w : pretokenize(text)) segment(w, ids);
    if (add_special) {
      if (max_len > 0 && (int)ids.size() + 1 > max_len) ids.resize(std::max(1, max_len - 1));
      ids.push_back(eos_);
    } else if (max_len > 0 && (int)ids.size() > max_len) {
      ids.resize(max_len);
    }
    return ids;
  }

#ifndef SYMB_NO_PYTHON
  py::tuple encode_packed(const std::vector<std::string>& texts, int max_len) const {
    std::vector<std::vector<int>> all;
    all.reserve(texts.size());
    {
      py::gil_scoped_release nogil;
      for (const auto& t : texts) all.push_back(encode(t, max_len, true));
    }
    return pack_varlen(all);
  }
#endif

  std::vector<std::string> tokenize(const std::string& text) const {
    std::vector<int> ids = encode(text, 0, false);
    std::vector<std::string> out;
    for (int i : ids) out.push_back(pieces_[i]);
    return out;
  }

  int id_of(const std::string& t) const {
    auto it = ids_.find(t);
    return it == ids_.end() ? -1 : it->second;
  }
  size_t size() const { return pieces_.size(); }

 private:
  static constexpr char32_t kMeta = U'\u2581';
  std::vector<std::string> pieces_;
  std::vector<double> scores_;
  std::unordered_map<std::string, int> ids_;
  int unk_, bos_, eos_;
  int max_chars_ = 1;
  double unk_score_ = -10.0;
  bool builtin_norm_ = true;
  char32_t meta_ = kMeta;
  int prepend_ = 1;
  bool split_ = true;
};

#ifndef SYMB_NO_PYTHON
void register_text(py::module_& m) {
  m.def("normalize_whitespace", &normalize_whitespace);
  m.def("split_sentences", &split_sentences);
  m.def("split_whitespace", &split_whitespace);
  m.def("rust_trim", &rust_trim);
  py::class_<MarkovModel>(m, "MarkovModel")
      .def(py::init<uint64_t>(), py::arg("seed") = 0)
      .def("train", &MarkovModel::train)
      .def("generate", &MarkovModel::generate)
      .def("num_states", &MarkovModel::num_states)
      .def("starters", &MarkovModel::starters)
      .def("successors", &MarkovModel::successors);
  py::class_<Unigram>(m, "Unigram")
      .def(py::init<const std::vector<std::string>&, const std::vector<double>&, int, int, int>(),
           py::arg("pieces"), py::arg("scores"), py::arg("unk_id"), py::arg("bos_id"),
           py::arg("eos_id"))
      .def("set_pretokenizer", &Unigram::set_pretokenizer, py::arg("builtin_norm"),
           py::arg("replacement") = "\u2581", py::arg("prepend") = 1, py::arg("split") = true)
      .def("tokenize", &Unigram::tokenize)
      .def("encode", &Unigram::encode, py::arg("text"), py::arg("max_len") = 0,
           py::arg("add_special") = true)
      .def("encode_packed", &Unigram::encode_packed)
      .def("id_of", &Unigram::id_of)
      .def("__len__", &Unigram::size);
  py::class_<WordPiece>(m, "WordPiece")
      .def(py::init<std::vector<std::string>, bool, std::string, std::string, std::string, int>(),
           py::arg("vocab"), py::arg("lowercase") = true, py::arg("unk") = "[UNK]",
           py::arg("cls") = "[CLS]", py::arg("sep") = "[SEP]", py::arg("max_chars_per_word") = 100)
      .def("basic", &WordPiece::basic)
      .def("tokenize", &WordPiece::tokenize)
      .def("encode", &WordPiece::encode, py::arg("text"), py::arg("max_len") = 0,
           py::arg("add_special") = true)
      .def("encode_packed", &WordPiece::encode_packed)
      .def("id_of", &WordPiece::id_of)
      .def("__len__", &WordPiece::size)
      .def_property_readonly("unk_id", &WordPiece::unk_id)
      .def_property_readonly("cls_id", &WordPiece::cls_id)
      .def_property_readonly("sep_id", &WordPiece::sep_id);
}

#endif

}  // namespace symbn
