// Sanitizer self-test of the host C++ cores (SURVEY.md §5 "race detection / sanitizers").
// Built WITHOUT Python (SYMB_NO_PYTHON) and with -fsanitize=address,undefined by
// tests/test_native_sanitize_cpu.py; exercises the text, tokenizer, Markov, HTML and JSON cores on
// fixed cases plus seeded random inputs (invalid UTF-8, truncated markup, hostile JSON), so any
// out-of-bounds access, use-after-free, leak or UB aborts the run.
#define SYMB_NO_PYTHON 1
#include "../text.cpp"
#include "../json.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

namespace symbn {
std::pair<std::string, std::string> extract_text_core(const std::string& html);
std::string decode_entities(const std::string& s);
}

using namespace symbn;

static int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

static std::string rand_bytes(std::mt19937_64& r, size_t n, bool ascii_heavy) {
  static const char* frags[] = {"<p>", "</p>", "<article>", "<div class=\"content\">", "&amp;",
                                "&#x41;", "&#", "<!--", "-->", "<script>", ". ", "? ", "! ",
                                "Привет", "\xF0\x9F\x98\x80", "\xC3", "\xFF", "  ", "\t", "\"",
                                "\\u00e9", "\\", "{", "}", "[", "]", ",", ":", "1e999", "-0.0"};
  std::string s;
  while (s.size() < n) {
    if (ascii_heavy && r() % 3 == 0) {
      s += frags[r() % (sizeof(frags) / sizeof(frags[0]))];
    } else {
      s.push_back((char)(r() % 256));
    }
  }
  return s;
}

int main() {
  // ---- sentence splitting / whitespace (fixed cases) ----
  CHECK(normalize_whitespace("  a \t b\n") == "a b");
  auto ss = split_sentences("One. Two? Three!");
  CHECK(ss.size() == 3 && ss[1] == "Two?");
  CHECK(split_whitespace(" x  y ").size() == 2);

  // ---- tokenizers ----
  std::vector<std::string> vocab = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "hello", "world", "##s", "h",
                                    "##e", "##l", "##o"};
  WordPiece wp(vocab, true, "[UNK]", "[CLS]", "[SEP]", 100);
  auto ids = wp.encode("Hello worlds!", 0, true);
  CHECK(ids.size() >= 4 && ids.front() == 2 && ids.back() == 3);
  std::vector<std::string> pieces = {"<s>", "<pad>", "</s>", "<unk>", "\xE2\x96\x81",
                                     "\xE2\x96\x81hello", "lo", "h", "e", "l", "o"};
  std::vector<double> scores = {0, 0, 0, 0, -2, -3, -4, -8, -8, -8, -8};
  Unigram ug(pieces, scores, 3, 0, 2);
  auto u = ug.encode("hello  xyz", 0, true);
  CHECK(u.size() >= 4 && u.front() == 0 && u.back() == 2);

  // ---- Markov ----
  MarkovModel mk(7);
  CHECK(mk.train("a b c a b d"));
  CHECK(!mk.generate(20).empty());

  // ---- HTML ----
  auto h = extract_text_core("<html><body><article><h1>T</h1><p>x &amp; y</p></article></body></html>");
  CHECK(h.second == "article" && h.first == "T\nx & y");

  // ---- JSON f32 formatting round-trip ----
  std::mt19937_64 r(12345);
  for (int i = 0; i < 20000; ++i) {
    uint32_t bits = (uint32_t)r();
    float f;
    std::memcpy(&f, &bits, 4);
    if (!std::isfinite(f)) continue;
    std::string out;
    append_f32(out, f);
    const float back = std::strtof(out.c_str(), nullptr);
    CHECK(back == f || (f == 0 && back == 0));
  }

  // ---- fuzz: every core on random / hostile input ----
  for (int it = 0; it < 3000; ++it) {
    const std::string s = rand_bytes(r, r() % 600, it % 2 == 0);
    (void)normalize_whitespace(s);
    (void)split_sentences(normalize_whitespace(s));
    (void)split_whitespace(s);
    (void)wp.encode(s, 64, true);
    (void)wp.tokenize(s);
    (void)ug.encode(s, 64, true);
    (void)extract_text_core(s);
    (void)decode_entities(s);
    MarkovModel m2(it);
    m2.train(s);
    (void)m2.generate(10);
    try {
      Parser p(s.data(), s.size());
      p.ws();
      if (!p.at_end() && p.peek() == '"') (void)p.string();
      else if (!p.at_end()) (void)p.number();
    } catch (const JsonError&) {
    }
    std::string js;
    append_json_string(js, s.data(), s.size());
  }
  if (g_fail) {
    std::fprintf(stderr, "selftest: %d failures\n", g_fail);
    return 1;
  }
  std::printf("selftest ok\n");
  return 0;
}
