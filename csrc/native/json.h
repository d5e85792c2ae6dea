#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace symbn {

void append_f32(std::string& out, float f);
void append_f32_array(std::string& out, const float* v, size_t n);
void append_json_string(std::string& out, const char* s, size_t n);

// Decimal text -> double, correctly rounded (strtod's result) -- Clinger's fast path for the
// numbers JSON embeddings consist of (<= 15 significant digits, |decimal exponent| <= 22: the
// mantissa and 10^e are exact doubles, so one IEEE multiply/divide rounds correctly), strtod
// otherwise.  f32 fields use (float)parse_f64(...): serde_json parses an f32 as f64 then casts,
// and so do we (bit-identical to the reference, double rounding included).
double parse_f64(const char* s, size_t n);

struct JsonError : std::runtime_error {
  JsonError(const std::string& m, size_t line, size_t col);
  std::string msg;
  size_t line, column;
};

struct Number {
  bool is_float = false;
  std::string text;
};

struct NumSpan {  // a validated number token, by position (no allocation)
  size_t start, len;
  bool is_float;
};

// Low-level tokenizer shared by the Python-object builder (json_py.cpp).
class Parser {
 public:
  Parser(const char* p, size_t n);
  void ws();
  char peek();
  bool at_end();
  std::string string();
  Number number();
  NumSpan number_span();
  double number_f64();  // number_span + parse_f64 in one pass
  const char* data() const { return p_; }
  void expect_lit(const char* lit);
  [[noreturn]] void fail(const std::string& m) const;
  void advance() { ++i_; }
  size_t pos() const { return i_; }

 private:
  uint32_t hex4();
  const char* p_;
  size_t n_;
  size_t i_ = 0;
};

}  // namespace symbn
