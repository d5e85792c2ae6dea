#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace symbn {

void append_f32(std::string& out, float f);
void append_f32_array(std::string& out, const float* v, size_t n);
void append_json_string(std::string& out, const char* s, size_t n);

struct JsonError : std::runtime_error {
  JsonError(const std::string& m, size_t line, size_t col);
  std::string msg;
  size_t line, column;
};

struct Number {
  bool is_float = false;
  std::string text;
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
