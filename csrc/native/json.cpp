// serde_json-compatible JSON codec for the wire contracts (libs/shared_models/src/lib.rs:3-110).
//
// Encoding matches `serde_json::to_vec` byte for byte:
//   * compact (no whitespace), keys in insertion order (= Rust struct field order),
//   * Option::None -> null, bool -> true/false, integers in decimal,
//   * floats are f32 (every float on the wire is f32: Vec<f32> embeddings, f32 scores) printed in
//     ryu's shortest round-trip "pretty" layout: 0.1 / 1.0 / 12.34 / 0.001234 / 1e-7 / 1.5e20,
//     non-finite -> null,
//   * strings: UTF-8 passes through; escapes \" \\ \n \r \t \b \f and \u00XX (lowercase hex)
//     for the other control characters.
// Decoding is a strict RFC 8259 parser (rejects trailing garbage, bad escapes, lone surrogates,
// invalid UTF-8) that returns Python objects; numeric arrays can be returned as float32 numpy
// buffers to keep 384-1024-float embeddings off the Python object path.
#include "json.h"

#include <charconv>
#include <cmath>
#include <cstring>
#include <stdexcept>

namespace symbn {

// ------------------------------------------------------------------ f32 shortest (ryu layout)
static int decimal_digits(uint32_t v) {
  int n = 1;
  while (v >= 10) {
    v /= 10;
    ++n;
  }
  return n;
}

void append_f32(std::string& out, float f) {
  if (!std::isfinite(f)) {
    out += "null";
    return;
  }
  if (f == 0.0f) {
    out += std::signbit(f) ? "-0.0" : "0.0";
    return;
  }
  // Shortest round-trip digits via to_chars(scientific): "d.ddddde[+-]XX"
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof(buf), f, std::chars_format::scientific);
  std::string s(buf, res.ptr);
  bool neg = false;
  size_t i = 0;
  if (s[0] == '-') {
    neg = true;
    i = 1;
  }
  size_t epos = s.find('e');
  std::string mant = s.substr(i, epos - i);
  int e10 = std::stoi(s.substr(epos + 1));
  std::string digits;
  for (char c : mant)
    if (c != '.') digits.push_back(c);
  // strip trailing zeros of the digit string (to_chars shortest has none, be safe)
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const int length = (int)digits.size();
  const int k = e10 - (length - 1);  // value = digits * 10^k
  const int kk = length + k;          // 10^(kk-1) <= v < 10^kk
  if (neg) out.push_back('-');
  if (0 <= k && kk <= 13) {
    out += digits;
    out.append(k, '0');
    out += ".0";
  } else if (0 < kk && kk <= 13) {
    out.append(digits, 0, kk);
    out.push_back('.');
    out.append(digits, kk, std::string::npos);
  } else if (-6 < kk && kk <= 0) {
    out += "0.";
    out.append(-kk, '0');
    out += digits;
  } else if (length == 1) {
    out += digits;
    out.push_back('e');
    out += std::to_string(kk - 1);
  } else {
    out.push_back(digits[0]);
    out.push_back('.');
    out.append(digits, 1, std::string::npos);
    out.push_back('e');
    out += std::to_string(kk - 1);
  }
}

void append_f32_array(std::string& out, const float* v, size_t n) {
  out.push_back('[');
  for (size_t i = 0; i < n; ++i) {
    if (i) out.push_back(',');
    append_f32(out, v[i]);
  }
  out.push_back(']');
}

void append_json_string(std::string& out, const char* s, size_t n) {
  static const char* hex = "0123456789abcdef";
  out.push_back('"');
  for (size_t i = 0; i < n; ++i) {
    const unsigned char c = (unsigned char)s[i];
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          out += "\\u00";
          out.push_back(hex[c >> 4]);
          out.push_back(hex[c & 15]);
        } else {
          out.push_back((char)c);
        }
    }
  }
  out.push_back('"');
}

// ------------------------------------------------------------------ parser
JsonError::JsonError(const std::string& m, size_t line, size_t col)
    : std::runtime_error(m + " at line " + std::to_string(line) + " column " + std::to_string(col)),
      msg(m), line(line), column(col) {}

Parser::Parser(const char* p, size_t n) : p_(p), n_(n) {}

void Parser::fail(const std::string& m) const {
  // serde_json reports the 1-based line and the column of the last consumed character
  size_t line = 1, col = 0;
  for (size_t i = 0; i < i_ && i < n_; ++i) {
    if (p_[i] == '\n') {
      ++line;
      col = 0;
    } else {
      ++col;
    }
  }
  throw JsonError(m, line, col);
}

void Parser::ws() {
  while (i_ < n_ && (p_[i_] == ' ' || p_[i_] == '\n' || p_[i_] == '\r' || p_[i_] == '\t')) ++i_;
}

char Parser::peek() {
  ws();
  if (i_ >= n_) fail("EOF while parsing a value");
  return p_[i_];
}

bool Parser::at_end() {
  ws();
  return i_ >= n_;
}

static void put_utf8(std::string& s, uint32_t cp) {
  if (cp < 0x80) {
    s.push_back((char)cp);
  } else if (cp < 0x800) {
    s.push_back((char)(0xC0 | (cp >> 6)));
    s.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    s.push_back((char)(0xE0 | (cp >> 12)));
    s.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    s.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    s.push_back((char)(0xF0 | (cp >> 18)));
    s.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    s.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    s.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

uint32_t Parser::hex4() {
  if (i_ + 4 > n_) {
    i_ = n_;
    fail("EOF while parsing a string");
  }
  uint32_t v = 0;
  for (int k = 0; k < 4; ++k) {
    const char c = p_[i_++];
    v <<= 4;
    if (c >= '0' && c <= '9') v |= c - '0';
    else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
    else fail("invalid escape");
  }
  return v;
}

std::string Parser::string() {
  if (p_[i_] != '"') fail("expected string");
  ++i_;
  std::string s;
  for (;;) {
    if (i_ >= n_) fail("EOF while parsing a string");
    const unsigned char c = (unsigned char)p_[i_];
    if (c == '"') {
      ++i_;
      return s;
    }
    if (c == '\\') {
      ++i_;
      if (i_ >= n_) fail("EOF while parsing a string");
      const char e = p_[i_++];
      switch (e) {
        case '"': s.push_back('"'); break;
        case '\\': s.push_back('\\'); break;
        case '/': s.push_back('/'); break;
        case 'b': s.push_back('\b'); break;
        case 'f': s.push_back('\f'); break;
        case 'n': s.push_back('\n'); break;
        case 'r': s.push_back('\r'); break;
        case 't': s.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (i_ + 2 > n_ || p_[i_] != '\\' || p_[i_ + 1] != 'u')
              fail("unexpected end of hex escape");
            i_ += 2;
            const uint32_t lo = hex4();
            if (lo < 0xDC00 || lo > 0xDFFF) fail("lone leading surrogate in hex escape");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            fail("lone leading surrogate in hex escape");
          }
          put_utf8(s, cp);
          break;
        }
        default: fail("invalid escape");
      }
      continue;
    }
    if (c < 0x20) fail("control character (\\u0000-\\u001F) found while parsing a string");
    // validate UTF-8 sequence
    int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (len == 0 || i_ + len > n_) fail("invalid unicode code point");
    for (int k = 1; k < len; ++k)
      if (((unsigned char)p_[i_ + k] >> 6) != 2) fail("invalid unicode code point");
    s.append(p_ + i_, len);
    i_ += len;
  }
}

Number Parser::number() {
  const size_t st = i_;
  bool is_float = false;
  if (p_[i_] == '-') ++i_;
  if (i_ >= n_) fail("EOF while parsing a value");
  if (p_[i_] == '0') {
    ++i_;
  } else if (p_[i_] >= '1' && p_[i_] <= '9') {
    while (i_ < n_ && isdigit((unsigned char)p_[i_])) ++i_;
  } else {
    fail("invalid number");
  }
  if (i_ < n_ && p_[i_] == '.') {
    is_float = true;
    ++i_;
    if (i_ >= n_ || !isdigit((unsigned char)p_[i_])) fail("invalid number");
    while (i_ < n_ && isdigit((unsigned char)p_[i_])) ++i_;
  }
  if (i_ < n_ && (p_[i_] == 'e' || p_[i_] == 'E')) {
    is_float = true;
    ++i_;
    if (i_ < n_ && (p_[i_] == '+' || p_[i_] == '-')) ++i_;
    if (i_ >= n_ || !isdigit((unsigned char)p_[i_])) fail("invalid number");
    while (i_ < n_ && isdigit((unsigned char)p_[i_])) ++i_;
  }
  Number num;
  num.is_float = is_float;
  num.text.assign(p_ + st, i_ - st);
  return num;
}

void Parser::expect_lit(const char* lit) {
  const size_t L = strlen(lit);
  if (i_ + L > n_ || memcmp(p_ + i_, lit, L) != 0) fail("expected value");
  i_ += L;
}

}  // namespace symbn
