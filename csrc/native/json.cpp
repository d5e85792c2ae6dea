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

#include <cstdlib>

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

static inline bool is_dig(char c) { return (unsigned)(c - '0') < 10u; }

NumSpan Parser::number_span() {
  const size_t st = i_;
  bool is_float = false;
  if (p_[i_] == '-') ++i_;
  if (i_ >= n_) fail("EOF while parsing a value");
  if (p_[i_] == '0') {
    ++i_;
  } else if (p_[i_] >= '1' && p_[i_] <= '9') {
    while (i_ < n_ && is_dig(p_[i_])) ++i_;
  } else {
    fail("invalid number");
  }
  if (i_ < n_ && p_[i_] == '.') {
    is_float = true;
    ++i_;
    if (i_ >= n_ || !is_dig(p_[i_])) fail("invalid number");
    while (i_ < n_ && is_dig(p_[i_])) ++i_;
  }
  if (i_ < n_ && (p_[i_] == 'e' || p_[i_] == 'E')) {
    is_float = true;
    ++i_;
    if (i_ < n_ && (p_[i_] == '+' || p_[i_] == '-')) ++i_;
    if (i_ >= n_ || !is_dig(p_[i_])) fail("invalid number");
    while (i_ < n_ && is_dig(p_[i_])) ++i_;
  }
  return NumSpan{st, i_ - st, is_float};
}

static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

double Parser::number_f64() {
  // one pass: JSON number grammar (number_span's checks) + the decimal mantissa/exponent for
  // parse_f64's fast path; strtod on the token when the fast path does not apply
  const size_t st = i_;
  const bool neg = p_[i_] == '-';
  if (neg) ++i_;
  if (i_ >= n_) fail("EOF while parsing a value");
  // m accumulates every digit (leading zeros add nothing); the digit count from the first
  // non-zero one decides the fast path (<= 15 significant digits: m < 2^53, exact)
  const char* p = p_;
  size_t i = i_;
  const size_t n = n_;
  uint64_t m = 0;
  int e10 = 0;
  size_t first_sig = SIZE_MAX, frac_digits = 0, int_end;
  if (p[i] == '0') {
    ++i;
  } else if (p[i] >= '1' && p[i] <= '9') {
    first_sig = i;
    while (i < n && is_dig(p[i])) m = m * 10 + (uint64_t)(p[i++] - '0');
  } else {
    i_ = i;
    fail("invalid number");
  }
  int_end = i;
  size_t sig_digits = first_sig == SIZE_MAX ? 0 : int_end - first_sig;
  if (i < n && p[i] == '.') {
    ++i;
    if (i >= n || !is_dig(p[i])) {
      i_ = i;
      fail("invalid number");
    }
    const size_t fs = i;
    while (i < n && is_dig(p[i])) {
      if (first_sig == SIZE_MAX && p[i] != '0') first_sig = i;
      m = m * 10 + (uint64_t)(p[i++] - '0');
    }
    frac_digits = i - fs;
    if (first_sig != SIZE_MAX) sig_digits = first_sig < fs ? (int_end - first_sig) + frac_digits
                                                          : i - first_sig;
  }
  e10 = -(int)frac_digits;
  bool fast = sig_digits <= 15;
  i_ = i;
  if (i_ < n_ && (p_[i_] == 'e' || p_[i_] == 'E')) {
    ++i_;
    bool eneg = false;
    if (i_ < n_ && (p_[i_] == '+' || p_[i_] == '-')) eneg = p_[i_++] == '-';
    if (i_ >= n_ || !is_dig(p_[i_])) fail("invalid number");
    int x = 0, nd = 0;
    while (i_ < n_ && is_dig(p_[i_])) {
      if (++nd > 4) fast = false;
      x = x * 10 + (p_[i_++] - '0');
    }
    e10 += eneg ? -x : x;
  }
  if (fast && m == 0) return neg ? -0.0 : 0.0;
  if (fast && e10 >= -22 && e10 <= 22) {
    const double d = e10 >= 0 ? (double)m * kPow10[e10] : (double)m / kPow10[-e10];
    return neg ? -d : d;
  }
  return std::strtod(std::string(p_ + st, i_ - st).c_str(), nullptr);
}

Number Parser::number() {
  const NumSpan sp = number_span();
  Number num;
  num.is_float = sp.is_float;
  num.text.assign(p_ + sp.start, sp.len);
  return num;
}

void Parser::expect_lit(const char* lit) {
  const size_t L = strlen(lit);
  if (i_ + L > n_ || memcmp(p_ + i_, lit, L) != 0) fail("expected value");
  i_ += L;
}


static bool f64_fast(const char* s, size_t n, double& out) {
  static const double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                  1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                  1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  size_t i = 0;
  const bool neg = i < n && s[i] == '-';
  if (neg) ++i;
  uint64_t m = 0;
  int sig = 0, e10 = 0;
  bool any = false;
  for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i, any = true) {
    if ((sig || s[i] != '0') && ++sig > 15) return false;
    m = m * 10 + (uint64_t)(s[i] - '0');
  }
  if (i < n && s[i] == '.') {
    for (++i; i < n && s[i] >= '0' && s[i] <= '9'; ++i, any = true) {
      if ((sig || s[i] != '0') && ++sig > 15) return false;
      m = m * 10 + (uint64_t)(s[i] - '0');
      --e10;
    }
  }
  if (!any) return false;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    bool eneg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) eneg = s[i++] == '-';
    int x = 0, nd = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i) {
      if (++nd > 4) return false;
      x = x * 10 + (s[i] - '0');
    }
    if (!nd) return false;
    e10 += eneg ? -x : x;
  }
  if (i != n) return false;
  if (m == 0) {
    out = neg ? -0.0 : 0.0;
    return true;
  }
  if (e10 < -22 || e10 > 22) return false;
  const double d = e10 >= 0 ? (double)m * kP10[e10] : (double)m / kP10[-e10];
  out = neg ? -d : d;
  return true;
}

double parse_f64(const char* s, size_t n) {
  double d;
  if (f64_fast(s, n, d)) return d;
  return std::strtod(std::string(s, n).c_str(), nullptr);
}
}  // namespace symbn
