// HTML text extraction for the perception service (replaces the scraper/html5ever usage of
// services/perception_service/src/main.rs:86-170).
//
// Behaviour reproduced:
//  1. container = first element (document order) matching, in priority order,
//       article | main | div[role='main'] | div.content | div.post-content | div.entry-content | body
//  2. inside the container, for each text selector in order h1 h2 h3 h4 h5 h6 p li span, every
//     matching element in document order contributes the concatenation of its descendant text
//     nodes, each trimmed and followed by one space, the whole trimmed (empty -> skipped);
//     nested matches contribute again (the reference's duplication quirk);
//  3. parts joined with "\n", then re-split into lines, each trimmed, empties dropped.
// Parsing: a tolerant tokenizer + open-element stack with the HTML auto-closing rules that
// matter for these selectors (p closed by block starts, li by li, void elements, raw-text
// script/style/textarea/title, comments, doctype, character references).
#ifndef SYMB_NO_PYTHON
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif

#include <algorithm>
#include <cctype>
#include <memory>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#ifndef SYMB_NO_PYTHON
namespace py = pybind11;
#endif

namespace symbn {

struct Node {
  bool is_text = false;
  std::string tag;   // lower-case element name
  std::string text;  // text node content (entities decoded)
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<Node*> kids;
  Node* parent = nullptr;
};

static void put_utf8(std::string& s, uint32_t cp) {
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

std::string decode_entities(const std::string& s) {
  static const std::unordered_map<std::string, uint32_t> named = {
      {"amp", '&'}, {"lt", '<'}, {"gt", '>'}, {"quot", '"'}, {"apos", '\''}, {"nbsp", 0xA0},
      {"copy", 0xA9}, {"reg", 0xAE}, {"trade", 0x2122}, {"hellip", 0x2026}, {"mdash", 0x2014},
      {"ndash", 0x2013}, {"laquo", 0xAB}, {"raquo", 0xBB}, {"lsquo", 0x2018}, {"rsquo", 0x2019},
      {"ldquo", 0x201C}, {"rdquo", 0x201D}, {"bull", 0x2022}, {"middot", 0xB7}, {"deg", 0xB0},
      {"euro", 0x20AC}, {"pound", 0xA3}, {"yen", 0xA5}, {"cent", 0xA2}, {"sect", 0xA7},
      {"para", 0xB6}, {"times", 0xD7}, {"divide", 0xF7}, {"shy", 0xAD}, {"thinsp", 0x2009},
      {"ensp", 0x2002}, {"emsp", 0x2003}, {"zwnj", 0x200C}, {"zwj", 0x200D}};
  std::string out;
  out.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    if (s[i] != '&') { out.push_back(s[i++]); continue; }
    size_t semi = s.find(';', i + 1);
    if (semi == std::string::npos || semi - i > 32) { out.push_back(s[i++]); continue; }
    std::string ent = s.substr(i + 1, semi - i - 1);
    uint32_t cp = 0;
    bool ok = false;
    if (!ent.empty() && ent[0] == '#') {
      try {
        if (ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X')) cp = std::stoul(ent.substr(2), nullptr, 16);
        else cp = std::stoul(ent.substr(1), nullptr, 10);
        ok = cp > 0 && cp < 0x110000 && !(cp >= 0xD800 && cp <= 0xDFFF);
      } catch (...) { ok = false; }
    } else {
      auto it = named.find(ent);
      if (it != named.end()) { cp = it->second; ok = true; }
    }
    if (ok) { put_utf8(out, cp); i = semi + 1; }
    else out.push_back(s[i++]);
  }
  return out;
}

class Document {
 public:
  explicit Document(const std::string& html) { parse(html); }
  Node* root() { return root_; }

  std::vector<Node*> select(Node* scope, const std::string& tag, const std::string& cls,
                            const std::string& attr, const std::string& val, bool include_scope) {
    std::vector<Node*> out;
    walk(scope, [&](Node* n) {
      if (n->is_text) return;
      if (!include_scope && n == scope) return;
      if (n->tag != tag) return;
      if (!cls.empty()) {
        bool has = false;
        for (auto& a : n->attrs)
          if (a.first == "class") {
            size_t i = 0;
            const std::string& v = a.second;
            while (i < v.size()) {
              while (i < v.size() && isspace((unsigned char)v[i])) ++i;
              size_t j = i;
              while (j < v.size() && !isspace((unsigned char)v[j])) ++j;
              if (v.compare(i, j - i, cls) == 0 && j - i == cls.size()) has = true;
              i = j;
            }
          }
        if (!has) return;
      }
      if (!attr.empty()) {
        bool has = false;
        for (auto& a : n->attrs)
          if (a.first == attr && a.second == val) has = true;
        if (!has) return;
      }
      out.push_back(n);
    });
    return out;
  }

  static void text_of(Node* n, std::vector<std::string>& out) {
    walk(n, [&](Node* c) {
      if (c->is_text) out.push_back(c->text);
    });
  }

 private:
  template <class F>
  static void walk(Node* n, F&& f) {
    f(n);
    for (Node* k : n->kids) walk(k, f);
  }

  Node* make(bool text) {
    pool_.emplace_back(new Node());
    pool_.back()->is_text = text;
    return pool_.back().get();
  }

  void add_text(const std::string& raw, bool decode) {
    if (raw.empty()) return;
    Node* t = make(true);
    t->text = decode ? decode_entities(raw) : raw;
    t->parent = cur_;
    cur_->kids.push_back(t);
  }

  bool in_stack(const std::string& tag) const {
    for (Node* n = cur_; n && n != root_; n = n->parent)
      if (n->tag == tag) return true;
    return false;
  }

  void close(const std::string& tag) {
    for (Node* n = cur_; n && n != root_; n = n->parent)
      if (n->tag == tag) { cur_ = n->parent; return; }
  }

  void open(const std::string& tag, std::vector<std::pair<std::string, std::string>> attrs,
            bool self_closing) {
    static const std::unordered_set<std::string> closes_p = {
        "address", "article", "aside", "blockquote", "details", "div", "dl", "fieldset",
        "figcaption", "figure", "footer", "form", "h1", "h2", "h3", "h4", "h5", "h6", "header",
        "hgroup", "hr", "main", "menu", "nav", "ol", "p", "pre", "section", "table", "ul", "li"};
    static const std::unordered_set<std::string> voids = {
        "area", "base", "br", "col", "embed", "hr", "img", "input", "link", "meta", "param",
        "source", "track", "wbr"};
    if (tag == "html" || tag == "head" || tag == "body") {
      // single html/head/body: keep attributes on the synthesized element
      if (tag == "body") {
        if (!body_) {
          body_ = make(false);
          body_->tag = "body";
          body_->attrs = std::move(attrs);
          body_->parent = root_;
          root_->kids.push_back(body_);
          cur_ = body_;
        }
      }
      return;
    }
    if (closes_p.count(tag) && in_stack("p")) close("p");
    if (tag == "li" && in_stack("li")) close("li");
    if ((tag == "dt" || tag == "dd") && (in_stack("dt") || in_stack("dd"))) {
      close("dt");
      close("dd");
    }
    Node* e = make(false);
    e->tag = tag;
    e->attrs = std::move(attrs);
    e->parent = cur_;
    cur_->kids.push_back(e);
    if (!self_closing && !voids.count(tag)) cur_ = e;
  }

  void parse(const std::string& h) {
    pool_.emplace_back(new Node());
    root_ = pool_.back().get();
    root_->tag = "#document";
    cur_ = root_;
    size_t i = 0;
    const size_t n = h.size();
    std::string text;
    auto flush = [&]() {
      add_text(text, true);
      text.clear();
    };
    while (i < n) {
      if (h[i] != '<') { text.push_back(h[i++]); continue; }
      if (h.compare(i, 4, "<!--") == 0) {
        flush();
        size_t e = h.find("-->", i + 4);
        i = e == std::string::npos ? n : e + 3;
        continue;
      }
      if (i + 1 < n && (h[i + 1] == '!' || h[i + 1] == '?')) {
        flush();
        size_t e = h.find('>', i);
        i = e == std::string::npos ? n : e + 1;
        continue;
      }
      const bool end_tag = i + 1 < n && h[i + 1] == '/';
      size_t j = i + (end_tag ? 2 : 1);
      if (j >= n || !isalpha((unsigned char)h[j])) { text.push_back(h[i++]); continue; }
      flush();
      size_t k = j;
      while (k < n && !isspace((unsigned char)h[k]) && h[k] != '>' && h[k] != '/') ++k;
      std::string tag = h.substr(j, k - j);
      std::transform(tag.begin(), tag.end(), tag.begin(), ::tolower);
      std::vector<std::pair<std::string, std::string>> attrs;
      bool self_closing = false;
      // attributes
      while (k < n && h[k] != '>') {
        while (k < n && (isspace((unsigned char)h[k]))) ++k;
        if (k < n && h[k] == '/') { self_closing = true; ++k; continue; }
        if (k >= n || h[k] == '>') break;
        size_t a = k;
        while (k < n && !isspace((unsigned char)h[k]) && h[k] != '=' && h[k] != '>' && h[k] != '/') ++k;
        std::string name = h.substr(a, k - a);
        std::transform(name.begin(), name.end(), name.begin(), ::tolower);
        while (k < n && isspace((unsigned char)h[k])) ++k;
        std::string val;
        if (k < n && h[k] == '=') {
          ++k;
          while (k < n && isspace((unsigned char)h[k])) ++k;
          if (k < n && (h[k] == '"' || h[k] == '\'')) {
            const char q = h[k++];
            size_t e = h.find(q, k);
            if (e == std::string::npos) e = n;
            val = h.substr(k, e - k);
            k = e < n ? e + 1 : n;
          } else {
            size_t a2 = k;
            while (k < n && !isspace((unsigned char)h[k]) && h[k] != '>') ++k;
            val = h.substr(a2, k - a2);
          }
        }
        if (!name.empty()) attrs.emplace_back(name, decode_entities(val));
      }
      i = k < n ? k + 1 : n;
      if (end_tag) {
        if (tag == "p" && !in_stack("p")) {  // stray </p> creates an empty paragraph
          open("p", {}, false);
          close("p");
        } else if (tag != "html" && tag != "body" && tag != "head") {
          close(tag);
        }
        continue;
      }
      if (!body_ && tag != "html" && tag != "head" && tag != "body" && !head_only(tag)) {
        open("body", {}, false);
      }
      open(tag, std::move(attrs), self_closing);
      if (tag == "script" || tag == "style" || tag == "textarea" || tag == "title" ||
          tag == "xmp" || tag == "noscript") {
        const std::string endt = "</" + tag;
        size_t e = i;
        for (;;) {
          e = h.find("</", e);
          if (e == std::string::npos) break;
          std::string cand = h.substr(e, endt.size());
          std::transform(cand.begin(), cand.end(), cand.begin(), ::tolower);
          if (cand == endt) break;
          e += 2;
        }
        if (e == std::string::npos) e = n;
        add_text(h.substr(i, e - i), tag == "textarea" || tag == "title");
        close(tag);
        size_t g = h.find('>', e);
        i = (e == n || g == std::string::npos) ? n : g + 1;
      }
    }
    if (!body_ && !text.empty()) open("body", {}, false);
    flush();
    if (!body_) open("body", {}, false);
  }

  static bool head_only(const std::string& t) {
    return t == "meta" || t == "link" || t == "title" || t == "style" || t == "base" ||
           t == "script" || t == "noscript";
  }

  std::vector<std::unique_ptr<Node>> pool_;
  Node* root_ = nullptr;
  Node* cur_ = nullptr;
  Node* body_ = nullptr;
};

static std::string trim_ws(const std::string& s) {
  // Rust str::trim over ASCII + common Unicode spaces (NBSP, ideographic)
  size_t b = 0, e = s.size();
  auto ws_at = [&](size_t i, size_t& len) -> bool {
    const unsigned char c = (unsigned char)s[i];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) { len = 1; return true; }
    if (c == 0xC2 && i + 1 < s.size() && ((unsigned char)s[i + 1] == 0xA0 || (unsigned char)s[i + 1] == 0x85)) { len = 2; return true; }
    if (c == 0xE3 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 && (unsigned char)s[i + 2] == 0x80) { len = 3; return true; }
    if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
        (((unsigned char)s[i + 2] >= 0x80 && (unsigned char)s[i + 2] <= 0x8A) ||
         (unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9 || (unsigned char)s[i + 2] == 0xAF)) { len = 3; return true; }
    return false;
  };
  size_t L;
  while (b < e && ws_at(b, L)) b += L;
  for (;;) {
    if (e <= b) break;
    size_t st = e - 1;
    while (st > b && (((unsigned char)s[st]) >> 6) == 2) --st;
    if (ws_at(st, L) && st + L == e) e = st;
    else break;
  }
  return s.substr(b, e - b);
}

// -> (text, container selector); pure C++ core (the sanitizer self-test links it directly)
std::pair<std::string, std::string> extract_text_core(const std::string& html) {
  Document doc(html);
  struct Sel { const char* tag; const char* cls; const char* attr; const char* val; const char* name; };
  static const Sel containers[] = {
      {"article", "", "", "", "article"}, {"main", "", "", "", "main"},
      {"div", "", "role", "main", "div[role='main']"}, {"div", "content", "", "", "div.content"},
      {"div", "post-content", "", "", "div.post-content"},
      {"div", "entry-content", "", "", "div.entry-content"}, {"body", "", "", "", "body"}};
  Node* scope = doc.root();
  std::string used = "";
  for (const auto& s : containers) {
    auto found = doc.select(doc.root(), s.tag, s.cls, s.attr, s.val, true);
    if (!found.empty()) {
      scope = found.front();
      used = s.name;
      break;
    }
  }
  static const char* text_sel[] = {"h1", "h2", "h3", "h4", "h5", "h6", "p", "li", "span"};
  std::vector<std::string> parts;
  for (const char* t : text_sel) {
    for (Node* e : doc.select(scope, t, "", "", "", false)) {
      std::vector<std::string> texts;
      Document::text_of(e, texts);
      std::string acc;
      for (auto& x : texts) {
        std::string tr = trim_ws(x);
        if (!tr.empty()) {
          acc += tr;
          acc.push_back(' ');
        }
      }
      std::string c = trim_ws(acc);
      if (!c.empty()) parts.push_back(c);
    }
  }
  std::string joined;
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i) joined.push_back('\n');
    joined += parts[i];
  }
  // .lines() (split on \n, strip a trailing \r), trim, drop empty, join "\n"
  std::string out;
  size_t pos = 0;
  while (pos <= joined.size()) {
    size_t e = joined.find('\n', pos);
    if (e == std::string::npos) e = joined.size();
    std::string line = joined.substr(pos, e - pos);
    if (!line.empty() && line.back() == '\r') line.pop_back();
    line = trim_ws(line);
    if (!line.empty()) {
      if (!out.empty()) out.push_back('\n');
      out += line;
    }
    if (e == joined.size()) break;
    pos = e + 1;
  }
  return {out, used};
}

#ifndef SYMB_NO_PYTHON
void register_html(py::module_& m) {
  m.def("html_extract_text", [](const std::string& html) {
    auto r = extract_text_core(html);
    return py::make_tuple(r.first, r.second);
  }, "Reference-compatible main-content text extraction -> (text, container selector)");
  m.def("html_decode_entities", &decode_entities);
}
#endif

}  // namespace symbn
