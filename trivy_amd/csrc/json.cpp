#include "json.h"

#include <cstdio>
#include <cstdlib>

#include "goregexp.h"

namespace tsg {
namespace {

struct P {
  const std::string& s;
  size_t i = 0;
  std::string err;
  explicit P(const std::string& t) : s(t) {}

  void ws() { while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i; }
  bool fail(const char* m) { if (err.empty()) err = std::string(m) + " at offset " + std::to_string(i); return false; }

  bool hex4(uint32_t* v) {
    if (i + 4 > s.size()) return fail("bad \\u escape");
    *v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
      if (d < 0) return fail("bad \\u escape");
      *v = *v * 16 + d;
    }
    return true;
  }

  bool str(std::string* out) {
    if (s[i] != '"') return fail("expected string");
    ++i;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c != '\\') { out->push_back(c); continue; }
      if (i >= s.size()) return fail("bad escape");
      char e = s[i++];
      switch (e) {
        case '"': out->push_back('"'); break;
        case '\\': out->push_back('\\'); break;
        case '/': out->push_back('/'); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          uint32_t v;
          if (!hex4(&v)) return false;
          if (v >= 0xD800 && v <= 0xDBFF && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
            size_t save = i;
            i += 2;
            uint32_t lo;
            if (!hex4(&lo)) return false;
            if (lo >= 0xDC00 && lo <= 0xDFFF) {
              re::append_utf8(out, 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00));
              break;
            }
            i = save;
          }
          if (v >= 0xDC80 && v <= 0xDCFF) { out->push_back(static_cast<char>(v - 0xDC00)); break; }
          re::append_utf8(out, v);
          break;
        }
        default: return fail("bad escape");
      }
    }
    if (i >= s.size()) return fail("unterminated string");
    ++i;
    return true;
  }

  bool value(JValue* v) {
    ws();
    if (i >= s.size()) return fail("unexpected end");
    char c = s[i];
    if (c == '{') {
      v->kind = JValue::Obj;
      ++i; ws();
      if (i < s.size() && s[i] == '}') { ++i; return true; }
      for (;;) {
        ws();
        std::string k;
        if (!str(&k)) return false;
        ws();
        if (i >= s.size() || s[i] != ':') return fail("expected :");
        ++i;
        JValue x;
        if (!value(&x)) return false;
        v->obj.emplace_back(std::move(k), std::move(x));
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == '}') { ++i; return true; }
        return fail("expected , or }");
      }
    }
    if (c == '[') {
      v->kind = JValue::Arr;
      ++i; ws();
      if (i < s.size() && s[i] == ']') { ++i; return true; }
      for (;;) {
        JValue x;
        if (!value(&x)) return false;
        v->arr.push_back(std::move(x));
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == ']') { ++i; return true; }
        return fail("expected , or ]");
      }
    }
    if (c == '"') { v->kind = JValue::Str; return str(&v->str); }
    if (s.compare(i, 4, "true") == 0) { v->kind = JValue::Bool; v->b = true; i += 4; return true; }
    if (s.compare(i, 5, "false") == 0) { v->kind = JValue::Bool; v->b = false; i += 5; return true; }
    if (s.compare(i, 4, "null") == 0) { v->kind = JValue::Null; i += 4; return true; }
    char* end = nullptr;
    double d = strtod(s.c_str() + i, &end);
    if (end == s.c_str() + i) return fail("bad value");
    v->kind = JValue::Num;
    v->num = d;
    i = end - s.c_str();
    return true;
  }
};

}  // namespace

bool json_parse(const std::string& text, JValue* out, std::string* err) {
  P p(text);
  if (!p.value(out)) { *err = p.err; return false; }
  p.ws();
  if (p.i != text.size()) { *err = "trailing data"; return false; }
  return true;
}

}  // namespace tsg
