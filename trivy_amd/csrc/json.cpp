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

void go_json_string(std::string* out, const char* src, size_t n, bool escape_html) {
  static const char hex[] = "0123456789abcdef";
  const uint8_t* p = reinterpret_cast<const uint8_t*>(src);
  out->push_back('"');
  size_t start = 0, i = 0;
  while (i < n) {
    const uint8_t b = p[i];
    if (b < 0x80) {
      const bool html = b == '<' || b == '>' || b == '&';
      if (b >= 0x20 && b != '"' && b != '\\' && !(escape_html && html)) { ++i; continue; }
      out->append(src + start, i - start);
      switch (b) {
        case '\\': case '"': out->push_back('\\'); out->push_back(static_cast<char>(b)); break;
        case '\b': *out += "\\b"; break;
        case '\f': *out += "\\f"; break;
        case '\n': *out += "\\n"; break;
        case '\r': *out += "\\r"; break;
        case '\t': *out += "\\t"; break;
        default:
          *out += "\\u00";
          out->push_back(hex[b >> 4]);
          out->push_back(hex[b & 0xF]);
      }
      start = ++i;
      continue;
    }
    // utf8.DecodeRune
    uint32_t r = 0xFFFD;
    size_t w = 1;
    auto cont = [&](size_t k) { return i + k < n && (p[i + k] & 0xC0) == 0x80; };
    if (b >= 0xC2 && b <= 0xDF && cont(1)) {
      r = ((b & 0x1Fu) << 6) | (p[i + 1] & 0x3Fu); w = 2;
    } else if (b >= 0xE0 && b <= 0xEF && i + 2 < n) {
      const uint8_t lo = b == 0xE0 ? 0xA0 : 0x80, hi = b == 0xED ? 0x9F : 0xBF;
      if (p[i + 1] >= lo && p[i + 1] <= hi && cont(2)) {
        r = ((b & 0x0Fu) << 12) | ((p[i + 1] & 0x3Fu) << 6) | (p[i + 2] & 0x3Fu); w = 3;
      }
    } else if (b >= 0xF0 && b <= 0xF4 && i + 3 < n) {
      const uint8_t lo = b == 0xF0 ? 0x90 : 0x80, hi = b == 0xF4 ? 0x8F : 0xBF;
      if (p[i + 1] >= lo && p[i + 1] <= hi && cont(2) && cont(3)) {
        r = ((b & 0x07u) << 18) | ((p[i + 1] & 0x3Fu) << 12) | ((p[i + 2] & 0x3Fu) << 6) | (p[i + 3] & 0x3Fu); w = 4;
      }
    }
    if (r == 0xFFFD && w == 1) {
      out->append(src + start, i - start);
      *out += "\\ufffd";
      start = ++i;
      continue;
    }
    if (r == 0x2028 || r == 0x2029) {
      out->append(src + start, i - start);
      *out += "\\u202";
      out->push_back(hex[r & 0xF]);
      i += w;
      start = i;
      continue;
    }
    i += w;
  }
  out->append(src + start, n - start);
  out->push_back('"');
}

}  // namespace tsg
