// Minimal JSON reader for rule configs crossing the C-ABI (the parsed
// trivy-secret.yaml schema, pkg/fanal/secret/scanner.go:29-43) and for the
// embedded builtin rule data.  Strings decode \uXXXX; a lone low surrogate
// U+DC80..U+DCFF denotes a raw byte 0x80..0xFF (Python 'surrogateescape'),
// so Go byte strings survive the round trip.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace tsg {

struct JValue {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<JValue> arr;
  std::vector<std::pair<std::string, JValue>> obj;

  const JValue* get(const std::string& k) const {
    for (const auto& kv : obj) if (kv.first == k) return &kv.second;
    return nullptr;
  }
  bool is_null() const { return kind == Null; }
  // Scalar as Go string (yaml.v3 decodes scalars into string fields).
  std::string as_string() const {
    if (kind == Str) return str;
    if (kind == Bool) return b ? "true" : "false";
    if (kind == Num) {
      char buf[64];
      if (num == static_cast<long long>(num)) snprintf(buf, sizeof buf, "%lld", static_cast<long long>(num));
      else snprintf(buf, sizeof buf, "%g", num);
      return buf;
    }
    return "";
  }
};

// Returns false and sets *err on malformed input.
bool json_parse(const std::string& text, JValue* out, std::string* err);

// Go encoding/json string encoding (go1.23 encoding/json/encode.go
// appendString): '"' and '\\' backslashed; \\b \\f \\n \\r \\t short escapes;
// other bytes < 0x20 as \\u00XX; with escape_html (json.Marshal's default)
// '<' '>' '&' as \\u003c \\u003e \\u0026; an invalid UTF-8 byte as \\ufffd;
// U+2028 / U+2029 as \\u2028 / \\u2029; everything else raw.
void go_json_string(std::string* out, const char* s, size_t n, bool escape_html = true);
inline void go_json_string(std::string* out, const std::string& s, bool escape_html = true) {
  go_json_string(out, s.data(), s.size(), escape_html);
}

}  // namespace tsg
