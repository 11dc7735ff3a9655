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

}  // namespace tsg
