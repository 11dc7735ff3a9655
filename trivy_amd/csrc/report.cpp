// Secret report assembly and Go JSON encoding (see report.h for the
// reference functions restated here).
#include "report.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>

#include "gosort.h"

namespace tsg {

namespace {

// ------------------------------------------------------------ JSON decoding
// Go's decoder matches an object key to a struct field by exact name, else
// case-insensitively (bytes.EqualFold: ASCII letters, plus U+212A -> k and
// U+017F -> s, the only non-ASCII runes that fold onto ASCII); a later key
// overwrites an earlier one.
std::string fold_key(const std::string& k) {
  std::string o;
  for (size_t i = 0; i < k.size(); ++i) {
    const unsigned char c = static_cast<unsigned char>(k[i]);
    if (c == 0xE2 && i + 2 < k.size() && static_cast<unsigned char>(k[i + 1]) == 0x84 &&
        static_cast<unsigned char>(k[i + 2]) == 0xAA) { o.push_back('k'); i += 2; continue; }
    if (c == 0xC5 && i + 1 < k.size() && static_cast<unsigned char>(k[i + 1]) == 0xBF) { o.push_back('s'); i += 1; continue; }
    o.push_back(static_cast<char>(c >= 'A' && c <= 'Z' ? c + 32 : c));
  }
  return o;
}

const JValue* field(const JValue* obj, const char* name) {
  if (!obj || obj->kind != JValue::Obj) return nullptr;
  const std::string want = fold_key(name);
  const JValue* v = nullptr;
  for (const auto& kv : obj->obj)
    if (kv.first == name || fold_key(kv.first) == want) v = &kv.second;
  return v;
}

struct Dec {
  std::string* err;
  bool fail(const std::string& m) { if (err->empty()) *err = m; return false; }
  // string field: absent / null -> "" (null is a no-op for a non-pointer field)
  bool str(const JValue* o, const char* k, std::string* out) {
    out->clear();
    const JValue* v = field(o, k);
    if (!v || v->is_null()) return true;
    if (v->kind != JValue::Str) return fail(std::string("json: cannot unmarshal into string field ") + k);
    *out = v->str;
    return true;
  }
  bool boolean(const JValue* o, const char* k, bool* out) {
    *out = false;
    const JValue* v = field(o, k);
    if (!v || v->is_null()) return true;
    if (v->kind != JValue::Bool) return fail(std::string("json: cannot unmarshal into bool field ") + k);
    *out = v->b;
    return true;
  }
  bool integer(const JValue* o, const char* k, long long* out) {
    *out = 0;
    const JValue* v = field(o, k);
    if (!v || v->is_null()) return true;
    if (v->kind != JValue::Num || v->num != static_cast<double>(static_cast<long long>(v->num)))
      return fail(std::string("json: cannot unmarshal into integer field ") + k);
    *out = static_cast<long long>(v->num);
    return true;
  }
  // []string: *present = false for absent / null (a nil slice)
  bool strings(const JValue* o, const char* k, std::vector<std::string>* out, bool* present) {
    out->clear();
    *present = false;
    const JValue* v = field(o, k);
    if (!v || v->is_null()) return true;
    if (v->kind != JValue::Arr) return fail(std::string("json: cannot unmarshal into []string field ") + k);
    *present = true;
    for (const auto& e : v->arr) {
      if (e.kind != JValue::Str) return fail(std::string("json: cannot unmarshal into []string field ") + k);
      out->push_back(e.str);
    }
    return true;
  }
  // map[string]X: sorted keys (encoding/json sorts map keys); values kept raw
  bool map(const JValue* o, const char* k, std::map<std::string, const JValue*>* out) {
    out->clear();
    const JValue* v = field(o, k);
    if (!v || v->is_null()) return true;
    if (v->kind != JValue::Obj) return fail(std::string("json: cannot unmarshal into map field ") + k);
    for (const auto& kv : v->obj) (*out)[kv.first] = &kv.second;
    return true;
  }
};

// ------------------------------------------------------------ JSON encoding
struct Enc {
  std::string o;
  bool first = true;
  void open(char c) { o.push_back(c); first = true; }
  void close(char c) { o.push_back(c); first = false; }
  void key(const char* k) {
    if (!first) o.push_back(',');
    first = false;
    go_json_string(&o, k, std::strlen(k));
    o.push_back(':');
  }
  void elem() { if (!first) o.push_back(','); first = false; }
  void str(const std::string& s) { go_json_string(&o, s); }
  void num(long long v) { o += std::to_string(v); }
  void boolean(bool b) { o += b ? "true" : "false"; }
  void null() { o += "null"; }
  void kv_str(const char* k, const std::string& v) { key(k); str(v); }
  void kv_str_omit(const char* k, const std::string& v) { if (!v.empty()) kv_str(k, v); }
  void kv_bool_omit(const char* k, bool v) { if (v) { key(k); boolean(true); } }
  void kv_num_omit(const char* k, long long v) { if (v) { key(k); num(v); } }
  void strings(const std::vector<std::string>& v) {
    open('[');
    for (const auto& s : v) { elem(); str(s); }
    close(']');
  }
  void kv_strings_omit(const char* k, const std::vector<std::string>& v) { if (!v.empty()) { key(k); strings(v); } }
};

// time.Time (pkg time, format.go / time.go MarshalJSON) ---------------------
bool digits(const std::string& s, size_t at, size_t n, int* out) {
  if (at + n > s.size()) return false;
  int v = 0;
  for (size_t i = 0; i < n; ++i) {
    const char c = s[at + i];
    if (c < '0' || c > '9') return false;
    v = v * 10 + (c - '0');
  }
  *out = v;
  return true;
}

int days_in(int year, int month) {
  static const int d[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (month == 2 && (year % 4 == 0 && (year % 100 != 0 || year % 400 == 0))) return 29;
  return d[month - 1];
}

bool encode_time_field(const JValue* v, Enc* e, Dec* d, const char* name) {
  std::string t = "0001-01-01T00:00:00Z";
  if (v && !v->is_null()) {
    if (v->kind != JValue::Str || !go_time_rfc3339(v->str, &t))
      return d->fail(std::string("parsing time field ") + name + ": not RFC 3339");
  }
  e->key(name);
  e->str(t);
  return true;
}

// v1.ConfigFile (go-containerregistry v0.20.3 pkg/v1/config.go) -----------
bool encode_health(const JValue* h, Enc* e, Dec* d) {
  std::vector<std::string> test;
  bool have = false;
  long long interval, timeout, start, retries;
  if (!d->strings(h, "Test", &test, &have) || !d->integer(h, "Interval", &interval) ||
      !d->integer(h, "Timeout", &timeout) || !d->integer(h, "StartPeriod", &start) || !d->integer(h, "Retries", &retries))
    return false;
  e->open('{');
  e->kv_strings_omit("Test", test);
  e->kv_num_omit("Interval", interval);
  e->kv_num_omit("Timeout", timeout);
  e->kv_num_omit("StartPeriod", start);
  e->kv_num_omit("Retries", retries);
  e->close('}');
  return true;
}

bool encode_set_map(const std::map<std::string, const JValue*>& m, Enc* e, Dec* d, const char* name) {
  if (m.empty()) return true;                       // omitempty
  e->key(name);
  e->open('{');
  for (const auto& kv : m) {
    if (!kv.second->is_null() && kv.second->kind != JValue::Obj)
      return d->fail(std::string("json: cannot unmarshal into struct{} in ") + name);
    e->key(kv.first.c_str());
    e->o += "{}";
  }
  e->close('}');
  return true;
}

bool encode_config(const JValue* c, Enc* e, Dec* d) {
  bool b;
  std::string s;
  std::vector<std::string> v;
  bool have;
  std::map<std::string, const JValue*> m;
  e->open('{');
  static const char* kBools1[] = {"AttachStderr", "AttachStdin", "AttachStdout"};
  for (const char* k : kBools1) { if (!d->boolean(c, k, &b)) return false; e->kv_bool_omit(k, b); }
  if (!d->strings(c, "Cmd", &v, &have)) return false;
  e->kv_strings_omit("Cmd", v);
  if (const JValue* h = field(c, "Healthcheck")) {
    if (!h->is_null()) {
      if (h->kind != JValue::Obj) return d->fail("json: cannot unmarshal into Healthcheck");
      e->key("Healthcheck");
      if (!encode_health(h, e, d)) return false;
    }
  }
  if (!d->str(c, "Domainname", &s)) return false;
  e->kv_str_omit("Domainname", s);
  if (!d->strings(c, "Entrypoint", &v, &have)) return false;
  e->kv_strings_omit("Entrypoint", v);
  if (!d->strings(c, "Env", &v, &have)) return false;
  e->kv_strings_omit("Env", v);
  static const char* kStr1[] = {"Hostname", "Image"};
  for (const char* k : kStr1) { if (!d->str(c, k, &s)) return false; e->kv_str_omit(k, s); }
  if (!d->map(c, "Labels", &m)) return false;
  if (!m.empty()) {
    e->key("Labels");
    e->open('{');
    for (const auto& kv : m) {
      if (!kv.second->is_null() && kv.second->kind != JValue::Str) return d->fail("json: cannot unmarshal into Labels");
      e->key(kv.first.c_str());
      e->str(kv.second->is_null() ? std::string() : kv.second->str);
    }
    e->close('}');
  }
  if (!d->strings(c, "OnBuild", &v, &have)) return false;
  e->kv_strings_omit("OnBuild", v);
  static const char* kBools2[] = {"OpenStdin", "StdinOnce", "Tty"};
  for (const char* k : kBools2) { if (!d->boolean(c, k, &b)) return false; e->kv_bool_omit(k, b); }
  if (!d->str(c, "User", &s)) return false;
  e->kv_str_omit("User", s);
  if (!d->map(c, "Volumes", &m) || !encode_set_map(m, e, d, "Volumes")) return false;
  if (!d->str(c, "WorkingDir", &s)) return false;
  e->kv_str_omit("WorkingDir", s);
  if (!d->map(c, "ExposedPorts", &m) || !encode_set_map(m, e, d, "ExposedPorts")) return false;
  static const char* kBools3[] = {"ArgsEscaped", "NetworkDisabled"};
  for (const char* k : kBools3) { if (!d->boolean(c, k, &b)) return false; e->kv_bool_omit(k, b); }
  static const char* kStr2[] = {"MacAddress", "StopSignal"};
  for (const char* k : kStr2) { if (!d->str(c, k, &s)) return false; e->kv_str_omit(k, s); }
  if (!d->strings(c, "Shell", &v, &have)) return false;
  e->kv_strings_omit("Shell", v);
  e->close('}');
  return true;
}

bool encode_config_file(const JValue* cf, Enc* e, Dec* d) {
  if (cf && !cf->is_null() && cf->kind != JValue::Obj) return d->fail("json: cannot unmarshal into v1.ConfigFile");
  std::string s;
  e->open('{');
  if (!d->str(cf, "architecture", &s)) return false;
  e->kv_str("architecture", s);
  static const char* kStr1[] = {"author", "container"};
  for (const char* k : kStr1) { if (!d->str(cf, k, &s)) return false; e->kv_str_omit(k, s); }
  if (!encode_time_field(field(cf, "created"), e, d, "created")) return false;
  if (!d->str(cf, "docker_version", &s)) return false;
  e->kv_str_omit("docker_version", s);
  if (const JValue* h = field(cf, "history")) {
    if (!h->is_null()) {
      if (h->kind != JValue::Arr) return d->fail("json: cannot unmarshal into history");
      if (!h->arr.empty()) {                          // omitempty
        e->key("history");
        e->open('[');
        for (const auto& it : h->arr) {
          if (!it.is_null() && it.kind != JValue::Obj) return d->fail("json: cannot unmarshal into v1.History");
          e->elem();
          e->open('{');
          bool el;
          if (!d->str(&it, "author", &s)) return false;
          e->kv_str_omit("author", s);
          if (!encode_time_field(field(&it, "created"), e, d, "created")) return false;
          static const char* kH[] = {"created_by", "comment"};
          for (const char* k : kH) { if (!d->str(&it, k, &s)) return false; e->kv_str_omit(k, s); }
          if (!d->boolean(&it, "empty_layer", &el)) return false;
          e->kv_bool_omit("empty_layer", el);
          e->close('}');
        }
        e->close(']');
      }
    }
  }
  if (!d->str(cf, "os", &s)) return false;
  e->kv_str("os", s);
  e->key("rootfs");
  const JValue* rf = field(cf, "rootfs");
  if (rf && !rf->is_null() && rf->kind != JValue::Obj) return d->fail("json: cannot unmarshal into v1.RootFS");
  e->open('{');
  if (!d->str(rf, "type", &s)) return false;
  e->kv_str("type", s);
  std::vector<std::string> ids;
  bool have = false;
  if (!d->strings(rf, "diff_ids", &ids, &have)) return false;
  for (const auto& h : ids)                          // v1.Hash: "algorithm:hex"
    if (h.find(':') == std::string::npos) return d->fail("cannot parse hash: \"" + h + "\"");
  e->key("diff_ids");
  if (have) e->strings(ids); else e->null();
  e->close('}');
  e->key("config");
  const JValue* cfg = field(cf, "config");
  if (cfg && !cfg->is_null() && cfg->kind != JValue::Obj) return d->fail("json: cannot unmarshal into v1.Config");
  if (!encode_config(cfg, e, d)) return false;
  if (!d->str(cf, "os.version", &s)) return false;
  e->kv_str_omit("os.version", s);
  if (!d->str(cf, "variant", &s)) return false;
  e->kv_str_omit("variant", s);
  std::vector<std::string> feats;
  if (!d->strings(cf, "os.features", &feats, &have)) return false;
  e->kv_strings_omit("os.features", feats);
  e->close('}');
  return true;
}

// types.Metadata (pkg/types/report.go:27-37) ------------------------------
bool encode_metadata(const JValue* md, Enc* e, Dec* d) {
  if (md && !md->is_null() && md->kind != JValue::Obj) return d->fail("json: cannot unmarshal into types.Metadata");
  long long size = 0;
  if (!d->integer(md, "Size", &size)) return false;
  e->open('{');
  e->kv_num_omit("Size", size);
  if (const JValue* os = field(md, "OS")) {
    if (!os->is_null()) {                             // *ftypes.OS (pkg/fanal/types/artifact.go:9-16)
      if (os->kind != JValue::Obj) return d->fail("json: cannot unmarshal into types.OS");
      std::string fam, name;
      bool eosl, ext;
      if (!d->str(os, "Family", &fam) || !d->str(os, "Name", &name) || !d->boolean(os, "EOSL", &eosl) ||
          !d->boolean(os, "extended", &ext))
        return false;
      e->key("OS");
      e->open('{');
      e->kv_str("Family", fam);
      e->kv_str("Name", name);
      e->kv_bool_omit("EOSL", eosl);
      e->kv_bool_omit("extended", ext);
      e->close('}');
    }
  }
  std::string s;
  std::vector<std::string> v;
  bool have;
  if (!d->str(md, "ImageID", &s)) return false;
  e->kv_str_omit("ImageID", s);
  static const char* kL[] = {"DiffIDs", "RepoTags", "RepoDigests"};
  for (const char* k : kL) { if (!d->strings(md, k, &v, &have)) return false; e->kv_strings_omit(k, v); }
  e->key("ImageConfig");
  if (!encode_config_file(field(md, "ImageConfig"), e, d)) return false;
  e->close('}');
  return true;
}

// ------------------------------------------------------------ secret merge
struct MFinding {
  const Secret* sec;
  const FindingRec* f;
  int layer;                          // index into refs, or -1 (image config: empty Layer)
};

struct MSecret {
  std::string path;
  std::vector<MFinding> findings;
};

void encode_finding(const MFinding& m, const std::vector<LayerRef>& refs, Enc* e) {
  const FindingRec& f = *m.f;
  const Secret& s = *m.sec;
  e->open('{');
  e->kv_str("RuleID", f.rule->id);
  e->kv_str("Category", f.rule->category);
  e->kv_str("Severity", Secret::severity(f));
  e->kv_str("Title", f.rule->title);
  e->key("StartLine"); e->num(f.start_line);
  e->key("EndLine"); e->num(f.end_line);
  e->key("Code");
  e->open('{');
  e->key("Lines");
  if (f.line_count == 0) {
    e->null();                        // types.Code{} of the binary rewrite (scanner.go:440-444)
  } else {
    e->open('[');
    for (uint32_t l = 0; l < f.line_count; ++l) {
      const LineRec& ln = s.lines()[f.line_begin + l];
      const std::string content(s.ptr(ln.content), ln.content.len);
      e->elem();
      e->open('{');
      e->key("Number"); e->num(ln.number);
      e->kv_str("Content", content);
      e->key("IsCause"); e->boolean(ln.is_cause);
      e->kv_str("Annotation", "");
      e->key("Truncated"); e->boolean(false);
      e->kv_str_omit("Highlighted", content);        // Highlighted == Content (scanner.go:538-545), omitempty
      e->key("FirstCause"); e->boolean(ln.first_cause);
      e->key("LastCause"); e->boolean(ln.last_cause);
      e->close('}');
    }
    e->close(']');
  }
  e->close('}');
  e->kv_str("Match", std::string(s.ptr(f.match), f.match.len));
  e->key("Layer");
  e->open('{');
  if (m.layer >= 0) {
    const LayerRef& r = refs[m.layer];
    e->kv_str_omit("Digest", r.digest);
    e->kv_str_omit("DiffID", r.diff_id);
    e->kv_str_omit("CreatedBy", r.created_by);
  }
  e->close('}');
  e->close('}');
}

}  // namespace

// ----------------------------------------------------------------- public
bool go_time_rfc3339(const std::string& in, std::string* out) {
  int Y, M, D, h, mi, sec;
  if (in.size() < 20 || !digits(in, 0, 4, &Y) || in[4] != '-' || !digits(in, 5, 2, &M) || in[7] != '-' ||
      !digits(in, 8, 2, &D) || in[10] != 'T' || !digits(in, 11, 2, &h) || in[13] != ':' || !digits(in, 14, 2, &mi) ||
      in[16] != ':' || !digits(in, 17, 2, &sec))
    return false;
  if (M < 1 || M > 12 || D < 1 || D > days_in(Y, M) || h > 23 || mi > 59 || sec > 59) return false;
  size_t i = 19;
  std::string frac;
  if (i < in.size() && in[i] == '.') {
    ++i;
    while (i < in.size() && in[i] >= '0' && in[i] <= '9') frac.push_back(in[i++]);
    if (frac.empty() || frac.size() > 9) return false;
  }
  int off = 0;
  if (i < in.size() && in[i] == 'Z') {
    ++i;
  } else if (i < in.size() && (in[i] == '+' || in[i] == '-')) {
    int oh, om;
    if (!digits(in, i + 1, 2, &oh) || i + 3 >= in.size() || in[i + 3] != ':' || !digits(in, i + 4, 2, &om) ||
        oh > 23 || om > 59)
      return false;
    off = (in[i] == '-' ? -1 : 1) * (oh * 60 + om);
    i += 6;
  } else {
    return false;
  }
  if (i != in.size()) return false;
  while (!frac.empty() && frac.back() == '0') frac.pop_back();
  char buf[64];
  snprintf(buf, sizeof buf, "%04d-%02d-%02dT%02d:%02d:%02d", Y, M, D, h, mi, sec);
  std::string t = buf;
  if (!frac.empty()) t += "." + frac;
  if (off == 0) {
    t += "Z";
  } else {
    const int a = off < 0 ? -off : off;
    snprintf(buf, sizeof buf, "%c%02d:%02d", off < 0 ? '-' : '+', a / 60, a % 60);
    t += buf;
  }
  *out = t;
  return true;
}

void go_indent(const std::string& src, const std::string& prefix, const std::string& indent, std::string* out) {
  bool need = false, in_str = false, esc = false;
  int depth = 0;
  auto newline = [&](int d) {
    out->push_back('\n');
    *out += prefix;
    for (int k = 0; k < d; ++k) *out += indent;
  };
  for (char c : src) {
    if (in_str) {
      out->push_back(c);
      if (esc) esc = false;
      else if (c == '\\') esc = true;
      else if (c == '"') in_str = false;
      continue;
    }
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r') continue;
    if (need && c != ']' && c != '}') {
      need = false;
      ++depth;
      newline(depth);
    }
    switch (c) {
      case '"': in_str = true; out->push_back(c); break;
      case '{': case '[': need = true; out->push_back(c); break;
      case ',': out->push_back(c); newline(depth); break;
      case ':': out->push_back(c); out->push_back(' '); break;
      case '}': case ']':
        if (need) need = false;                        // empty object / array stays "{}" / "[]"
        else { --depth; newline(depth); }
        out->push_back(c);
        break;
      default: out->push_back(c);
    }
  }
}

bool image_config_content(const std::string& config_json, std::string* out, std::string* err) {
  JValue cf;
  std::string perr;
  if (!json_parse(config_json, &cf, &perr)) { *err = "image config: " + perr; return false; }
  Enc e;
  Dec d{err};
  if (!encode_config_file(&cf, &e, &d)) return false;
  out->clear();
  go_indent(e.o, "  ", "", out);
  return true;
}

bool guess_base_layers(const std::string& config_json, const std::vector<std::string>& diff_ids,
                       std::vector<std::string>* base, std::string* err) {
  base->clear();
  JValue cf;
  std::string perr;
  if (!json_parse(config_json, &cf, &perr)) { *err = "image config: " + perr; return false; }
  struct H { std::string created_by; bool empty; };
  std::vector<H> hist;
  Dec d{err};
  if (const JValue* h = field(&cf, "history")) {
    if (h->kind == JValue::Arr) {
      for (const auto& it : h->arr) {
        H x;
        if (!d.str(&it, "created_by", &x.created_by) || !d.boolean(&it, "empty_layer", &x.empty)) return false;
        hist.push_back(x);
      }
    }
  }
  // image.GuessBaseImageIndex (pkg/fanal/image/image.go:111-137)
  int base_idx = -1;
  bool found_non_empty = false;
  for (int i = static_cast<int>(hist.size()) - 1; i >= 0; --i) {
    const H& h = hist[i];
    if (!found_non_empty) {
      if (h.empty) continue;
      found_non_empty = true;
    }
    if (!h.empty) continue;
    if (h.created_by.rfind("/bin/sh -c #(nop)  CMD", 0) == 0 || h.created_by.rfind("CMD", 0) == 0) {
      base_idx = i;
      break;
    }
  }
  // guessBaseLayers (pkg/fanal/artifact/image/image.go:526-554)
  size_t di = 0;
  for (int i = 0; i < static_cast<int>(hist.size()); ++i) {
    if (i > base_idx) break;
    if (hist[i].empty) continue;
    if (di >= diff_ids.size()) { base->clear(); return true; }   // "something wrong..."
    base->push_back(diff_ids[di++]);
  }
  return true;
}

bool report_json(const std::vector<const SecretVec*>& layers, const std::vector<LayerRef>& refs,
                 const Secret* image_config, const ReportOptions& opt, std::string* out, std::string* err) {
  // --- per layer: the analyzer keeps Secrets with findings (secret.go:139-141),
  // AnalysisResult.Sort orders them by FilePath and each one's findings by
  // (RuleID, StartLine) with sort.Slice (analyzer.go:224-235)
  std::map<std::string, MSecret> merged;             // ApplyLayers' secretsMap
  for (size_t li = 0; li < layers.size(); ++li) {
    std::vector<const Secret*> secs;
    for (const Secret& s : *layers[li])
      if (!s.findings().empty()) secs.push_back(&s);
    if (!opt.layers_sorted)
      GoSort<const Secret*>(&secs, [&secs](size_t i, size_t j) { return secs[i]->file_path() < secs[j]->file_path(); }).run();
    for (const Secret* s : secs) {
      MSecret ns;
      ns.path = std::string(s->file_path());
      for (const FindingRec& f : s->findings()) ns.findings.push_back({s, &f, static_cast<int>(li)});
      auto& fs = ns.findings;
      if (!opt.layers_sorted) {
        GoSort<MFinding>(&fs, [&fs](size_t i, size_t j) {
          if (fs[i].f->rule->id != fs[j].f->rule->id) return fs[i].f->rule->id < fs[j].f->rule->id;
          return fs[i].f->start_line < fs[j].f->start_line;
        }).run();
      }
      // mergeSecrets (docker.go:297-316): the newer layer's findings replace
      // older ones of the same RuleID; older ones of other rules stay, after them
      auto it = merged.find(ns.path);
      if (it != merged.end()) {
        for (const MFinding& prev : it->second.findings) {
          bool has = false;
          for (const MFinding& nf : ns.findings) if (nf.f->rule->id == prev.f->rule->id) { has = true; break; }
          if (!has) ns.findings.push_back(prev);
        }
        it->second = std::move(ns);
      } else {
        merged.emplace(ns.path, std::move(ns));
      }
    }
  }
  // Go iterates secretsMap in random order (docker.go:186-188); the report
  // lists merged secrets by FilePath, then the image-config secret under the
  // artifact name (local/scan.go:487-496)
  std::vector<MSecret> all;
  for (auto& kv : merged) all.push_back(std::move(kv.second));
  if (image_config && !image_config->findings().empty()) {
    MSecret cs;
    cs.path = opt.artifact_name;
    for (const FindingRec& f : image_config->findings()) cs.findings.push_back({image_config, &f, -1});
    all.push_back(std::move(cs));
  }
  // --- the report document
  Enc e;
  Dec d{err};
  e.open('{');
  e.kv_num_omit("SchemaVersion", opt.schema_version);
  std::string created;
  if (!go_time_rfc3339(opt.created_at, &created)) { *err = "CreatedAt is not RFC 3339: " + opt.created_at; return false; }
  e.kv_str("CreatedAt", created);
  e.kv_str_omit("ArtifactName", opt.artifact_name);
  e.kv_str_omit("ArtifactType", opt.artifact_type);
  e.key("Metadata");
  if (!encode_metadata(opt.metadata, &e, &d)) return false;
  // secretsToResults (local/scan.go:236-254) + filterSecrets (filter.go:154-169)
  // + JSONWriter's filter (json.go:36-38: Target != "" || !IsEmpty())
  std::string results;
  Enc r;
  r.open('[');
  size_t nres = 0;
  for (const MSecret& s : all) {
    std::vector<const MFinding*> kept;
    for (const MFinding& f : s.findings)
      if (std::find(opt.severities.begin(), opt.severities.end(), Secret::severity(*f.f)) != opt.severities.end())
        kept.push_back(&f);
    if (s.path.empty() && kept.empty()) continue;
    r.elem();
    r.open('{');
    r.kv_str("Target", s.path);
    r.kv_str("Class", "secret");
    if (!kept.empty()) {
      r.key("Secrets");
      r.open('[');
      for (const MFinding* f : kept) { r.elem(); encode_finding(*f, refs, &r); }
      r.close(']');
    }
    r.close('}');
    ++nres;
  }
  r.close(']');
  if (nres) {                                        // Results `json:",omitempty"`
    e.key("Results");
    e.o += r.o;
  }
  e.close('}');
  out->clear();
  go_indent(e.o, "", "  ", out);
  out->push_back('\n');                              // fmt.Fprintln
  return true;
}

}  // namespace tsg
