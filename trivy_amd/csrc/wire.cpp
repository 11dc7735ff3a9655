// Protobuf wire format of the secret results for Trivy's client/server mode
// (SURVEY.md 8f row 4): trivy.common.Secret / SecretFinding / Code / Line /
// Layer (rpc/common/service.proto:152-156, 191-223) as produced by
// ConvertToRPCSecrets / ConvertToRPCSecretFindings / ConvertToRPCCode /
// ConvertToRPCLayer (pkg/rpc/convert.go:127-175, 370-376) and proto.Marshal,
// and read back as ConvertFromRPCSecrets (convert.go:476-533, 655-664).
//
// proto3 rules restated: fields in field-number order; scalar fields equal to
// their default ("" / 0 / false) are not written; message fields set by the
// converters (code, layer, every line) are written even when empty; int32 is
// a varint of the sign-extended 64-bit value; a string field must hold valid
// UTF-8 (proto.Marshal fails otherwise, so the encoder does too).
#include "wire.h"

#include <cstring>

namespace tsg {

namespace {

void varint(std::string* o, uint64_t v) {
  while (v >= 0x80) { o->push_back(static_cast<char>((v & 0x7f) | 0x80)); v >>= 7; }
  o->push_back(static_cast<char>(v));
}

void tag(std::string* o, uint32_t field, uint32_t wt) { varint(o, (static_cast<uint64_t>(field) << 3) | wt); }

bool valid_utf8(const char* s, size_t n) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(s);
  size_t i = 0;
  while (i < n) {
    const uint8_t c = p[i];
    if (c < 0x80) { ++i; continue; }
    int32_t r;
    int w;
    re::decode_rune(p + i, n - i, &r, &w);
    if (r == 0xFFFD && w == 1) return false;
    i += w;
  }
  return true;
}

struct Enc {
  std::string* err;
  bool str(std::string* o, uint32_t f, const char* s, size_t n, const char* name) {
    if (!n) return true;
    if (!valid_utf8(s, n)) {
      if (err->empty()) *err = std::string("proto: field trivy.common.") + name + " contains invalid UTF-8";
      return false;
    }
    tag(o, f, 2);
    varint(o, n);
    o->append(s, n);
    return true;
  }
  bool str(std::string* o, uint32_t f, const std::string& s, const char* name) { return str(o, f, s.data(), s.size(), name); }
  void i32(std::string* o, uint32_t f, int v) {
    if (!v) return;
    tag(o, f, 0);
    varint(o, static_cast<uint64_t>(static_cast<int64_t>(v)));
  }
  void boolean(std::string* o, uint32_t f, bool v) {
    if (!v) return;
    tag(o, f, 0);
    o->push_back(1);
  }
  void msg(std::string* o, uint32_t f, const std::string& body) {
    tag(o, f, 2);
    varint(o, body.size());
    *o += body;
  }
};

// ------------------------------------------------------------------ decode
struct Reader {
  const uint8_t* p;
  size_t n, i = 0;
  bool ok = true;
  bool more() const { return ok && i < n; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (i >= n) { ok = false; return 0; }
      const uint8_t b = p[i++];
      v |= static_cast<uint64_t>(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  bool bytes(const uint8_t** s, size_t* len) {
    const uint64_t l = varint();
    if (!ok || l > n - i) { ok = false; return false; }
    *s = p + i;
    *len = static_cast<size_t>(l);
    i += *len;
    return true;
  }
  // skip a field of wire type wt (unknown fields are ignored by proto.Unmarshal)
  void skip(uint32_t wt) {
    const uint8_t* s;
    size_t l;
    switch (wt) {
      case 0: varint(); break;
      case 1: if (n - i < 8) ok = false; else i += 8; break;
      case 2: bytes(&s, &l); break;
      case 5: if (n - i < 4) ok = false; else i += 4; break;
      default: ok = false;
    }
  }
};

StrRef put(SecretBuilder* s, const uint8_t* p, size_t n) { return s->put(reinterpret_cast<const char*>(p), n); }

bool read_string(Reader* r, uint32_t wt, std::string* out) {
  const uint8_t* s;
  size_t l;
  if (wt != 2 || !r->bytes(&s, &l)) return false;
  out->assign(reinterpret_cast<const char*>(s), l);
  return valid_utf8(out->data(), out->size());
}

}  // namespace

bool secret_to_proto(const Secret& sec, const std::vector<LayerRef>* layer_of_finding, std::string* out,
                     std::string* err) {
  Enc e{err};
  std::string o;
  const std::string_view fp = sec.file_path();
  if (!e.str(&o, 1, fp.data(), fp.size(), "Secret.filepath")) return false;
  const auto sf = sec.findings();
  const auto sl = sec.lines();
  for (size_t k = 0; k < sf.size(); ++k) {
    const FindingRec& f = sf[k];
    std::string fm;
    if (!e.str(&fm, 1, f.rule->id, "SecretFinding.rule_id") || !e.str(&fm, 2, f.rule->category, "SecretFinding.category") ||
        !e.str(&fm, 3, Secret::severity(f), "SecretFinding.severity") || !e.str(&fm, 4, f.rule->title, "SecretFinding.title"))
      return false;
    e.i32(&fm, 5, f.start_line);
    e.i32(&fm, 6, f.end_line);
    std::string code;                        // ConvertToRPCCode: always a message
    for (uint32_t l = 0; l < f.line_count; ++l) {
      const LineRec& ln = sl[f.line_begin + l];
      std::string lm;
      e.i32(&lm, 1, ln.number);
      if (!e.str(&lm, 2, sec.ptr(ln.content), ln.content.len, "Line.content")) return false;
      e.boolean(&lm, 3, ln.is_cause);
      // annotation (4) "" and truncated (5) false: defaults, not written
      if (!e.str(&lm, 6, sec.ptr(ln.content), ln.content.len, "Line.highlighted")) return false;
      e.boolean(&lm, 7, ln.first_cause);
      e.boolean(&lm, 8, ln.last_cause);
      e.msg(&code, 1, lm);
    }
    e.msg(&fm, 7, code);
    if (!e.str(&fm, 8, sec.ptr(f.match), f.match.len, "SecretFinding.match")) return false;
    std::string lay;                         // ConvertToRPCLayer: always a message
    if (layer_of_finding && k < layer_of_finding->size()) {
      const LayerRef& r = (*layer_of_finding)[k];
      if (!e.str(&lay, 1, r.digest, "Layer.digest") || !e.str(&lay, 2, r.diff_id, "Layer.diff_id") ||
          !e.str(&lay, 3, r.created_by, "Layer.created_by"))
        return false;
    }
    e.msg(&fm, 10, lay);
    e.msg(&o, 2, fm);
  }
  *out = std::move(o);
  return true;
}

bool secret_from_proto(const uint8_t* data, size_t len, std::deque<Rule>* rules, Secret* out,
                       std::vector<LayerRef>* layers, std::string* err) {
  *out = Secret();
  SecretBuilder sb;
  layers->clear();
  Reader r{data, len};
  auto bad = [&](const char* what) { *err = std::string("proto: cannot parse ") + what; return false; };
  while (r.more()) {
    const uint64_t key = r.varint();
    const uint32_t f = static_cast<uint32_t>(key >> 3), wt = static_cast<uint32_t>(key & 7);
    if (f == 1) {
      if (!read_string(&r, wt, &sb.file_path)) return bad("Secret.filepath");
    } else if (f == 2 && wt == 2) {
      const uint8_t* s;
      size_t l;
      if (!r.bytes(&s, &l)) return bad("Secret.findings");
      Rule rule;
      FindingRec fr;
      LayerRef lr;
      std::string match;
      std::vector<LineRec> lines;
      std::string sev;
      Reader fm{s, l};
      while (fm.more()) {
        const uint64_t k2 = fm.varint();
        const uint32_t f2 = static_cast<uint32_t>(k2 >> 3), w2 = static_cast<uint32_t>(k2 & 7);
        bool ok = true;
        switch (f2) {
          case 1: ok = read_string(&fm, w2, &rule.id); break;
          case 2: ok = read_string(&fm, w2, &rule.category); break;
          case 3: ok = read_string(&fm, w2, &sev); break;
          case 4: ok = read_string(&fm, w2, &rule.title); break;
          case 5: ok = w2 == 0; fr.start_line = static_cast<int32_t>(fm.varint()); break;
          case 6: ok = w2 == 0; fr.end_line = static_cast<int32_t>(fm.varint()); break;
          case 7: {
            const uint8_t* cs;
            size_t cl;
            if (w2 != 2 || !fm.bytes(&cs, &cl)) { ok = false; break; }
            Reader cm{cs, cl};
            while (cm.more() && ok) {
              const uint64_t k3 = cm.varint();
              if ((k3 >> 3) != 1 || (k3 & 7) != 2) { cm.skip(static_cast<uint32_t>(k3 & 7)); continue; }
              const uint8_t* ls;
              size_t ll;
              if (!cm.bytes(&ls, &ll)) { ok = false; break; }
              Reader lm{ls, ll};
              LineRec ln;
              std::string content, ann, hl;
              bool trunc = false;
              while (lm.more() && ok) {
                const uint64_t k4 = lm.varint();
                const uint32_t f4 = static_cast<uint32_t>(k4 >> 3), w4 = static_cast<uint32_t>(k4 & 7);
                switch (f4) {
                  case 1: ok = w4 == 0; ln.number = static_cast<int32_t>(lm.varint()); break;
                  case 2: ok = read_string(&lm, w4, &content); break;
                  case 3: ok = w4 == 0; ln.is_cause = lm.varint() != 0; break;
                  case 4: ok = read_string(&lm, w4, &ann); break;
                  case 5: ok = w4 == 0; trunc = lm.varint() != 0; break;
                  case 6: ok = read_string(&lm, w4, &hl); break;
                  case 7: ok = w4 == 0; ln.first_cause = lm.varint() != 0; break;
                  case 8: ok = w4 == 0; ln.last_cause = lm.varint() != 0; break;
                  default: lm.skip(w4);
                }
              }
              // the result model keeps Highlighted == Content, Annotation "" and
              // Truncated false (all the scanner produces, scanner.go:538-545)
              if (!lm.ok || !ann.empty() || trunc || hl != content) { ok = false; break; }
              ln.content = put(&sb, reinterpret_cast<const uint8_t*>(content.data()), content.size());
              lines.push_back(ln);
            }
            ok = ok && cm.ok;
            break;
          }
          case 8: ok = read_string(&fm, w2, &match); break;
          case 10: {
            const uint8_t* ls;
            size_t ll;
            if (w2 != 2 || !fm.bytes(&ls, &ll)) { ok = false; break; }
            Reader lm{ls, ll};
            while (lm.more() && ok) {
              const uint64_t k4 = lm.varint();
              const uint32_t f4 = static_cast<uint32_t>(k4 >> 3), w4 = static_cast<uint32_t>(k4 & 7);
              if (f4 == 1) ok = read_string(&lm, w4, &lr.digest);
              else if (f4 == 2) ok = read_string(&lm, w4, &lr.diff_id);
              else if (f4 == 3) ok = read_string(&lm, w4, &lr.created_by);
              else lm.skip(w4);
            }
            ok = ok && lm.ok;
            break;
          }
          default: fm.skip(w2);
        }
        if (!ok || !fm.ok) return bad("SecretFinding");
      }
      rule.severity = sev;
      rules->push_back(rule);
      fr.rule = &rules->back();
      fr.match = put(&sb, reinterpret_cast<const uint8_t*>(match.data()), match.size());
      fr.line_begin = static_cast<uint32_t>(sb.lines.size());
      for (const LineRec& ln : lines) sb.lines.push_back(ln);
      fr.line_count = static_cast<uint32_t>(lines.size());
      sb.findings.push_back(fr);
      layers->push_back(lr);
    } else {
      r.skip(wt);
    }
    if (!r.ok) return bad("Secret");
  }
  if (!r.ok) return bad("Secret");
  *out = Secret::build(sb);
  return true;
}

}  // namespace tsg
