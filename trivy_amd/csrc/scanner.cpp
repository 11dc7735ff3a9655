// Exact restatement of pkg/fanal/secret/scanner.go on the host (see scanner.h).
#include "scanner.h"

#include <array>
#include "gosort.h"
#include "guard.h"
#include "prefilter.h"

#include <algorithm>
#include <atomic>
#include <emmintrin.h>
#include <chrono>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <sys/mman.h>
#include <cstdlib>

namespace tsg {

#include "builtin_rules.inc"   // kBuiltinRulesJson: trivy_amd/data/builtin_rules.json

namespace {

RegexpPtr compile_or_err(const JValue* v, std::string* err) {
  if (!v || v->is_null()) return nullptr;
  std::string e;
  auto re = re::Regexp::compile(v->as_string(), &e);
  if (!re) {
    // scanner.go:80-83: xerrors.Errorf("regexp compile error: %w", err)
    if (err->empty()) *err = "regexp compile error: " + e;
    return nullptr;
  }
  re::LitGate g;
  bool bounded = false;
  uint32_t dmin = 0, dmax = 0;
  if (literal_gate(*re->ast(), &g, &bounded, &dmin, &dmax)) re->set_gate(std::move(g), bounded, dmin, dmax);
  return RegexpPtr(re.release());
}

std::vector<std::string> str_list(const JValue* v) {
  std::vector<std::string> out;
  if (!v) return out;
  if (v->kind == JValue::Arr) {
    for (const auto& x : v->arr) out.push_back(x.as_string());
  }
  return out;
}

std::string field(const JValue* o, const char* k) {
  const JValue* v = o ? o->get(k) : nullptr;
  return v ? v->as_string() : "";
}

bool allow_rules_from(const JValue* v, std::vector<AllowRule>* out, std::string* err) {
  if (!v || v->kind != JValue::Arr) return true;
  for (const auto& a : v->arr) {
    AllowRule r;
    r.id = field(&a, "id");
    r.description = field(&a, "description");
    r.regex = compile_or_err(a.get("regex"), err);
    r.path = compile_or_err(a.get("path"), err);
    if (!err->empty()) return false;
    out->push_back(std::move(r));
  }
  return true;
}

bool exclude_from(const JValue* v, std::vector<RegexpPtr>* out, std::string* err) {
  if (!v || v->kind != JValue::Obj) return true;
  const JValue* rx = v->get("regexes");
  if (!rx || rx->kind != JValue::Arr) return true;
  for (const auto& r : rx->arr) {
    RegexpPtr p = compile_or_err(&r, err);
    if (!err->empty()) return false;
    out->push_back(p);
  }
  return true;
}

// scanner.go:309-318
std::string convert_severity(const std::string& s) {
  std::string lo, up;
  for (char c : s) { lo.push_back(static_cast<char>(tolower(static_cast<unsigned char>(c)))); }
  if (lo == "low" || lo == "medium" || lo == "high" || lo == "critical" || lo == "unknown") {
    for (char c : s) up.push_back(static_cast<char>(toupper(static_cast<unsigned char>(c))));
    return up;
  }
  return "UNKNOWN";
}

void finish_rule(Rule* r) {
  for (const auto& k : r->keywords) r->keywords_lower.push_back(go_str_to_lower(k));
  r->secret_groups.clear();
  if (r->regex && !r->secret_group_name.empty()) {
    const auto& names = r->regex->subexp_names();
    for (size_t i = 0; i < names.size(); ++i) {
      if (names[i] == r->secret_group_name) r->secret_groups.push_back(static_cast<int>(i));
    }
  }
}

bool load_builtins(std::vector<Rule>* rules, std::vector<AllowRule>* allows, std::string* err) {
  static std::once_flag once;
  static std::vector<Rule> b_rules;
  static std::vector<AllowRule> b_allow;
  static std::string b_err;
  std::call_once(once, [] {
    JValue doc;
    if (!json_parse(kBuiltinRulesJson, &doc, &b_err)) return;
    for (const auto& j : doc.get("rules")->arr) {
      Rule r;
      r.id = field(&j, "id");
      r.category = field(&j, "category");
      r.title = field(&j, "title");
      r.severity = field(&j, "severity");
      r.regex = compile_or_err(j.get("regex"), &b_err);
      r.keywords = str_list(j.get("keywords"));
      r.secret_group_name = field(&j, "secret_group_name");
      finish_rule(&r);
      b_rules.push_back(std::move(r));
    }
    allow_rules_from(doc.get("allow_rules"), &b_allow, &b_err);
  });
  if (!b_err.empty()) { *err = "builtin rules: " + b_err; return false; }
  *rules = b_rules;
  *allows = b_allow;
  return true;
}

bool contains(const std::vector<std::string>& v, const std::string& s) {
  return std::find(v.begin(), v.end(), s) != v.end();
}

void index_excludes(Ruleset* rs) {
  rs->excludes.clear();
  for (const auto& r : rs->exclude_block) rs->excludes.push_back(r.get());
  for (auto& rule : rs->rules) {
    rule.exclude_base = static_cast<uint32_t>(rs->excludes.size());
    for (const auto& r : rule.exclude_block) rs->excludes.push_back(r.get());
  }
}

}  // namespace

// Ruleset::AllowPathIndex: the literals of every global allow rule's path
// (or, for the match index, text) regex's gate (each unit's alternatives
// expanded, at most kMaxLits per regex; a regex past that or without a gate
// is always run) in one Aho-Corasick DFA.
static void build_allow_index(Ruleset* rs, RegexpPtr AllowRule::*field, Ruleset::AllowPathIndex* ixp) {
  Ruleset::AllowPathIndex& ix = *ixp;
  ix = Ruleset::AllowPathIndex();
  if (rs->allow_rules.size() > 64) return;
  constexpr size_t kMaxLits = 512, kMaxStates = 4096;
  std::vector<std::array<int32_t, 256>> go(1);
  go[0].fill(-1);
  std::vector<uint64_t> out(1, 0);
  for (size_t j = 0; j < rs->allow_rules.size(); ++j) {
    const auto& path = rs->allow_rules[j].*field;
    if (!path) continue;
    std::vector<std::string> lits;
    bool ok = path->has_gate();
    for (const auto& seq : path->gate()) {
      if (!ok) break;
      std::vector<std::string> cur{""};
      for (const auto& unit : seq) {
        std::vector<std::string> nx;
        for (const auto& c : cur)
          for (const auto& alt : unit) nx.push_back(c + alt);
        if (nx.size() > kMaxLits) { ok = false; break; }
        cur.swap(nx);
      }
      if (ok) lits.insert(lits.end(), cur.begin(), cur.end());
      if (lits.size() > kMaxLits) ok = false;
    }
    if (!ok || lits.empty()) { ix.always |= 1ull << j; continue; }
    for (const auto& l : lits) {
      int32_t st = 0;
      for (unsigned char c : l) {
        if (go[st][c] < 0) {
          go[st][c] = static_cast<int32_t>(go.size());
          go.emplace_back();
          go.back().fill(-1);
          out.push_back(0);
        }
        st = go[st][c];
      }
      out[st] |= 1ull << j;
    }
    if (go.size() > kMaxStates) return;    // unusable: the plain loop
  }
  // BFS: failure links folded into a full DFA
  const size_t ns = go.size();
  ix.next.assign(ns * 256, 0);
  std::vector<int32_t> fail(ns, 0), order;
  for (int c = 0; c < 256; ++c) {
    const int32_t t = go[0][c];
    if (t >= 0) { fail[t] = 0; order.push_back(t); ix.next[c] = static_cast<uint16_t>(t); }
  }
  for (size_t k = 0; k < order.size(); ++k) {
    const int32_t s = order[k];
    out[s] |= out[fail[s]];
    for (int c = 0; c < 256; ++c) {
      const int32_t t = go[s][c];
      if (t >= 0) {
        fail[t] = ix.next[static_cast<size_t>(fail[s]) * 256 + c];
        order.push_back(t);
        ix.next[static_cast<size_t>(s) * 256 + c] = static_cast<uint16_t>(t);
      } else {
        ix.next[static_cast<size_t>(s) * 256 + c] = ix.next[static_cast<size_t>(fail[s]) * 256 + c];
      }
    }
  }
  ix.out = std::move(out);
  ix.usable = true;
}

bool build_ruleset(const JValue* cfg, Ruleset* out, std::string* err) {
  std::vector<Rule> b_rules;
  std::vector<AllowRule> b_allow;
  if (!load_builtins(&b_rules, &b_allow, err)) return false;
  if (!cfg || cfg->is_null()) {                       // scanner.go:324-332
    out->rules = std::move(b_rules);
    out->allow_rules = std::move(b_allow);
    out->exclude_block.clear();
    index_excludes(out);
    build_allow_index(out, &AllowRule::path, &out->allow_index);
    build_allow_index(out, &AllowRule::regex, &out->allow_match_index);
    return true;
  }
  std::vector<std::string> enable = str_list(cfg->get("enable-builtin-rules"));
  std::vector<std::string> disable = str_list(cfg->get("disable-rules"));
  std::vector<std::string> disable_allow = str_list(cfg->get("disable-allow-rules"));
  std::vector<Rule> custom;
  if (const JValue* rl = cfg->get("rules")) {
    if (rl->kind == JValue::Arr) {
      for (const auto& j : rl->arr) {
        Rule r;
        r.id = field(&j, "id");
        r.category = field(&j, "category");
        r.title = field(&j, "title");
        r.severity = convert_severity(field(&j, "severity"));   // scanner.go:301-304
        r.regex = compile_or_err(j.get("regex"), err);
        r.keywords = str_list(j.get("keywords"));
        r.path = compile_or_err(j.get("path"), err);
        if (!allow_rules_from(j.get("allow-rules"), &r.allow_rules, err)) return false;
        if (!exclude_from(j.get("exclude-block"), &r.exclude_block, err)) return false;
        r.secret_group_name = field(&j, "secret-group-name");
        if (!err->empty()) return false;
        finish_rule(&r);
        custom.push_back(std::move(r));
      }
    }
  }
  std::vector<AllowRule> custom_allow;
  if (!allow_rules_from(cfg->get("allow-rules"), &custom_allow, err)) return false;
  std::vector<RegexpPtr> excl;
  if (!exclude_from(cfg->get("exclude-block"), &excl, err)) return false;

  std::vector<Rule> enabled;                          // scanner.go:334-348
  for (auto& r : b_rules) {
    if (enable.empty() || contains(enable, r.id)) enabled.push_back(r);
  }
  for (auto& r : custom) enabled.push_back(std::move(r));
  out->rules.clear();
  for (auto& r : enabled) {
    if (!contains(disable, r.id)) out->rules.push_back(std::move(r));
  }
  out->allow_rules.clear();                           // scanner.go:350-354
  for (auto& a : b_allow) if (!contains(disable_allow, a.id)) out->allow_rules.push_back(a);
  for (auto& a : custom_allow) if (!contains(disable_allow, a.id)) out->allow_rules.push_back(a);
  out->exclude_block = std::move(excl);
  index_excludes(out);
  build_allow_index(out, &AllowRule::path, &out->allow_index);
  build_allow_index(out, &AllowRule::regex, &out->allow_match_index);
  return true;
}

namespace {
// Some global allow rule's `field` regex matches p[0, n) (scanner.go:52-59):
// the rules whose gate literals occur in the text, found in one pass of the
// index, are the only ones that can; the plain loop when the index is unusable.
bool global_allow_indexed(const Ruleset& rs, const Ruleset::AllowPathIndex& ix, RegexpPtr AllowRule::*field,
                          const uint8_t* p, size_t n) {
  if (!ix.usable) {
    for (const auto& r : rs.allow_rules)
      if ((r.*field) && (r.*field)->match_string(p, n)) return true;
    return false;
  }
  uint64_t cand = ix.always;
  uint32_t st = 0;
  for (size_t i = 0; i < n; ++i) {
    st = ix.next[st * 256u + p[i]];
    cand |= ix.out[st];
  }
  while (cand) {                       // a rule none of whose gate literals occurs cannot match
    const int j = __builtin_ctzll(cand);
    cand &= cand - 1;
    if ((rs.allow_rules[j].*field)->match_string(p, n)) return true;
  }
  return false;
}
}  // namespace

bool global_allow_path(const Ruleset& rs, const uint8_t* p, size_t n) {
  return global_allow_indexed(rs, rs.allow_index, &AllowRule::path, p, n);
}

bool global_allow_match(const Ruleset& rs, const uint8_t* m, size_t n) {
  return global_allow_indexed(rs, rs.allow_match_index, &AllowRule::regex, m, n);
}

// ---------------------------------------------------------------- helpers
std::string go_bytes_to_lower(const uint8_t* s, size_t n) {
  bool ascii = true;
  for (size_t i = 0; i < n; ++i) if (s[i] >= 0x80) { ascii = false; break; }
  std::string out;
  out.resize(n);
  if (ascii) {
    for (size_t i = 0; i < n; ++i) {
      uint8_t c = s[i];
      out[i] = static_cast<char>((c >= 'A' && c <= 'Z') ? c + 32 : c);
    }
    return out;
  }
  out.clear();
  out.reserve(n + 16);
  size_t i = 0;
  while (i < n) {
    int32_t r; int w;
    re::decode_rune(s + i, n - i, &r, &w);
    re::append_utf8(&out, re::to_lower(static_cast<uint32_t>(r)));   // invalid byte: r == U+FFFD
    i += w;
  }
  return out;
}

std::string go_str_to_lower(const std::string& s) {
  return go_bytes_to_lower(reinterpret_cast<const uint8_t*>(s.data()), s.size());
}

std::string go_quote(const std::string& s) {
  std::string out = "\"";
  const uint8_t* p = reinterpret_cast<const uint8_t*>(s.data());
  size_t i = 0, n = s.size();
  char buf[16];
  while (i < n) {
    int32_t r; int w;
    re::decode_rune(p + i, n - i, &r, &w);
    if (r == 0xFFFD && w == 1) { snprintf(buf, sizeof buf, "\\x%02x", p[i]); out += buf; i += 1; continue; }
    if (r == '"' || r == '\\') { out.push_back('\\'); out.push_back(static_cast<char>(r)); }
    else if (r < 0x80 && r >= 0x20 && r != 0x7f) out.push_back(static_cast<char>(r));
    else if (r >= 0x80 && re::is_print(static_cast<uint32_t>(r))) out.append(s, i, w);
    else {
      switch (r) {
        case '\a': out += "\\a"; break;
        case '\b': out += "\\b"; break;
        case '\f': out += "\\f"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        case '\v': out += "\\v"; break;
        default:
          if (r < 0x80) snprintf(buf, sizeof buf, "\\x%02x", r);
          else if (r < 0x10000) snprintf(buf, sizeof buf, "\\u%04x", r);
          else snprintf(buf, sizeof buf, "\\U%08x", r);
          out += buf;
      }
    }
    i += w;
  }
  out += "\"";
  return out;
}

bool go_is_binary(const uint8_t* head, size_t n) {          // utils.go:68-86
  n = std::min<size_t>(n, 300);
  for (size_t i = 0; i < n; ++i) {
    uint8_t b = head[i];
    if (b < 7 || b == 11 || (13 < b && b < 27) || (27 < b && b < 0x20) || b == 0x7f) return true;
  }
  return false;
}

std::string go_extract_printable(const uint8_t* s, size_t n) {   // utils.go:111-143
  std::string out, cur;
  for (size_t i = 0; i < n; ++i) {
    if (re::is_print(s[i])) { cur.push_back(static_cast<char>(s[i])); continue; }
    if (cur.size() > 4) { cur.push_back('\n'); out += cur; }
    cur.clear();
  }
  if (cur.size() > 4) { cur.push_back('\n'); out += cur; }
  return out;
}

// ------------------------------------------------------ candidate find-all
namespace {

// Is `s` a rune boundary of the decoding chain that starts at boundary `pos`?
bool chain_boundary(const uint8_t* t, size_t len, size_t pos, size_t s) {
  if (s == pos || s >= len) return s <= len;
  if ((t[s] & 0xC0) != 0x80) return true;            // not a continuation byte
  size_t q = s;
  while (q > pos && (t[q] & 0xC0) == 0x80 && s - q < 4) --q;
  if ((t[q] & 0xC0) == 0x80 && q != pos) return true;  // >=4 continuation bytes: all invalid, width 1
  // decode forward from q (a chain boundary) until reaching >= s
  size_t x = q;
  while (x < s) {
    int32_t r; int w;
    re::decode_rune(t + x, len - x, &r, &w);
    x += w;
  }
  return x == s;
}

}  // namespace

void find_all_from_candidates(const re::Regexp& re, const uint8_t* text, size_t len,
                              const std::vector<uint64_t>& starts, bool submatch,
                              std::vector<re::Cap>* out) {
  const int ncap = 2 * (re.num_subexp() + 1);
  thread_local std::vector<re::Cap> caps;        // per-thread scratch (no allocation per call)
  caps.resize(ncap);
  size_t pos = 0;
  long prev_end = -1;
  size_t idx = 0;
  while (pos <= len) {
    // leftmost match with start >= pos: first candidate with an anchored match
    bool found = false;
    while (idx < starts.size()) {
      size_t s = starts[idx];
      if (s < pos) { ++idx; continue; }
      if (s > len) { idx = starts.size(); break; }
      if (chain_boundary(text, len, pos, s)) {
        // submatch rules go straight to the VM: the GPU's verify leaves few
        // candidates that do not match (config 2: 84% match), so a lazy-DFA
        // pre-check mostly costs twice (table model: find 4.5 vs 6.4 ms warm);
        // other rules take the lazy DFA's anchored match end
        if (submatch) {
          if (re.match_at(text, len, s, true, ncap, caps.data())) { found = true; break; }
          ++idx;
          continue;
        }
        const long e = re.match_end(text, len, s);
        if (e >= 0) {
          caps[0] = static_cast<re::Cap>(s);
          caps[1] = static_cast<re::Cap>(e);
          found = true;
          break;
        }
      }
      ++idx;
    }
    if (!found) break;
    bool accept = true;
    if (static_cast<size_t>(caps[1]) == pos) {
      if (caps[0] == prev_end) accept = false;
      int32_t r; int w;
      re::decode_rune(text + pos, len - pos, &r, &w);
      pos = w > 0 ? pos + w : len + 1;
    } else {
      pos = static_cast<size_t>(caps[1]);
    }
    prev_end = caps[1];
    if (accept) {
      if (submatch) out->insert(out->end(), caps.begin(), caps.end());
      else { out->push_back(caps[0]); out->push_back(caps[1]); }
    }
  }
}

// ------------------------------------------------------------------- Scan
namespace {

bool allow_path(const std::vector<AllowRule>& rules, const std::string& path) {
  for (const auto& r : rules) {
    if (r.path && r.path->match_string(reinterpret_cast<const uint8_t*>(path.data()), path.size())) return true;
  }
  return false;
}

bool allow_match(const std::vector<AllowRule>& rules, const uint8_t* m, size_t n) {
  for (const auto& r : rules) {
    if (r.regex && r.regex->match_string(m, n)) return true;
  }
  return false;
}

struct Loc { long start, end; };

// ExcludeBlock (scanner.go:237-275): on first use, every exclude regex's
// find-all over the whole file.  With a plan, exclude regex k (pseudo-rule
// plan_base + k) is evaluated like a rule: from its GPU candidate starts, not
// at all when it has none, or in full when it has no bounded anchor.
class Blocks {
 public:
  Blocks(const uint8_t* c, size_t n, const std::vector<RegexpPtr>& rx, const FilePlan* plan, size_t plan_base)
      : c_(c), n_(n), rx_(rx), plan_(plan), base_(plan_base) {}
  bool match(const Loc& l) {
    if (!done_) {
      done_ = true;
      std::vector<re::Cap> m;
      for (size_t j = 0; j < rx_.size(); ++j) {
        const auto& r = rx_[j];
        if (!r) continue;
        m.clear();
        const size_t id = base_ + j;
        const uint8_t kind = plan_ && id < plan_->kind.size() ? plan_->kind[id] : static_cast<uint8_t>(kPlanFull);
        if (kind == kPlanFull) {
          r->find_all(c_, n_, false, &m);
        } else if (kind == kPlanCandidates || kind == kPlanCandHostGate) {
          auto it = std::lower_bound(plan_->cands.begin(), plan_->cands.end(), id,
                                     [](const RuleCandidates& a, size_t v) { return a.rule < v; });
          if (it != plan_->cands.end() && it->rule == id) find_all_from_candidates(*r, c_, n_, it->starts, false, &m);
        }
        for (size_t k = 0; k + 1 < m.size(); k += 2) locs_.push_back({m[k], m[k + 1]});
      }
    }
    for (const auto& b : locs_) if (b.start <= l.start && l.end <= b.end) return true;
    return false;
  }

 private:
  const uint8_t* c_;
  size_t n_;
  const std::vector<RegexpPtr>& rx_;
  const FilePlan* plan_;
  size_t base_;
  bool done_ = false;
  std::vector<Loc> locs_;
};

// scanner.go:102-148
void find_locations(const Ruleset& rs, const Rule& rule, const uint8_t* c, size_t n,
                    const std::vector<uint64_t>* starts, std::vector<Loc>* locs, int* error) {
  if (!rule.regex) return;
  const bool sub = !rule.secret_group_name.empty();
  thread_local std::vector<re::Cap> m;           // per-thread scratch
  m.clear();
  if (starts) find_all_from_candidates(*rule.regex, c, n, *starts, sub, &m);
  else rule.regex->find_all(c, n, sub, &m);
  const size_t stride = sub ? 2 * (rule.regex->num_subexp() + 1) : 2;
  for (size_t k = 0; k + stride <= m.size(); k += stride) {
    const long s = m[k], e = m[k + 1];
    // AllowLocation (scanner.go:150-153): global then rule allow regexes on the whole match
    if (global_allow_match(rs, c + s, e - s) || allow_match(rule.allow_rules, c + s, e - s)) continue;
    if (!sub) { locs->push_back({s, e}); continue; }
    for (int gi : rule.secret_groups) {                // scanner.go:155-168
      Loc l{m[k + 2 * gi], m[k + 2 * gi + 1]};
      if (l.start < 0) *error = 1;                     // reference: censorLocation panics on {-1,-1}
      locs->push_back(l);
    }
  }
}

// '\n' bytes in p[0, n): eight at a time (bit 7 of a byte of t is set
// exactly when that byte of v is '\n')
// SSE2: per 16 bytes one compare subtracted into byte counters, summed by
// psadbw every 255 vectors (~16 B/cycle; the 8-byte SWAR form ran ~3)
uint64_t count_newlines(const uint8_t* p, size_t n) {
  const __m128i nl = _mm_set1_epi8('\n');
  uint64_t cnt = 0;
  size_t i = 0;
  while (i + 16 <= n) {
    const size_t stop = std::min(n - 15, i + 255 * 16);
    __m128i acc = _mm_setzero_si128();
    for (; i < stop; i += 16)
      acc = _mm_sub_epi8(acc, _mm_cmpeq_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i)), nl));
    const __m128i sum = _mm_sad_epu8(acc, _mm_setzero_si128());
    cnt += static_cast<uint64_t>(_mm_cvtsi128_si32(sum)) + static_cast<uint64_t>(_mm_extract_epi16(sum, 4));
  }
  for (; i < n; ++i) cnt += p[i] == '\n';
  return cnt;
}

// The censored buffer of scanner.go:431-435 (content with every matched span
// overwritten by '*'), represented virtually: original bytes + merged spans.
class CensoredView {
 public:
  // `spans` is merged in place and kept as the view's span list; `scratch`
  // holds the newline prefix (both the caller's per-thread buffers: no
  // allocation per confirmed file)
  CensoredView(const uint8_t* c, size_t n, std::vector<Loc>& spans, std::vector<uint64_t>& scratch, const NlSource* nl)
      : c_(c), n_(n), iv_(spans), local_(scratch) {
    std::sort(spans.begin(), spans.end(), [](const Loc& a, const Loc& b) { return a.start < b.start; });
    size_t m = 0;
    for (size_t i = 0; i < spans.size(); ++i) {
      const Loc l = spans[i];
      if (l.end <= l.start) continue;
      if (m > 0 && l.start <= spans[m - 1].end) spans[m - 1].end = std::max(spans[m - 1].end, l.end);
      else spans[m++] = l;
    }
    spans.resize(m);
    if (nl && nl->chunk_nl) {
      // local prefix over the batch chunks this file touches
      ch_ = nl->chunk;
      data_ = nl->data;
      off_ = nl->file_off;
      first_ = off_ / ch_;
      // prefix_at(g) reads local_[g / ch_ - first_] for g <= off_ + n: only
      // chunks strictly below (off_ + n) / ch_ are summed, so a file ending
      // exactly on the batch's last chunk boundary reads no count past the end
      // filled on demand (prefix_at): a finding near the start of a large
      // file does not pay for the chunks after it
      chunk_nl_ = nl->chunk_nl;
      local_.assign(1, 0);
    } else {
      // local prefix over this file (reference / host-only paths)
      ch_ = 4096;
      data_ = c_;
      off_ = 0;
      first_ = 0;
      const size_t nch = n / ch_ + 1;
      local_.assign(nch + 1, 0);
      for (size_t k = 0; k < nch; ++k) {
        const size_t b = std::min<size_t>(n, k * ch_), e = std::min<size_t>(n, b + ch_);
        local_[k + 1] = local_[k] + count_newlines(c_ + b, e - b);
      }
    }
  }
  uint8_t at(size_t i) const { return censored(static_cast<long>(i)) ? '*' : c_[i]; }
  bool censored(long i) const {
    auto it = std::upper_bound(iv_.begin(), iv_.end(), i, [](long v, const Loc& l) { return v < l.start; });
    if (it == iv_.begin()) return false;
    --it;
    return i < it->end;
  }
  // '\n' count of the censored buffer in [a, b)
  uint64_t count_nl(size_t a, size_t b) const {
    if (b <= a) return 0;
    uint64_t n = orig_nl(a, b);
    for (auto it = first_ending_after(a); it != iv_.end() && static_cast<size_t>(it->start) < b; ++it) {
      size_t x = std::max<size_t>(a, it->start), y = std::min<size_t>(b, it->end);
      if (x < y) n -= orig_nl(x, y);
    }
    return n;
  }
  // last censored-buffer '\n' position < pos, or -1
  long prev_nl(size_t pos) const {
    long i = static_cast<long>(pos) - 1;
    while (i >= 0) {
      const void* q = memrchr(c_, '\n', static_cast<size_t>(i) + 1);
      if (!q) return -1;
      long k = static_cast<const uint8_t*>(q) - c_;
      if (!censored(k)) return k;
      auto it = std::upper_bound(iv_.begin(), iv_.end(), k, [](long v, const Loc& l) { return v < l.start; });
      --it;
      i = it->start - 1;
    }
    return -1;
  }
  // first censored-buffer '\n' position >= pos, or n
  size_t next_nl(size_t pos) const {
    size_t i = pos;
    while (i < n_) {
      const void* q = memchr(c_ + i, '\n', n_ - i);
      if (!q) return n_;
      size_t k = static_cast<const uint8_t*>(q) - c_;
      if (!censored(static_cast<long>(k))) return k;
      auto it = std::upper_bound(iv_.begin(), iv_.end(), static_cast<long>(k), [](long v, const Loc& l) { return v < l.start; });
      --it;
      i = static_cast<size_t>(it->end);
    }
    return n_;
  }
  // the censored bytes [a, b) appended to `arena` (no temporary string)
  StrRef put(std::string* arena, size_t a, size_t b) const {
    StrRef r{static_cast<uint32_t>(arena->size()), static_cast<uint32_t>(b - a)};
    arena->append(reinterpret_cast<const char*>(c_) + a, b - a);
    char* d = &(*arena)[r.off];
    for (auto it = first_ending_after(a); it != iv_.end() && static_cast<size_t>(it->start) < b; ++it) {
      size_t x = std::max<size_t>(a, it->start), y = std::min<size_t>(b, it->end);
      for (size_t k = x; k < y; ++k) d[k - a] = '*';
    }
    return r;
  }
  size_t size() const { return n_; }

 private:
  const uint8_t* c_;
  size_t n_;
  const std::vector<Loc>& iv_;
  std::vector<uint64_t>& local_;          // local_[k] = '\n' in data_[first_*ch_, (first_+k)*ch_)
  const uint16_t* chunk_nl_ = nullptr;      // per-chunk counts (K1's), summed into local_ on demand
  const uint8_t* data_ = nullptr;
  uint64_t off_ = 0, first_ = 0;
  uint32_t ch_ = 4096;

  // the merged spans are sorted and disjoint: the first one ending after a
  std::vector<Loc>::const_iterator first_ending_after(size_t a) const {
    return std::upper_bound(iv_.begin(), iv_.end(), static_cast<long>(a), [](long v, const Loc& l) { return v < l.end; });
  }
  uint64_t prefix_at(uint64_t g) const {   // '\n' in data_[first_*ch_, g)
    const uint64_t k = g / ch_;
    if (chunk_nl_) {
      while (local_.size() <= k - first_) {   // g <= off_ + n: only chunks below (off_ + n) / ch_ are summed
        const uint64_t j = first_ + local_.size() - 1;
        local_.push_back(local_.back() + chunk_nl_[j]);
      }
    }
    return local_[k - first_] + count_newlines(data_ + k * ch_, g - k * ch_);
  }
  uint64_t orig_nl(size_t a, size_t b) const {
    if (b - a <= 2 * static_cast<size_t>(ch_)) return count_newlines(c_ + a, b - a);
    return prefix_at(off_ + b) - prefix_at(off_ + a);
  }
};

StrRef put(std::string* arena, const std::string& v) {
  StrRef r{static_cast<uint32_t>(arena->size()), static_cast<uint32_t>(v.size())};
  arena->append(v);
  return r;
}

// scanner.go:475-558 on the (virtual) censored buffer; appends to `out`.
void to_finding(const Rule& rule, Loc loc, const CensoredView& cv, SecretBuilder* out) {
  FindingRec f;
  f.rule = &rule;
  const size_t n = cv.size();
  const size_t start = static_cast<size_t>(loc.start), end = static_cast<size_t>(loc.end);
  const size_t start_line = cv.count_nl(0, start);
  const long pn = cv.prev_nl(start);
  const size_t line0_b = pn < 0 ? 0 : static_cast<size_t>(pn) + 1;   // LastIndex('\n') + 1
  const size_t line0_e = cv.next_nl(start);                             // Index('\n') from start
  size_t line_start = line0_b, line_end = line0_e;
  if (line_end - line_start > 100) {
    line_start = (static_cast<long>(start) - static_cast<long>(line_start) - 30 < 0) ? line_start : start - 30;
    line_end = (end + 20 > line_end) ? line_end : end + 20;
  }
  f.match = cv.put(&out->arena, line_start, line_end);
  const size_t end_line = start_line + cv.count_nl(start, end);
  const size_t code_start = start_line >= 2 ? start_line - 2 : 0;
  // lines code_start .. min(end_line + 2, len(lines)) - 1 of bytes.Split of
  // the censored buffer: walking forward, a line ending at n (no '\n' after
  // it) is the last one
  size_t code_end = end_line + 2;
  std::pair<size_t, size_t> lines[8];
  size_t nl = 0;
  {
    std::pair<size_t, size_t> before[2];
    size_t nb = 0;
    size_t b = line0_b;
    for (size_t k = start_line; k > code_start; --k) {   // walk back (at most 2 lines)
      const size_t e = b - 1;                            // the '\n' ending line k-1
      const long q = cv.prev_nl(e);
      const size_t bb = q < 0 ? 0 : static_cast<size_t>(q) + 1;
      before[nb++] = {bb, e};
      b = bb;
    }
    while (nb > 0) lines[nl++] = before[--nb];
    size_t e = line0_e;
    lines[nl++] = {line0_b, line0_e};
    size_t k = start_line + 1;
    for (; k < code_end && nl < 8 && e < n; ++k) {
      const size_t bb = e + 1;
      e = cv.next_nl(bb);
      lines[nl++] = {bb, e};
    }
    code_end = k;
  }
  f.line_begin = static_cast<uint32_t>(out->lines.size());
  bool found_first = false;
  size_t last_cause = SIZE_MAX;
  for (size_t idx = 0; idx < nl; ++idx) {
    const size_t k = code_start + idx;
    if (k >= code_end) break;
    const size_t b = lines[idx].first, e = lines[idx].second;
    const bool in_cause = k >= start_line && k <= end_line;
    LineRec ln;
    ln.number = static_cast<int>(k + 1);
    if (e - b > 100) ln.content = in_cause ? f.match : cv.put(&out->arena, b, b + 100);
    else ln.content = cv.put(&out->arena, b, e);
    ln.is_cause = in_cause;
    ln.first_cause = !found_first && in_cause;
    found_first = found_first || in_cause;
    if (in_cause) last_cause = out->lines.size();
    out->lines.push_back(ln);
  }
  if (last_cause != SIZE_MAX) out->lines[last_cause].last_cause = true;
  f.line_count = static_cast<uint32_t>(out->lines.size()) - f.line_begin;
  f.start_line = static_cast<int>(start_line + 1);
  f.end_line = static_cast<int>(end_line + 1);
  out->findings.push_back(f);
}

bool keywords_match(const Rule& r, const std::string& lower) {   // scanner.go:174-186
  if (r.keywords.empty()) return true;
  for (const auto& kw : r.keywords_lower) {
    if (kw.empty()) return true;
    if (lower.find(kw) != std::string::npos) return true;
  }
  return false;
}

// Case-insensitive (ASCII) search of a lowercase ASCII keyword in raw bytes.
bool ascii_ci_find(const uint8_t* s, size_t n, const std::string& kw) {
  const size_t m = kw.size();
  if (m == 0) return true;
  if (m > n) return false;
  const uint8_t k0 = static_cast<uint8_t>(kw[0]);
  const bool alpha0 = k0 >= 'a' && k0 <= 'z';
  const uint8_t u0 = alpha0 ? static_cast<uint8_t>(k0 - 32) : k0;
  auto at = [&](size_t i) {
    for (size_t j = 1; j < m; ++j) {
      uint8_t b = s[i + j];
      if (b >= 'A' && b <= 'Z') b = static_cast<uint8_t>(b + 32);
      if (b != static_cast<uint8_t>(kw[j])) return false;
    }
    return true;
  };
  const size_t last = n - m;                     // candidate starts 0..last
  size_t i = 0;
  // 16 starts at a time: positions whose byte is the first keyword byte in
  // either case (SSE2 compares), then the rest of the keyword
  const __m128i v0 = _mm_set1_epi8(static_cast<char>(k0)), v1 = _mm_set1_epi8(static_cast<char>(u0));
  for (; i + 16 <= last + 1; i += 16) {
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i));
    uint32_t mask = static_cast<uint32_t>(_mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(x, v0), _mm_cmpeq_epi8(x, v1))));
    while (mask) {
      const size_t k = i + static_cast<size_t>(__builtin_ctz(mask));
      if (at(k)) return true;
      mask &= mask - 1;
    }
  }
  for (; i <= last; ++i) {
    const uint8_t c = s[i];
    if ((c == k0 || c == u0) && at(i)) return true;
  }
  return false;
}

// U+0130 (C4 B0) or U+212A (E2 84 AA): the only runes bytes.ToLower turns
// into ASCII letters ('i', 'k')
bool has_ascii_folding_rune(const uint8_t* s, size_t n) {
  for (const uint8_t* p = s; (p = static_cast<const uint8_t*>(memchr(p, 0xC4, n - (p - s)))) != nullptr; ++p) {
    if (p + 1 < s + n && p[1] == 0xB0) return true;
  }
  for (const uint8_t* p = s; (p = static_cast<const uint8_t*>(memchr(p, 0xE2, n - (p - s)))) != nullptr; ++p) {
    if (p + 2 < s + n && p[1] == 0x84 && p[2] == 0xAA) return true;
  }
  return false;
}

// MatchKeywords (scanner.go:174-186) without the lowered copy where the raw
// bytes decide it: ASCII bytes are single runes that bytes.ToLower keeps in
// place (A-Z lowered), so an ASCII keyword found case-insensitively in the raw
// bytes is in the lowered text; if it is not found, only U+0130 / U+212A can
// still produce it, and files without them are decided too.  Everything else
// (non-ASCII keywords, files with those runes) takes the exact lowered path.
template <typename Lowered>
bool keywords_match_raw(const Rule& r, const uint8_t* content, size_t len, Lowered&& lowered) {
  if (r.keywords.empty()) return true;
  bool undecided = false;
  for (const auto& kw : r.keywords_lower) {
    if (kw.empty()) return true;
    bool ascii = true;
    for (unsigned char c : kw) ascii &= c < 0x80;
    if (!ascii) { undecided = true; continue; }
    if (ascii_ci_find(content, len, kw)) return true;
  }
  if (!undecided && !has_ascii_folding_rune(content, len)) return false;
  return keywords_match(r, lowered());
}

}  // namespace

std::atomic<bool> g_scan_prof_on{false};

namespace {
struct Matched { const Rule* rule; Loc loc; };
}  // namespace
std::atomic<uint64_t> g_scan_prof[8];   // phase ns [0..4]; [5] ns of whole-file find-alls, [7] their count

namespace {
struct PhaseClock {
  bool on = g_scan_prof_on.load(std::memory_order_relaxed);
  uint64_t acc[5] = {0, 0, 0, 0, 0};
  std::chrono::steady_clock::time_point t = on ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  void lap(int k) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    acc[k] += static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(n - t).count());
    t = n;
  }
  ~PhaseClock() {
    if (on) for (int k = 0; k < 5; ++k) if (acc[k]) g_scan_prof[k].fetch_add(acc[k], std::memory_order_relaxed);
  }
};
}  // namespace

Secret scan_file(const Ruleset& rs, std::string path, const uint8_t* content, size_t len,
                 bool binary, const FilePlan* plan, const NlSource* nl) {
  return scan_file(rs, path.data(), path.size(), content, len, binary, plan, nl);
}

// (the path by pointer and length: it is copied into the per-thread builder,
// whose buffer is reused from file to file -- the engine's confirm pool made a
// std::string of every confirmed file's path, a heap allocation and a free per
// file once paths pass 15 bytes)
Secret scan_file(const Ruleset& rs, const char* path_p, size_t path_n, const uint8_t* content, size_t len,
                 bool binary, const FilePlan* plan, const NlSource* nl) {
  PhaseClock pc;
  if (global_allow_path(rs, reinterpret_cast<const uint8_t*>(path_p), path_n))
    return Secret::path_only(path_p, path_n);    // scanner.go:381-386
  thread_local SecretBuilder out_tl;             // (per-thread: no allocation per file once warm)
  SecretBuilder& out = out_tl;
  out.clear();
  out.file_path.assign(path_p, path_n);
  const std::string& path = out.file_path;
  std::string lower;
  bool have_lower = false;
  auto lowered = [&]() -> const std::string& {
    if (!have_lower) { lower = go_bytes_to_lower(content, len); have_lower = true; }
    return lower;
  };
  Blocks gblocks(content, len, rs.exclude_block, plan, rs.rules.size());
  // per-thread working vectors (kept across files: no allocation per file)
  thread_local std::vector<Matched> matched_tl;
  thread_local std::vector<Loc> locs_tl, spans_tl;
  thread_local std::vector<uint64_t> nl_tl;
  std::vector<Matched>& matched = matched_tl;
  std::vector<Loc>& locs = locs_tl;
  matched.clear();
  size_t cand_i = 0;
  const bool listed = plan && plan->active_set;
  const size_t niter = listed ? plan->active.size() : rs.rules.size();
  for (size_t it = 0; it < niter; ++it) {
    const size_t ri = listed ? plan->active[it] : it;
    if (ri >= rs.rules.size()) break;                // exclude-regex pseudo-rules (listed last)
    const Rule& rule = rs.rules[ri];
    const uint8_t kind = plan ? plan->kind[ri] : static_cast<uint8_t>(kPlanFull);
    const std::vector<uint64_t>* starts = nullptr;
    if (plan) {
      while (cand_i < plan->cands.size() && plan->cands[cand_i].rule < ri) ++cand_i;
      if (cand_i < plan->cands.size() && plan->cands[cand_i].rule == ri) starts = &plan->cands[cand_i].starts;
    }
    // rules the plan rules out (gate false, no match possible, or a
    // host-gated rule without candidate starts) add nothing whatever their
    // path filters say: skipped before the path regexes
    if (kind == kPlanSkip || kind == kPlanNoMatch) continue;
    if (kind == kPlanCandHostGate && (!starts || starts->empty())) continue;
    if (rule.path && !rule.path->match_string(reinterpret_cast<const uint8_t*>(path.data()), path.size())) continue;
    if (allow_path(rule.allow_rules, path)) continue;
    pc.lap(0);
    const bool kw_ok = !(kind == kPlanFull || kind == kPlanCandHostGate) || keywords_match_raw(rule, content, len, lowered);
    pc.lap(0);
    if (!kw_ok) continue;
    locs.clear();
    static const std::vector<uint64_t> kEmpty;
    const std::vector<uint64_t>* use = nullptr;
    if (kind == kPlanCandidates || kind == kPlanCandHostGate) use = starts ? starts : &kEmpty;
    if (pc.on && !use) {
      const auto tf = std::chrono::steady_clock::now();
      find_locations(rs, rule, content, len, use, &locs, &out.error);
      g_scan_prof[5].fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tf).count());
      g_scan_prof[7].fetch_add(1);
    } else {
      find_locations(rs, rule, content, len, use, &locs, &out.error);
    }
    pc.lap(1);
    if (locs.empty()) continue;
    Blocks lblocks(content, len, rule.exclude_block, plan, rs.rules.size() + rule.exclude_base);
    for (const Loc& l : locs) {
      if (l.start < 0) continue;                      // reference panics here (error flagged)
      if (gblocks.match(l) || lblocks.match(l)) continue;
      matched.push_back({&rule, l});                  // censorLocation: applied virtually below
    }
    pc.lap(2);
  }
  if (matched.empty()) {                              // types.Secret{}
    Secret empty;
    empty.error = out.error;
    return empty;
  }
  std::vector<Loc>& spans = spans_tl;
  spans.clear();
  for (const auto& m : matched) spans.push_back(m.loc);
  CensoredView cv(content, len, spans, nl_tl, nl);
  for (const auto& m : matched) {
    to_finding(*m.rule, m.loc, cv, &out);
    if (binary) {                                     // scanner.go:440-444
      FindingRec& f = out.findings.back();
      out.lines.resize(f.line_begin);
      f.line_count = 0;
      f.match = put(&out.arena, "Binary file " + go_quote(path) + " matches a rule " + go_quote(m.rule->title));
    }
  }
  pc.lap(3);
  auto& fs = out.findings;
  const std::string& ar = out.arena;
  GoSort<FindingRec>(&fs, [&fs, &ar](size_t i, size_t j) {
    if (fs[i].rule->id != fs[j].rule->id) return fs[i].rule->id < fs[j].rule->id;
    return ar.compare(fs[i].match.off, fs[i].match.len, ar, fs[j].match.off, fs[j].match.len) < 0;
  }).run();
  Secret res = Secret::build(out);
  pc.lap(4);
  return res;
}

Secret Secret::build(const SecretBuilder& b) {
  Secret s;
  s.error = b.error;
  if (b.file_path.empty() && b.findings.empty()) return s;
  const size_t nf = b.findings.size(), nl = b.lines.size();
  const size_t bytes = kHdr + nf * sizeof(FindingRec) + nl * sizeof(LineRec) + b.file_path.size() + b.arena.size();
  char* blk = static_cast<char*>(std::malloc(bytes));
  if (!blk) throw std::bad_alloc();
  Hdr h{static_cast<uint32_t>(nf), static_cast<uint32_t>(nl), static_cast<uint32_t>(b.file_path.size()),
        static_cast<uint32_t>(b.arena.size())};
  std::memcpy(blk, &h, kHdr);
  char* q = blk + kHdr;
  if (nf) std::memcpy(q, b.findings.data(), nf * sizeof(FindingRec));
  q += nf * sizeof(FindingRec);
  if (nl) std::memcpy(q, b.lines.data(), nl * sizeof(LineRec));
  q += nl * sizeof(LineRec);
  if (!b.file_path.empty()) std::memcpy(q, b.file_path.data(), b.file_path.size());
  q += b.file_path.size();
  if (!b.arena.empty()) std::memcpy(q, b.arena.data(), b.arena.size());
  s.blk_ = blk;
  return s;
}

Secret Secret::path_only(const char* p, size_t n) {
  Secret s;
  if (n == 0) return s;
  char* blk = static_cast<char*>(std::malloc(kHdr + n));
  if (!blk) throw std::bad_alloc();
  Hdr h{0, 0, static_cast<uint32_t>(n), 0};
  std::memcpy(blk, &h, kHdr);
  std::memcpy(blk + kHdr, p, n);
  s.blk_ = blk;
  return s;
}

}  // namespace tsg

namespace tsg {

namespace {
// Result blocks of 4 MiB and more are 2 MiB-aligned and marked for
// transparent huge pages: 297k result slots (36 MB) were 9k page faults,
// 2.2 ms even on 8 threads before a resident config-5 step could confirm
// its first piece (profiles/rd4x_bench_c5prof.log).  Smaller blocks use new.
constexpr size_t kHugeBlock = 4u << 20, kHugePage = 2u << 20;
void* block_alloc(size_t bytes) {
  if (bytes < kHugeBlock) return ::operator new(bytes);
  const size_t n = (bytes + kHugePage - 1) & ~(kHugePage - 1);
  void* p = std::aligned_alloc(kHugePage, n);
  if (!p) throw std::bad_alloc();
  madvise(p, n, MADV_HUGEPAGE);                  // a hint: no effect where THP is off
  return p;
}
void block_free(void* p, size_t bytes) {
  if (!p) return;
  if (bytes < kHugeBlock) ::operator delete(p);
  else std::free(p);
}
}  // namespace

void SecretVec::reserve(size_t c) {
  if (c <= cap_) return;
  Secret* q = static_cast<Secret*>(block_alloc(c * sizeof(Secret)));
  for (size_t i = 0; i < n_; ++i) {
    new (q + i) Secret(std::move(p_[i]));
    p_[i].~Secret();
  }
  block_free(p_, cap_ * sizeof(Secret));
  p_ = q;
  cap_ = c;
}

void SecretVec::clear() {
  for (size_t i = 0; i < n_; ++i) p_[i].~Secret();
  n_ = 0;
}

void SecretVec::destroy() {
  clear();
  block_free(p_, cap_ * sizeof(Secret));
  p_ = nullptr;
  cap_ = 0;
}

void SecretVec::resize(size_t n) {
  if (n <= n_) {
    for (size_t i = n; i < n_; ++i) p_[i].~Secret();
    n_ = n;
    return;
  }
  reserve(n);
  const size_t add = n - n_;
  constexpr size_t kPerThread = 32768;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t nt = std::min<size_t>({add / kPerThread, 8, hw});
  // exception safety (a Secret() that throws bad_alloc): every element
  // constructed before the throw is destroyed again before it propagates, so
  // n_ still describes the live range and a retried resize starts clean
  if (nt <= 1) {
    size_t i = n_;
    try {
      for (; i < n; ++i) new (p_ + i) Secret();
    } catch (...) {
      for (size_t k = n_; k < i; ++k) p_[k].~Secret();
      throw;
    }
  } else {
    const size_t per = (add + nt - 1) / nt;
    std::vector<size_t> built(nt, 0);                // elements constructed in each block
    std::atomic<size_t> next{0};
    try {
      run_threads(static_cast<int>(nt), [&] {
        for (size_t t; (t = next.fetch_add(1)) < nt;) {
          const size_t a = n_ + t * per, b = std::min(n, a + per);
          for (size_t i = a; i < b; ++i) {
            new (p_ + i) Secret();
            built[t] = i + 1 - a;
          }
        }
      });
    } catch (...) {
      for (size_t t = 0; t < nt; ++t)
        for (size_t k = 0; k < built[t]; ++k) p_[n_ + t * per + k].~Secret();
      throw;
    }
  }
  n_ = n;
}

}  // namespace tsg

extern "C" const char* tsg_builtin_json_ptr() { return tsg::kBuiltinRulesJson; }
