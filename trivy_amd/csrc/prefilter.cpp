// Rule -> GPU table compiler.  See prefilter.h for what is produced and
// DESIGN.md ("Why candidates are a superset") for the correctness argument.
#include "prefilter.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <bitset>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>

namespace tsg {

using re::Node;
using re::Op;

namespace {

constexpr uint32_t kInf = 0x3fffffff;
constexpr int kMaxSetSize = 64;          // literal-set cap
constexpr int kMaxUnits = 6;             // literal length cap (units): longer adds DFA states, little selectivity
constexpr uint32_t kMaxPrefixBytes = 96; // dmax cap for a usable anchor
constexpr uint32_t kVerifyStateCap = 3000;
constexpr uint32_t kScanStateCap = 60000;
// K2 gives up on a verify walk after this many bytes and passes the start on
// (the host decides it exactly): one thread walking an exclude block's
// `.*?END NOSCAN` over 8 KiB held a 3 GB config-5 piece's K2 for 2.4 ms
// (profiles/rd4z_bench_c5k2.log, max_hit_bytes 8193).  Round 5: 1024 -> 64
// bytes: a K2 launch lasts as long as its longest walk (one dependent
// transition per byte), and the few walks past 64 bytes (lane maxima p90 66,
// max 159 on config 2) set it: K2 per 4 GB 0.378 -> 0.338 ms, per resident
// step config 2 1.45 -> 1.27 ms, config 5 1.69 -> 1.26 ms, for +2% / +0.8%
// host candidates (profiles/r6x_verify_cap.log)
constexpr uint32_t kVerifyLimitCap = 64;
constexpr double kWeakAnchor = 3.0;
constexpr size_t kHostKeywordLen = 3;     // keywords this short gate on the host      // literal anchors scoring below this get class extensions

using Bits = std::bitset<256>;

// ------------------------------------------------------------------ NFA
struct NState {
  std::vector<int> eps;
  std::vector<std::pair<int, int>> edges;   // (set index, target)
  int out = -1;                             // scan: output id; verify: 0 = accept
};

struct Nfa {
  bool rev = false;                         // build the reversed language (reverse anchors, mode 4)
  std::vector<NState> st;
  std::vector<Bits> sets;
  std::map<std::string, int> set_index;
  int add() { st.emplace_back(); return static_cast<int>(st.size()) - 1; }
  void eps(int a, int b) { st[a].eps.push_back(b); }
  int set_id(const Bits& b) {
    std::string k = b.to_string();
    auto it = set_index.find(k);
    if (it != set_index.end()) return it->second;
    sets.push_back(b);
    int id = static_cast<int>(sets.size()) - 1;
    set_index.emplace(std::move(k), id);
    return id;
  }
  void edge(int a, const Bits& b, int to) { st[a].edges.push_back({set_id(b), to}); }
  void byte_chain(int from, const std::string& fwd, int to) {
    const std::string bytes = rev ? std::string(fwd.rbegin(), fwd.rend()) : fwd;
    int cur = from;
    for (size_t i = 0; i < bytes.size(); ++i) {
      int nx = (i + 1 == bytes.size()) ? to : add();
      Bits b;
      b.set(static_cast<uint8_t>(bytes[i]));
      edge(cur, b, nx);
      cur = nx;
    }
    if (bytes.empty()) eps(from, to);
  }
  // [\x80-\xFF]{1,4}: any non-ASCII rune (valid 2-4 byte sequence or an invalid byte)
  void high_unit(int from, int to) {
    Bits hi;
    for (int c = 0x80; c < 256; ++c) hi.set(c);
    int cur = from;
    for (int k = 0; k < 4; ++k) {
      int nx = add();
      edge(cur, hi, nx);
      eps(nx, to);
      cur = nx;
    }
  }
};

std::string utf8(uint32_t r) { std::string s; re::append_utf8(&s, r); return s; }

uint64_t class_size(const Node& n) {
  uint64_t c = 0;
  for (const auto& r : n.ranges) c += static_cast<uint64_t>(r.hi) - r.lo + 1;
  return c;
}

// Relaxed rune class -> NFA fragment from `from` to `to`.
void class_frag(Nfa* nfa, const std::vector<re::Range>& ranges, int from, int to) {
  Bits ascii;
  uint64_t nonascii = 0;
  bool has_fffd = false;
  std::vector<uint32_t> small;
  for (const auto& r : ranges) {
    for (uint32_t c = r.lo; c <= std::min<uint32_t>(r.hi, 0x7f); ++c) ascii.set(c);
    if (r.hi >= 0x80) {
      uint32_t lo = std::max<uint32_t>(r.lo, 0x80);
      nonascii += r.hi - lo + 1;
      if (lo <= 0xFFFD && 0xFFFD <= r.hi) has_fffd = true;
      if (nonascii <= 16) for (uint32_t c = lo; c <= r.hi; ++c) small.push_back(c);
    }
  }
  if (ascii.any()) nfa->edge(from, ascii, to);
  if (nonascii == 0) return;
  if (nonascii <= 16 && !has_fffd) {
    for (uint32_t c : small) nfa->byte_chain(from, utf8(c), to);
  } else {
    nfa->high_unit(from, to);
  }
}

// Relaxed (superset) NFA of an AST node.
int build(Nfa* nfa, const Node& n, int from);

int build_repeat(Nfa* nfa, const Node& sub, int mn, int mx, int from) {
  // relaxation: X{m,n} with m > 64 or n-m > 8 becomes X{min(m,64)}X*
  int m = std::min(mn, 64);
  bool loose = mx < 0 || mn > 64 || (mx - mn) > 8;
  int cur = from;
  for (int k = 0; k < m; ++k) cur = build(nfa, sub, cur);
  if (loose) {
    int loop = nfa->add();
    nfa->eps(cur, loop);
    int body_end = build(nfa, sub, loop);
    nfa->eps(body_end, loop);
    return loop;
  }
  int end = nfa->add();
  nfa->eps(cur, end);
  for (int k = m; k < mx; ++k) {
    cur = build(nfa, sub, cur);
    nfa->eps(cur, end);
  }
  return end;
}

int build(Nfa* nfa, const Node& n, int from) {
  switch (n.op) {
    case Op::NoMatch: {
      return nfa->add();   // unreachable end
    }
    case Op::EmptyMatch: case Op::BeginLine: case Op::EndLine: case Op::BeginText:
    case Op::EndText: case Op::WordBoundary: case Op::NoWordBoundary:
      return from;
    case Op::Literal: {
      int to = nfa->add();
      if (n.rune < 0x80) { Bits b; b.set(n.rune); nfa->edge(from, b, to); }
      else nfa->byte_chain(from, utf8(n.rune), to);
      return to;
    }
    case Op::CharClass: {
      int to = nfa->add();
      class_frag(nfa, n.ranges, from, to);
      return to;
    }
    case Op::AnyCharNotNL: {
      int to = nfa->add();
      class_frag(nfa, {{0, 9}, {11, 0x10FFFF}}, from, to);
      return to;
    }
    case Op::AnyChar: {
      int to = nfa->add();
      class_frag(nfa, {{0, 0x10FFFF}}, from, to);
      return to;
    }
    case Op::Capture:
      return build(nfa, *n.sub[0], from);
    case Op::Concat: {
      int cur = from;
      if (nfa->rev) for (size_t i = n.sub.size(); i-- > 0;) cur = build(nfa, *n.sub[i], cur);
      else for (const auto& s : n.sub) cur = build(nfa, *s, cur);
      return cur;
    }
    case Op::Alternate: {
      int end = nfa->add();
      for (const auto& s : n.sub) {
        int st = nfa->add();
        nfa->eps(from, st);
        nfa->eps(build(nfa, *s, st), end);
      }
      return end;
    }
    case Op::Star: return build_repeat(nfa, *n.sub[0], 0, -1, from);
    case Op::Plus: return build_repeat(nfa, *n.sub[0], 1, -1, from);
    case Op::Quest: return build_repeat(nfa, *n.sub[0], 0, 1, from);
    case Op::Repeat: return build_repeat(nfa, *n.sub[0], n.min, n.max, from);
  }
  return from;
}

// Byte-length bounds of a match of n (relaxed; runes >= 0x80 may be 1..4 bytes).
void len_bounds(const Node& n, uint32_t* lo, uint32_t* hi) {
  auto add = [](uint32_t a, uint32_t b) { return (a >= kInf || b >= kInf) ? kInf : std::min(a + b, kInf); };
  auto mul = [](uint32_t a, uint32_t k) { return a >= kInf ? kInf : static_cast<uint32_t>(std::min<uint64_t>(static_cast<uint64_t>(a) * k, kInf)); };
  switch (n.op) {
    case Op::NoMatch: *lo = kInf; *hi = 0; return;
    case Op::EmptyMatch: case Op::BeginLine: case Op::EndLine: case Op::BeginText:
    case Op::EndText: case Op::WordBoundary: case Op::NoWordBoundary:
      *lo = *hi = 0; return;
    case Op::Literal: *lo = *hi = static_cast<uint32_t>(utf8(n.rune).size()); return;
    case Op::CharClass: {
      bool ascii = false, non = false;
      for (const auto& r : n.ranges) { if (r.lo < 0x80) ascii = true; if (r.hi >= 0x80) non = true; }
      *lo = ascii ? 1 : (non ? 1 : kInf);
      *hi = non ? 4 : 1;
      return;
    }
    case Op::AnyCharNotNL: case Op::AnyChar: *lo = 1; *hi = 4; return;
    case Op::Capture: len_bounds(*n.sub[0], lo, hi); return;
    case Op::Concat: {
      uint32_t a = 0, b = 0;
      for (const auto& s : n.sub) { uint32_t x, y; len_bounds(*s, &x, &y); a = add(a, x); b = add(b, y); }
      *lo = a; *hi = b; return;
    }
    case Op::Alternate: {
      uint32_t a = kInf, b = 0;
      for (const auto& s : n.sub) { uint32_t x, y; len_bounds(*s, &x, &y); a = std::min(a, x); b = std::max(b, y); }
      *lo = a; *hi = b; return;
    }
    case Op::Star: { uint32_t x, y; len_bounds(*n.sub[0], &x, &y); *lo = 0; *hi = y == 0 ? 0 : kInf; return; }
    case Op::Plus: { uint32_t x, y; len_bounds(*n.sub[0], &x, &y); *lo = x; *hi = y == 0 ? 0 : kInf; return; }
    case Op::Quest: { uint32_t x, y; len_bounds(*n.sub[0], &x, &y); *lo = 0; *hi = y; return; }
    case Op::Repeat: {
      uint32_t x, y; len_bounds(*n.sub[0], &x, &y);
      *lo = mul(x, n.min);
      *hi = n.max < 0 ? (y == 0 ? 0 : kInf) : mul(y, n.max);
      return;
    }
  }
  *lo = 0; *hi = kInf;
}

// --------------------------------------------------------- literal sets
using Unit = std::vector<std::string>;     // sorted alternative byte strings
using Seq = std::vector<Unit>;
using SeqSet = std::set<Seq>;

bool small_class(const Node& n, Unit* u) {
  if (class_size(n) > 4) return false;
  for (const auto& r : n.ranges)
    for (uint32_t c = r.lo; c <= r.hi; ++c) {
      if (c == 0xFFFD) return false;       // would also stand for every invalid byte
      u->push_back(utf8(c));
    }
  std::sort(u->begin(), u->end());
  return true;
}

bool cross(const SeqSet& a, const SeqSet& b, SeqSet* out) {
  out->clear();
  for (const auto& x : a) {
    for (const auto& y : b) {
      Seq s = x;
      for (const auto& u : y) { if (static_cast<int>(s.size()) >= kMaxUnits) break; s.push_back(u); }
      out->insert(std::move(s));
      if (static_cast<int>(out->size()) > kMaxSetSize) return false;
    }
  }
  return true;
}

// Exact finite set of literal sequences matched by n, if small.
bool finite_set(const Node& n, SeqSet* out) {
  out->clear();
  switch (n.op) {
    case Op::EmptyMatch: case Op::BeginLine: case Op::EndLine: case Op::BeginText:
    case Op::EndText: case Op::WordBoundary: case Op::NoWordBoundary:
      out->insert(Seq{});
      return true;
    case Op::Literal: out->insert(Seq{Unit{utf8(n.rune)}}); return true;
    case Op::CharClass: {
      Unit u;
      if (!small_class(n, &u)) return false;
      out->insert(Seq{u});
      return true;
    }
    case Op::Capture: return finite_set(*n.sub[0], out);
    case Op::Concat: {
      SeqSet acc{Seq{}};
      for (const auto& s : n.sub) {
        SeqSet f, t;
        if (!finite_set(*s, &f)) return false;
        if (!cross(acc, f, &t)) return false;
        acc.swap(t);
      }
      *out = std::move(acc);
      return true;
    }
    case Op::Alternate: {
      for (const auto& s : n.sub) {
        SeqSet f;
        if (!finite_set(*s, &f)) return false;
        out->insert(f.begin(), f.end());
        if (static_cast<int>(out->size()) > kMaxSetSize) return false;
      }
      return true;
    }
    case Op::Quest: {
      SeqSet f;
      if (!finite_set(*n.sub[0], &f)) return false;
      *out = std::move(f);
      out->insert(Seq{});
      return static_cast<int>(out->size()) <= kMaxSetSize;
    }
    case Op::Repeat: {
      if (n.max < 0 || n.max > 4) return false;
      SeqSet f;
      if (!finite_set(*n.sub[0], &f)) return false;
      SeqSet acc{Seq{}}, all;
      for (int k = 0; k <= n.max; ++k) {
        if (k >= n.min) all.insert(acc.begin(), acc.end());
        SeqSet t;
        if (!cross(acc, f, &t)) return false;
        acc.swap(t);
      }
      *out = std::move(all);
      return static_cast<int>(out->size()) <= kMaxSetSize;
    }
    default:
      return false;
  }
}

// A character class of ASCII characters only, as one unit of single-byte
// alternatives (anchor extensions: a weak literal followed by such a class).
bool class_unit(const Node& n, Unit* u) {
  if (n.op != Op::CharClass) return false;
  for (const auto& r : n.ranges) {
    if (r.hi >= 0x80) return false;
    for (uint32_t c = r.lo; c <= r.hi; ++c) u->push_back(std::string(1, static_cast<char>(c)));
  }
  return !u->empty() && u->size() <= 96;
}

// Set of sequences one of which begins every match of items[k..] (Seq{} = no
// info).  ext: a class item that ends the literal part contributes up to
// kExtUnits class units (used for weak anchors only: they add scan states).
int ext_units() {
  static const int n = [] { const char* e = std::getenv("TSG_ANCHOR_EXT"); return e ? std::atoi(e) : 0; }();
  return n;
}
// Reverse anchors (mode 4) on unless TSG_REVERSE_ANCHORS=0.
bool ext_rev() {
  static const bool on = [] { const char* e = std::getenv("TSG_REVERSE_ANCHORS"); return !e || std::atoi(e) != 0; }();
  return on;
}
SeqSet prefix_of_items(const std::vector<const Node*>& items, size_t k, bool ext = false);

SeqSet prefix_set(const Node& n, bool ext = false) {
  SeqSet f;
  if (finite_set(n, &f)) return f;
  Unit u;
  switch (n.op) {
    case Op::Capture: return prefix_set(*n.sub[0], ext);
    case Op::Concat: {
      std::vector<const Node*> items;
      for (const auto& s : n.sub) items.push_back(s.get());
      return prefix_of_items(items, 0, ext);
    }
    case Op::Alternate: {
      SeqSet out;
      for (const auto& s : n.sub) {
        SeqSet p = prefix_set(*s, ext);
        out.insert(p.begin(), p.end());
        if (static_cast<int>(out.size()) > kMaxSetSize) return SeqSet{Seq{}};
      }
      return out;
    }
    case Op::CharClass:
      if (ext && ext_units() > 0 && class_unit(n, &u)) return SeqSet{Seq{u}};
      return SeqSet{Seq{}};
    case Op::Plus: return prefix_set(*n.sub[0], ext);
    case Op::Repeat:
      if (n.min < 1) return SeqSet{Seq{}};
      if (ext && class_unit(*n.sub[0], &u)) return SeqSet{Seq(std::min(n.min, ext_units()), u)};
      return prefix_set(*n.sub[0], ext);
    default: return SeqSet{Seq{}};
  }
}

SeqSet prefix_of_items(const std::vector<const Node*>& items, size_t k, bool ext) {
  SeqSet acc{Seq{}};
  for (size_t i = k; i < items.size(); ++i) {
    SeqSet f, t;
    if (finite_set(*items[i], &f)) {
      if (!cross(acc, f, &t)) return acc;   // keep what we have (still a valid prefix set)
      acc.swap(t);
      continue;
    }
    SeqSet p = prefix_set(*items[i], ext);
    if (!cross(acc, p, &t)) return acc;
    acc.swap(t);
    break;
  }
  return acc;
}

void flatten(const Node& n, std::vector<const Node*>* items) {
  if (n.op == Op::Concat) { for (const auto& s : n.sub) flatten(*s, items); return; }
  if (n.op == Op::Capture) { flatten(*n.sub[0], items); return; }
  items->push_back(&n);
}

uint32_t seq_min_len(const Seq& s) {
  uint32_t l = 0;
  for (const auto& u : s) { size_t m = 1000; for (const auto& a : u) m = std::min(m, a.size()); l += static_cast<uint32_t>(m); }
  return l;
}
uint32_t seq_max_len(const Seq& s) {
  uint32_t l = 0;
  for (const auto& u : s) { size_t m = 0; for (const auto& a : u) m = std::max(m, a.size()); l += static_cast<uint32_t>(m); }
  return l;
}

// Selectivity score of a literal unit sequence: longer and case-sensitive is better.
// "abc" for single-string units, "(a|A)" for alternatives (report only)
std::string seq_str(const Seq& s) {
  std::string o;
  auto esc = [&](const std::string& b) {
    for (unsigned char c : b) {
      if (c >= 0x20 && c < 0x7f && c != '|' && c != '(' && c != ')' && c != '\\') o.push_back(static_cast<char>(c));
      else { char t[8]; snprintf(t, sizeof t, "\\x%02x", c); o += t; }
    }
  };
  for (const auto& u : s) {
    if (u.size() == 1) { esc(u[0]); continue; }
    o.push_back('(');
    for (size_t i = 0; i < u.size(); ++i) { if (i) o.push_back('|'); esc(u[i]); }
    o.push_back(')');
  }
  return o;
}

std::string seqs_str(const SeqSet& ss) {
  std::string o;
  for (const auto& s : ss) { if (!o.empty()) o += " "; o += seq_str(s); }
  return o;
}

double seq_score(const Seq& s) {
  double sc = 0;
  for (const auto& u : s) {
    if (u.size() > 8) { sc += 0.3; continue; }      // a class unit (anchor extension)
    const char c = static_cast<char>(tolower(static_cast<unsigned char>(u[0][0])));
    bool common = u[0].size() == 1 && strchr(" etaoinsr\"'=:_-.,", c) != nullptr;
    sc += common ? 0.7 : 1.0;
  }
  return sc;
}

// --------------------------------------------------------- DFA building
struct ClassMap { uint8_t cls[256]; uint32_t n; };

ClassMap byte_classes(const Nfa& nfa) {
  std::map<std::vector<bool>, uint8_t> sig;
  ClassMap cm;
  for (int b = 0; b < 256; ++b) {
    std::vector<bool> s(nfa.sets.size());
    for (size_t i = 0; i < nfa.sets.size(); ++i) s[i] = nfa.sets[i].test(b);
    auto it = sig.find(s);
    if (it == sig.end()) it = sig.emplace(s, static_cast<uint8_t>(sig.size())).first;
    cm.cls[b] = it->second;
  }
  cm.n = static_cast<uint32_t>(sig.size());
  return cm;
}

void closure(const Nfa& nfa, std::vector<int>* set) {
  std::vector<int> stack(set->begin(), set->end());
  std::vector<char> in(nfa.st.size(), 0);
  for (int s : *set) in[s] = 1;
  while (!stack.empty()) {
    int s = stack.back();
    stack.pop_back();
    for (int t : nfa.st[s].eps) if (!in[t]) { in[t] = 1; set->push_back(t); stack.push_back(t); }
  }
  std::sort(set->begin(), set->end());
}

struct RawDfa {
  std::vector<std::vector<int>> subsets;
  std::vector<std::vector<uint32_t>> next;   // per state, per class
  ClassMap cm;
};

// Subset construction.  `loop_start`: scan DFA (the start closure is re-added
// after every byte).  `absorb_accept`: verify DFA (accepting subsets stop).
bool determinize(const Nfa& nfa, int start, bool loop_start, int accept_state, uint32_t cap, RawDfa* out,
                 bool absorb_accept = true) {
  out->cm = byte_classes(nfa);
  const uint32_t C = out->cm.n;
  std::vector<int> s0{start};
  closure(nfa, &s0);
  std::map<std::vector<int>, uint32_t> ids;
  out->subsets.push_back(s0);
  ids[s0] = 0;
  // representative byte of each class
  std::vector<int> rep(C, -1);
  for (int b = 0; b < 256; ++b) if (rep[out->cm.cls[b]] < 0) rep[out->cm.cls[b]] = b;
  for (size_t i = 0; i < out->subsets.size(); ++i) {
    if (out->subsets.size() > cap) return false;
    std::vector<uint32_t> row(C, 0);
    const std::vector<int> cur = out->subsets[i];
    bool acc = absorb_accept && accept_state >= 0 && std::binary_search(cur.begin(), cur.end(), accept_state);
    for (uint32_t c = 0; c < C; ++c) {
      std::vector<int> nx;
      if (acc) { row[c] = static_cast<uint32_t>(i); continue; }
      std::vector<char> seen(0);
      for (int s : cur) {
        for (const auto& e : nfa.st[s].edges) {
          if (nfa.sets[e.first].test(rep[c])) nx.push_back(e.second);
        }
      }
      if (loop_start) nx.push_back(start);
      std::sort(nx.begin(), nx.end());
      nx.erase(std::unique(nx.begin(), nx.end()), nx.end());
      closure(nfa, &nx);
      auto it = ids.find(nx);
      uint32_t id;
      if (it == ids.end()) {
        id = static_cast<uint32_t>(out->subsets.size());
        ids.emplace(nx, id);
        out->subsets.push_back(std::move(nx));
      } else {
        id = it->second;
      }
      row[c] = id;
    }
    out->next.push_back(std::move(row));
  }
  return true;
}

// Add a literal unit sequence as a chain into the scan NFA; returns max bytes.
uint32_t add_seq(Nfa* nfa, int start, const Seq& s, int out_id) {
  int cur = start;
  uint32_t maxb = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    int nx = nfa->add();
    size_t m = 0;
    for (const auto& alt : s[i]) { nfa->byte_chain(cur, alt, nx); m = std::max(m, alt.size()); }
    maxb += static_cast<uint32_t>(m);
    cur = nx;
  }
  nfa->st[cur].out = out_id;
  return maxb;
}

// Scan-DFA unit for one ASCII byte: the byte and, for letters, its other case.
Unit folded_unit(unsigned char c) {
  Unit u;
  u.push_back(std::string(1, static_cast<char>(c)));
  if (c >= 'a' && c <= 'z') u.push_back(std::string(1, static_cast<char>(c - 32)));
  if (c >= 'A' && c <= 'Z') u.push_back(std::string(1, static_cast<char>(c + 32)));
  std::sort(u.begin(), u.end());
  return u;
}

// Keyword (already strings.ToLower'ed, ASCII) under bytes.ToLower semantics.
// The two non-ASCII runes that lower to ASCII (U+0130 -> 'i', U+212A -> 'k')
// are only in the host variant DFA: K1 flags files containing them.
Seq keyword_seq(const std::string& kw, bool variants) {
  Seq s;
  for (char ch : kw) {
    Unit u = folded_unit(static_cast<unsigned char>(ch));
    if (variants && ch == 'i') u.push_back("\xC4\xB0");
    if (variants && ch == 'k') u.push_back("\xE2\x84\xAA");
    std::sort(u.begin(), u.end());
    s.push_back(u);
  }
  return s;
}

// Anchor literals of at most TSG_EXACT_ANCHORS units (default 3; 0 = none)
// keep the regex's own case: a case-sensitive `SK` or `pk.` then fires only on
// that case, while (?i) units already list both cases.  Longer ones are
// case-folded (a superset; the verify DFA re-checks case).
int exact_anchors() {
  static const int n = [] { const char* e = std::getenv("TSG_EXACT_ANCHORS"); return e ? std::atoi(e) : 3; }();
  return n;
}

// Scan-DFA form of an anchor literal: the unit's ASCII alternatives (or, with
// exact_anchors() off, every unit case-folded over ASCII: a superset; the
// verify DFA re-checks case).  Non-ASCII alternatives that are
// the fold images of ASCII letters (U+212A, U+017F) are dropped -- files that
// contain them are flagged by K1 and scanned exactly on the host.  The literal
// is cut before any unit with another non-ASCII alternative.
Seq scan_form(const Seq& lit, bool keep_special = false) {
  Seq out;
  // exact case only for short literals: they fire most often, and folded
  // long literals share their trie states with the (folded) keywords
  const int ex = exact_anchors();
  const bool exact = ex != 0 && (ex >= 99 || static_cast<int>(lit.size()) <= ex);
  for (const Unit& u : lit) {
    Unit f;
    bool ok = true;
    for (const auto& alt : u) {
      if (alt == "\xE2\x84\xAA" || alt == "\xC5\xBF") { if (keep_special) f.push_back(alt); continue; }
      if (alt.size() != 1 || static_cast<unsigned char>(alt[0]) >= 0x80) { ok = false; break; }
      if (exact) f.push_back(alt);
      else for (const auto& x : folded_unit(static_cast<unsigned char>(alt[0]))) f.push_back(x);
    }
    if (!ok || f.empty()) break;
    std::sort(f.begin(), f.end());
    f.erase(std::unique(f.begin(), f.end()), f.end());
    out.push_back(f);
  }
  return out;
}

bool is_ascii(const std::string& s) {
  for (unsigned char c : s) if (c >= 0x80) return false;
  return true;
}

struct AnchorChoice {
  bool ok = false;
  size_t k = 0;
  SeqSet lits;
  SeqSet raw;
  uint32_t dmin = 0, dmax = 0;         // dmax = kInf: unbounded prefix
  double score = -1;
};

// bounded: the literal's offset from the match start must be bounded (a
// candidate-start anchor); otherwise any literal set every match contains
// will do (a presence gate for a rule evaluated in full on the host).
AnchorChoice choose_anchor(const std::vector<const Node*>& items, bool bounded = true) {
  AnchorChoice best;
  double best_score = -1;
  uint32_t plo = 0, phi = 0;
  for (size_t k = 0; k < items.size(); ++k) {
    if (!bounded || phi <= kMaxPrefixBytes) {
      auto form = [&](bool ext, SeqSet* raw, SeqSet* lits, double* score) {
        *raw = prefix_of_items(items, k, ext);
        lits->clear();
        for (const auto& s : *raw) lits->insert(scan_form(s));
        *score = 1e9;
        bool ok = !lits->empty();
        for (const auto& s : *lits) {
          if (s.empty()) { ok = false; break; }
          *score = std::min(*score, seq_score(s));
        }
        return ok;
      };
      SeqSet raw, lits;
      double score;
      bool usable = form(false, &raw, &lits, &score);
      if (usable && score < kWeakAnchor) {
        // a weak literal ("ey", "sk"): extend it by the class that follows
        // (ey[a-zA-Z0-9]{17,} -> ey + 2 alnum units), far fewer K1 hits
        SeqSet xraw, xlits;
        double xscore;
        if (form(true, &xraw, &xlits, &xscore) && xscore > score) {
          raw.swap(xraw);
          lits.swap(xlits);
          score = xscore;
        }
      }
      if (usable) {
        // every extra literal costs scan-DFA states: prefer small sets
        score -= 0.05 * static_cast<double>(lits.size() - 1);
        if (score > best_score) {
          best_score = score;
          best.ok = true;
          best.k = k;
          best.lits = lits;
          best.raw = raw;
          best.dmin = plo;
          best.dmax = phi;
        }
      }
    }
    uint32_t lo, hi;
    len_bounds(*items[k], &lo, &hi);
    plo = std::min(plo + lo, kInf);
    phi = (phi >= kInf || hi >= kInf) ? kInf : std::min(phi + hi, kInf);
  }
  if (best.ok && best_score < 1.5) best.ok = false;   // a 1-unit anchor is useless
  best.score = best_score;
  return best;
}

DfaTable to_table(const RawDfa& raw, const std::vector<uint32_t>& order, int accept_state) {
  DfaTable t;
  t.nstates = static_cast<uint32_t>(raw.subsets.size());
  t.nclasses = raw.cm.n;
  std::copy(raw.cm.cls, raw.cm.cls + 256, t.byte_class);
  std::vector<uint32_t> inv(order.size());
  for (size_t i = 0; i < order.size(); ++i) inv[order[i]] = static_cast<uint32_t>(i);
  t.next.resize(static_cast<size_t>(t.nstates) * t.nclasses);
  t.accept.assign(t.nstates, 0);
  for (uint32_t i = 0; i < t.nstates; ++i) {
    uint32_t old = order[i];
    for (uint32_t c = 0; c < t.nclasses; ++c) t.next[static_cast<size_t>(i) * t.nclasses + c] = static_cast<uint16_t>(inv[raw.next[old][c]]);
    if (accept_state >= 0 && std::binary_search(raw.subsets[old].begin(), raw.subsets[old].end(), accept_state)) t.accept[i] = 1;
    if (raw.subsets[old].empty()) t.dead = i;
  }
  return t;
}

bool build_verify(const std::vector<const Node*>& items, size_t min_items, DfaTable* out, uint32_t* limit,
                  std::string* note) {
  for (size_t j = items.size(); j >= min_items && j > 0; --j) {
    Nfa nfa;
    int start = nfa.add();
    int cur = start;
    uint32_t lo = 0, hi = 0;
    for (size_t i = 0; i < j; ++i) {
      cur = build(&nfa, *items[i], cur);
      uint32_t a, b;
      len_bounds(*items[i], &a, &b);
      hi = (hi >= kInf || b >= kInf) ? kInf : std::min(hi + b, kInf);
    }
    int acc = nfa.add();
    nfa.eps(cur, acc);
    nfa.st[acc].out = 0;
    RawDfa raw;
    if (!determinize(nfa, start, false, acc, kVerifyStateCap, &raw)) continue;
    // make sure a dead (empty) state exists
    bool has_dead = false;
    for (const auto& s : raw.subsets) if (s.empty()) has_dead = true;
    if (!has_dead) {
      raw.subsets.push_back({});
      raw.next.push_back(std::vector<uint32_t>(raw.cm.n, static_cast<uint32_t>(raw.subsets.size() - 1)));
    }
    std::vector<uint32_t> order(raw.subsets.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = static_cast<uint32_t>(i);
    *out = to_table(raw, order, acc);
    // TSG_VERIFY_CAP (measurement): a lower cap on the bytes a K2 walk may
    // take before it gives up and emits the start for the host (exact either way)
    uint32_t cap = kVerifyLimitCap;
    if (const char* v = std::getenv("TSG_VERIFY_CAP")) cap = static_cast<uint32_t>(std::max(16, std::min(4096, std::atoi(v))));
    *limit = std::min(hi, cap);
    if (j < items.size()) *note += " verify-truncated:" + std::to_string(j) + "/" + std::to_string(items.size());
    return true;
  }
  return false;
}

// Reverse DFA of a mode-4 anchor: the anchor literals (raw units, cut to the
// length of their scan form, which is where a K1 hit ends) preceded by the
// relaxed prefix items[0..k), all read BACKWARDS from the hit's last byte.
// After consuming the byte at p the DFA is accepting iff text[p..hit] is in
// relaxed(prefix) . literal, i.e. p may start a match; accepting states are
// not absorbing, so one walk visits every possible start until the DFA dies.
bool build_reverse(const std::vector<const Node*>& items, size_t k, const SeqSet& raw, DfaTable* out) {
  Nfa nfa;
  nfa.rev = true;
  const int start = nfa.add();
  const int lit_end = nfa.add();
  for (const Seq& r : raw) {
    const size_t n = scan_form(r).size();
    if (n == 0) return false;
    int cur = start;
    for (size_t i = n; i-- > 0;) {
      const int nx = i == 0 ? lit_end : nfa.add();
      for (const auto& alt : r[i]) nfa.byte_chain(cur, alt, nx);
      cur = nx;
    }
  }
  int cur = lit_end;
  for (size_t i = k; i-- > 0;) cur = build(&nfa, *items[i], cur);
  const int acc = nfa.add();
  nfa.eps(cur, acc);
  nfa.st[acc].out = 0;
  RawDfa rd;
  if (!determinize(nfa, start, false, acc, kVerifyStateCap, &rd, /*absorb_accept=*/false)) return false;
  bool has_dead = false;
  for (const auto& sub : rd.subsets) if (sub.empty()) has_dead = true;
  if (!has_dead) {
    rd.subsets.push_back({});
    rd.next.push_back(std::vector<uint32_t>(rd.cm.n, static_cast<uint32_t>(rd.subsets.size() - 1)));
  }
  std::vector<uint32_t> order(rd.subsets.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = static_cast<uint32_t>(i);
  *out = to_table(rd, order, acc);
  return true;
}

// Byte classes whose transition columns are identical are one class for the
// automaton (exact: no state tells them apart).  The subset construction's
// classes come from the NFA's edge sets, which can distinguish bytes the DFA
// does not (the builtin scan DFA: 64 -> 50 classes), so merging shrinks every
// K1 table row.
void merge_classes(DfaTable* t) {
  const uint32_t C = t->nclasses, N = t->nstates;
  std::map<std::vector<uint16_t>, uint32_t> colid;
  std::vector<uint32_t> newc(C);
  for (uint32_t c = 0; c < C; ++c) {
    std::vector<uint16_t> col(N);
    for (uint32_t s = 0; s < N; ++s) col[s] = t->next[static_cast<size_t>(s) * C + c];
    newc[c] = colid.emplace(std::move(col), static_cast<uint32_t>(colid.size())).first->second;
  }
  const uint32_t C2 = static_cast<uint32_t>(colid.size());
  if (C2 == C) return;
  std::vector<uint16_t> nx(static_cast<size_t>(N) * C2);
  for (uint32_t s = 0; s < N; ++s)
    for (uint32_t c = 0; c < C; ++c) nx[static_cast<size_t>(s) * C2 + newc[c]] = t->next[static_cast<size_t>(s) * C + c];
  t->next.swap(nx);
  for (int b = 0; b < 256; ++b) t->byte_class[b] = static_cast<uint8_t>(newc[t->byte_class[b]]);
  t->nclasses = C2;
}

bool make_scan_dfa(const Nfa& nfa, int s0, uint32_t maxb, ScanDfa* out, std::string* err) {
  RawDfa raw;
  if (!determinize(nfa, s0, true, -1, kScanStateCap, &raw)) { *err = "scan DFA exceeds state cap"; return false; }
  // outputs per subset; renumber: states without outputs first (start stays 0)
  std::vector<std::vector<uint32_t>> outs(raw.subsets.size());
  for (size_t i = 0; i < raw.subsets.size(); ++i) {
    for (int s : raw.subsets[i]) if (nfa.st[s].out >= 0) outs[i].push_back(static_cast<uint32_t>(nfa.st[s].out));
    std::sort(outs[i].begin(), outs[i].end());
    outs[i].erase(std::unique(outs[i].begin(), outs[i].end()), outs[i].end());
  }
  if (!outs[0].empty()) { *err = "scan DFA start state has outputs"; return false; }
  std::vector<uint32_t> order;
  for (size_t i = 0; i < raw.subsets.size(); ++i) if (outs[i].empty()) order.push_back(static_cast<uint32_t>(i));
  out->first_out_state = static_cast<uint32_t>(order.size());
  for (size_t i = 0; i < raw.subsets.size(); ++i) if (!outs[i].empty()) order.push_back(static_cast<uint32_t>(i));
  if (order.size() > 65535) { *err = "scan DFA too large for 16-bit states"; return false; }
  out->t = to_table(raw, order, -1);
  out->out_off.assign(1, 0);
  out->out_ids.clear();
  for (size_t i = out->first_out_state; i < order.size(); ++i) {
    const auto& o = outs[order[i]];
    out->out_ids.insert(out->out_ids.end(), o.begin(), o.end());
    out->out_off.push_back(static_cast<uint32_t>(out->out_ids.size()));
  }
  out->max_pattern_bytes = maxb;
  merge_classes(&out->t);
  return true;
}

// The two passes on the host over one file with the given scan DFAs (K1 runs
// each group's DFA over the whole batch; outputs are unioned).
void two_pass(const Prefilter& pf, const ScanDfa* dfas, size_t ndfa, const std::vector<AnchorInfo>& anchors,
              const uint8_t* data, size_t len, std::vector<std::vector<uint64_t>>* cand, std::vector<uint8_t>* gate,
              const CompressedScan* comp = nullptr) {
  std::vector<uint8_t> kwbit(pf.nkw, 0);
  struct Hit { uint64_t end; uint32_t anchor; };
  std::vector<Hit> hits;
  if (comp) {
    // K1c: the compressed table's packed states (k1c_step), outputs through
    // the state's DESC record -> output record (keyword masks + list)
    uint32_t s = comp->state_val[0];
    for (size_t p = 0; p < len; ++p) {
      s = k1c_step(*comp, s, data[p]);
      if (!(s & 1u)) continue;
      const uint32_t oi = comp->image[((s & 0xfff0u) - 256) / 4 + 3];
      const CompressedScan::Out& o = comp->outs[oi];
      for (uint32_t k = 0; k < 64; ++k) if ((o.kw0 >> k) & 1u) kwbit[k] = 1;
      for (uint32_t k = 0; k < 64; ++k) if ((o.kw1 >> k) & 1u) kwbit[64 + k] = 1;
      for (uint32_t j = 0; j < o.list_count; ++j) {
        const uint32_t id = comp->out_list[o.list_begin + j];
        if (id < pf.nkw) kwbit[id] = 1; else hits.push_back({p, id - pf.nkw});
      }
    }
    ndfa = 0;
  }
  for (size_t g = 0; g < ndfa; ++g) {
    const ScanDfa& sd = dfas[g];
    const DfaTable& t = sd.t;
    uint32_t s = 0;
    for (size_t p = 0; p < len; ++p) {
      s = t.next[static_cast<size_t>(s) * t.nclasses + t.byte_class[data[p]]];
      if (s >= sd.first_out_state) {
        uint32_t o = s - sd.first_out_state;
        for (uint32_t k = sd.out_off[o]; k < sd.out_off[o + 1]; ++k) {
          uint32_t id = sd.out_ids[k];
          if (id < pf.nkw) kwbit[id] = 1; else hits.push_back({p, id - pf.nkw});
        }
      }
    }
  }
  gate->assign(pf.rules.size(), 0);
  for (size_t r = 0; r < pf.rules.size(); ++r) {
    const RuleGpuInfo& gi = pf.rules[r];
    uint8_t g = gi.always_gate;
    for (uint32_t k = 0; k < gi.kw_count; ++k) g |= kwbit[pf.rule_kw[gi.kw_begin + k]];
    (*gate)[r] = g;
  }
  cand->assign(pf.rules.size(), {});
  for (const Hit& h : hits) {
    const AnchorInfo& a = anchors[h.anchor];
    if (!(*gate)[a.rule] && pf.rules[a.rule].gate_on_gpu) continue;
    const RuleGpuInfo& gi = pf.rules[a.rule];
    if (gi.mode == 3) {                                 // presence gate: the hit itself
      (*cand)[a.rule].push_back(h.end);
      continue;
    }
    const DfaTable& v = pf.verify[gi.verify_dfa];
    auto verify_from = [&](size_t st) {
      uint32_t q = 0;
      bool emit = v.accept[0];
      size_t p = st;
      for (; !emit && p < len && p - st < gi.verify_limit; ++p) {
        q = v.next[static_cast<size_t>(q) * v.nclasses + v.byte_class[data[p]]];
        if (v.accept[q]) emit = true;
        else if (q == v.dead) break;
      }
      if (!emit && q != v.dead && p < len && p - st >= gi.verify_limit) emit = true;   // gave up: conservative
      return emit;
    };
    if (gi.mode == 4) {
      // backward walk of the reverse DFA from the hit's last byte: every
      // accepting position may start a match (then verified forwards)
      const DfaTable& rv = pf.verify[gi.rev_dfa];
      uint32_t q = 0;
      for (size_t p = h.end + 1; p-- > 0;) {
        if (h.end - p >= kRevLimit) { (*cand)[a.rule].push_back(kFullScanStart); break; }
        q = rv.next[static_cast<size_t>(q) * rv.nclasses + rv.byte_class[data[p]]];
        if (q == rv.dead) break;
        if (rv.accept[q] && verify_from(p)) (*cand)[a.rule].push_back(static_cast<uint64_t>(p));
      }
      continue;
    }
    long hi = static_cast<long>(h.end) + 1 - a.min_len - a.dmin;
    long lo = static_cast<long>(h.end) + 1 - a.max_len - a.dmax;
    if (lo < 0) lo = 0;
    for (long st = lo; st <= hi; ++st) {
      if (verify_from(static_cast<size_t>(st))) (*cand)[a.rule].push_back(static_cast<uint64_t>(st));
    }
  }
  for (auto& c : *cand) {
    std::sort(c.begin(), c.end());
    c.erase(std::unique(c.begin(), c.end()), c.end());
  }
}

// ------------------------------------------------------ K1 scan groups
struct Pattern {
  Seq seq;          // scan form (ASCII units, case-folded)
  uint32_t id;      // output id: keyword (< nkw) or nkw + anchor
};

// Sort key: the lowered first alternative of every unit, so patterns that
// share a prefix (a vendor keyword and the same rule's anchor) sit together
// and share trie states inside a group.
std::string pattern_key(const Seq& s) {
  std::string k;
  for (const auto& u : s) k.push_back(static_cast<char>(tolower(static_cast<unsigned char>(u.front().front()))));
  return k;
}

bool build_group(const std::vector<Pattern>& ps, ScanDfa* out, std::string* err) {
  Nfa nfa;
  int s0 = nfa.add();
  uint32_t maxb = 1;
  for (const auto& p : ps) maxb = std::max(maxb, add_seq(&nfa, s0, p.seq, static_cast<int>(p.id)));
  if (!make_scan_dfa(nfa, s0, maxb, out, err)) return false;
  out->npatterns = static_cast<uint32_t>(ps.size());
  return true;
}

// One group when everything fits K1 (the builtin rules).  Otherwise the
// patterns, sorted so shared prefixes sit together, are cut into the fewest
// balanced runs (by estimated trie nodes) whose DFAs all fit K1's LDS budget:
// each group is one K1 pass over the data, so fewer groups is the lever on a
// large ruleset's K1 time.  A run that still does not fit at many runs is
// halved until it does.
bool make_groups(Prefilter* pf, std::vector<Pattern> pats, ScanDfa* all_out, std::string* err) {
  pf->groups.clear();
  std::string e;
  {
    ScanDfa& all = *all_out;
    if (build_group(pats, &all, &e) && k1_fits(all)) {
      pf->groups.push_back(std::move(all));
      *all_out = ScanDfa();
      return true;
    }
    if (!e.empty()) *all_out = ScanDfa();                       // no one-group DFA (state cap)
    if (std::getenv("TSG_PREFILTER_DEBUG"))
      fprintf(stderr, "one-group scan DFA: %u states x %u classes (%u silent), %zu table words, LDS %zu B\n",
              all.t.nstates, all.t.nclasses, all.first_out_state, static_cast<size_t>(k1_table_words16(all)),
              k1_lds_table_bytes(all));
  }
  std::vector<std::string> keys(pats.size());
  std::vector<size_t> order(pats.size());
  for (size_t i = 0; i < pats.size(); ++i) { keys[i] = pattern_key(pats[i].seq); order[i] = i; }
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    return keys[a] != keys[b] ? keys[a] < keys[b] : pats[a].id < pats[b].id;
  });
  auto lcp_of = [](const std::string& a, const std::string& b) {
    size_t l = 0;
    while (l < a.size() && l < b.size() && a[l] == b[l]) ++l;
    return l;
  };
  uint64_t total = 0;
  for (size_t j = 0; j < order.size(); ++j)
    total += keys[order[j]].size() - (j ? lcp_of(keys[order[j]], keys[order[j - 1]]) : 0);
  auto split = [&](uint64_t nruns) {
    const uint64_t share = (total + nruns - 1) / nruns;
    std::vector<std::vector<Pattern>> runs(1);
    uint64_t est = 0;
    std::string prev;
    for (size_t i : order) {
      const std::string& k = keys[i];
      size_t lcp = lcp_of(k, prev);
      if (est + (k.size() - lcp) > share && !runs.back().empty() && runs.size() < nruns) { runs.emplace_back(); est = 0; lcp = 0; }
      est += k.size() - lcp;
      runs.back().push_back(pats[i]);
      prev = k;
    }
    return runs;
  };
  // ~130 bytes of LDS per trie node (a row of ~64 classes): the first guess
  constexpr uint64_t kNodesPerGroup = (kK1LdsBytes - kK1HitLdsMin - 8192) / 130;
  const uint64_t first = std::max<uint64_t>(2, (total + kNodesPerGroup - 1) / kNodesPerGroup);
  for (uint64_t nruns = first; nruns <= 4 * first; ++nruns) {
    std::vector<ScanDfa> gs;
    bool ok = true;
    for (auto& run : split(nruns)) {
      ScanDfa d;
      e.clear();
      if (!build_group(run, &d, &e) || !k1_fits(d)) { ok = false; break; }
      gs.push_back(std::move(d));
    }
    if (ok) {
      pf->groups = std::move(gs);
      return true;
    }
  }
  std::vector<std::vector<Pattern>> runs = split(4 * first);
  std::vector<std::vector<Pattern>> todo(runs.rbegin(), runs.rend());
  while (!todo.empty()) {
    std::vector<Pattern> ps = std::move(todo.back());
    todo.pop_back();
    ScanDfa d;
    e.clear();
    if (build_group(ps, &d, &e) && k1_fits(d)) { pf->groups.push_back(std::move(d)); continue; }
    if (ps.size() == 1) { *err = "scan pattern does not fit K1 (" + (e.empty() ? std::string("LDS") : e) + ")"; return false; }
    const size_t h = ps.size() / 2;
    todo.emplace_back(ps.begin() + h, ps.end());
    todo.emplace_back(ps.begin(), ps.begin() + h);
  }
  return true;
}

// ------------------------------------------------------ K1c compressed table
// Exceptions of state s against full state f: the classes whose next state
// differs.  Representable in one DESC record when there are at most four such
// classes going to at most two targets, and when there are two targets each
// takes at most two of the four class slots.
struct Exc { uint32_t n = 0; uint32_t cls[4]; uint16_t tgt[4]; };

bool exceptions(const DfaTable& t, uint32_t s, uint32_t f, Exc* e) {
  const uint32_t C = t.nclasses;
  const uint16_t* a = &t.next[static_cast<size_t>(s) * C];
  const uint16_t* b = &t.next[static_cast<size_t>(f) * C];
  e->n = 0;
  for (uint32_t c = 0; c < C; ++c) {
    if (a[c] == b[c]) continue;
    if (e->n == 4) return false;
    e->cls[e->n] = c;
    e->tgt[e->n] = a[c];
    ++e->n;
  }
  uint16_t tg[2] = {0, 0};
  uint32_t cnt[2] = {0, 0}, nt = 0;
  for (uint32_t i = 0; i < e->n; ++i) {
    uint32_t k = 0;
    while (k < nt && tg[k] != e->tgt[i]) ++k;
    if (k == nt) {
      if (nt == 2) return false;
      tg[nt++] = e->tgt[i];
    }
    ++cnt[k];
  }
  return nt <= 1 || (cnt[0] <= 2 && cnt[1] <= 2);
}

// The DFA of all scan patterns as a K1c table (prefilter.h).  Full rows are
// chosen greedily: the start state, then, while some state has no full state
// it can be expressed against, the shallowest such states.  Every (state,
// class) transition and every output flag is checked against the DFA before
// the table is accepted.
bool compress_scan(const ScanDfa& d, uint32_t nkw, size_t lds_budget, CompressedScan* out, std::string* why) {
  const DfaTable& t = d.t;
  const uint32_t N = t.nstates, C = t.nclasses;
  *out = CompressedScan();
  if (N == 0 || C == 0 || C > 63) { *why = "classes"; return false; }
  std::vector<uint32_t> depth(N, UINT32_MAX);
  {
    std::vector<uint32_t> fr{0}, nf;
    depth[0] = 0;
    while (!fr.empty()) {
      nf.clear();
      for (uint32_t s : fr)
        for (uint32_t c = 0; c < C; ++c) {
          const uint32_t x = t.next[static_cast<size_t>(s) * C + c];
          if (depth[x] == UINT32_MAX) { depth[x] = depth[s] + 1; nf.push_back(x); }
        }
      fr.swap(nf);
    }
  }
  for (uint32_t s = 0; s < N; ++s) if (depth[s] == UINT32_MAX) depth[s] = 0xfffffu;   // unreachable: keep anyway
  std::vector<uint8_t> is_full(N, 0);
  std::vector<uint32_t> full{0}, def(N, UINT32_MAX);
  is_full[0] = 1;
  Exc e;
  for (;;) {
    std::vector<uint32_t> bad;
    for (uint32_t s = 0; s < N; ++s) {
      if (is_full[s]) continue;
      if (def[s] != UINT32_MAX && exceptions(t, s, def[s], &e)) continue;
      def[s] = UINT32_MAX;
      uint32_t best = UINT32_MAX, bestn = 5;
      for (uint32_t f : full) {
        if (exceptions(t, s, f, &e) && e.n < bestn) {
          best = f;
          bestn = e.n;
          if (bestn == 0) break;
        }
      }
      if (best == UINT32_MAX) bad.push_back(s);
      else def[s] = best;
    }
    if (bad.empty()) break;
    uint32_t md = UINT32_MAX;
    for (uint32_t s : bad) md = std::min(md, depth[s]);
    for (uint32_t s : bad)
      if (depth[s] == md) { is_full[s] = 1; full.push_back(s); }
    if (full.size() > 8192) { *why = "too many full rows"; return false; }
  }
  // records: 0 = no exceptions, then every compact state and every output state
  const uint32_t fo = d.first_out_state;
  std::vector<uint32_t> rec(N, 0);
  uint32_t ndesc = 1;
  for (uint32_t s = 0; s < N; ++s) if (!is_full[s] || s >= fo) rec[s] = ndesc++;
  if (256 + 16ull * ndesc > 0x10000) { *why = "too many DESC records for 16-bit addresses"; return false; }
  uint32_t stride = C | 1u;                                     // odd dword stride: a class spreads over banks
  const uint64_t desc_dw = 4ull * ndesc;
  const uint64_t full_base_dw = 64 + desc_dw;                   // LDS dword address of the first full row
  const uint64_t image_dw = desc_dw + static_cast<uint64_t>(full.size()) * stride;
  if (full_base_dw + static_cast<uint64_t>(full.size()) * stride > 0x10000) { *why = "full rows beyond 256 KiB"; return false; }
  if (256 + image_dw * 4 > lds_budget) {
    *why = "table " + std::to_string(256 + image_dw * 4) + " B > LDS budget " + std::to_string(lds_budget) + " B";
    return false;
  }
  std::vector<uint32_t> row_of(N, 0);                           // full row index of each full state
  for (size_t i = 0; i < full.size(); ++i) row_of[full[i]] = static_cast<uint32_t>(i);
  std::vector<uint32_t> val(N);
  for (uint32_t s = 0; s < N; ++s) {
    const uint32_t f = is_full[s] ? s : def[s];
    val[s] = (static_cast<uint32_t>(full_base_dw + static_cast<uint64_t>(row_of[f]) * stride) << 16) |
             (256u + 16u * rec[s]) | (s >= fo ? 1u : 0u);
  }
  out->image.assign(image_dw, 0);
  uint32_t* desc = out->image.data();
  desc[0] = kK1cNoRecord; desc[1] = desc[2] = 0; desc[3] = kK1cNoRecord;
  for (uint32_t s = 0; s < N; ++s) {
    if (rec[s] == 0) continue;
    uint32_t* r = desc + 4ull * rec[s];
    uint8_t slot[4] = {0xff, 0xff, 0xff, 0xff};
    uint32_t tA = 0, tB = 0;
    if (!is_full[s]) {
      if (!exceptions(t, s, def[s], &e)) { *why = "internal: exception set"; return false; }
      // group the classes by target: target 1 in slots 0-1, target 2 in slots 2-3 (one target: slots 0-3)
      uint16_t first = e.n ? e.tgt[0] : 0;
      uint32_t na = 0, nb = 0;
      bool two = false;
      for (uint32_t i = 0; i < e.n; ++i) two |= e.tgt[i] != first;
      for (uint32_t i = 0; i < e.n; ++i) {
        const uint8_t c4 = static_cast<uint8_t>(e.cls[i] * 4);
        if (!two) { slot[na++] = c4; continue; }
        if (e.tgt[i] == first) slot[na++] = c4;
        else { slot[2 + nb++] = c4; tB = val[e.tgt[i]]; }
      }
      if (e.n) tA = val[first];
      if (!two) tB = tA;
    }
    r[0] = static_cast<uint32_t>(slot[0]) | (static_cast<uint32_t>(slot[1]) << 8) |
           (static_cast<uint32_t>(slot[2]) << 16) | (static_cast<uint32_t>(slot[3]) << 24);
    r[1] = tA;
    r[2] = tB;
    r[3] = kK1cNoRecord;
    if (s >= fo) {
      // outputs: keyword ids < 128 in two masks, the others (anchors, keywords >= 128) listed
      const uint32_t o = s - fo;
      CompressedScan::Out om{0, 0, static_cast<uint32_t>(out->out_list.size()), 0};
      for (uint32_t k = d.out_off[o]; k < d.out_off[o + 1]; ++k) {
        const uint32_t id = d.out_ids[k];
        if (id < nkw && id < 64) om.kw0 |= 1ull << id;
        else if (id < nkw && id < 128) om.kw1 |= 1ull << (id - 64);
        else out->out_list.push_back(id);
      }
      om.list_count = static_cast<uint32_t>(out->out_list.size()) - om.list_begin;
      r[3] = static_cast<uint32_t>(out->outs.size());
      out->outs.push_back(om);
    }
  }
  for (size_t i = 0; i < full.size(); ++i) {
    uint32_t* row = out->image.data() + desc_dw + i * stride;
    for (uint32_t c = 0; c < C; ++c) row[c] = val[t.next[static_cast<size_t>(full[i]) * C + c]];
  }
  for (int b = 0; b < 256; ++b) out->cls4[b] = static_cast<uint8_t>(t.byte_class[b] * 4);
  out->nclasses = C;
  out->row_stride = stride;
  out->ndesc = ndesc;
  out->nfull = static_cast<uint32_t>(full.size());
  out->nstates = N;
  out->state_val = val;
  out->max_pattern_bytes = d.max_pattern_bytes;
  // exhaustive self-check against the DFA: every transition, every output flag
  for (uint32_t s = 0; s < N; ++s) {
    if (((val[s] & 1u) != 0) != (s >= fo)) { *why = "internal: output flag"; return false; }
    for (int b = 0; b < 256; ++b) {
      const uint32_t want = val[t.next[static_cast<size_t>(s) * C + t.byte_class[b]]];
      if (k1c_step(*out, val[s], static_cast<uint32_t>(b)) != want) {
        *why = "internal: transition check failed at state " + std::to_string(s) + " byte " + std::to_string(b);
        return false;
      }
    }
  }
  out->ok = true;
  return true;
}

// Keyword ids are renumbered so that each group's keywords are contiguous:
// K1 then ORs them into register masks relative to the group's kw_base.
void renumber_keywords(Prefilter* pf, ScanDfa* all) {
  std::vector<uint32_t> newid(pf->nkw, 0xffffffffu);
  uint32_t next = 0;
  for (auto& g : pf->groups) {
    std::vector<uint32_t> ids;
    for (uint32_t id : g.out_ids) if (id < pf->nkw) ids.push_back(id);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    for (uint32_t id : ids) if (newid[id] == 0xffffffffu) newid[id] = next++;
  }
  for (uint32_t k = 0; k < pf->nkw; ++k) if (newid[k] == 0xffffffffu) newid[k] = next++;
  auto remap = [&](std::vector<uint32_t>* v) { for (auto& id : *v) if (id < pf->nkw) id = newid[id]; };
  for (auto& g : pf->groups) {
    remap(&g.out_ids);
    uint32_t lo = 0xffffffffu;
    for (uint32_t id : g.out_ids) if (id < pf->nkw) lo = std::min(lo, id);
    g.kw_base = lo == 0xffffffffu ? 0 : (lo & ~31u);
  }
  remap(&pf->host_scan.out_ids);
  remap(&all->out_ids);
  remap(&pf->rule_kw);
  std::vector<std::string> text(pf->nkw);
  for (uint32_t k = 0; k < pf->nkw; ++k) text[newid[k]] = pf->kw_text[k];
  pf->kw_text.swap(text);
}

}  // namespace

uint32_t k1_row_stride(uint32_t nclasses) {
  uint32_t s = (nclasses + 2) & ~1u;      // >= nclasses + 1: slot nclasses holds the output-state index
  if (((s / 2) & 1u) == 0) s += 2;        // odd dword stride spreads a class over LDS banks
  return s;
}

uint32_t k1_out_row_stride(uint32_t nclasses) {
  uint32_t s = k1_row_stride(nclasses) + 10;
  if (((s / 2) & 1u) == 0) s += 2;
  return s;
}

uint64_t k1_table_words16(const ScanDfa& d) {
  return static_cast<uint64_t>(d.first_out_state) * k1_row_stride(d.t.nclasses) +
         static_cast<uint64_t>(d.t.nstates - d.first_out_state) * k1_out_row_stride(d.t.nclasses);
}

size_t k1_lds_table_bytes(const ScanDfa& d) {
  const size_t tab = (k1_table_words16(d) * 2 + 15) & ~size_t(15);
  const size_t list = (d.out_ids.size() * 4 + 15) & ~size_t(15);   // (at most) every output id listed
  return tab + 256 + list;
}

// K1 entries are dword row offsets in 16 bits (tables up to 256 KiB); the
// per-wave hit buffers shrink to kK1WaveHitsMin entries for large groups
bool k1_fits(const ScanDfa& d) {
  return k1_table_words16(d) <= 2 * 65535 && kK1HitLdsMin + k1_lds_table_bytes(d) <= kK1LdsBytes;
}

bool literal_gate(const re::Node& ast, re::LitGate* out, bool* bounded, uint32_t* dmin, uint32_t* dmax) {
  std::vector<const Node*> items;
  flatten(ast, &items);
  for (bool b : {true, false}) {
    out->clear();
    AnchorChoice a = choose_anchor(items, b);
    if (!a.ok) continue;
    for (const Seq& raw : a.raw) {
      Seq f = scan_form(raw, /*keep_special=*/true);   // ASCII case-folded superset, fold runes kept
      if (f.empty()) { out->clear(); break; }
      out->push_back(f);
    }
    if (out->empty()) continue;
    *bounded = b;
    *dmin = a.dmin;
    *dmax = a.dmax;
    return true;
  }
  return false;
}

bool build_prefilter(const Ruleset& rs, Prefilter* pf, std::string* err) {
  *pf = Prefilter();
  // --- keywords: distinct ASCII lowered keywords get a GPU pattern id
  std::map<std::string, uint32_t> kw_ids;
  // rules, then one keyword-less pseudo-rule per exclude-block regex
  const size_t nr = rs.rules.size();
  pf->rules.resize(nr + rs.excludes.size());
  for (size_t k = 0; k < rs.excludes.size(); ++k) {
    RuleGpuInfo& gi = pf->rules[nr + k];
    gi.kw_begin = gi.kw_count = 0;
    gi.always_gate = 1;
    gi.gate_on_gpu = 1;
  }
  for (size_t r = 0; r < nr; ++r) {
    const Rule& rule = rs.rules[r];
    RuleGpuInfo& gi = pf->rules[r];
    gi.kw_begin = static_cast<uint32_t>(pf->rule_kw.size());
    gi.always_gate = rule.keywords.empty();
    gi.gate_on_gpu = 1;
    for (const auto& kw : rule.keywords_lower) {
      if (kw.empty()) { gi.always_gate = 1; continue; }
      // non-ASCII keywords, and short ones ("sk", "key": outputs at a few
      // positions per KB of text, the most expensive part of K1), are
      // evaluated on the host, only for files with candidates of the rule
      if (!is_ascii(kw) || kw.size() <= kHostKeywordLen) { gi.gate_on_gpu = 0; continue; }
      auto it = kw_ids.find(kw);
      if (it == kw_ids.end()) {
        it = kw_ids.emplace(kw, static_cast<uint32_t>(pf->kw_text.size())).first;
        pf->kw_text.push_back(kw);
      }
      pf->rule_kw.push_back(it->second);
    }
    gi.kw_count = static_cast<uint32_t>(pf->rule_kw.size()) - gi.kw_begin;
    if (gi.always_gate) gi.gate_on_gpu = 1;
  }
  pf->nkw = static_cast<uint32_t>(pf->kw_text.size());

  // --- scan patterns (GPU form, partitioned into K1 groups below) and the
  // host variant NFA
  std::vector<Pattern> pats;
  Nfa host;
  int h0 = host.add();
  uint32_t maxb = 1, hmaxb = 1;
  for (uint32_t k = 0; k < pf->nkw; ++k) {
    pats.push_back({keyword_seq(pf->kw_text[k], false), k});
    hmaxb = std::max(hmaxb, add_seq(&host, h0, keyword_seq(pf->kw_text[k], true), static_cast<int>(k)));
  }
  std::string rep;
  for (size_t r = 0; r < pf->rules.size(); ++r) {
    const re::Regexp* rx = r < nr ? rs.rules[r].regex.get() : rs.excludes[r - nr];
    const std::string name = r < nr ? rs.rules[r].id : "exclude-block #" + std::to_string(r - nr);
    RuleGpuInfo& gi = pf->rules[r];
    gi.mode = 1;
    if (!rx) { gi.mode = 2; continue; }              // no regex: never any location
    std::vector<const Node*> items;
    flatten(*rx->ast(), &items);
    AnchorChoice ch = rx->nullable() ? AnchorChoice() : choose_anchor(items);
    std::string note;
    DfaTable vt, rt;
    uint32_t limit = 0;
    // a far better literal behind an unbounded (or long) prefix: reverse-anchored
    // (mode 4), its prefix walked backwards from each hit (jwt-token's `.ey`
    // after `ey[a-zA-Z0-9]{17,}` instead of `ey` itself)
    bool reverse = false;
    if (!rx->nullable() && ext_rev()) {
      AnchorChoice rv = choose_anchor(items, false);
      // only when the bounded anchor is weak: a strong one ("-----") is kept
      // even if a higher-scoring literal ("PRIVAT", common in source code)
      // sits further in
      if (rv.ok && rv.dmax > kMaxPrefixBytes && (!ch.ok || (ch.score < kWeakAnchor && rv.score >= ch.score + 0.5)) &&
          build_reverse(items, rv.k, rv.raw, &rt)) {
        ch = rv;
        reverse = true;
      }
    }
    const char* why = !ch.ok ? "no bounded anchor" : nullptr;
    if (!why && !build_verify(items, ch.k + 1, &vt, &limit, &note)) why = "verify DFA too large";
    if (why) {
      // FULL on the host -- but only in files that contain one of a literal
      // set every match contains (mode 3: K2 turns such a hit straight into
      // a presence candidate, no verify)
      AnchorChoice req = rx->nullable() ? AnchorChoice() : choose_anchor(items, false);
      if (!req.ok) { rep += name + ": FULL (" + why + ")\n"; continue; }
      gi.mode = 3;
      gi.verify_dfa = 0;
      gi.verify_limit = 0;
      for (const auto& s : req.lits) {
        AnchorInfo a{static_cast<uint32_t>(r), seq_min_len(s), seq_max_len(s), 0, 0};
        uint32_t id = pf->nkw + static_cast<uint32_t>(pf->anchors.size());
        pf->anchors.push_back(a);
        pats.push_back({s, id});
        maxb = std::max(maxb, seq_max_len(s));
        AnchorInfo ha = a;
        ha.min_len = 0xffffffffu;
        ha.max_len = 0;
        SeqSet vforms;
        for (const auto& rawlit : req.raw) if (scan_form(rawlit) == s) vforms.insert(scan_form(rawlit, true));
        for (const auto& v : vforms) {
          ha.min_len = std::min(ha.min_len, seq_min_len(v));
          ha.max_len = std::max(ha.max_len, seq_max_len(v));
          hmaxb = std::max(hmaxb, add_seq(&host, h0, v, static_cast<int>(id)));
        }
        pf->host_anchors.push_back(ha);
      }
      rep += name + ": FULL (" + why + ") where present: item " + std::to_string(req.k) + ", " +
             std::to_string(req.lits.size()) + " literal(s) {" + seqs_str(req.lits) + "}\n";
      continue;
    }
    gi.mode = reverse ? 4 : 0;
    gi.verify_dfa = static_cast<uint32_t>(pf->verify.size());
    gi.verify_limit = std::max<uint32_t>(limit, 1);
    pf->verify.push_back(std::move(vt));
    if (reverse) {
      gi.rev_dfa = static_cast<uint32_t>(pf->verify.size());
      note += " reverse " + std::to_string(rt.nstates) + " states x " + std::to_string(rt.nclasses) + " classes";
      pf->verify.push_back(std::move(rt));
    }
    for (const auto& s : ch.lits) {
      AnchorInfo a;
      a.rule = static_cast<uint32_t>(r);
      a.min_len = seq_min_len(s);
      a.max_len = seq_max_len(s);
      a.dmin = ch.dmin;
      a.dmax = ch.dmax;
      uint32_t id = pf->nkw + static_cast<uint32_t>(pf->anchors.size());
      pf->anchors.push_back(a);
      pats.push_back({s, id});
      maxb = std::max(maxb, seq_max_len(s));
      // host variant forms of every raw literal with this scan form
      AnchorInfo ha = a;
      ha.min_len = 0xffffffffu;
      ha.max_len = 0;
      SeqSet vforms;
      for (const auto& rawlit : ch.raw) if (scan_form(rawlit) == s) vforms.insert(scan_form(rawlit, true));
      for (const auto& v : vforms) {
        ha.min_len = std::min(ha.min_len, seq_min_len(v));
        ha.max_len = std::max(ha.max_len, seq_max_len(v));
        hmaxb = std::max(hmaxb, add_seq(&host, h0, v, static_cast<int>(id)));
      }
      pf->host_anchors.push_back(ha);
    }
    rep += name + (reverse ? ": reverse-anchored item " : ": anchored item ") + std::to_string(ch.k) + ", " +
           std::to_string(ch.lits.size()) + " literal(s), offset [" + std::to_string(ch.dmin) + "," +
           (ch.dmax >= kInf ? std::string("inf") : std::to_string(ch.dmax)) + "], verify " +
           std::to_string(pf->verify[gi.verify_dfa].nstates) + " states x " +
           std::to_string(pf->verify[gi.verify_dfa].nclasses) +
           " classes, limit " + std::to_string(gi.verify_limit) + note + " {" + seqs_str(ch.lits) + "}\n";
  }
  ScanDfa all;
  if (!make_groups(pf, pats, &all, err)) return false;
  if (!make_scan_dfa(host, h0, hmaxb, &pf->host_scan, err)) return false;
  renumber_keywords(pf, &all);
  std::string k1c_note;
  const char* k1c_env = std::getenv("TSG_K1C");
  if (pf->groups.size() > 1 && all.t.nstates > 0 && !(k1c_env && std::atoi(k1c_env) == 0)) {
    if (!compress_scan(all, pf->nkw, kK1LdsBytes - kK1HitLdsMin, &pf->compressed, &k1c_note)) pf->compressed = CompressedScan();
  }
  std::string grep;
  for (size_t g = 0; g < pf->groups.size(); ++g) {
    const ScanDfa& d = pf->groups[g];
    maxb = std::max(maxb, d.max_pattern_bytes);
    grep += "scan DFA group " + std::to_string(g) + ": " + std::to_string(d.npatterns) + " patterns, " +
            std::to_string(d.t.nstates) + " states x " + std::to_string(d.t.nclasses) + " classes (" +
            std::to_string(d.first_out_state) + " silent), keyword base " + std::to_string(d.kw_base) +
            ", max pattern " + std::to_string(d.max_pattern_bytes) + " B, LDS " +
            std::to_string(k1_lds_table_bytes(d)) + " B\n";
  }
  if (pf->compressed.ok) {
    const CompressedScan& c = pf->compressed;
    grep += "K1c one-pass table: " + std::to_string(c.nstates) + " states x " + std::to_string(c.nclasses) +
            " classes, " + std::to_string(c.nfull) + " full rows (stride " + std::to_string(c.row_stride) + "), " +
            std::to_string(c.ndesc) + " DESC records, " + std::to_string(c.outs.size()) + " output records, LDS " +
            std::to_string(c.lds_bytes()) + " B\n";
  } else if (pf->groups.size() > 1) {
    grep += "K1c one-pass table: not used (" + (k1c_note.empty() ? std::string("disabled") : k1c_note) + ")\n";
  }
  pf->report = "host variant DFA: " + std::to_string(pf->host_scan.t.nstates) + " states x " +
               std::to_string(pf->host_scan.t.nclasses) + " classes\n" +
               std::to_string(pf->groups.size()) + " scan DFA group(s), " + std::to_string(pf->nkw) +
               " keywords, " + std::to_string(pf->anchors.size()) + " anchor literals, max pattern " +
               std::to_string(maxb) + " B\n" + grep + rep;
  const auto& ix = rs.allow_index;
  pf->report += "global allow-path index: " +
                (ix.usable ? std::to_string(ix.out.size()) + " AC states, " +
                                 std::to_string(__builtin_popcountll(ix.always)) + " ungated regexes"
                           : std::string("unused (plain loop)")) + "\n";
  return true;
}

bool prefilter_reference_file(const Prefilter& pf, const uint8_t* data, size_t len,
                              std::vector<std::vector<uint64_t>>* cand, std::vector<uint8_t>* gate) {
  bool special = false;
  for (size_t p = 1; p < len; ++p) {
    if (fold_special_at(p >= 2 ? data[p - 2] : 0, data[p - 1], data[p])) { special = true; break; }
  }
  // the tables the engine runs: K1c's compressed one-pass table when the
  // rule set has one, else the scan-DFA groups
  two_pass(pf, pf.groups.data(), pf.groups.size(), pf.anchors, data, len, cand, gate,
           pf.compressed.ok ? &pf.compressed : nullptr);
  return special;
}

void plan_from_candidates(const Prefilter& pf, std::vector<std::vector<uint64_t>>* cands, FilePlan* plan) {
  const size_t nr = pf.rules.size();
  plan->kind.assign(nr, kPlanNoMatch);
  plan->cands.clear();
  plan->active.clear();
  plan->active_set = true;
  for (size_t k = 0; k < nr; ++k) {
    const RuleGpuInfo& gi = pf.rules[k];
    if (gi.mode == 1 || (gi.mode == 3 && !(*cands)[k].empty()) ||
        (gi.mode == 4 && !(*cands)[k].empty() && (*cands)[k].back() == kFullScanStart)) {
      plan->kind[k] = kPlanFull;
      plan->active.push_back(static_cast<uint32_t>(k));
    } else if ((gi.mode == 0 || gi.mode == 4) && !(*cands)[k].empty()) {
      plan->kind[k] = gi.gate_on_gpu ? kPlanCandidates : kPlanCandHostGate;
      plan->cands.push_back({static_cast<uint32_t>(k), std::move((*cands)[k])});
      plan->active.push_back(static_cast<uint32_t>(k));
    }
  }
}

void prefilter_variant_file(const Prefilter& pf, const uint8_t* data, size_t len,
                            std::vector<std::vector<uint64_t>>* cand, std::vector<uint8_t>* gate) {
  two_pass(pf, &pf.host_scan, 1, pf.host_anchors, data, len, cand, gate);
}

}  // namespace tsg
