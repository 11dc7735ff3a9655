// Go regexp semantics restated in C++ -- see goregexp.h for the contract and
// the Go sources each part follows (regexp/syntax parse.go, simplify.go,
// compile.go; regexp/exec.go, regexp.go allMatches).
#include "goregexp.h"

#include <unordered_map>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <cstring>

namespace tsg {
namespace re {

namespace {
#include "unicode_tables.inc"

constexpr uint32_t kMaxRune = 0x10FFFF;
constexpr int kMaxRepeat = 1000;

bool lookup_pair(const uint32_t (*tab)[2], size_t n, uint32_t r, uint32_t* out) {
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (tab[m][0] == r) { *out = tab[m][1]; return true; }
    if (tab[m][0] < r) lo = m + 1; else hi = m;
  }
  return false;
}

void add_range(std::vector<Range>* v, uint32_t lo, uint32_t hi) { v->push_back({lo, hi}); }

void normalize(std::vector<Range>* v) {
  std::sort(v->begin(), v->end(), [](const Range& a, const Range& b) { return a.lo < b.lo; });
  std::vector<Range> out;
  for (const Range& r : *v) {
    if (!out.empty() && r.lo <= out.back().hi + 1) {
      out.back().hi = std::max(out.back().hi, r.hi);
    } else {
      out.push_back(r);
    }
  }
  *v = std::move(out);
}

void negate(std::vector<Range>* v) {
  normalize(v);
  std::vector<Range> out;
  uint32_t next = 0;
  for (const Range& r : *v) {
    if (r.lo > next) out.push_back({next, r.lo - 1});
    next = r.hi + 1;
  }
  if (next <= kMaxRune) out.push_back({next, kMaxRune});
  *v = std::move(out);
}

// Add every SimpleFold orbit member of every rune in [lo,hi] (appendFoldedRange).
void add_folded(std::vector<Range>* v, uint32_t lo, uint32_t hi) {
  add_range(v, lo, hi);
  const size_t n = sizeof(kFoldOrbit) / sizeof(kFoldOrbit[0]);
  // kFoldOrbit is sorted by rune; walk the entries inside [lo,hi]
  size_t a = 0, b = n;
  while (a < b) {
    size_t m = (a + b) / 2;
    if (kFoldOrbit[m][0] < lo) a = m + 1; else b = m;
  }
  for (size_t k = a; k < n && kFoldOrbit[k][0] <= hi; ++k) {
    uint32_t r = kFoldOrbit[k][0];
    for (uint32_t f = kFoldOrbit[k][1]; f != r;) {
      add_range(v, f, f);
      uint32_t nx;
      if (!lookup_pair(kFoldOrbit, n, f, &nx)) break;
      f = nx;
    }
  }
}

bool is_word(int32_t r) {
  return (r >= '0' && r <= '9') || (r >= 'a' && r <= 'z') || (r >= 'A' && r <= 'Z') || r == '_';
}

// syntax.EmptyOpContext(r1, r2)
uint8_t empty_context(int32_t r1, int32_t r2) {
  uint8_t op = kEmptyNoWordBoundary;
  int boundary = 0;
  if (is_word(r1)) boundary = 1;
  else if (r1 == '\n') op |= kEmptyBeginLine;
  else if (r1 < 0) op |= kEmptyBeginText | kEmptyBeginLine;
  if (is_word(r2)) boundary ^= 1;
  else if (r2 == '\n') op |= kEmptyEndLine;
  else if (r2 < 0) op |= kEmptyEndText | kEmptyEndLine;
  if (boundary) op ^= (kEmptyWordBoundary | kEmptyNoWordBoundary);
  return op;
}

// Rune before position pos: only ASCII word chars / '\n' matter for contexts,
// so a non-ASCII predecessor is reported as U+FFFD (never word, never '\n').
int32_t rune_before(const uint8_t* s, size_t pos) {
  if (pos == 0) return -1;
  uint8_t c = s[pos - 1];
  return c < 0x80 ? c : 0xFFFD;
}

// ------------------------------------------------------------------ parser
struct Flags { bool i = false, m = false, s = false, U = false; };

std::unique_ptr<Node> mk(Op op) { auto n = std::make_unique<Node>(); n->op = op; return n; }

class Parser {
 public:
  Parser(const std::string& p) : p_(p) {}
  std::unique_ptr<Node> parse(std::string* err, std::vector<std::string>* names) {
    names_.push_back("");
    Flags f;
    auto n = alternation(&f);
    if (err_.empty() && i_ < p_.size()) err_ = "unexpected ): `" + p_ + "`";
    if (!err_.empty()) { *err = "error parsing regexp: " + err_; return nullptr; }
    *names = names_;
    return n;
  }

 private:
  const std::string& p_;
  size_t i_ = 0;
  std::string err_;
  int ncap_ = 0;
  int depth_ = 0;  // open groups; Go's maxHeight (regexp/syntax parse.go) bounds nesting at 1000
  std::vector<std::string> names_;

  bool eof() const { return i_ >= p_.size(); }
  char peek(size_t k = 0) const { return i_ + k < p_.size() ? p_[i_ + k] : '\0'; }
  void fail(const std::string& m) { if (err_.empty()) err_ = m; }

  uint32_t next_rune() {
    int32_t r; int w;
    decode_rune(reinterpret_cast<const uint8_t*>(p_.data()) + i_, p_.size() - i_, &r, &w);
    if (r == 0xFFFD && w == 1) fail("invalid UTF-8: `" + p_ + "`");
    i_ += w;
    return static_cast<uint32_t>(r);
  }

  std::unique_ptr<Node> alternation(Flags* f) {
    std::vector<std::unique_ptr<Node>> alts;
    alts.push_back(concat(f));
    while (err_.empty() && peek() == '|') {
      ++i_;
      alts.push_back(concat(f));
    }
    if (alts.size() == 1) return std::move(alts[0]);
    auto n = mk(Op::Alternate);
    n->sub = std::move(alts);
    return n;
  }

  std::unique_ptr<Node> concat(Flags* f) {
    auto n = mk(Op::Concat);
    while (err_.empty() && !eof() && peek() != '|' && peek() != ')') {
      auto a = atom(f);
      if (!err_.empty()) break;
      if (!a) continue;   // flag group (?i)
      a = repeat(std::move(a), *f);
      n->sub.push_back(std::move(a));
    }
    if (n->sub.size() == 1) return std::move(n->sub[0]);
    if (n->sub.empty()) return mk(Op::EmptyMatch);
    return n;
  }

  bool try_brace(int* lo, int* hi) {
    size_t j = i_ + 1, k = j;
    while (k < p_.size() && isdigit(static_cast<unsigned char>(p_[k]))) ++k;
    if (k == j) return false;
    if (k - j > 8) { fail("invalid repeat count"); return false; }
    *lo = std::stoi(p_.substr(j, k - j));
    *hi = *lo;
    if (k < p_.size() && p_[k] == ',') {
      ++k;
      size_t m = k;
      while (m < p_.size() && isdigit(static_cast<unsigned char>(p_[m]))) ++m;
      if (m - k > 8) { fail("invalid repeat count"); return false; }
      *hi = m > k ? std::stoi(p_.substr(k, m - k)) : -1;
      k = m;
    }
    if (k >= p_.size() || p_[k] != '}') return false;
    i_ = k + 1;
    return true;
  }

  std::unique_ptr<Node> repeat(std::unique_ptr<Node> a, const Flags& f) {
    bool seen = false;
    for (;;) {
      char c = peek();
      Op op;
      int lo = 0, hi = 0;
      size_t save = i_;
      if (c == '*') { op = Op::Star; ++i_; }
      else if (c == '+') { op = Op::Plus; ++i_; }
      else if (c == '?') { op = Op::Quest; ++i_; }
      else if (c == '{') {
        if (!try_brace(&lo, &hi)) { if (err_.empty()) i_ = save; return a; }
        if (lo > kMaxRepeat || hi > kMaxRepeat || (hi >= 0 && hi < lo)) {
          fail("invalid repeat count: `" + p_.substr(save, i_ - save) + "`");
          return a;
        }
        op = Op::Repeat;
      } else {
        return a;
      }
      if (seen) { fail("invalid nested repetition operator: `" + p_.substr(save, i_ - save) + "`"); return a; }
      seen = true;
      bool ng = false;
      if (peek() == '?') { ++i_; ng = true; }
      if (f.U) ng = !ng;
      auto n = mk(op);
      n->nongreedy = ng;
      n->min = lo;
      n->max = hi;
      n->sub.push_back(std::move(a));
      a = std::move(n);
      // regexp/syntax parser.repeat: nested counted repeats may not multiply
      // past 1000 (simplify would expand them into that many copies)
      if (op == Op::Repeat && (lo >= 2 || hi >= 2) && !repeat_is_valid(a.get(), kMaxRepeat)) {
        fail("invalid repeat count: `" + p_.substr(save, i_ - save) + "`");
        return a;
      }
    }
  }

  // regexp/syntax repeatIsValid
  static bool repeat_is_valid(const Node* re, int n) {
    if (re->op == Op::Repeat) {
      int m = re->max;
      if (m == 0) return true;
      if (m < 0) m = re->min;
      if (m > n) return false;
      if (m > 0) n /= m;
    }
    for (const auto& s : re->sub)
      if (!repeat_is_valid(s.get(), n)) return false;
    return true;
  }

  std::unique_ptr<Node> literal(uint32_t r, const Flags& f) {
    if (f.i) {
      std::vector<uint32_t> orb = fold_orbit(r);
      if (orb.size() > 1) {
        auto n = mk(Op::CharClass);
        for (uint32_t x : orb) add_range(&n->ranges, x, x);
        normalize(&n->ranges);
        return n;
      }
    }
    auto n = mk(Op::Literal);
    n->rune = r;
    return n;
  }

  std::unique_ptr<Node> atom(Flags* f) {
    char c = peek();
    if (c == '(') return group(f);
    if (c == '[') return char_class(*f);
    if (c == '*' || c == '+' || c == '?') { fail("missing argument to repetition operator: `" + std::string(1, c) + "`"); return nullptr; }
    if (c == '{') {
      size_t save = i_;
      int lo, hi;
      if (try_brace(&lo, &hi)) { fail("missing argument to repetition operator"); return nullptr; }
      i_ = save + 1;
      return literal('{', *f);
    }
    if (c == '.') {
      ++i_;
      return mk(f->s ? Op::AnyChar : Op::AnyCharNotNL);
    }
    if (c == '^') { ++i_; return mk(f->m ? Op::BeginLine : Op::BeginText); }
    if (c == '$') { ++i_; return mk(f->m ? Op::EndLine : Op::EndText); }
    if (c == '\\') return escape(*f);
    return literal(next_rune(), *f);
  }

  // Go rejects trees higher than 1000 (ErrNestingDepth): 1000 nested
  // capture groups around an atom are 1001 levels.  The cap also bounds this
  // parser's and compile()'s recursion on hostile configs (Go, whose
  // non-capturing groups add no level, accepts deeper (?: nesting).
  std::unique_ptr<Node> group(Flags* f) {
    if (++depth_ >= 1000) { fail("expression nests too deeply: `" + p_ + "`"); --depth_; return nullptr; }
    auto n = group_body(f);
    --depth_;
    return n;
  }

  std::unique_ptr<Node> group_body(Flags* f) {
    ++i_;  // '('
    std::string name;
    bool named = false;
    if (peek() == '?') {
      if (p_.compare(i_, 3, "?P<") == 0 || (p_.compare(i_, 2, "?<") == 0 && peek(2) != '=' && peek(2) != '!')) {
        size_t start = i_ + (peek(1) == 'P' ? 3 : 2);
        size_t end = p_.find('>', start);
        if (end == std::string::npos) { fail("invalid named capture: `" + p_ + "`"); return nullptr; }
        name = p_.substr(start, end - start);
        bool ok = !name.empty();
        for (char ch : name) ok = ok && (isalnum(static_cast<unsigned char>(ch)) || ch == '_');
        if (!ok) { fail("invalid named capture: `" + p_ + "`"); return nullptr; }
        named = true;
        i_ = end + 1;
      } else {
        ++i_;
        Flags nf = *f;
        bool neg = false, sawflag = false;
        for (;;) {
          if (eof()) { fail("missing closing ): `" + p_ + "`"); return nullptr; }
          char ch = p_[i_++];
          if (ch == 'i' || ch == 'm' || ch == 's' || ch == 'U') {
            bool v = !neg;
            if (ch == 'i') nf.i = v; else if (ch == 'm') nf.m = v; else if (ch == 's') nf.s = v; else nf.U = v;
            sawflag = true;
          } else if (ch == '-') {
            if (neg) { fail("invalid or unsupported Perl syntax: `" + p_ + "`"); return nullptr; }
            neg = true;
            sawflag = false;
          } else if (ch == ')' || ch == ':') {
            if (neg && !sawflag) { fail("invalid or unsupported Perl syntax: `" + p_ + "`"); return nullptr; }
            if (ch == ')') { *f = nf; return nullptr; }
            auto inner = alternation(&nf);
            if (peek() != ')') { fail("missing closing ): `" + p_ + "`"); return nullptr; }
            ++i_;
            return inner;
          } else {
            fail("invalid or unsupported Perl syntax: `" + p_ + "`");
            return nullptr;
          }
        }
      }
    }
    int cap = ++ncap_;
    names_.push_back(named ? name : "");
    Flags inner_flags = *f;
    auto inner = alternation(&inner_flags);
    if (peek() != ')') { fail("missing closing ): `" + p_ + "`"); return nullptr; }
    ++i_;
    auto n = mk(Op::Capture);
    n->cap = cap;
    n->name = name;
    n->sub.push_back(std::move(inner));
    return n;
  }

  bool escape_rune(uint32_t* out) {
    if (eof()) { fail("trailing backslash at end of expression"); return false; }
    char c = p_[i_++];
    if (c >= '1' && c <= '7') {
      if (!(peek() >= '0' && peek() <= '7')) { fail("invalid escape sequence: `\\" + std::string(1, c) + "`"); return false; }
    }
    if (c >= '0' && c <= '7') {
      uint32_t v = c - '0';
      for (int k = 0; k < 2 && peek() >= '0' && peek() <= '7'; ++k) v = v * 8 + (p_[i_++] - '0');
      *out = v;
      return true;
    }
    if (c == 'x') {
      if (peek() == '{') {
        size_t end = p_.find('}', i_);
        if (end == std::string::npos || end == i_ + 1) { fail("invalid escape sequence"); return false; }
        uint32_t v = 0;
        for (size_t k = i_ + 1; k < end; ++k) {
          char h = p_[k];
          if (!isxdigit(static_cast<unsigned char>(h))) { fail("invalid escape sequence"); return false; }
          v = v * 16 + (isdigit(static_cast<unsigned char>(h)) ? h - '0' : (tolower(h) - 'a' + 10));
          if (v > kMaxRune) { fail("invalid escape sequence"); return false; }
        }
        i_ = end + 1;
        *out = v;
        return true;
      }
      if (i_ + 2 > p_.size() || !isxdigit(static_cast<unsigned char>(p_[i_])) || !isxdigit(static_cast<unsigned char>(p_[i_ + 1]))) {
        fail("invalid escape sequence");
        return false;
      }
      *out = static_cast<uint32_t>(std::stoul(p_.substr(i_, 2), nullptr, 16));
      i_ += 2;
      return true;
    }
    switch (c) {
      case 'a': *out = 7; return true;
      case 'f': *out = 12; return true;
      case 'n': *out = 10; return true;
      case 'r': *out = 13; return true;
      case 't': *out = 9; return true;
      case 'v': *out = 11; return true;
    }
    if (static_cast<unsigned char>(c) < 0x80 && !isalnum(static_cast<unsigned char>(c))) { *out = static_cast<uint8_t>(c); return true; }
    fail(std::string("invalid escape sequence: `\\") + c + "`");
    return false;
  }

  // Go parser.appendGroup: the group is case folded under (?i) first, then
  // negated for \D \S \W / [:^name:].
  static void perl_class(char k, bool fold, std::vector<Range>* v) {
    std::vector<Range> tmp;
    switch (tolower(k)) {
      case 'd': add_range(&tmp, '0', '9'); break;
      case 's': add_range(&tmp, '\t', '\n'); add_range(&tmp, '\f', '\r'); add_range(&tmp, ' ', ' '); break;
      case 'w': add_range(&tmp, '0', '9'); add_range(&tmp, 'A', 'Z'); add_range(&tmp, 'a', 'z'); add_range(&tmp, '_', '_'); break;
    }
    group_into(tmp, fold, isupper(static_cast<unsigned char>(k)), v);
  }

  static void group_into(const std::vector<Range>& g, bool fold, bool neg, std::vector<Range>* v) {
    std::vector<Range> tmp;
    if (fold) { for (const Range& r : g) add_folded(&tmp, r.lo, r.hi); }
    else tmp = g;
    if (neg) negate(&tmp); else normalize(&tmp);
    v->insert(v->end(), tmp.begin(), tmp.end());
  }

  bool posix_class(const std::string& name, std::vector<Range>* v) {
    struct P { const char* n; const char* r; };
    static const P tab[] = {
      {"alnum", "09AZaz"}, {"alpha", "AZaz"}, {"ascii", "\x01\x7f"}, {"blank", "\t\t  "},
      {"cntrl", "\x01\x1f\x7f\x7f"}, {"digit", "09"}, {"graph", "!~"}, {"lower", "az"},
      {"print", " ~"}, {"punct", "!/:@[`{~"}, {"space", "\t\r  "}, {"upper", "AZ"},
      {"word", "09AZ__az"}, {"xdigit", "09AFaf"}};
    for (const P& p : tab) {
      if (name == p.n) {
        const char* r = p.r;
        size_t len = strlen(r);
        for (size_t k = 0; k + 1 < len; k += 2) add_range(v, static_cast<uint8_t>(r[k]), static_cast<uint8_t>(r[k + 1]));
        if (name == "ascii" || name == "cntrl") add_range(v, 0, 0);  // \x00 can't live in a C string
        return true;
      }
    }
    return false;
  }

  bool unicode_class(char pc, bool fold, std::vector<Range>* v) {
    std::string name;
    if (peek() == '{') {
      size_t end = p_.find('}', i_);
      if (end == std::string::npos) { fail("invalid character class range"); return false; }
      name = p_.substr(i_ + 1, end - i_ - 1);
      i_ = end + 1;
    } else {
      if (eof()) { fail("invalid character class range"); return false; }
      name = std::string(1, p_[i_++]);
    }
    bool neg = pc == 'P';
    if (!name.empty() && name[0] == '^') { neg = !neg; name = name.substr(1); }
    std::vector<Range> tmp;
    if (name == "Any") {
      add_range(&tmp, 0, kMaxRune);
    } else {
      bool found = false;
      for (const CatTable& t : kCats) {
        if (name == t.name) {
          for (size_t k = 0; k < t.n; ++k) add_range(&tmp, t.r[k][0], t.r[k][1]);
          found = true;
          break;
        }
      }
      if (!found) { fail("invalid character class range: `\\p{" + name + "}` (unsupported)"); return false; }
    }
    group_into(tmp, fold, neg, v);
    return true;
  }

  std::unique_ptr<Node> escape(const Flags& f) {
    ++i_;  // '\\'
    char c = peek();
    if (c == 'd' || c == 's' || c == 'w' || c == 'D' || c == 'S' || c == 'W') {
      ++i_;
      auto n = mk(Op::CharClass);
      perl_class(c, f.i, &n->ranges);
      normalize(&n->ranges);
      return n;
    }
    if (c == 'p' || c == 'P') {
      ++i_;
      auto n = mk(Op::CharClass);
      if (!unicode_class(c, f.i, &n->ranges)) return nullptr;
      normalize(&n->ranges);
      return n;
    }
    if (c == 'A') { ++i_; return mk(Op::BeginText); }
    if (c == 'z') { ++i_; return mk(Op::EndText); }
    if (c == 'b') { ++i_; return mk(Op::WordBoundary); }
    if (c == 'B') { ++i_; return mk(Op::NoWordBoundary); }
    if (c == 'Q') {
      ++i_;
      size_t end = p_.find("\\E", i_);
      std::string lit = end == std::string::npos ? p_.substr(i_) : p_.substr(i_, end - i_);
      i_ = end == std::string::npos ? p_.size() : end + 2;
      auto n = mk(Op::Concat);
      size_t k = 0;
      while (k < lit.size()) {
        int32_t r; int w;
        decode_rune(reinterpret_cast<const uint8_t*>(lit.data()) + k, lit.size() - k, &r, &w);
        k += w;
        n->sub.push_back(literal(static_cast<uint32_t>(r), f));
      }
      if (n->sub.size() == 1) return std::move(n->sub[0]);
      if (n->sub.empty()) return mk(Op::EmptyMatch);
      return n;
    }
    uint32_t r;
    if (!escape_rune(&r)) return nullptr;
    return literal(r, f);
  }

  bool class_rune(uint32_t* r) {
    if (peek() == '\\') { ++i_; return escape_rune(r); }
    *r = next_rune();
    return err_.empty();
  }

  std::unique_ptr<Node> char_class(const Flags& f) {
    ++i_;  // '['
    bool neg = false;
    if (peek() == '^') { neg = true; ++i_; }
    std::vector<Range> cls;
    bool first = true;
    auto add = [&](uint32_t lo, uint32_t hi) {
      if (f.i) add_folded(&cls, lo, hi); else add_range(&cls, lo, hi);
    };
    while (first || peek() != ']') {
      if (eof()) { fail("missing closing ]: `" + p_ + "`"); return nullptr; }
      first = false;
      if (peek() == '[' && peek(1) == ':') {
        size_t end = p_.find(":]", i_ + 2);
        if (end != std::string::npos) {
          std::string name = p_.substr(i_ + 2, end - i_ - 2);
          bool pneg = !name.empty() && name[0] == '^';
          if (pneg) name = name.substr(1);
          std::vector<Range> tmp;
          if (!posix_class(name, &tmp)) { fail("invalid character class range: `[:" + name + ":]`"); return nullptr; }
          group_into(tmp, f.i, pneg, &cls);
          i_ = end + 2;
          continue;
        }
      }
      if (peek() == '\\' && strchr("dswDSW", peek(1)) && peek(1) != '\0') {
        perl_class(peek(1), f.i, &cls);
        i_ += 2;
        continue;
      }
      if (peek() == '\\' && (peek(1) == 'p' || peek(1) == 'P')) {
        char pc = peek(1);
        i_ += 2;
        if (!unicode_class(pc, f.i, &cls)) return nullptr;
        continue;
      }
      uint32_t lo;
      if (!class_rune(&lo)) return nullptr;
      uint32_t hi = lo;
      if (peek() == '-' && peek(1) != ']' && peek(1) != '\0') {
        ++i_;
        if (!class_rune(&hi)) return nullptr;
        if (hi < lo) { fail("invalid character class range"); return nullptr; }
      }
      add(lo, hi);
    }
    ++i_;  // ']'
    if (neg) negate(&cls); else normalize(&cls);
    auto n = mk(Op::CharClass);
    n->ranges = std::move(cls);
    return n;
  }
};

// ---------------------------------------------------------------- simplify
std::unique_ptr<Node> clone(const Node& n) {
  auto c = std::make_unique<Node>();
  c->op = n.op; c->nongreedy = n.nongreedy; c->rune = n.rune; c->ranges = n.ranges;
  c->min = n.min; c->max = n.max; c->cap = n.cap; c->name = n.name;
  for (const auto& s : n.sub) c->sub.push_back(clone(*s));
  return c;
}

std::unique_ptr<Node> simplify1(Op op, bool ng, std::unique_ptr<Node> sub) {
  if (sub->op == Op::EmptyMatch) return sub;
  if (sub->op == op && sub->nongreedy == ng) return sub;
  auto n = mk(op);
  n->nongreedy = ng;
  n->sub.push_back(std::move(sub));
  return n;
}

std::unique_ptr<Node> simplify(std::unique_ptr<Node> n) {
  for (auto& s : n->sub) s = simplify(std::move(s));
  switch (n->op) {
    case Op::Star: case Op::Plus: case Op::Quest:
      return simplify1(n->op, n->nongreedy, std::move(n->sub[0]));
    case Op::Repeat: {
      const Node& sub = *n->sub[0];
      int mn = n->min, mx = n->max;
      bool ng = n->nongreedy;
      if (mn == 0 && mx == 0) return mk(Op::EmptyMatch);
      if (mx == -1) {
        if (mn == 0) return simplify1(Op::Star, ng, clone(sub));
        if (mn == 1) return simplify1(Op::Plus, ng, clone(sub));
        auto c = mk(Op::Concat);
        for (int k = 0; k < mn - 1; ++k) c->sub.push_back(clone(sub));
        c->sub.push_back(simplify1(Op::Plus, ng, clone(sub)));
        return c;
      }
      if (mn == 1 && mx == 1) return clone(sub);
      std::unique_ptr<Node> prefix;
      if (mn > 0) {
        prefix = mk(Op::Concat);
        for (int k = 0; k < mn; ++k) prefix->sub.push_back(clone(sub));
      }
      if (mx > mn) {
        auto suffix = simplify1(Op::Quest, ng, clone(sub));
        for (int k = mn + 1; k < mx; ++k) {
          auto c = mk(Op::Concat);
          c->sub.push_back(clone(sub));
          c->sub.push_back(std::move(suffix));
          suffix = simplify1(Op::Quest, ng, std::move(c));
        }
        if (!prefix) return suffix;
        prefix->sub.push_back(std::move(suffix));
      }
      if (prefix) return prefix;
      return mk(Op::NoMatch);
    }
    default:
      return n;
  }
}

// ----------------------------------------------------------------- compile
struct Frag {
  uint32_t i = 0;
  std::vector<uint32_t> out;   // patch list: (inst << 1) | is_arg
  bool nullable = false;
};

class Compiler {
 public:
  Prog* p;
  explicit Compiler(Prog* prog) : p(prog) { inst(IOp::Fail); }

  uint32_t inst(IOp op) {
    Inst in;
    in.op = op;
    p->inst.push_back(in);
    return static_cast<uint32_t>(p->inst.size() - 1);
  }
  void patch(const std::vector<uint32_t>& l, uint32_t to) {
    for (uint32_t x : l) {
      if (x & 1) p->inst[x >> 1].arg = to; else p->inst[x >> 1].out = to;
    }
  }
  static std::vector<uint32_t> cat_list(std::vector<uint32_t> a, const std::vector<uint32_t>& b) {
    a.insert(a.end(), b.begin(), b.end());
    return a;
  }

  Frag nop() { Frag f; f.i = inst(IOp::Nop); f.out = {f.i << 1}; f.nullable = true; return f; }
  Frag fail() { Frag f; return f; }
  Frag empty(uint8_t flags) {
    Frag f; f.i = inst(IOp::Empty); p->inst[f.i].arg = flags; f.out = {f.i << 1}; f.nullable = true; return f;
  }
  Frag cap(uint32_t slot) {
    Frag f; f.i = inst(IOp::Capture); p->inst[f.i].arg = slot; f.out = {f.i << 1}; f.nullable = true;
    if (static_cast<int>(slot) + 1 > p->num_cap * 2 + 2) {}
    return f;
  }
  Frag rune(const std::vector<Range>& rs) {
    Frag f;
    if (rs.size() == 1 && rs[0].lo == rs[0].hi) {
      f.i = inst(IOp::Rune1);
      p->inst[f.i].arg = rs[0].lo;
    } else if (rs.size() == 1 && rs[0].lo == 0 && rs[0].hi == kMaxRune) {
      f.i = inst(IOp::RuneAny);
    } else if (rs.size() == 2 && rs[0].lo == 0 && rs[0].hi == 9 && rs[1].lo == 11 && rs[1].hi == kMaxRune) {
      f.i = inst(IOp::RuneAnyNotNL);
    } else {
      f.i = inst(IOp::Rune);
    }
    Inst& in = p->inst[f.i];
    in.rbeg = static_cast<uint32_t>(p->ranges.size());
    in.rcnt = static_cast<uint32_t>(rs.size());
    for (const Range& r : rs) {
      p->ranges.push_back(r);
      for (uint32_t c = r.lo; c <= std::min<uint32_t>(r.hi, 127); ++c) in.ascii[c >> 6] |= 1ull << (c & 63);
      if (r.hi >= 0x80) in.nonascii = true;
    }
    f.out = {f.i << 1};
    return f;
  }
  Frag cat(Frag f1, Frag f2) {
    if (f1.i == 0 || f2.i == 0) return fail();
    patch(f1.out, f2.i);
    Frag f; f.i = f1.i; f.out = std::move(f2.out); f.nullable = f1.nullable && f2.nullable;
    return f;
  }
  Frag alt(Frag f1, Frag f2) {
    if (f1.i == 0) return f2;
    if (f2.i == 0) return f1;
    Frag f; f.i = inst(IOp::Alt);
    p->inst[f.i].out = f1.i;
    p->inst[f.i].arg = f2.i;
    f.out = cat_list(std::move(f1.out), f2.out);
    f.nullable = f1.nullable || f2.nullable;
    return f;
  }
  Frag quest(Frag f1, bool ng) {
    Frag f; f.i = inst(IOp::Alt); f.nullable = true;
    if (ng) { p->inst[f.i].arg = f1.i; f.out = {f.i << 1}; }
    else { p->inst[f.i].out = f1.i; f.out = {(f.i << 1) | 1}; }
    f.out = cat_list(std::move(f.out), f1.out);
    return f;
  }
  Frag loop(Frag f1, bool ng) {
    Frag f; f.i = inst(IOp::Alt);
    if (ng) { p->inst[f.i].arg = f1.i; f.out = {f.i << 1}; }
    else { p->inst[f.i].out = f1.i; f.out = {(f.i << 1) | 1}; }
    patch(f1.out, f.i);
    f.nullable = f1.nullable;
    return f;
  }
  Frag star(Frag f1, bool ng) {
    if (f1.nullable) return quest(plus(f1, ng), ng);
    return loop(f1, ng);
  }
  Frag plus(Frag f1, bool ng) {
    uint32_t start = f1.i;
    bool nl = f1.nullable;
    Frag l = loop(std::move(f1), ng);
    Frag f; f.i = start; f.out = std::move(l.out); f.nullable = nl;
    return f;
  }

  Frag compile(const Node& n) {
    switch (n.op) {
      case Op::NoMatch: return fail();
      case Op::EmptyMatch: return nop();
      case Op::Literal: return rune({{n.rune, n.rune}});
      case Op::CharClass: return rune(n.ranges);
      case Op::AnyCharNotNL: return rune({{0, 9}, {11, kMaxRune}});
      case Op::AnyChar: return rune({{0, kMaxRune}});
      case Op::BeginLine: return empty(kEmptyBeginLine);
      case Op::EndLine: return empty(kEmptyEndLine);
      case Op::BeginText: return empty(kEmptyBeginText);
      case Op::EndText: return empty(kEmptyEndText);
      case Op::WordBoundary: return empty(kEmptyWordBoundary);
      case Op::NoWordBoundary: return empty(kEmptyNoWordBoundary);
      case Op::Capture: {
        Frag bra = cap(static_cast<uint32_t>(n.cap << 1));
        Frag sub = compile(*n.sub[0]);
        Frag ket = cap(static_cast<uint32_t>((n.cap << 1) | 1));
        return cat(cat(std::move(bra), std::move(sub)), std::move(ket));
      }
      case Op::Star: return star(compile(*n.sub[0]), n.nongreedy);
      case Op::Plus: return plus(compile(*n.sub[0]), n.nongreedy);
      case Op::Quest: return quest(compile(*n.sub[0]), n.nongreedy);
      case Op::Concat: {
        if (n.sub.empty()) return nop();
        Frag f;
        for (size_t k = 0; k < n.sub.size(); ++k) {
          if (k == 0) f = compile(*n.sub[k]); else f = cat(std::move(f), compile(*n.sub[k]));
        }
        return f;
      }
      case Op::Alternate: {
        Frag f;
        for (const auto& s : n.sub) f = alt(std::move(f), compile(*s));
        return f;
      }
      case Op::Repeat: break;  // removed by simplify
    }
    return fail();
  }
};

int max_cap(const Node& n) {
  int m = n.op == Op::Capture ? n.cap : 0;
  for (const auto& s : n.sub) m = std::max(m, max_cap(*s));
  return m;
}

// ----------------------------------------------------------------- Pike VM
inline bool rune_match(const Prog& p, const Inst& in, int32_t c) {
  if (c < 0) return false;
  if (c < 128) return (in.ascii[c >> 6] >> (c & 63)) & 1;
  if (!in.nonascii) return false;
  const Range* r = &p.ranges[in.rbeg];
  uint32_t lo = 0, hi = in.rcnt;
  uint32_t uc = static_cast<uint32_t>(c);
  while (lo < hi) {
    uint32_t m = (lo + hi) / 2;
    if (uc < r[m].lo) hi = m;
    else if (uc > r[m].hi) lo = m + 1;
    else return true;
  }
  return false;
}

// The bit-state backtracker's visited set of one thread (see backtrack()).
struct VisitStamps {
  std::vector<uint16_t> stamp;
  uint16_t gen = 0;
};
VisitStamps& visit_stamps() {
  thread_local VisitStamps v;
  return v;
}

class Machine {
 public:
  Machine(const Prog& p, int ncap) : p_(p), ncap_(ncap) {
    if (p.has_first) {
      for (int b = 0; b < 256; ++b) first_[b] = (p.first[b >> 6] >> (b & 63)) & 1;
    }
    size_t n = p.inst.size();
    for (int q = 0; q < 2; ++q) {
      sparse_[q].assign(n, 0);
      dense_pc_[q].assign(n, 0);
      dense_has_[q].assign(n, 0);
      caps_[q].assign(n * std::max(ncap, 1), -1);
      size_[q] = 0;
    }
    matchcap_.assign(std::max(ncap, 1), -1);
    scratch_.assign(std::max(ncap, 1), -1);
    stack_.reserve(64);
  }

  bool match(const uint8_t* s, size_t len, size_t pos0, bool anchored, Cap* caps_out) {
    matched_ = false;
    std::fill(matchcap_.begin(), matchcap_.end(), -1);
    int rq = 0, nq = 1;
    size_[0] = size_[1] = 0;
    size_t pos = pos0;
    int32_t r, r1 = -1;
    int w, w1 = 0;
    decode_rune(s + pos, len - pos, &r, &w);
    if (r >= 0) decode_rune(s + pos + w, len - pos - w, &r1, &w1);
    uint8_t flag = pos == 0 ? empty_context(-1, r) : empty_context(rune_before(s, pos), r);
    for (;;) {
      if (size_[rq] == 0) {
        if (anchored && pos != pos0) break;
        if (matched_) break;
        if (!anchored && p_.has_first && pos < len && !first_[s[pos]]) {
          // no live thread and no match can start here: skip ahead
          size_t np = pos + 1;
          while (np < len && !first_[s[np]]) ++np;
          if (np >= len) break;          // every match consumes a byte
          pos = np;
          decode_rune(s + pos, len - pos, &r, &w);
          if (r >= 0) decode_rune(s + pos + w, len - pos - w, &r1, &w1); else { r1 = -1; w1 = 0; }
          flag = empty_context(rune_before(s, pos), r);
        }
      }
      if (!matched_ && (!anchored || pos == pos0)) {
        if (ncap_ > 0) {
          std::fill(scratch_.begin(), scratch_.end(), -1);
          scratch_[0] = static_cast<Cap>(pos);
        }
        add(rq, p_.start, pos, scratch_.data(), flag);
      }
      uint8_t nflag = empty_context(r, r1);
      step(rq, nq, pos, pos + w, r, nflag);
      if (w == 0) break;
      if (ncap_ == 0 && matched_) break;
      pos += w;
      r = r1; w = w1;
      if (r >= 0) decode_rune(s + pos + w, len - pos - w, &r1, &w1);
      else { r1 = -1; w1 = 0; }
      flag = nflag;
      std::swap(rq, nq);
    }
    size_[nq] = 0;
    if (matched_ && caps_out) std::copy(matchcap_.begin(), matchcap_.begin() + ncap_, caps_out);
    return matched_;
  }

  // Go's backtrack.go for an anchored leftmost-first match whose threads
  // consume at most `window` bytes past pos0: every (pc, pos) pair is
  // explored once, in priority order (the Pike VM's thread order), so the
  // first Match reached is the VM's match with the same submatches.
  // Returns 1 match, 0 none, -1 a thread ran past the window (caller: VM).
  int backtrack(const uint8_t* s, size_t len, size_t pos0, size_t window, Cap* caps_out) {
    const size_t end = std::min(len, pos0 + window);
    const size_t npos = end - pos0 + 1;
    // visited (pc, pos) pairs: generation stamps in one per-thread array
    // shared by every Machine of the thread (calls never nest), so a call
    // clears nothing -- clearing Go's bitmap (program size x window bits,
    // ~5 KB for config 5's custom rules) was a fifth of a candidate's cost
    VisitStamps& vs = visit_stamps();
    const size_t nvis = p_.inst.size() * npos;
    if (vs.stamp.size() < nvis) { vs.stamp.assign(nvis, 0); vs.gen = 0; }
    if (++vs.gen == 0) { std::fill(vs.stamp.begin(), vs.stamp.end(), 0); vs.gen = 1; }
    uint16_t* const stamp = vs.stamp.data();
    const uint16_t gen = vs.gen;
    const int nc = std::max(ncap_, 2);
    bcap_.assign(nc, -1);
    jobs_.clear();
    jobs_.push_back({p_.start, pos0, -1, 0});
    while (!jobs_.empty()) {
      const BJob j = jobs_.back();
      jobs_.pop_back();
      if (j.slot >= 0) { bcap_[j.slot] = j.old; continue; }
      uint32_t pc = j.pc;
      size_t pos = j.pos;
      for (;;) {
        if (pc == 0) break;
        const size_t bit = static_cast<size_t>(pc) * npos + (pos - pos0);
        if (stamp[bit] == gen) break;
        stamp[bit] = gen;
        const Inst& in = p_.inst[pc];
        bool fail = false;
        switch (in.op) {
          case IOp::Fail: fail = true; break;
          case IOp::Alt: case IOp::AltMatch:
            jobs_.push_back({in.arg, pos, -1, 0});
            pc = in.out;
            break;
          case IOp::Nop: pc = in.out; break;
          case IOp::Capture:
            if (static_cast<int>(in.arg) < ncap_) {
              jobs_.push_back({0, 0, static_cast<int>(in.arg), bcap_[in.arg]});
              bcap_[in.arg] = static_cast<Cap>(pos);
            }
            pc = in.out;
            break;
          case IOp::Empty: {
            int32_t r; int w;
            decode_rune(s + pos, len - pos, &r, &w);
            const uint8_t flag = empty_context(pos == 0 ? -1 : rune_before(s, pos), r);
            if (in.arg & ~flag) fail = true; else pc = in.out;
            break;
          }
          case IOp::Match:
            bcap_[0] = static_cast<Cap>(pos0);
            bcap_[1] = static_cast<Cap>(pos);
            if (caps_out && ncap_ > 0) std::copy(bcap_.begin(), bcap_.begin() + ncap_, caps_out);
            return 1;
          default: {   // Rune*: consume one rune
            int32_t c; int w;
            decode_rune(s + pos, len - pos, &c, &w);
            bool ok = false;
            switch (in.op) {
              case IOp::Rune: ok = rune_match(p_, in, c); break;
              case IOp::Rune1: ok = c == static_cast<int32_t>(in.arg); break;
              case IOp::RuneAny: ok = c >= 0; break;
              case IOp::RuneAnyNotNL: ok = c >= 0 && c != '\n'; break;
              default: break;
            }
            if (!ok) { fail = true; break; }
            if (pos + w > end) return -1;
            pos += w;
            pc = in.out;
            break;
          }
        }
        if (fail) break;
      }
    }
    return 0;
  }

 private:
  const Prog& p_;
  int ncap_;
  std::vector<uint32_t> sparse_[2], dense_pc_[2];
  std::vector<uint8_t> dense_has_[2];
  std::vector<Cap> caps_[2];
  uint32_t size_[2];
  std::vector<Cap> matchcap_, scratch_;
  bool matched_ = false;
  uint8_t first_[256] = {0};
  struct Frame { uint32_t pc; int slot; Cap old; };
  std::vector<Frame> stack_;
  struct BJob { uint32_t pc; size_t pos; int slot; Cap old; };   // slot >= 0: a capture restore
  std::vector<BJob> jobs_;
  std::vector<Cap> bcap_;

  bool contains(int q, uint32_t pc) const {
    uint32_t j = sparse_[q][pc];
    return j < size_[q] && dense_pc_[q][j] == pc;
  }

  // Go machine.add: DFS in priority order; capture slots restored on unwind.
  void add(int q, uint32_t pc0, size_t pos, Cap* cap, uint8_t cond) {
    // explicit stack: entries are either (pc) to visit or a capture-restore
    stack_.clear();
    stack_.push_back({pc0, -1, 0});
    while (!stack_.empty()) {
      Frame fr = stack_.back();
      stack_.pop_back();
      if (fr.slot >= 0) { cap[fr.slot] = fr.old; continue; }
      uint32_t pc = fr.pc;
      if (pc == 0) continue;
      if (contains(q, pc)) continue;
      uint32_t j = size_[q]++;
      sparse_[q][pc] = j;
      dense_pc_[q][j] = pc;
      dense_has_[q][j] = 0;
      const Inst& in = p_.inst[pc];
      switch (in.op) {
        case IOp::Fail: break;
        case IOp::Alt: case IOp::AltMatch:
          stack_.push_back({in.arg, -1, 0});
          stack_.push_back({in.out, -1, 0});
          break;
        case IOp::Empty:
          if ((in.arg & ~cond) == 0) stack_.push_back({in.out, -1, 0});
          break;
        case IOp::Nop:
          stack_.push_back({in.out, -1, 0});
          break;
        case IOp::Capture:
          if (static_cast<int>(in.arg) < ncap_) {
            stack_.push_back({0, static_cast<int>(in.arg), cap[in.arg]});   // restore after subtree
            cap[in.arg] = static_cast<Cap>(pos);
            stack_.push_back({in.out, -1, 0});
          } else {
            stack_.push_back({in.out, -1, 0});
          }
          break;
        default:  // Match / Rune*: a thread lives here
          dense_has_[q][j] = 1;
          if (ncap_ > 0) std::copy(cap, cap + ncap_, &caps_[q][static_cast<size_t>(j) * ncap_]);
          break;
      }
    }
  }

  void step(int rq, int nq, size_t pos, size_t npos, int32_t c, uint8_t ncond) {
    for (uint32_t j = 0; j < size_[rq]; ++j) {
      if (!dense_has_[rq][j]) continue;
      const Inst& in = p_.inst[dense_pc_[rq][j]];
      Cap* tcap = ncap_ > 0 ? &caps_[rq][static_cast<size_t>(j) * ncap_] : nullptr;
      bool addit = false;
      switch (in.op) {
        case IOp::Match:
          if (ncap_ > 0) {
            tcap[1] = static_cast<Cap>(pos);
            std::copy(tcap, tcap + ncap_, matchcap_.begin());
          }
          matched_ = true;
          size_[rq] = j + 1;   // cut off lower-priority threads
          break;
        case IOp::Rune: addit = rune_match(p_, in, c); break;
        case IOp::Rune1: addit = c == static_cast<int32_t>(in.arg); break;
        case IOp::RuneAny: addit = c >= 0; break;
        case IOp::RuneAnyNotNL: addit = c >= 0 && c != '\n'; break;
        default: break;
      }
      if (addit) {
        if (ncap_ > 0) {
          std::copy(tcap, tcap + ncap_, scratch_.begin());
          add(nq, in.out, npos, scratch_.data(), ncond);
        } else {
          add(nq, in.out, npos, scratch_.data(), ncond);
        }
      }
    }
    size_[rq] = 0;
  }
};

// ------------------------------------------------------------- lazy DFA
// End of the leftmost-first match anchored at a position, without captures,
// as a DFA built lazily from the program (the RE2 construction).  A state is
// the priority-ordered list of pcs the Pike VM above would add() to its
// queue (before the closure), plus the category of the previous rune; the
// closure is taken when the next rune is known, so empty-width assertions
// see exactly the context Machine::match gives them.  Captures never affect
// which thread wins (priority and dedupe are by pc only), so the match end
// equals Machine::match's caps[1].
class LazyDfa {
 public:
  explicit LazyDfa(const Prog& p) : p_(p) {
    mark_.assign(p.inst.size(), 0);
    for (uint32_t pc = 0; pc < p.inst.size(); ++pc) {
      const IOp op = p.inst[pc].op;
      if (op == IOp::Rune || op == IOp::Rune1 || op == IOp::RuneAny || op == IOp::RuneAnyNotNL) rinst_.push_back(pc);
    }
    for (int c = 0; c < 128; ++c) ascii_cls_[c] = class_of(c);
    states_.push_back(State());                    // state 0: dead (no seeds)
  }

  // -1: no match; -2: state budget exceeded (caller falls back to the VM)
  long match_end(const uint8_t* s, size_t len, size_t pos) {
    const int32_t pr = pos == 0 ? -1 : rune_before(s, pos);
    const uint8_t c0 = cat(pr);
    int st = start_[c0];                             // the start state per previous-rune category
    if (st < 0) {
      seeds_.assign(1, p_.start);
      st = intern(seeds_, c0);
      if (st < 0) return -2;                         // state budget exceeded
      start_[c0] = st;
    }
    long end = -1;
    size_t p = pos;
    for (;;) {
      if (st == 0) break;
      if (p >= len) {
        if (eot(st)) end = static_cast<long>(len);
        break;
      }
      int k, w;
      if (s[p] < 0x80) { k = ascii_cls_[s[p]]; w = 1; }
      else { int32_t r; decode_rune(s + p, len - p, &r, &w); k = class_of(r); }
      int32_t t = states_[st].next.size() > static_cast<size_t>(k) ? states_[st].next[k] : -1;
      if (t < 0) {
        t = transition(st, k);
        if (t < 0) return -2;
      }
      if (t & 1) end = static_cast<long>(p);
      st = t >> 1;
      p += w;
    }
    return end;
  }

 private:
  struct State {
    std::vector<uint32_t> seeds;
    uint8_t prev = 0;                // category of the previous rune
    std::vector<int32_t> next;       // per class: (state << 1) | match-before-this-rune; -1 unknown
    int8_t eot = -1;
  };
  static constexpr size_t kMaxStates = 4096;
  int start_[4] = {-1, -1, -1, -1};
  const Prog& p_;
  std::vector<uint32_t> rinst_;
  int ascii_cls_[128];
  std::vector<int32_t> cls_rep_;                 // class -> representative rune
  std::unordered_map<std::string, int> cls_ids_;
  std::unordered_map<int32_t, int> nonascii_cls_;
  std::vector<State> states_;
  std::unordered_map<std::string, int> state_ids_;
  std::vector<uint32_t> mark_, seeds_, threads_, stack_;
  uint32_t gen_ = 0;

  // rune categories that decide empty-width contexts: 0 begin/end of text,
  // 1 '\n', 2 word character, 3 anything else
  static uint8_t cat(int32_t r) { return r < 0 ? 0 : r == '\n' ? 1 : is_word(r) ? 2 : 3; }
  static int32_t rep_of_cat(uint8_t c) { static const int32_t k[4] = {-1, '\n', 'a', ' '}; return k[c]; }

  bool consumes(uint32_t pc, int32_t c) const {
    const Inst& in = p_.inst[pc];
    switch (in.op) {
      case IOp::Rune: return rune_match(p_, in, c);
      case IOp::Rune1: return c == static_cast<int32_t>(in.arg);
      case IOp::RuneAny: return c >= 0;
      case IOp::RuneAnyNotNL: return c >= 0 && c != '\n';
      default: return false;
    }
  }

  int class_of(int32_t r) {
    if (r >= 0x80) {
      auto it = nonascii_cls_.find(r);
      if (it != nonascii_cls_.end()) return it->second;
    }
    std::string sig(1, static_cast<char>(cat(r)));
    sig.resize(1 + (rinst_.size() + 7) / 8, 0);
    for (size_t i = 0; i < rinst_.size(); ++i)
      if (consumes(rinst_[i], r)) sig[1 + i / 8] = static_cast<char>(sig[1 + i / 8] | (1 << (i & 7)));
    auto ins = cls_ids_.emplace(sig, static_cast<int>(cls_rep_.size()));
    if (ins.second) cls_rep_.push_back(r);
    if (r >= 0x80) nonascii_cls_.emplace(r, ins.first->second);
    return ins.first->second;
  }

  int intern(const std::vector<uint32_t>& seeds, uint8_t prev) {
    if (seeds.empty()) return 0;
    std::string key(1, static_cast<char>(prev));
    key.append(reinterpret_cast<const char*>(seeds.data()), seeds.size() * sizeof(uint32_t));
    auto it = state_ids_.find(key);
    if (it != state_ids_.end()) return it->second;
    if (states_.size() >= kMaxStates) return -1;
    State st;
    st.seeds = seeds;
    st.prev = prev;
    states_.push_back(std::move(st));
    const int id = static_cast<int>(states_.size()) - 1;
    state_ids_.emplace(std::move(key), id);
    return id;
  }

  // Machine::add over every seed in order (shared visited set): the thread
  // pcs (Match / Rune*) in priority order
  void closure(const std::vector<uint32_t>& seeds, uint8_t cond) {
    if (++gen_ == 0) { std::fill(mark_.begin(), mark_.end(), 0); gen_ = 1; }
    threads_.clear();
    for (uint32_t s0 : seeds) {
      stack_.assign(1, s0);
      while (!stack_.empty()) {
        const uint32_t pc = stack_.back();
        stack_.pop_back();
        if (pc == 0 || mark_[pc] == gen_) continue;
        mark_[pc] = gen_;
        const Inst& in = p_.inst[pc];
        switch (in.op) {
          case IOp::Fail: break;
          case IOp::Alt: case IOp::AltMatch: stack_.push_back(in.arg); stack_.push_back(in.out); break;
          case IOp::Empty: if ((in.arg & ~cond) == 0) stack_.push_back(in.out); break;
          case IOp::Nop: case IOp::Capture: stack_.push_back(in.out); break;
          default: threads_.push_back(pc); break;
        }
      }
    }
  }

  int32_t transition(int st, int k) {
    const int32_t c = cls_rep_[k];
    const uint8_t cond = empty_context(rep_of_cat(states_[st].prev), c);
    closure(states_[st].seeds, cond);
    bool matched = false;
    std::vector<uint32_t> nseeds;
    const uint32_t g = gen_;
    (void)g;
    for (uint32_t pc : threads_) {
      const Inst& in = p_.inst[pc];
      if (in.op == IOp::Match) { matched = true; break; }   // lower-priority threads are cut
      if (consumes(pc, c) && std::find(nseeds.begin(), nseeds.end(), in.out) == nseeds.end()) nseeds.push_back(in.out);
    }
    const int to = intern(nseeds, cat(c));
    if (to < 0) return -1;
    const int32_t t = (to << 1) | (matched ? 1 : 0);
    State& S = states_[st];
    if (S.next.size() < cls_rep_.size()) S.next.resize(cls_rep_.size(), -1);
    S.next[k] = t;
    return t;
  }

  bool eot(int st) {
    State& S = states_[st];
    if (S.eot < 0) {
      closure(S.seeds, empty_context(rep_of_cat(S.prev), -1));
      bool m = false;
      for (uint32_t pc : threads_) if (p_.inst[pc].op == IOp::Match) { m = true; break; }
      S.eot = m ? 1 : 0;
    }
    return S.eot == 1;
  }
};

// First-byte set of a program: follow non-consuming instructions from start
// (assertions treated as passable); a reachable Match means no filter.
void compute_first(Prog* p) {
  p->has_first = false;
  if (p->start == 0) return;
  std::vector<char> seen(p->inst.size(), 0);
  std::vector<uint32_t> st{p->start};
  uint64_t f[4] = {0, 0, 0, 0};
  auto set = [&](uint32_t b) { f[b >> 6] |= 1ull << (b & 63); };
  while (!st.empty()) {
    uint32_t pc = st.back();
    st.pop_back();
    if (pc == 0 || seen[pc]) continue;
    seen[pc] = 1;
    const Inst& in = p->inst[pc];
    switch (in.op) {
      case IOp::Alt: case IOp::AltMatch: st.push_back(in.out); st.push_back(in.arg); break;
      case IOp::Capture: case IOp::Empty: case IOp::Nop: st.push_back(in.out); break;
      case IOp::Fail: break;
      case IOp::Match: case IOp::RuneAny: case IOp::RuneAnyNotNL: return;
      case IOp::Rune1: case IOp::Rune:
        for (uint32_t b = 0; b < 128; ++b) if ((in.ascii[b >> 6] >> (b & 63)) & 1) set(b);
        if (in.nonascii || (in.op == IOp::Rune1 && in.arg >= 0x80)) for (uint32_t b = 0x80; b < 256; ++b) set(b);
        break;
    }
  }
  std::copy(f, f + 4, p->first);
  p->has_first = true;
}

}  // namespace

std::vector<uint32_t> fold_orbit(uint32_t r) {
  std::vector<uint32_t> out{r};
  const size_t n = sizeof(kFoldOrbit) / sizeof(kFoldOrbit[0]);
  uint32_t f;
  if (!lookup_pair(kFoldOrbit, n, r, &f)) return out;
  while (f != r) {
    out.push_back(f);
    if (!lookup_pair(kFoldOrbit, n, f, &f)) break;
  }
  std::sort(out.begin(), out.end());
  return out;
}

bool is_print(uint32_t r) {
  if (r == 0x20) return true;
  static const char* cats[] = {"L", "M", "N", "P", "S"};
  for (const char* c : cats) {
    for (const CatTable& t : kCats) {
      if (t.name[0] == c[0] && t.name[1] == 0) {
        size_t lo = 0, hi = t.n;
        while (lo < hi) {
          size_t m = (lo + hi) / 2;
          if (r < t.r[m][0]) hi = m; else if (r > t.r[m][1]) lo = m + 1; else return true;
        }
      }
    }
  }
  return false;
}

uint32_t to_lower(uint32_t r) {
  if (r < 0x80) return (r >= 'A' && r <= 'Z') ? r + 32 : r;
  uint32_t l;
  if (lookup_pair(kLower, sizeof(kLower) / sizeof(kLower[0]), r, &l)) return l;
  return r;
}

void append_utf8(std::string* out, uint32_t r) {
  if (r < 0x80) { out->push_back(static_cast<char>(r)); return; }
  if (r < 0x800) { out->push_back(static_cast<char>(0xC0 | (r >> 6))); out->push_back(static_cast<char>(0x80 | (r & 0x3F))); return; }
  if (r < 0x10000) {
    out->push_back(static_cast<char>(0xE0 | (r >> 12)));
    out->push_back(static_cast<char>(0x80 | ((r >> 6) & 0x3F)));
    out->push_back(static_cast<char>(0x80 | (r & 0x3F)));
    return;
  }
  out->push_back(static_cast<char>(0xF0 | (r >> 18)));
  out->push_back(static_cast<char>(0x80 | ((r >> 12) & 0x3F)));
  out->push_back(static_cast<char>(0x80 | ((r >> 6) & 0x3F)));
  out->push_back(static_cast<char>(0x80 | (r & 0x3F)));
}

namespace {

// Rune ranges a one-rune node matches (false: not a one-rune node).
bool rune_cover(const Node& n, std::vector<Range>* out) {
  switch (n.op) {
    case Op::AnyChar: out->push_back({0, 0x10FFFF}); return true;
    case Op::AnyCharNotNL: out->push_back({0, 9}); out->push_back({11, 0x10FFFF}); return true;
    case Op::CharClass: out->insert(out->end(), n.ranges.begin(), n.ranges.end()); return true;
    case Op::Literal: out->push_back({n.rune, n.rune}); return true;
    case Op::Capture: return rune_cover(*n.sub[0], out);
    case Op::Alternate:
      for (const auto& c : n.sub) if (!rune_cover(*c, out)) return false;
      return true;
    default: return false;
  }
}

bool matches_every_rune(const Node& n) {
  std::vector<Range> r;
  if (!rune_cover(n, &r)) return false;
  std::sort(r.begin(), r.end(), [](const Range& a, const Range& b) { return a.lo < b.lo; });
  uint32_t next = 0;                     // every rune below `next` is covered
  for (const Range& x : r) {
    if (x.lo > next) return false;
    if (x.hi >= next) next = x.hi + 1;
  }
  return next > 0x10FFFF;
}

void flatten_concat(const Node& n, std::vector<const Node*>* items) {
  if (n.op == Op::Concat) { for (const auto& c : n.sub) flatten_concat(*c, items); return; }
  items->push_back(&n);
}

// L1 X* L2 (X matches every rune; L1, L2 non-empty ASCII literal runs)
int span_shape(const Node& ast, std::string* l1, std::string* l2) {
  std::vector<const Node*> items;
  flatten_concat(ast, &items);
  size_t k = 0;
  l1->clear();
  l2->clear();
  while (k < items.size() && items[k]->op == Op::Literal && items[k]->rune < 0x80) l1->push_back(static_cast<char>(items[k++]->rune));
  if (l1->empty() || k >= items.size() || items[k]->op != Op::Star || !matches_every_rune(*items[k]->sub[0])) return 0;
  const int shape = items[k]->nongreedy ? 2 : 1;
  ++k;
  while (k < items.size() && items[k]->op == Op::Literal && items[k]->rune < 0x80) l2->push_back(static_cast<char>(items[k++]->rune));
  if (l2->empty() || k != items.size()) return 0;
  return shape;
}

}  // namespace

static bool begins_with_text_start(const Node& n);

// Longest match of n in bytes, -1 when unbounded.  A rune node takes at most
// the UTF-8 length of its largest rune (an invalid byte decodes to U+FFFD
// with width 1, never more).
static long max_width(const Node& n) {
  auto rune_bytes = [](uint32_t r) -> long { return r < 0x80 ? 1 : r < 0x800 ? 2 : r < 0x10000 ? 3 : 4; };
  switch (n.op) {
    case Op::NoMatch: case Op::EmptyMatch: case Op::BeginLine: case Op::EndLine: case Op::BeginText:
    case Op::EndText: case Op::WordBoundary: case Op::NoWordBoundary:
      return 0;
    case Op::Literal: return rune_bytes(n.rune);
    case Op::CharClass: {
      uint32_t hi = 0;
      for (const Range& r : n.ranges) hi = std::max(hi, r.hi);
      return n.ranges.empty() ? 0 : rune_bytes(hi);
    }
    case Op::AnyChar: case Op::AnyCharNotNL: return 4;
    case Op::Capture: case Op::Quest: return n.sub.empty() ? 0 : max_width(*n.sub[0]);
    case Op::Star: case Op::Plus: {
      const long w = n.sub.empty() ? 0 : max_width(*n.sub[0]);
      return w == 0 ? 0 : -1;
    }
    case Op::Repeat: {
      const long w = n.sub.empty() ? 0 : max_width(*n.sub[0]);
      if (w < 0) return -1;
      if (w == 0) return 0;
      return n.max < 0 ? -1 : w * n.max;
    }
    case Op::Concat: {
      long t = 0;
      for (const auto& c : n.sub) {
        const long w = max_width(*c);
        if (w < 0) return -1;
        t += w;
      }
      return t;
    }
    case Op::Alternate: {
      long t = 0;
      for (const auto& c : n.sub) {
        const long w = max_width(*c);
        if (w < 0) return -1;
        t = std::max(t, w);
      }
      return t;
    }
  }
  return -1;
}

std::unique_ptr<Regexp> Regexp::compile(const std::string& pattern, std::string* err) {
  static std::atomic<uint64_t> next_id{1};
  auto re = std::unique_ptr<Regexp>(new Regexp());
  re->id_ = next_id.fetch_add(1);
  re->pattern_ = pattern;
  Parser ps(pattern);
  re->ast_ = ps.parse(err, &re->names_);
  if (!re->ast_) return nullptr;
  re->prog_.num_cap = max_cap(*re->ast_);
  auto simp = simplify(clone(*re->ast_));
  Compiler c(&re->prog_);
  Frag f = c.compile(*simp);
  uint32_t m = c.inst(IOp::Match);
  c.patch(f.out, m);
  re->prog_.start = f.i;
  re->nullable_ = f.nullable;
  compute_first(&re->prog_);
  re->span_shape_ = span_shape(*re->ast_, &re->span_l1_, &re->span_l2_);
  re->start_anchored_ = begins_with_text_start(*re->ast_);
  re->max_width_ = max_width(*re->ast_);
  return re;
}

bool Regexp::match_at(const uint8_t* text, size_t len, size_t pos, bool anchored, int ncap_wanted,
                      Cap* caps) const {
  if (prog_.start == 0) return false;
  // one Machine per (thread, Regexp): a direct-mapped per-thread cache keyed
  // by the Regexp's unique (sequential) id -- one probe per call, where a
  // scan over every cached regexp cost more than the match itself on the
  // short paths of image layers
  constexpr size_t kSlots = 4096;
  thread_local std::vector<std::pair<uint64_t, std::unique_ptr<Machine>>> cache(kSlots);
  auto& slot = cache[id_ & (kSlots - 1)];
  (void)ncap_wanted;
  if (slot.first != id_ || !slot.second) {
    slot.second.reset(new Machine(prog_, 2 * (prog_.num_cap + 1)));
    slot.first = id_;
  }
  // TSG_RE_NO_BACKTRACK=1: the Pike VM only (differential tests)
  static const bool no_bt = std::getenv("TSG_RE_NO_BACKTRACK") && std::atoi(std::getenv("TSG_RE_NO_BACKTRACK")) != 0;
  if (!no_bt && anchored && max_width_ >= 0 && pos <= len) {
    // Go's bit-state limit: (program size) x (window + 1) <= 256 Kbit
    const size_t window = std::min<size_t>(static_cast<size_t>(max_width_), len - pos);
    if (prog_.inst.size() * (window + 1) <= 256 * 1024) {
      const int r = slot.second->backtrack(text, len, pos, window, caps);
      if (r >= 0) return r == 1;
    }
  }
  return slot.second->match(text, len, pos, anchored, caps);
}

long Regexp::match_end(const uint8_t* text, size_t len, size_t pos) const {
  if (prog_.start == 0) return -1;
  // Bounded-width patterns take Go's bit-state backtracker (match_at's): a
  // per-thread lazy DFA builds its states and transitions over the first
  // hundreds of calls of each regexp (config 5: 7.7 us per call against ~1 us
  // backtracking), which a batch's few candidates per rule and thread never
  // amortise.  TSG_RE_MATCH_END_DFA=1 keeps the lazy DFA (A/B runs).
  static const bool dfa_only = std::getenv("TSG_RE_MATCH_END_DFA") && std::atoi(std::getenv("TSG_RE_MATCH_END_DFA")) != 0;
  if (!span_shape_ && !dfa_only && max_width_ >= 0 && pos <= len &&
      prog_.inst.size() * (std::min<size_t>(static_cast<size_t>(max_width_), len - pos) + 1) <= 256 * 1024) {
    thread_local std::vector<Cap> bcaps;
    bcaps.resize(2 * (prog_.num_cap + 1));
    return match_at(text, len, pos, true, 0, bcaps.data()) ? bcaps[1] : -1;
  }
  return match_end_dfa(text, len, pos);
}

long Regexp::match_end_dfa(const uint8_t* text, size_t len, size_t pos) const {
  if (prog_.start == 0) return -1;
  if (span_shape_) {
    // L1 X* L2: X* takes any run of runes, and L2 (ASCII) starts on a rune
    // boundary wherever it occurs, so the match ends after the last (greedy)
    // or first (lazy) occurrence of L2 at or after pos + |L1|
    const size_t n1 = span_l1_.size(), n2 = span_l2_.size();
    if (pos + n1 + n2 > len || std::memcmp(text + pos, span_l1_.data(), n1) != 0) return -1;
    const size_t lo = pos + n1;
    if (span_shape_ == 2) {
      const void* q = memmem(text + lo, len - lo, span_l2_.data(), n2);
      return q ? static_cast<long>(static_cast<const uint8_t*>(q) - text + n2) : -1;
    }
    for (size_t hi = len - n2 + 1; hi > lo;) {       // candidate starts in [lo, hi)
      const void* q = memrchr(text + lo, span_l2_[0], hi - lo);
      if (!q) break;
      const size_t at = static_cast<const uint8_t*>(q) - text;
      if (std::memcmp(text + at, span_l2_.data(), n2) == 0) return static_cast<long>(at + n2);
      hi = at;
    }
    return -1;
  }
  // per-thread DFA cache, direct-mapped by the Regexp's sequential id (as
  // match_at's): config 5 has ~600 regexes, a linear probe cost ~300 compares
  constexpr size_t kSlots = 4096;
  thread_local std::vector<std::pair<uint64_t, std::unique_ptr<LazyDfa>>> cache(kSlots);
  auto& slot = cache[id_ & (kSlots - 1)];
  if (slot.first != id_ || !slot.second) {
    slot.second.reset(new LazyDfa(prog_));
    slot.first = id_;
  }
  LazyDfa* d = slot.second.get();
  long e = d->match_end(text, len, pos);
  if (e == -2) {                        // state budget exceeded: start a fresh DFA next time, use the VM now
    slot.second.reset(new LazyDfa(prog_));
    std::vector<Cap> caps(2 * (prog_.num_cap + 1));
    e = match_at(text, len, pos, true, 0, caps.data()) ? caps[1] : -1;
  }
  return e;
}

// Length of the gate sequence `seq` occurring at text[i..] (0: none there).
static size_t seq_at(const std::vector<std::vector<std::string>>& seq, const uint8_t* text, size_t len, size_t i) {
  size_t p = i;
  for (const auto& unit : seq) {
    bool any = false;
    for (const auto& alt : unit) {
      // alternatives of a unit are whole runes (1-byte ASCII or a complete
      // UTF-8 sequence): none is a proper prefix of another
      if (p + alt.size() <= len && std::memcmp(text + p, alt.data(), alt.size()) == 0) {
        p += alt.size();
        any = true;
        break;
      }
    }
    if (!any) return 0;
  }
  return p - i;
}

// Every match of n starts at the beginning of the text: n begins with
// BeginText (Go's ^ without (?m), \A) on every alternative.
static bool begins_with_text_start(const Node& n) {
  switch (n.op) {
    case Op::BeginText: return true;
    case Op::Capture:
    case Op::Concat: return !n.sub.empty() && begins_with_text_start(*n.sub[0]);
    case Op::Alternate:
      if (n.sub.empty()) return false;
      for (const auto& s : n.sub) if (!begins_with_text_start(*s)) return false;
      return true;
    default: return false;
  }
}

bool Regexp::gate_hit_at(const uint8_t* text, size_t len, size_t i) const {
  if (gate_.empty()) return true;
  if (i >= len || !gate_first_[text[i]]) return false;
  for (const auto& seq : gate_) if (seq_at(seq, text, len, i)) return true;
  return false;
}

bool Regexp::match_string(const uint8_t* text, size_t len) const {
  if (gate_.empty()) {
    thread_local std::vector<Cap> caps0;
    caps0.resize(2 * (prog_.num_cap + 1));
    return match_at(text, len, 0, false, 0, caps0.data());
  }
  auto hit_at = [&](size_t i) {
    if (!gate_first_[text[i]]) return false;
    for (const auto& seq : gate_) if (seq_at(seq, text, len, i)) return true;
    return false;
  };
  if (start_anchored_) {
    // a match can only start at 0, so its gate literal lies at
    // gate_dmin_..gate_dmax_ (bounded) or anywhere (unbounded)
    const size_t hi = gate_bounded_ ? std::min<size_t>(gate_dmax_ + 1, len) : len;
    bool hit = false;
    for (size_t i = gate_bounded_ ? gate_dmin_ : 0; i < hi && !hit; ++i) hit = hit_at(i);
    if (!hit) return false;
    thread_local std::vector<Cap> caps2;
    caps2.resize(2 * (prog_.num_cap + 1));
    return match_at(text, len, 0, true, 0, caps2.data());
  }
  if (!gate_bounded_) {
    for (size_t i = 0; i < len; ++i) {
      if (hit_at(i)) {
        thread_local std::vector<Cap> caps1;
        caps1.resize(2 * (prog_.num_cap + 1));
        return match_at(text, len, 0, false, 0, caps1.data());
      }
    }
    return false;                                  // no gate literal: no match can exist
  }
  // every match starts gate_dmin_..gate_dmax_ bytes before a gate literal;
  // starts already tried are skipped (a per-thread scratch, no allocation
  // per call)
  thread_local std::vector<uint8_t> tried;
  thread_local std::vector<Cap> caps;
  bool first = true;
  for (size_t i = gate_dmin_; i < len; ++i) {
    if (!hit_at(i)) continue;
    if (first) {
      first = false;
      tried.assign(len + 1, 0);
      caps.resize(2 * (prog_.num_cap + 1));
    }
    const size_t lo = i >= gate_dmax_ ? i - gate_dmax_ : 0, hi = i - gate_dmin_;
    for (size_t s0 = lo; s0 <= hi; ++s0) {
      if (tried[s0]) continue;
      tried[s0] = 1;
      if (match_at(text, len, s0, true, 0, caps.data())) return true;
    }
  }
  return false;
}

void Regexp::find_all(const uint8_t* text, size_t len, bool submatch, std::vector<Cap>* out) const {
  const int ncap = 2 * (prog_.num_cap + 1);
  std::vector<Cap> caps(ncap);
  size_t pos = 0;
  long prev_end = -1;
  while (pos <= len) {
    if (!match_at(text, len, pos, false, ncap, caps.data())) break;
    bool accept = true;
    if (static_cast<size_t>(caps[1]) == pos) {
      if (caps[0] == prev_end) accept = false;
      int32_t r; int w;
      decode_rune(text + pos, len - pos, &r, &w);
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

}  // namespace re
}  // namespace tsg
