// Go `regexp` semantics (RE2 syntax, leftmost-first, UTF-8 runes) for the host
// side of the secret scanner.  The reference compiles every rule with Go's
// regexp.Compile (pkg/fanal/secret/scanner.go:66-87) and calls FindAllIndex /
// FindAllSubmatchIndex / MatchString (scanner.go:112,130,171,207,216,264).
// Go is not available to link against, so this engine restates the semantics:
//   * parser: Perl flags (i m s U), (?P<n>..)/(?<n>..), classes, \pX, POSIX
//     classes, repeats <= 1000, ClassNL/OneLine (syntax.Perl defaults)
//   * simplify: x{n,m} -> n copies + nested quests, x** -> x* (syntax.Simplify)
//   * program: Go-shaped instruction list (Alt/Capture/EmptyWidth/Rune...),
//     star of a nullable body compiled as (x+)?  (syntax/compile.go)
//   * Pike VM: priority-ordered threads, first thread to reach a pc wins,
//     first match cuts lower-priority threads (regexp/exec.go)
//   * allMatches: empty match right after a previous match is skipped.
// Invalid UTF-8 bytes decode as U+FFFD with width 1 (utf8.DecodeRune).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace tsg {
namespace re {

enum class Op : uint8_t {
  NoMatch, EmptyMatch, Literal, CharClass, AnyCharNotNL, AnyChar,
  BeginLine, EndLine, BeginText, EndText, WordBoundary, NoWordBoundary,
  Capture, Star, Plus, Quest, Repeat, Concat, Alternate
};

struct Range { uint32_t lo, hi; };

// Match offsets (64-bit: files of 2 GiB and more are valid Go []byte inputs).
using Cap = int64_t;

struct Node {
  Op op = Op::EmptyMatch;
  bool nongreedy = false;
  uint32_t rune = 0;              // Literal (one rune; case folding already expanded to CharClass)
  std::vector<Range> ranges;      // CharClass: sorted, non-overlapping, merged
  int min = 0, max = 0;           // Repeat (max == -1: unbounded)
  int cap = 0;                    // Capture index (1-based)
  std::string name;               // Capture name
  std::vector<std::unique_ptr<Node>> sub;
};

// Empty-width assertion bits (syntax.EmptyOp)
enum : uint8_t {
  kEmptyBeginLine = 1, kEmptyEndLine = 2, kEmptyBeginText = 4, kEmptyEndText = 8,
  kEmptyWordBoundary = 16, kEmptyNoWordBoundary = 32
};

enum class IOp : uint8_t { Alt, AltMatch, Capture, Empty, Match, Fail, Nop, Rune, Rune1, RuneAny, RuneAnyNotNL };

struct Inst {
  IOp op;
  uint32_t out = 0, arg = 0;      // Alt: out (preferred) / arg; Capture: arg = slot; Empty: arg = flags; Rune1: arg = rune
  uint32_t rbeg = 0, rcnt = 0;    // Rune: ranges in Prog::ranges
  uint64_t ascii[2] = {0, 0};     // Rune/Rune1: ASCII membership bitmap
  bool nonascii = false;          // Rune: has any range >= 0x80
};

struct Prog {
  std::vector<Inst> inst;
  std::vector<Range> ranges;
  uint32_t start = 0;
  int num_cap = 0;                // capture groups, excluding group 0
  // Bytes that can begin a match (first byte of the first rune); used to skip
  // positions in an unanchored search while no thread is alive.  Performance
  // only: has_first == false when a match may be empty or start anywhere.
  bool has_first = false;
  uint64_t first[4] = {0, 0, 0, 0};
};

// Go utf8.DecodeRune: rune + width; invalid -> 0xFFFD width 1; at end width 0.
inline void decode_rune(const uint8_t* s, size_t n, int32_t* r, int* w) {
  if (n == 0) { *r = -1; *w = 0; return; }
  uint8_t c = s[0];
  if (c < 0x80) { *r = c; *w = 1; return; }
  auto cont = [](uint8_t b) { return (b & 0xC0) == 0x80; };
  if (c >= 0xC2 && c <= 0xDF) {
    if (n >= 2 && cont(s[1])) { *r = ((c & 0x1F) << 6) | (s[1] & 0x3F); *w = 2; return; }
  } else if (c >= 0xE0 && c <= 0xEF) {
    uint8_t lo = 0x80, hi = 0xBF;
    if (c == 0xE0) lo = 0xA0;
    if (c == 0xED) hi = 0x9F;
    if (n >= 3 && s[1] >= lo && s[1] <= hi && cont(s[2])) {
      *r = ((c & 0x0F) << 12) | ((s[1] & 0x3F) << 6) | (s[2] & 0x3F); *w = 3; return;
    }
  } else if (c >= 0xF0 && c <= 0xF4) {
    uint8_t lo = 0x80, hi = 0xBF;
    if (c == 0xF0) lo = 0x90;
    if (c == 0xF4) hi = 0x8F;
    if (n >= 4 && s[1] >= lo && s[1] <= hi && cont(s[2]) && cont(s[3])) {
      *r = ((c & 0x07) << 18) | ((s[1] & 0x3F) << 12) | ((s[2] & 0x3F) << 6) | (s[3] & 0x3F); *w = 4; return;
    }
  }
  *r = 0xFFFD; *w = 1;
}

// Go unicode.SimpleFold orbit of r (including r), sorted.
std::vector<uint32_t> fold_orbit(uint32_t r);
// Go unicode.ToLower (simple mapping).
uint32_t to_lower(uint32_t r);
// Go unicode.IsPrint: categories L, M, N, P, S and U+0020.
bool is_print(uint32_t r);
// Append UTF-8 encoding of rune r.
void append_utf8(std::string* out, uint32_t r);

// Required-literal gate: alternatives of literal sequences (each unit a set of
// alternative byte strings); every match of the regexp contains at least one.
using LitGate = std::vector<std::vector<std::vector<std::string>>>;

class Regexp {
 public:
  // Returns nullptr and sets *err on a syntax error (Go: "error parsing regexp: ...").
  static std::unique_ptr<Regexp> compile(const std::string& pattern, std::string* err);

  const std::string& pattern() const { return pattern_; }
  const Node* ast() const { return ast_.get(); }
  const Prog& prog() const { return prog_; }
  int num_subexp() const { return prog_.num_cap; }
  // SubexpNames(): index 0 is "" (the whole match).
  const std::vector<std::string>& subexp_names() const { return names_; }

  // Leftmost-first match search starting at `pos` (context from the whole text).
  // If `anchored`, only a match starting exactly at `pos` is considered.
  // caps receives 2*(num_subexp+1) offsets (-1 for non-participating groups).
  bool match_at(const uint8_t* text, size_t len, size_t pos, bool anchored, int ncap_wanted,
                Cap* caps) const;
  // End offset of the leftmost-first match anchored at `pos` (-1: none),
  // from a lazily built DFA (no captures); equals match_at(.., true, ..)'s caps[1].
  long match_end(const uint8_t* text, size_t len, size_t pos) const;
  // match_end's lazy-DFA path alone (bounded-width patterns otherwise take
  // the backtracker): the same result, for tests
  long match_end_dfa(const uint8_t* text, size_t len, size_t pos) const;
  // Regexp.MatchString (with a gate set: false without running the VM when
  // no gate literal occurs in the text -- no match can exist then)
  bool match_string(const uint8_t* text, size_t len) const;
  // bounded gate: every match starts dmin..dmax bytes before a gate literal,
  // so only those starts are tried (anchored)
  void set_gate(LitGate g, bool bounded = false, uint32_t dmin = 0, uint32_t dmax = 0) {
    gate_ = std::move(g); gate_bounded_ = bounded; gate_dmin_ = dmin; gate_dmax_ = dmax;
    for (auto& f : gate_first_) f = 0;
    for (const auto& seq : gate_)
      for (const auto& alt : seq[0]) gate_first_[static_cast<uint8_t>(alt[0])] = 1;
  }
  const LitGate& gate() const { return gate_; }
  bool has_gate() const { return !gate_.empty(); }
  const uint8_t* gate_first() const { return gate_first_; }   // first bytes of the gate literals
  // Some gate literal occurs at text[i..] (always true without a gate).
  bool gate_hit_at(const uint8_t* text, size_t len, size_t i) const;
  // Regexp.FindAll(Submatch)Index(text, -1): flattened vectors of 2 (or 2*(ncap+1)) ints.
  void find_all(const uint8_t* text, size_t len, bool submatch, std::vector<Cap>* out) const;
  // Minimal byte length of a match (used by the prefilter to reject nullable rules).
  bool nullable() const { return nullable_; }

 private:
  std::string pattern_;
  std::unique_ptr<Node> ast_;     // parsed + simplified
  Prog prog_;
  std::vector<std::string> names_;
  bool nullable_ = false;
  uint64_t id_ = 0;
  LitGate gate_;
  bool start_anchored_ = false;     // every match starts at text offset 0 (leading \A / non-multiline ^)
  uint8_t gate_first_[256] = {};    // first bytes of the gate literals
  bool gate_bounded_ = false;
  uint32_t gate_dmin_ = 0, gate_dmax_ = 0;
  // L1 (any-rune)* L2 with ASCII literals (e.g. the exclude-block idiom
  // `--- ignore block start ---(.|\s)*--- ignore block stop ---`): the
  // anchored leftmost-first end is the last (greedy) / first (lazy) L2 after L1
  int span_shape_ = 0;               // 0 none, 1 greedy star, 2 lazy star
  std::string span_l1_, span_l2_;
  long max_width_ = -1;              // longest match in bytes (-1: unbounded); anchored submatches of a
                                     // bounded regexp take the backtracker (Go's backtrack.go)
};

}  // namespace re
}  // namespace tsg
