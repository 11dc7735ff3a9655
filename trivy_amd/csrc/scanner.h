// Host side of the secret scanner: rule model and the exact `Scan` semantics of
// pkg/fanal/secret/scanner.go, restricted by a per-(file, rule) plan that the
// GPU prefilter produces.  With no plan this is the reference algorithm
// (every rule's keyword gate and full find-all evaluated on the host).
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <new>
#include <string>
#include <string_view>
#include <cstdlib>
#include <vector>

#include "goregexp.h"
#include "json.h"

namespace tsg {

using RegexpPtr = std::shared_ptr<re::Regexp>;

struct AllowRule {                       // scanner.go:196-201
  std::string id, description;
  RegexpPtr regex, path;
};

struct Rule {                            // scanner.go:89-100
  std::string id, category, title, severity;
  RegexpPtr regex;                       // may be null (scanner.go:103-105)
  std::vector<std::string> keywords;
  std::vector<std::string> keywords_lower;   // strings.ToLower(kw)
  RegexpPtr path;
  std::vector<AllowRule> allow_rules;
  std::vector<RegexpPtr> exclude_block;
  uint32_t exclude_base = 0;             // exclude_block[j] has exclude id exclude_base + j
  std::string secret_group_name;
  std::vector<int> secret_groups;        // i with SubexpNames()[i] == SecretGroupName
};

struct Ruleset {                         // scanner.go:45-49 (Global)
  std::vector<Rule> rules;
  std::vector<AllowRule> allow_rules;
  std::vector<RegexpPtr> exclude_block;  // exclude ids [0, size)
  // Every exclude-block regex (global ones, then each rule's in rule order)
  // by exclude id.  The prefilter treats exclude id k as pseudo-rule
  // rules.size() + k, so block locations come from GPU candidates too.
  std::vector<const re::Regexp*> excludes;
  // The global allow-path regexes indexed by the first bytes of their gate
  // literals: AllowPath over hundreds of thousands of image paths makes one
  // pass over each path to find the few regexes worth running
  // (global_allow_path).  Built by build_ruleset.
  struct AllowPathIndex {
    // Aho-Corasick DFA over every gate literal (case variants expanded) of
    // every global allow-path regex: out[s] = rules with a literal ending in
    // state s (suffix links folded in)
    std::vector<uint16_t> next;  // nstates x 256
    std::vector<uint64_t> out;
    uint64_t always = 0;         // allow rules with a path regex but no (expandable) gate
    bool usable = false;         // <= 64 allow rules and the automaton fits
  } allow_index;
  AllowPathIndex allow_match_index;   // the same over the global allow rules' text regexes
};

// Scanner.AllowPath (scanner.go:205-212): some global allow rule's path regex
// matches `path`; equals the loop over rs.allow_rules.
bool global_allow_path(const Ruleset& rs, const uint8_t* path, size_t n);
inline bool global_allow_path(const Ruleset& rs, const std::string& path) {
  return global_allow_path(rs, reinterpret_cast<const uint8_t*>(path.data()), path.size());
}

// AllowRules.Allow over the global allow rules (scanner.go:52-54, called from
// AllowLocation :150-153): some rule's text regex matches the match text.
bool global_allow_match(const Ruleset& rs, const uint8_t* m, size_t n);

// ParseConfig (already decoded from YAML to JSON) + NewScanner: builtin rules
// and allow rules, enable/disable filters, custom rules appended
// (scanner.go:277-364).  cfg == nullptr -> builtins only.
bool build_ruleset(const JValue* cfg, Ruleset* out, std::string* err);

// Results are stored compactly: every string of one file's findings lives in
// that Secret's arena (one allocation per file instead of ~13 per finding).
struct StrRef { uint32_t off = 0, len = 0; };

struct LineRec {                         // types.Line (misconf.go:51-60)
  int number = 0;
  StrRef content;                        // Highlighted == Content (scanner.go:538-545);
  bool is_cause = false;                 // Annotation "" and Truncated false always
  bool first_cause = false, last_cause = false;
};

struct FindingRec {                      // types.SecretFinding (secret.go:10-20)
  const Rule* rule = nullptr;            // RuleID, Category, Title; Severity ("" -> "UNKNOWN")
  int start_line = 0, end_line = 0;
  StrRef match;
  uint32_t line_begin = 0, line_count = 0;
};

// A read-only view of a contiguous array inside a Secret's block.
template <typename T>
struct PodView {
  const T* p = nullptr;
  size_t n = 0;
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const T& operator[](size_t i) const { return p[i]; }
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
  const T& back() const { return p[n - 1]; }
};

// A Secret under construction (scan_file, the JSON / protobuf decoders):
// growable parts, turned into one compact Secret by build().
struct SecretBuilder {
  std::string file_path;
  std::string arena;
  std::vector<FindingRec> findings;
  std::vector<LineRec> lines;
  int error = 0;
  void clear() { file_path.clear(); arena.clear(); findings.clear(); lines.clear(); error = 0; }
  StrRef put(const char* p, size_t n) {
    StrRef r{static_cast<uint32_t>(arena.size()), static_cast<uint32_t>(n)};
    arena.append(p, n);
    return r;
  }
};

// types.Secret, compact: a file's path, findings, code lines and their text
// live in ONE heap block (none for the empty Secret{} that most files get), so
// a result of hundreds of thousands of files is freed with one free per
// finding file -- round 5 kept four containers per Secret (120 bytes a slot,
// four frees per finding file): a config-5 result took 15-23 ms to free, on
// the reaper beside the next resident step or inline when the reaper lagged.
class Secret {
 public:
  int error = 0;                         // nonzero: the reference would panic on this file
  Secret() = default;
  Secret(Secret&& o) noexcept : error(o.error), blk_(o.blk_) { o.blk_ = nullptr; o.error = 0; }
  Secret& operator=(Secret&& o) noexcept {
    if (this != &o) {
      release();
      blk_ = o.blk_; error = o.error;
      o.blk_ = nullptr; o.error = 0;
    }
    return *this;
  }
  Secret(const Secret&) = delete;
  Secret& operator=(const Secret&) = delete;
  ~Secret() { release(); }

  static Secret build(const SecretBuilder& b);
  static Secret path_only(const char* p, size_t n);   // Secret{FilePath} (a globally allowed path)

  std::string_view file_path() const {
    return blk_ ? std::string_view(path_data(), hdr()->plen) : std::string_view();
  }
  PodView<FindingRec> findings() const {
    return blk_ ? PodView<FindingRec>{reinterpret_cast<const FindingRec*>(blk_ + kHdr), hdr()->nf} : PodView<FindingRec>{};
  }
  PodView<LineRec> lines() const {
    return blk_ ? PodView<LineRec>{reinterpret_cast<const LineRec*>(blk_ + kHdr + hdr()->nf * sizeof(FindingRec)), hdr()->nl}
                : PodView<LineRec>{};
  }
  const char* ptr(StrRef r) const { return text_data() + r.off; }
  static const std::string& severity(const FindingRec& f) {
    static const std::string kUnknown = "UNKNOWN";
    return f.rule->severity.empty() ? kUnknown : f.rule->severity;
  }

 private:
  struct Hdr { uint32_t nf, nl, plen, tlen; };
  static constexpr size_t kHdr = 16;
  static_assert(sizeof(Hdr) == kHdr && alignof(FindingRec) <= kHdr, "block layout");
  char* blk_ = nullptr;                   // [Hdr][FindingRec x nf][LineRec x nl][path][text]
  const Hdr* hdr() const { return reinterpret_cast<const Hdr*>(blk_); }
  const char* path_data() const { return blk_ + kHdr + hdr()->nf * sizeof(FindingRec) + hdr()->nl * sizeof(LineRec); }
  const char* text_data() const { return path_data() + hdr()->plen; }
  void release() { std::free(blk_); blk_ = nullptr; }
};

// The per-file results of a batch (one Secret per file).  A vector whose
// resize default-constructs large ranges on several threads: a batch of
// image-layer files holds hundreds of thousands of Secrets (16 bytes each; 120 until round 5),
// and constructing them on one thread before the first segment's
// confirmation cost 2.7 ms of a 7.9 ms resident config-3 step (page faults
// and stores of ~29 MB; profiles/rd4o_bench_c3prof.log).
class SecretVec {
 public:
  SecretVec() = default;
  ~SecretVec() { destroy(); }
  SecretVec(SecretVec&& o) noexcept : p_(o.p_), n_(o.n_), cap_(o.cap_) { o.p_ = nullptr; o.n_ = o.cap_ = 0; }
  SecretVec& operator=(SecretVec&& o) noexcept {
    if (this != &o) {
      destroy();
      p_ = o.p_; n_ = o.n_; cap_ = o.cap_;
      o.p_ = nullptr; o.n_ = o.cap_ = 0;
    }
    return *this;
  }
  SecretVec(const SecretVec&) = delete;
  SecretVec& operator=(const SecretVec&) = delete;

  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  Secret* data() { return p_; }
  const Secret* data() const { return p_; }
  Secret& operator[](size_t i) { return p_[i]; }
  const Secret& operator[](size_t i) const { return p_[i]; }
  Secret* begin() { return p_; }
  Secret* end() { return p_ + n_; }
  const Secret* begin() const { return p_; }
  const Secret* end() const { return p_ + n_; }
  Secret& back() { return p_[n_ - 1]; }
  void reserve(size_t c);
  void push_back(Secret&& s) {
    if (n_ == cap_) reserve(cap_ < 16 ? 16 : 2 * cap_);
    new (p_ + n_) Secret(std::move(s));
    ++n_;
  }
  void clear();
  // n default-constructed (or kept) Secrets; large growth on several threads
  void resize(size_t n);

 private:
  void destroy();
  Secret* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

// Per-(file, rule) plan from the GPU prefilter.
enum PlanKind : uint8_t {
  kPlanSkip = 0,        // keyword gate false (MatchKeywords == false)
  kPlanNoMatch = 1,     // gate true; no regex match can exist in the file
  kPlanCandidates = 2,  // gate true; every match start lies in `starts`
  kPlanFull = 3,        // host evaluates the gate and a full find-all
  kPlanCandHostGate = 4 // host evaluates the gate exactly; matches only from `starts`
};

struct RuleCandidates {
  uint32_t rule;
  std::vector<uint64_t> starts;          // sorted, unique byte offsets (superset of match starts)
};

struct FilePlan {
  std::vector<uint8_t> kind;             // one PlanKind per rule, then one per exclude regex
  std::vector<RuleCandidates> cands;     // sorted by rule (exclude regexes after the rules)
  // with active_set: every index whose kind is kPlanFull / kPlanCandidates /
  // kPlanCandHostGate, ascending -- scan_file visits only these rules (config
  // 5: 1-3 of 587 per file) instead of testing every rule's kind
  std::vector<uint32_t> active;
  bool active_set = false;
};

// Newline counts for findLocation without rescanning a file: K1's per-chunk
// '\n' counts over the packed batch (chunk c covers data[c*chunk, (c+1)*chunk)).
struct NlSource {
  const uint16_t* chunk_nl = nullptr;
  const uint8_t* data = nullptr;      // packed batch (host)
  uint64_t file_off = 0;              // global offset of this file in data
  uint32_t chunk = 0;
};

// bytes.ToLower (ASCII fast path; Map(unicode.ToLower) with invalid bytes -> U+FFFD)
std::string go_bytes_to_lower(const uint8_t* s, size_t n);
std::string go_str_to_lower(const std::string& s);
// fmt "%q"
std::string go_quote(const std::string& s);

// Scanner.Scan (scanner.go:377-463).  plan == nullptr: reference algorithm.
// TSG_HOST_PROFILE: scan_file's time per phase (ns, summed over threads):
// 0 keyword gate, 1 find_locations, 2 exclude blocks, 3 censor + findings, 4 sort
extern std::atomic<bool> g_scan_prof_on;
extern std::atomic<uint64_t> g_scan_prof[8];
Secret scan_file(const Ruleset& rs, std::string path, const uint8_t* content, size_t len,
                 bool binary, const FilePlan* plan, const NlSource* nl = nullptr);
Secret scan_file(const Ruleset& rs, const char* path, size_t path_len, const uint8_t* content, size_t len,
                 bool binary, const FilePlan* plan, const NlSource* nl = nullptr);

// Exact Go FindAll(Submatch)Index restricted to candidate start offsets.
// `starts` must be a sorted superset of every position where an anchored
// match can start; the result equals re.find_all(text).
void find_all_from_candidates(const re::Regexp& re, const uint8_t* text, size_t len,
                              const std::vector<uint64_t>& starts, bool submatch,
                              std::vector<re::Cap>* out);

// SecretAnalyzer helpers (pkg/fanal/analyzer/secret/secret.go:103-190, utils.go:68-143)
bool go_is_binary(const uint8_t* head, size_t n);
std::string go_extract_printable(const uint8_t* s, size_t n);

}  // namespace tsg
