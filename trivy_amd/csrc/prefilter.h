// Rule compiler for the GPU prefilter (host side, run once per ruleset, the
// equivalent of where the reference compiles its regexes: ParseConfig /
// NewScanner, pkg/fanal/secret/scanner.go:75-87,320-364).
//
// Produces, from the Go regexp ASTs and keywords of every rule:
//  * one SCAN DFA over bytes (`.*(p1|p2|...)`) whose patterns are
//      - every distinct ASCII keyword under bytes.ToLower semantics
//        (A-Z folded; U+0130 -> 'i', U+212A -> 'k' as in unicode.ToLower),
//        exact, giving the per-(file, rule) keyword gate of
//        Rule.MatchKeywords (scanner.go:174-186);
//      - ANCHOR literals: for each rule a set of literal unit sequences such
//        that every match of the rule's regex contains one of them at a
//        byte offset d in [dmin, dmax] from the match start;
//  * one anchored VERIFY DFA per rule: a relaxed superset of the regex
//    (assertions -> empty, non-ASCII runes -> 1-4 high bytes, long repeats
//    loosened, tail truncated to fit a state budget), accepting as soon as a
//    prefix of the text from a candidate start is in the relaxed language.
// A rule with no usable anchor (nullable regex, unbounded prefix) is marked
// FULL: the host evaluates it exactly over the whole file.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "scanner.h"

namespace tsg {

struct DfaTable {
  uint32_t nstates = 0;     // state 0 = start; state `dead` = no match possible
  uint32_t nclasses = 0;
  uint32_t dead = 0;
  uint8_t byte_class[256] = {0};
  std::vector<uint16_t> next;          // nstates * nclasses
  std::vector<uint8_t> accept;         // verify DFA: absorbing accept flag per state
};

struct ScanDfa {
  DfaTable t;
  uint32_t first_out_state = 0;        // states >= this have outputs (renumbered)
  std::vector<uint32_t> out_off;       // (nstates - first_out_state + 1) offsets into out_ids
  std::vector<uint32_t> out_ids;       // output ids: [0, nkw) keywords, [nkw, nkw+nanchor) anchors
  uint32_t max_pattern_bytes = 1;      // warm-up window = max_pattern_bytes - 1
  uint32_t kw_base = 0;                // GPU group: keyword ids [kw_base, kw_base+128) kept in register masks
  uint32_t npatterns = 0;
};

// K1 keeps one scan DFA in LDS next to 16 per-wave hit buffers of 4 KiB; its
// transitions are uint16 row offsets (state * stride), so a GPU scan DFA
// must satisfy nstates * stride <= 65535 and fit the LDS left over.
constexpr uint32_t kK1LdsBytes = 160 * 1024;
constexpr uint32_t kK1WaveHits = 512;    // per-wave LDS hit buffer entries (K1) when the table leaves room
constexpr uint32_t kK1WaveHitsMin = 64;  // ... and the least a group is planned with; further hits go to global
constexpr uint32_t kK1HitLdsBytes = 16 * kK1WaveHits * 4 + 16 * 4 + 16;
constexpr uint32_t kK1HitLdsMin = 16 * kK1WaveHitsMin * 4 + 16 * 4 + 16;
uint32_t k1_row_stride(uint32_t nclasses);          // >= nclasses + 1, odd number of dwords
// Output-state rows carry their output metadata inline after the spare slot:
// keyword masks (8 x uint16) and the output list's begin / count (2 x uint16).
uint32_t k1_out_row_stride(uint32_t nclasses);      // k1_row_stride + 10, rounded to an odd number of dwords
uint64_t k1_table_words16(const ScanDfa& d);        // silent rows then output rows
size_t k1_lds_table_bytes(const ScanDfa& d);        // scan table + class map + output metadata
bool k1_fits(const ScanDfa& d);

// K1c: the scan DFA of ALL patterns as one compressed LDS table, for rule
// sets whose full table does not fit K1's LDS (config 5: 4020 states x 53
// classes = 426 KB as a full table, 3 K1 passes; compressed ~140 KB, 1 pass).
//
// A few states keep a FULL row (uint32 packed next states per class); every
// other state is its "default" full state's row plus at most four classes
// that go elsewhere (at most two targets, each reached by at most two of the
// four classes when there are two), kept in a 16-byte DESC record.  A state
// is one packed uint32:
//   bit   0      the state has outputs (its DESC record holds the output index)
//   bits  4..15  LDS byte address of its DESC record (256 = the shared record
//                with no exceptions; records are 16-byte aligned, below 64 KiB)
//   bits 16..31  LDS dword address of its full row (its own, or its default's)
// so one byte is: the row entry FULL[row + class] and the record DESC[idx],
// both addressed from the state alone (issued together, one LDS round trip),
// then the record's classes decide between its targets and the row entry.
// LDS image: [class map 256 B][DESC ndesc x 16 B][FULL nfull x row_stride x 4 B].
struct CompressedScan {
  bool ok = false;
  uint32_t nclasses = 0, row_stride = 0;      // row_stride: odd number of dwords >= nclasses
  uint32_t ndesc = 0, nfull = 0, nstates = 0;
  uint8_t cls4[256] = {0};                    // byte -> class * 4
  std::vector<uint32_t> image;                // DESC then FULL, dwords (LDS bytes 256 ..)
  std::vector<uint32_t> state_val;            // packed value of every DFA state (state 0 = start)
  // per output record (indexed by DESC .w): keyword ids < 128 as two masks, then a list
  struct Out { uint64_t kw0, kw1; uint32_t list_begin, list_count; };
  std::vector<Out> outs;
  std::vector<uint32_t> out_list;
  uint32_t max_pattern_bytes = 1;
  size_t lds_bytes() const { return 256 + image.size() * 4; }
};
constexpr uint32_t kK1cNoRecord = 0xffffffffu;

// One K1c step on the host (the kernel's arithmetic; tests and self-checks).
inline uint32_t k1c_step(const CompressedScan& c, uint32_t s, uint32_t b) {
  const uint32_t c4 = c.cls4[b];
  const uint32_t f = c.image[(s >> 16) - 64 + c4 / 4];       // the image starts at LDS byte 256 = dword 64
  const uint32_t* d = c.image.data() + ((s & 0xfff0u) - 256) / 4;
  const uint32_t x = d[0] ^ (c4 * 0x01010101u);
  const uint32_t z = (x - 0x01010101u) & ~x & 0x80808080u;
  return (z & 0x8080u) ? d[1] : (z & 0x80800000u) ? d[2] : f;
}

struct AnchorInfo {                    // one literal of one rule
  uint32_t rule;
  uint32_t min_len, max_len;           // byte length range of the literal
  uint32_t dmin, dmax;                 // byte offset of the literal from the match start
};

struct RuleGpuInfo {
  uint8_t mode;                        // 0 = anchored (GPU candidates), 1 = FULL (host), 2 = no regex,
                                       // 3 = FULL in files containing a required literal (presence anchors),
                                       // 4 = reverse-anchored: candidate starts from a backward walk of
                                       //     the reverse DFA `rev_dfa` from the hit (unbounded prefixes)
  uint8_t gate_on_gpu;                 // keyword gate exact on GPU (ASCII keywords)
  uint8_t always_gate;                 // no keywords (or an empty keyword): gate always true
  uint32_t kw_begin, kw_count;         // keyword ids in Prefilter::rule_kw
  uint32_t verify_dfa;                 // index into verify
  uint32_t verify_limit;               // bytes scanned before giving up (emit conservatively)
  uint32_t rev_dfa = 0;                // mode 4: index into verify of the reverse DFA
};

// Mode 4: a backward walk longer than this many bytes that is still alive
// gives up and asks for the rule in full on the host (candidate start
// kFullScanStart).
constexpr uint32_t kRevLimit = 4096;
constexpr uint64_t kFullScanStart = ~0ull;

struct Prefilter {
  uint32_t nkw = 0;                    // distinct keyword patterns
  // GPU scan DFAs (ASCII-only, case-folded units), one K1 pass each.  The
  // keyword and anchor patterns are partitioned over the groups (a pattern
  // is in exactly one group), so the union of the groups' outputs equals the
  // outputs of one DFA over all patterns.  The builtin rules need one group;
  // large custom rule sets (config 5) are split until every group fits K1.
  std::vector<ScanDfa> groups;
  // K1c: all groups' patterns as one compressed table (ok only when there is
  // more than one group and it fits); the engine then runs one K1c pass
  // instead of one K1 pass per group.  TSG_K1C=0 disables it.
  CompressedScan compressed;
  ScanDfa host_scan;                  // host: + U+0130/U+212A/U+017F alternatives (fold-special files)
  std::vector<AnchorInfo> anchors;
  std::vector<AnchorInfo> host_anchors;   // same ids; byte lengths of the variant forms
  std::vector<RuleGpuInfo> rules;
  std::vector<uint32_t> rule_kw;       // flattened keyword ids per rule
  std::vector<DfaTable> verify;
  std::vector<std::string> kw_text;    // for diagnostics
  std::string report;                  // human-readable compile summary
};

bool build_prefilter(const Ruleset& rs, Prefilter* out, std::string* err);

// Required-literal gate of a regexp (false: none found): every match contains
// one of the sequences.  Set on path / allow regexes so MatchString skips the
// VM on texts that contain none (scanner.go's per-file AllowPath/MatchPath).
// Bounded (*bounded): every match starts *dmin..*dmax bytes before one.
bool literal_gate(const re::Node& ast, re::LitGate* out, bool* bounded, uint32_t* dmin, uint32_t* dmax);

// CPU model of the two GPU passes (used by unit tests to check the compiled
// tables without a GPU, never by the product path): returns per-rule sorted
// candidate starts and keyword-gate bits for one file.
// Returns true when the file contains U+0130 (C4 B0), U+212A (E2 84 AA) or
// U+017F (C5 BF): the scan DFA is ASCII-only, so such files are evaluated
// exactly on the host (FilePlan == nullptr).
bool prefilter_reference_file(const Prefilter& pf, const uint8_t* data, size_t len,
                              std::vector<std::vector<uint64_t>>* cand_per_rule,
                              std::vector<uint8_t>* gate_per_rule);

// Host path for fold-special files: the same two passes with the variant scan
// DFA (exact for those runes).  Product code (used by Engine::scan).
void prefilter_variant_file(const Prefilter& pf, const uint8_t* data, size_t len,
                            std::vector<std::vector<uint64_t>>* cand_per_rule,
                            std::vector<uint8_t>* gate_per_rule);

// FilePlan from per-rule candidate lists (moves the lists into the plan).
void plan_from_candidates(const Prefilter& pf, std::vector<std::vector<uint64_t>>* cands, FilePlan* plan);

// True when bytes[i-2..i] end one of the fold-special sequences above.
inline bool fold_special_at(uint8_t p2, uint8_t p1, uint8_t b) {
  return (b == 0xB0 && p1 == 0xC4) || (b == 0xBF && p1 == 0xC5) || (b == 0xAA && p1 == 0x84 && p2 == 0xE2);
}

}  // namespace tsg
