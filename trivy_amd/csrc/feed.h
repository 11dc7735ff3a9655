// Host feed: batched SecretAnalyzer.Required + content preparation.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "scanner.h"

namespace tsg {

struct PreparedBatch {
  std::shared_ptr<uint8_t> data;   // kept files' ScanArgs.Content, back to back (+64 B pad)
  bool pinned = false;             // data is pinned host memory (tsg_alloc_pinned)
  std::vector<uint64_t> offsets;   // nkept + 1
  std::vector<uint32_t> index;     // source file index of each kept file
  std::vector<uint8_t> binary;     // ScanArgs.Binary (a .pyc scanned as printable runs)
};

namespace re { class Regexp; }

// AnalyzerGroup options the secret analyzer's feed depends on.
struct FeedOpts {
  std::string config_path;                         // SecretAnalyzer.configPath (Required skips its base name)
  std::vector<std::shared_ptr<re::Regexp>> patterns;   // --file-patterns "secret:<re>" (analyzer.go:332-350)
  bool assume_required = false;                    // Required/patterns already decided by the caller
};

// --file-patterns entries ("fileType:regexPattern"; only "secret" ones kept),
// with analyzer.go:332-350's errors for a malformed entry or regexp.
bool parse_file_patterns(const std::vector<std::string>& entries, FeedOpts* out, std::string* err);

// AnalyzeFile's gate for the secret analyzer (analyzer.go:403-419):
// filePatternMatch(TrimLeft(path, "/")) || Required(TrimLeft(path, "/"), size)
bool secret_analyzer_wants(const Ruleset& rs, const FeedOpts& opts, const std::string& path, uint64_t size);
// The same split for a walk that learns sizes later: 0 = not wanted, 1 =
// wanted by a file pattern (any size), 2 = wanted if size >= 10 (Required).
int secret_analyzer_wants_path(const Ruleset& rs, const FeedOpts& opts, const std::string& path);

// Output buffer for the packed contents: returns memory of `bytes` bytes and
// sets the deleter, or nullptr (the batch then uses the heap).  An empty
// FeedAlloc means the heap.
using FeedFree = std::function<void(uint8_t*)>;
using FeedAlloc = std::function<uint8_t*(size_t bytes, FeedFree* free_fn)>;

// keep(i) = (filePatternMatch || Required)(path_i, size_i) && (!IsBinary || ext == ".pyc")
bool prepare_batch(const Ruleset& rs, const FeedOpts& opts, const uint8_t* raw, const uint64_t* raw_off,
                   uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, int threads,
                   PreparedBatch* out, std::string* err, FeedAlloc alloc = {});
bool prepare_files(const Ruleset& rs, const FeedOpts& opts, const uint8_t* raw, const uint64_t* starts,
                   const uint64_t* sizes, const std::vector<std::string>& paths, int threads, PreparedBatch* out,
                   std::string* err, FeedAlloc alloc = {});

bool prepare_batch(const Ruleset& rs, const std::string& config_path, const uint8_t* raw, const uint64_t* raw_off,
                   uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, int threads,
                   PreparedBatch* out, std::string* err, FeedAlloc alloc = {});

// The same over files at arbitrary places of one buffer (a layer tar):
// file i is raw[starts[i], starts[i] + sizes[i]) with Required's path paths[i].
bool prepare_files(const Ruleset& rs, const std::string& config_path, const uint8_t* raw, const uint64_t* starts,
                   const uint64_t* sizes, const std::vector<std::string>& paths, int threads, PreparedBatch* out,
                   std::string* err, FeedAlloc alloc = {});

}  // namespace tsg
