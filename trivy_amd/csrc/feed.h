// Host feed: batched SecretAnalyzer.Required + content preparation.
#pragma once
#include <cstdint>
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

// Output buffer for the packed contents: returns memory of `bytes` bytes and
// sets the deleter, or nullptr (the batch then uses the heap).
using FeedAlloc = uint8_t* (*)(size_t bytes, void (**free_fn)(uint8_t*));

// keep(i) = Required(path_i, size_i) && (!IsBinary || ext == ".pyc")
bool prepare_batch(const Ruleset& rs, const std::string& config_path, const uint8_t* raw, const uint64_t* raw_off,
                   uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, int threads,
                   PreparedBatch* out, std::string* err, FeedAlloc alloc = nullptr);

// The same over files at arbitrary places of one buffer (a layer tar):
// file i is raw[starts[i], starts[i] + sizes[i]) with Required's path paths[i].
bool prepare_files(const Ruleset& rs, const std::string& config_path, const uint8_t* raw, const uint64_t* starts,
                   const uint64_t* sizes, const std::vector<std::string>& paths, int threads, PreparedBatch* out,
                   std::string* err, FeedAlloc alloc = nullptr);

}  // namespace tsg
