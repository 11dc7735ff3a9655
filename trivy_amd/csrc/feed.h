// Host feed: batched SecretAnalyzer.Required + content preparation.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "scanner.h"

namespace tsg {

struct PreparedBatch {
  std::unique_ptr<uint8_t[]> data; // kept files' ScanArgs.Content, back to back (+64 B pad)
  std::vector<uint64_t> offsets;   // nkept + 1
  std::vector<uint32_t> index;     // source file index of each kept file
  std::vector<uint8_t> binary;     // ScanArgs.Binary (a .pyc scanned as printable runs)
};

// keep(i) = Required(path_i, size_i) && (!IsBinary || ext == ".pyc")
bool prepare_batch(const Ruleset& rs, const std::string& config_path, const uint8_t* raw, const uint64_t* raw_off,
                   uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, int threads,
                   PreparedBatch* out, std::string* err);

}  // namespace tsg
