// GPU engine: device-resident rule tables + per-batch scan on one MI355X.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "prefilter.h"
#include "scanner.h"

namespace tsg {

struct ScanStats {
  double k1_ms = 0, k2_ms = 0, h2d_ms = 0, d2h_ms = 0, host_ms = 0, total_ms = 0;
  double gpu_wall_ms = 0;               // run_gpu() wall time (launches + syncs + copies)
  uint64_t bytes = 0, files = 0, hits = 0, candidates = 0, confirm_files = 0, findings = 0;
  uint32_t k1_blocks = 0, k1_threads = 0, chunk_bytes = 0, pieces = 1;
  int table_in_lds = 0;
};

struct BatchInput {
  const uint8_t* h_data = nullptr;     // host copy (needed by the exact confirmer)
  const void* d_data = nullptr;        // device copy; nullptr -> engine uploads h_data
  const uint64_t* offsets = nullptr;   // nfiles + 1 byte offsets into data
  uint32_t nfiles = 0;
  const char* const* paths = nullptr;  // nfiles NUL-terminated paths (ScanArgs.FilePath)
  const uint32_t* path_lens = nullptr; // optional explicit lengths
  const uint8_t* binary = nullptr;     // optional ScanArgs.Binary flags
};

class Engine {
 public:
  // Fails (returns nullptr, *err set) when no HIP device is available: the
  // product path has no CPU fallback.
  static std::unique_ptr<Engine> create(std::shared_ptr<const Ruleset> rs, int device, std::string* err);
  ~Engine();

  // Scan one batch; results[i] is Scanner.Scan(ScanArgs{paths[i], data[off[i]:off[i+1]], binary[i]}).
  bool scan(const BatchInput& in, std::vector<Secret>* results, ScanStats* stats, std::string* err);

  // Only the two GPU passes (no host confirmation): used by bench.py to time
  // the kernels in isolation and by tests to compare raw candidates.
  bool prefilter_only(const BatchInput& in, std::vector<uint8_t>* kw_gate /*nfiles*nrules or null*/,
                      std::vector<std::vector<std::vector<uint64_t>>>* cands /*[file][rule] or null*/,
                      ScanStats* stats, std::string* err);

  const Prefilter& prefilter() const { return pf_; }
  std::shared_ptr<const Ruleset> ruleset() const { return rs_; }
  int device() const { return device_; }
  void set_threads(int n) { threads_ = n; }

  struct Impl;
  struct GpuOut;

 private:
  Engine() = default;
  bool run_gpu(const BatchInput& in, ScanStats* stats, GpuOut* out, std::string* err);
  void confirm_piece(const BatchInput& in, const GpuOut& g, Secret* results, uint64_t* nconf, uint64_t* nfind,
                     bool gpu_in_flight);
  std::shared_ptr<const Ruleset> rs_;
  Prefilter pf_;
  int device_ = 0;
  int threads_ = 0;
  std::unique_ptr<Impl> impl_;
};

int device_count();

}  // namespace tsg
