// Per-file Scan for unchanged callers: SecretAnalyzer.Analyze calls
// Scanner.Scan once per file (pkg/fanal/analyzer/secret/secret.go:137) from
// --parallel goroutines (analyzer.go:434-451, default 5, pkg/flag/
// scan_flags.go:85).  Concurrent scan() calls are gathered into one engine
// batch: the first caller that finds no batch forming leads one, waits until
// as many callers as are expected (the recent peak of concurrent callers,
// less those inside a running batch) have joined -- or the batch is full, or
// max_wait has passed -- packs the contents into a pinned staging buffer and
// scans them; the others sleep until their result is set.
// Several batches may run at once (the engine is reentrant).
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "engine.h"

namespace tsg {

struct QueueStats {
  uint64_t calls = 0, batches = 0, files = 0, bytes = 0;
  uint32_t max_batch = 0;
  uint64_t timeouts = 0;       // leaders that waited the full max_wait
};

class ScanQueue {
 public:
  // scan: the batch stage (Engine::scan; a CPU model in tests)
  ScanQueue(BatchScanFn scan, uint32_t max_files, uint64_t max_bytes, uint32_t max_wait_us, uint32_t max_inflight);
  ~ScanQueue();
  // Scanner.Scan(ScanArgs{path, content, binary}) through a shared batch
  bool scan(const char* path, size_t path_len, const uint8_t* content, size_t len, bool binary, Secret* out,
            std::string* err);
  QueueStats stats();

  // How long a peak of concurrent callers is expected back: the --parallel
  // goroutines return one by one after their batch (read the next file,
  // call again, ~0.2 ms apart), so a peak not seen again for this long is
  // over (a lone caller after a burst does not wait for callers that left).
  static constexpr std::chrono::milliseconds kPeakHold{10};

 private:
  using Clock = std::chrono::steady_clock;
  struct Req {
    const char* path;
    size_t path_len;
    const uint8_t* data;
    size_t len;
    bool binary;
    Secret result;
    std::string err;
    bool done = false;
  };
  struct Staging { void* p = nullptr; size_t cap = 0; };
  void run_batch(std::vector<Req*>& batch);
  Staging take_staging(size_t bytes);
  void give_staging(Staging s);

  BatchScanFn scan_;
  uint32_t max_files_, max_wait_us_, max_inflight_;
  uint64_t max_bytes_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Req*> pending_;
  uint64_t pending_bytes_ = 0;
  uint32_t callers_ = 0;       // callers inside scan()
  uint32_t expect_ = 0;        // callers a leader waits for: the recent peak of callers_ (decays)
  Clock::time_point expect_at_;  // when callers_ last reached expect_
  uint32_t in_batches_ = 0;    // of them, in a running batch
  uint32_t inflight_ = 0;      // running batches
  bool forming_ = false;       // a leader is gathering a batch
  bool spread_ = true;         // expected callers split over the batch slots (TSG_QUEUE_SPREAD=0: one batch gathers them all)
  std::vector<Staging> free_staging_;
  QueueStats st_;
};

}  // namespace tsg
