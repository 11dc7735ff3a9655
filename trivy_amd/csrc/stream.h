// Streamed feed -> scan pipeline: a layer tar pulled
// from a reader (walker.LayerTar.Walk over an io.Reader,
// pkg/fanal/walker/tar.go:35-103) or a directory tree (walker.FS.Walk,
// fs.go:25-97), each file through AnalyzeFile's gate (analyzer.go:403-419)
// and SecretAnalyzer.Analyze's preparation (secret.go:103-150), packed into
// bounded batches that are scanned while the next batch is walked, read and
// prepared -- end-to-end time is the larger of feed and scan, not their sum,
// and host memory is bounded by the batch size (plus the largest file, which
// Analyze's io.ReadAll holds whole in the reference too).
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "engine.h"
#include "feed.h"
#include "scanner.h"
#include "walkfs.h"

namespace tsg {

// A reader (io.Reader): > 0 bytes read into buf, 0 at the end, < 0 on an error.
using StreamReadFn = int64_t (*)(void* user, uint8_t* buf, size_t cap);

struct StreamOpts {
  FeedOpts feed;
  std::vector<std::string> skip_files, skip_dirs;
  uint64_t batch_bytes = 256ull << 20;   // raw bytes per batch (a larger file is a batch of its own); host memory ~4 batches
  int threads = 16;                      // prepare / read threads of the producer
  bool pinned = true;                    // prepared batches in pinned host memory (the GPU engine)
};

struct StreamStats {
  double wall_ms = 0;        // first byte walked -> last result
  double feed_ms = 0;        // producer busy: walk + read + prepare
  double scan_ms = 0;        // consumer busy: the scan stage
  double wait_ms = 0;        // producer time blocked on a free batch buffer (scan-bound)
  uint64_t walked_bytes = 0; // bytes of every file handed to the analyzers (raw)
  uint64_t read_bytes = 0;   // raw bytes of the files the secret analyzer kept (read)
  uint64_t scanned_bytes = 0;// ScanArgs.Content bytes scanned
  uint64_t batches = 0, files = 0, peak_batch_bytes = 0;
};

struct StreamResult {
  SecretVec files;              // every scanned file, walk order
  std::vector<std::string> walked;        // every regular file handed to the analyzers, walk order
  std::vector<std::string> opq_dirs, wh_files;
  StreamStats st;
};

// scan_path_prefix: "/" for image layers (secret.go:131-135), "" for fs trees.
bool stream_layer(const Ruleset& rs, const StreamOpts& o, StreamReadFn read, void* user, const BatchScanFn& scan,
                  StreamResult* out, std::string* err);
bool stream_fs_tree(const Ruleset& rs, const StreamOpts& o, const std::string& root, const BatchScanFn& scan,
                    StreamResult* out, std::string* err);

// fs-tree planning shared with tsg_prepare_fs_tree: walk, d.Info() of every
// walked file, AnalyzeFile's gate; keep = indices of the files to read, walk order.
bool plan_fs_tree(const Ruleset& rs, const FeedOpts& fo, const std::string& root,
                  const std::vector<std::string>& skip_files, const std::vector<std::string>& skip_dirs, int threads,
                  FsWalk* walk, std::vector<uint32_t>* keep, std::string* err);

}  // namespace tsg
