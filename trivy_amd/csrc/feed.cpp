// Host feed: SecretAnalyzer.Required + Analyze's content preparation for a
// whole batch (pkg/fanal/analyzer/secret/secret.go:103-190,
// pkg/fanal/utils/utils.go:68-86,111-143), producing the packed ScanArgs
// contents the engine scans.  Two parallel passes (decide + size, then copy)
// around a prefix sum, so a batch of many small files (image layers) is
// prepared at memory speed instead of one Go goroutine per file.
#include "feed.h"

#include "goregexp.h"
#include "guard.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace tsg {
namespace {

const char* const kSkipFiles[] = {"go.mod", "go.sum", "package-lock.json", "yarn.lock", "pnpm-lock.yaml",
                                  "Pipfile.lock", "Gemfile.lock"};                         // secret.go:28-36
const char* const kSkipDirs[] = {".git", "node_modules"};                                 // secret.go:37-40
const char* const kSkipExts[] = {".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg", ".socket", ".deb",
                                 ".rpm", ".zip", ".gz", ".gzip", ".tar"};                  // secret.go:41-62

// filepath.Base (Unix)
std::string go_base(std::string p) {
  if (p.empty()) return ".";
  while (p.size() > 1 && p.back() == '/') p.pop_back();
  if (p == "/") return "/";
  const size_t i = p.rfind('/');
  return i == std::string::npos ? p : p.substr(i + 1);
}

// filepath.Ext of a final path element
std::string go_ext(const std::string& name) {
  for (size_t i = name.size(); i-- > 0;) {
    if (name[i] == '/') break;
    if (name[i] == '.') return name.substr(i);
  }
  return "";
}

bool required_path(const Ruleset& rs, const std::string& path, const std::string& cfg_base);

bool required(const Ruleset& rs, const std::string& path, uint64_t size, const std::string& cfg_base) {
  if (size < 10) return false;                                     // secret.go:154-156
  return required_path(rs, path, cfg_base);
}

// Required's checks other than the size (secret.go:158-188)
bool required_path(const Ruleset& rs, const std::string& path, const std::string& cfg_base) {
  const size_t slash = path.rfind('/');                            // filepath.Split
  const std::string dir = slash == std::string::npos ? "" : path.substr(0, slash + 1);
  const std::string name = slash == std::string::npos ? path : path.substr(slash + 1);
  size_t b = 0;                                                    // strings.Split(dir, "/")
  for (;;) {
    const size_t e = dir.find('/', b);
    const std::string part = dir.substr(b, e == std::string::npos ? std::string::npos : e - b);
    for (const char* sd : kSkipDirs) if (part == sd) return false;
    if (e == std::string::npos) break;
    b = e + 1;
  }
  for (const char* sf : kSkipFiles) if (name == sf) return false;
  if (cfg_base == path) return false;                              // secret.go:178-180
  const std::string ext = go_ext(name);
  for (const char* se : kSkipExts) if (ext == se) return false;
  return !global_allow_path(rs, path);                             // scanner.AllowPath (scanner.go:205-212)
}

// fn(i) for i in [0, n) on `threads` threads, files handed out dynamically
// (one at a time for batches of few, large files; in blocks of 64 otherwise)
template <typename F>
void parallel_for(uint32_t n, int threads, F&& fn) {
  const int nt = std::max(1, std::min<int>(threads, static_cast<int>(n)));
  if (nt == 1) { for (uint32_t i = 0; i < n; ++i) fn(i); return; }
  std::atomic<uint32_t> next{0};
  const uint32_t blk = n >= 256u * static_cast<uint32_t>(nt) ? 64 : 1;
  auto run = [&]() {
    for (;;) {
      const uint32_t b = next.fetch_add(blk);
      if (b >= n) break;
      for (uint32_t i = b, e = std::min(n, b + blk); i < e; ++i) fn(i);
    }
  };
  run_threads(nt, run);
}

std::string trim_left_slash(const std::string& p) {
  size_t i = 0;
  while (i < p.size() && p[i] == '/') ++i;
  return p.substr(i);
}

bool wants(const Ruleset& rs, const FeedOpts& opts, const std::string& path, uint64_t size,
           const std::string& cfg_base) {
  // filepath extracted from a tar file has no "/" prefix (analyzer.go:407-408)
  const std::string clean = trim_left_slash(path);
  for (const auto& rx : opts.patterns)                              // filePatternMatch (analyzer.go:522-530)
    if (rx->match_string(reinterpret_cast<const uint8_t*>(clean.data()), clean.size())) return true;
  return required(rs, clean, size, cfg_base);
}

// The two passes over nfiles files; file(i) gives (content, size, path).
template <typename File>
bool prepare_core(const Ruleset& rs, const FeedOpts& opts, uint32_t nfiles, File&& file, int threads,
                  PreparedBatch* out, FeedAlloc alloc) {
  const std::string cfg_base = go_base(opts.config_path);
  // pass 1: keep decision, binary flag and prepared size per file
  std::vector<uint8_t> keep(nfiles), bin(nfiles);
  std::vector<uint64_t> size(nfiles);
  parallel_for(nfiles, threads, [&](uint32_t i) {
    const uint8_t* c;
    uint64_t n;
    std::string path;
    file(i, &c, &n, &path);
    keep[i] = 0;
    if (!opts.assume_required && !wants(rs, opts, path, n, cfg_base)) return;
    const bool binary = go_is_binary(c, n);                        // secret.go:104-108
    if (binary && go_ext(path) != ".pyc") return;                  // allowedBinary
    bin[i] = binary;
    keep[i] = 1;
    if (binary) {
      size[i] = go_extract_printable(c, n).size();
    } else {
      size[i] = n - static_cast<uint64_t>(std::count(c, c + n, static_cast<uint8_t>('\r')));
    }
  });
  out->index.clear();
  for (uint32_t i = 0; i < nfiles; ++i) if (keep[i]) out->index.push_back(i);
  const uint32_t nk = static_cast<uint32_t>(out->index.size());
  out->offsets.assign(nk + 1, 0);
  out->binary.assign(nk, 0);
  for (uint32_t k = 0; k < nk; ++k) {
    out->offsets[k + 1] = out->offsets[k] + size[out->index[k]];
    out->binary[k] = bin[out->index[k]];
  }
  // not zero-filled (every byte below offsets[nk] is written in pass 2); only
  // the pad K1 may read past the last file is cleared
  const size_t bytes = out->offsets[nk] + 64;
  FeedFree free_fn;
  uint8_t* buf = alloc ? alloc(bytes, &free_fn) : nullptr;
  out->pinned = buf != nullptr;
  if (buf) out->data = std::shared_ptr<uint8_t>(buf, free_fn);
  else out->data = std::shared_ptr<uint8_t>(new uint8_t[bytes], std::default_delete<uint8_t[]>());
  std::memset(out->data.get() + out->offsets[nk], 0, 64);
  // pass 2: write ScanArgs.Content (CR stripped, or the printable runs of a .pyc)
  parallel_for(nk, threads, [&](uint32_t k) {
    const uint8_t* c;
    uint64_t n;
    std::string path;
    file(out->index[k], &c, &n, &path);
    uint8_t* d = out->data.get() + out->offsets[k];
    if (out->binary[k]) {
      const std::string p = go_extract_printable(c, n);
      std::memcpy(d, p.data(), p.size());
      return;
    }
    if (out->offsets[k + 1] - out->offsets[k] == n) { std::memcpy(d, c, n); return; }   // no CR
    for (uint64_t x = 0; x < n; ++x) if (c[x] != '\r') *d++ = c[x];
  });
  return true;
}

}  // namespace

bool parse_file_patterns(const std::vector<std::string>& entries, FeedOpts* out, std::string* err) {
  for (const std::string& p : entries) {
    const size_t colon = p.find(':');                              // strings.SplitN(p, ":", 2)
    if (colon == std::string::npos) {
      *err = "invalid file pattern (" + p + ") expected format: \"fileType:regexPattern\" e.g. "
             "\"dockerfile:my_dockerfile_*\"";
      return false;
    }
    std::string rerr;
    std::unique_ptr<re::Regexp> rx = re::Regexp::compile(p.substr(colon + 1), &rerr);   // regexp.Compile
    if (!rx) { *err = "invalid file regexp (" + p + "): " + rerr; return false; }
    if (p.compare(0, colon, "secret") == 0 && colon == 6) out->patterns.emplace_back(std::move(rx));
  }
  return true;
}

bool secret_analyzer_wants(const Ruleset& rs, const FeedOpts& opts, const std::string& path, uint64_t size) {
  return wants(rs, opts, path, size, go_base(opts.config_path));
}

int secret_analyzer_wants_path(const Ruleset& rs, const FeedOpts& opts, const std::string& path) {
  const std::string clean = trim_left_slash(path);
  for (const auto& rx : opts.patterns)
    if (rx->match_string(reinterpret_cast<const uint8_t*>(clean.data()), clean.size())) return 1;
  return required_path(rs, clean, go_base(opts.config_path)) ? 2 : 0;
}

bool prepare_batch(const Ruleset& rs, const std::string& config_path, const uint8_t* raw, const uint64_t* raw_off,
                   uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, int threads,
                   PreparedBatch* out, std::string* err, FeedAlloc alloc) {
  FeedOpts o;
  o.config_path = config_path;
  return prepare_batch(rs, o, raw, raw_off, nfiles, paths, path_lens, threads, out, err, alloc);
}

bool prepare_files(const Ruleset& rs, const std::string& config_path, const uint8_t* raw, const uint64_t* starts,
                   const uint64_t* sizes, const std::vector<std::string>& paths, int threads, PreparedBatch* out,
                   std::string* err, FeedAlloc alloc) {
  FeedOpts o;
  o.config_path = config_path;
  return prepare_files(rs, o, raw, starts, sizes, paths, threads, out, err, alloc);
}

bool prepare_batch(const Ruleset& rs, const FeedOpts& opts, const uint8_t* raw, const uint64_t* raw_off,
                   uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, int threads,
                   PreparedBatch* out, std::string* err, FeedAlloc alloc) {
  for (uint32_t i = 0; i < nfiles; ++i) {
    if (raw_off[i + 1] < raw_off[i]) { *err = "offsets must be non-decreasing"; return false; }
  }
  return prepare_core(rs, opts, nfiles, [&](uint32_t i, const uint8_t** c, uint64_t* n, std::string* path) {
    *c = raw + raw_off[i];
    *n = raw_off[i + 1] - raw_off[i];
    *path = path_lens ? std::string(paths[i], path_lens[i]) : std::string(paths[i]);
  }, threads, out, alloc);
}

bool prepare_files(const Ruleset& rs, const FeedOpts& opts, const uint8_t* raw, const uint64_t* starts,
                   const uint64_t* sizes, const std::vector<std::string>& paths, int threads, PreparedBatch* out,
                   std::string* err, FeedAlloc alloc) {
  (void)err;
  return prepare_core(rs, opts, static_cast<uint32_t>(paths.size()),
                      [&](uint32_t i, const uint8_t** c, uint64_t* n, std::string* path) {
                        *c = raw + starts[i];
                        *n = sizes[i];
                        *path = paths[i];
                      }, threads, out, alloc);
}

}  // namespace tsg
