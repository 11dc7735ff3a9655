// Layer-tar walk: walker.LayerTar.Walk
// (pkg/fanal/walker/tar.go:35-103) over an uncompressed layer tar held in
// memory, restated without Go's archive/tar: the regular files the walk hands
// to the analyzers, plus the layer's opaque directories and whiteout files.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace tsg {

struct TarFile {
  std::string path;        // path.Clean(hdr.Name) with leading '/' trimmed (tar.go:47-48)
  uint64_t offset = 0;     // content offset in the tar
  uint64_t size = 0;
};

struct LayerWalk {
  std::vector<TarFile> files;        // regular files, tar order
  std::vector<std::string> opq_dirs; // ".wh..wh..opq" parents (tar.go:52-55)
  std::vector<std::string> wh_files; // ".wh.<name>" targets (tar.go:57-61)
};

// The bytes of a layer tar: held in memory (tsg_prepare_layer_tar) or pulled
// from a reader (an io.Reader: tsg_scan_layer_stream), consumed in order.
class TarInput {
 public:
  virtual ~TarInput() = default;
  // up to n bytes into dst; *got = 0 only at the end of the data; false: read error (*err)
  virtual bool read(uint8_t* dst, size_t n, size_t* got, std::string* err) = 0;
  // skip up to n bytes; *got < n only at the end of the data
  virtual bool skip(uint64_t n, uint64_t* got, std::string* err);
  uint64_t pos = 0;                  // bytes consumed so far
};

// exactly n bytes unless the data ends first (*got < n); false: read error
bool read_full(TarInput& in, uint8_t* dst, size_t n, size_t* got, std::string* err);

class MemTarInput : public TarInput {
 public:
  MemTarInput(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  bool read(uint8_t* dst, size_t n, size_t* got, std::string* err) override;
  bool skip(uint64_t n, uint64_t* got, std::string* err) override;
 private:
  const uint8_t* p_;
  size_t n_;
};

// Called, positioned at its data, for every regular file Walk hands to the
// analyzers (processFile, tar.go:94-105): it may consume up to `size` bytes of
// `in` (the walker skips the rest); false stops the walk with *err.
using TarFileFn = std::function<bool(const std::string& path, uint64_t size, TarInput& in, std::string* err)>;

// skip_files / skip_dirs as given to walker.Option (cleaned here with
// utils.CleanSkipPaths, matched with doublestar.Match as utils.SkipPath does).
// Errors mirror Walk's: "failed to extract the archive: ..." for a malformed
// tar (archive/tar's ErrHeader, io.ErrUnexpectedEOF, ErrFieldTooLong for a
// PAX / GNU long-name entry over 1 MiB).
bool walk_layer(TarInput& in, const std::vector<std::string>& skip_files, const std::vector<std::string>& skip_dirs,
                LayerWalk* out, const TarFileFn& on_file, std::string* err);

// walk_layer over a tar in memory: out->files carry each file's content offset
bool walk_layer_tar(const uint8_t* tar, size_t len, const std::vector<std::string>& skip_files,
                    const std::vector<std::string>& skip_dirs, LayerWalk* out, std::string* err);

// Go path.Clean (Unix, slash-separated)
std::string go_path_clean(const std::string& p);
// github.com/bmatcuk/doublestar/v4 Match(pattern, name) for the syntax
// utils.SkipPath patterns use: '*', '**' path segments, '?', '[...]' classes
// ('!' / '^' negation, ranges), '{a,b}' alternatives, '\' escapes.  A bad
// pattern returns false (SkipPath treats the error as "no match").
bool doublestar_match(const std::string& pattern, const std::string& name);

}  // namespace tsg
