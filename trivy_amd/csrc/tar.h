// Layer-tar walk: walker.LayerTar.Walk
// (pkg/fanal/walker/tar.go:35-103) over an uncompressed layer tar held in
// memory, restated without Go's archive/tar: the regular files the walk hands
// to the analyzers, plus the layer's opaque directories and whiteout files.
#pragma once
#include <cstdint>
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

// skip_files / skip_dirs as given to walker.Option (cleaned here with
// utils.CleanSkipPaths, matched with doublestar.Match as utils.SkipPath does).
// Errors mirror Walk's: "failed to extract the archive: ..." for a malformed
// tar.
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
