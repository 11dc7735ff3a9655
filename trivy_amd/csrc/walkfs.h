// Filesystem walk: walker.FS.Walk
// (pkg/fanal/walker/fs.go:25-78) over a directory tree on disk -- Go's
// filepath.WalkDir order (lexical, directories entered as met, symlinks not
// followed), BuildSkipPaths (fs.go:99-149) + defaultSkipDirs (walk.go:11-16),
// utils.SkipPath (doublestar) on the slash path relative to the root,
// permission errors ignored (fs.go:81-96) -- then the regular files' contents
// read with several threads for the batched analyzer feed.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace tsg {

struct FsFile {
  std::string rel;      // filepath.ToSlash(filepath.Rel(root, path)): the analyzer's FilePath
  std::string path;     // path as opened (root joined with the entries)
  uint64_t size = 0;    // info.Size() (stat_fs_files; UINT64_MAX: vanished)
};

struct FsWalk {
  std::vector<FsFile> files;   // every regular file handed to the WalkFunc, walk order
};

// skip_files / skip_dirs as given on the command line (--skip-files /
// --skip-dirs); err mirrors Walk's "walk dir error: unknown error with ...".
// Directories are read by `threads` threads; the files come back in
// WalkDir's order.
bool walk_fs_tree(const std::string& root, const std::vector<std::string>& skip_files,
                  const std::vector<std::string>& skip_dirs, int threads, FsWalk* out, std::string* err);

// info.Size() of the files with want[i] (lstat, `threads` threads)
bool stat_fs_files(FsWalk* walk, const std::vector<uint8_t>& want, int threads);

// walker.FS.BuildSkipPaths(base, paths) with the process's working directory
std::string go_filepath_clean(const std::string& p);
std::vector<std::string> build_skip_paths(const std::string& base, const std::vector<std::string>& paths);

// Read files[i] (only i with want[i]) into buf + starts[i], sizes[i] bytes,
// `threads` readers; a file shorter than its walked size ends early
// (got[i] = bytes read).  Non-permission open/read errors fail like
// AnalyzeFile's "unable to open %s"; a permission error drops the file
// (got[i] = UINT64_MAX), as AnalyzeFile skips it.
bool read_fs_files(const FsWalk& walk, const std::vector<uint8_t>& want, const std::vector<uint64_t>& starts,
                   uint8_t* buf, int threads, std::vector<uint64_t>* got, std::string* err);

}  // namespace tsg
