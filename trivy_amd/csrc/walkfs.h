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
  // Go's walk stops at its first error in walk order; the walk records the
  // earliest one it met (a directory that could not be read, stat_fs_files'
  // d.Info() failures) with its position: err_key = the path relative to the
  // root where WalkDir meets it (walk_order_less orders keys)
  bool failed = false;
  std::string err, err_key;
  // the earliest error wins (the files before it are still walked)
  void fail_at(const std::string& key, const std::string& msg);
};

// WalkDir's order of two relative paths: a pre-order walk with every
// directory's entries in name order ('/' ranks below every other byte)
bool walk_order_less(const std::string& a, const std::string& b);

// skip_files / skip_dirs as given on the command line (--skip-files /
// --skip-dirs); err mirrors Walk's "walk dir error: unknown error with ...".
// Directories are read by `threads` threads; the files come back in
// WalkDir's order.  On an error (false) out->files still holds the files
// walked, out->err / err_key the first error in walk order.
bool walk_fs_tree(const std::string& root, const std::vector<std::string>& skip_files,
                  const std::vector<std::string>& skip_dirs, int threads, FsWalk* out, std::string* err);

// info.Size() (lstat, `threads` threads) of every walked file (WalkDirFunc
// calls d.Info() on each regular, non-skipped file before any analyzer gate,
// fs.go:67-70): a file that cannot be stat'ed (vanished since the walk, ...)
// halts Go's walk with "file info error" -- recorded in walk->err at its
// walk position (size UINT64_MAX).
bool stat_fs_files(FsWalk* walk, int threads);

// walker.FS.BuildSkipPaths(base, paths) with the process's working directory
std::string go_filepath_clean(const std::string& p);
std::vector<std::string> build_skip_paths(const std::string& base, const std::vector<std::string>& paths);

// Read files[i] for i in idx into buf + starts[k] (k = position in idx),
// files[i].size bytes, `threads` readers; a file shorter than its walked size
// ends early (got[k] = bytes read; a file that grew is read up to its walked
// size: Go's io.ReadAll reads to EOF -- a divergence only a concurrent writer
// sees).  A non-permission open error fails like AnalyzeFile's "unable to
// open %s" -- the one earliest in walk order when several files fail; a
// permission error drops the file (got[k] = UINT64_MAX), as AnalyzeFile skips
// it, and so does a read error (Analyze returns no result).
bool read_fs_files(const FsWalk& walk, const std::vector<uint32_t>& idx, const std::vector<uint64_t>& starts,
                   uint8_t* buf, int threads, std::vector<uint64_t>* got, std::string* err);

}  // namespace tsg
