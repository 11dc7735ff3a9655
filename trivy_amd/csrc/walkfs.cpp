// walker.FS.Walk (pkg/fanal/walker/fs.go:25-149) restated over POSIX
// directory reads, plus the threaded file reads of the analyzer feed.
#include "walkfs.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#include "guard.h"
#include "tar.h"

namespace tsg {
namespace {

// Go's syscall error text: strerror with a lower-case first letter
std::string go_errno(int e) {
  std::string s = std::strerror(e);
  if (!s.empty() && s[0] >= 'A' && s[0] <= 'Z') s[0] = static_cast<char>(s[0] - 'A' + 'a');
  return s;
}

bool is_permission(int e) { return e == EACCES || e == EPERM; }   // os.IsPermission

// filepath.Join(dir, name) for a name without separators
std::string join(const std::string& dir, const std::string& name) { return go_filepath_clean(dir + "/" + name); }

std::string getcwd_str() {
  std::vector<char> b(4096);
  while (!::getcwd(b.data(), b.size())) {
    if (errno != ERANGE) return "/";
    b.resize(b.size() * 2);
  }
  return b.data();
}

// filepath.Abs
std::string go_abs(const std::string& p) {
  if (!p.empty() && p[0] == '/') return go_filepath_clean(p);
  return go_filepath_clean(getcwd_str() + "/" + p);
}

// filepath.Rel (Unix; both arguments absolute here, so it cannot fail)
std::string go_rel(const std::string& basepath, const std::string& targpath) {
  const std::string base = go_filepath_clean(basepath), targ = go_filepath_clean(targpath);
  if (targ == base) return ".";
  const size_t bl = base.size(), tl = targ.size();
  size_t b0 = 0, bi = 0, t0 = 0, ti = 0;
  for (;;) {
    while (bi < bl && base[bi] != '/') ++bi;
    while (ti < tl && targ[ti] != '/') ++ti;
    if (targ.compare(t0, ti - t0, base, b0, bi - b0) != 0) break;
    if (bi < bl) ++bi;
    if (ti < tl) ++ti;
    b0 = bi;
    t0 = ti;
  }
  if (b0 != bl) {
    const size_t seps = static_cast<size_t>(std::count(base.begin() + static_cast<long>(b0), base.end(), '/'));
    std::string out = "..";
    for (size_t i = 0; i < seps; ++i) out += "/..";
    if (t0 != tl) out += "/" + targ.substr(t0);
    return out;
  }
  return targ.substr(t0);
}

bool skip_path(const std::string& path, const std::vector<std::string>& pats) {   // utils.SkipPath
  size_t i = 0;
  while (i < path.size() && path[i] == '/') ++i;
  const std::string p = path.substr(i);
  for (const auto& pat : pats) if (doublestar_match(pat, p)) return true;
  return false;
}


// The walk, directories read by several threads (each directory is one task;
// results are put back into WalkDir's order at the end).  Regular files are
// recorded from the directory entry's type; their size is taken when they
// are read (the analyzer's gate runs on the path first).
struct Walker {
  const std::vector<std::string>& skip_files;
  const std::vector<std::string>& skip_dirs;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<std::string, std::string>> todo;   // (path, rel) of directories to read
  size_t busy = 0;
  bool failed = false;
  std::string err, err_key;                                // the first error in walk order wins
  std::vector<FsFile> files;

  void fail(const std::string& key, const std::string& path, const std::string& what) {
    std::lock_guard<std::mutex> lk(mu);
    if (!failed || walk_order_less(key, err_key)) {
      err = "walk dir error: unknown error with " + path + ": " + what;
      err_key = key;
    }
    failed = true;
  }

  void dir(const std::string& path, const std::string& rel, std::vector<FsFile>* out,
           std::vector<std::pair<std::string, std::string>>* subdirs) {
    DIR* dp = ::opendir(path.c_str());
    if (!dp) {
      if (!is_permission(errno)) fail(rel, path, "open " + path + ": " + go_errno(errno));
      return;                                                     // onError: permission errors ignored
    }
    const int dfd = ::dirfd(dp);
    std::vector<std::pair<std::string, unsigned char>> ents;
    errno = 0;
    while (struct dirent* e = ::readdir(dp)) {
      if (!std::strcmp(e->d_name, ".") || !std::strcmp(e->d_name, "..")) continue;
      unsigned char type = e->d_type;
      if (type == DT_UNKNOWN) {
        struct stat sb;
        if (::fstatat(dfd, e->d_name, &sb, AT_SYMLINK_NOFOLLOW) != 0) {
          // os.ReadDir: an entry that vanished between readdir and lstat is
          // skipped as if it never existed (dir_unix.go); other errors end
          // the directory's read
          if (errno == ENOENT) { errno = 0; continue; }
          if (!is_permission(errno)) fail(rel, path + "/" + e->d_name, "lstat: " + go_errno(errno));
          continue;
        }
        type = S_ISDIR(sb.st_mode) ? DT_DIR : S_ISREG(sb.st_mode) ? DT_REG : DT_LNK;
      }
      ents.emplace_back(e->d_name, type);
      errno = 0;
    }
    const int rerr = errno;
    ::closedir(dp);
    if (rerr != 0 && !is_permission(rerr)) fail(rel, path, "readdirent " + path + ": " + go_errno(rerr));
    for (auto& [name, type] : ents) {
      const std::string crel = rel == "." ? name : rel + "/" + name;
      if (type == DT_DIR) {
        if (skip_path(crel, skip_dirs)) continue;                   // filepath.SkipDir
        subdirs->emplace_back(join(path, name), crel);
      } else if (type == DT_REG) {
        if (skip_path(crel, skip_files)) continue;
        out->push_back(FsFile{crel, join(path, name), 0});
      }                                                           // symlinks, devices, ...: not regular
    }
  }

  void run(int threads) {
    auto worker = [&]() {
      std::vector<FsFile> local;
      for (;;) {
        std::pair<std::string, std::string> task;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return !todo.empty() || busy == 0; });
          if (todo.empty()) break;
          task = std::move(todo.front());
          todo.pop_front();
          ++busy;
        }
        std::vector<std::pair<std::string, std::string>> subdirs;
        try {
          dir(task.first, task.second, &local, &subdirs);
        } catch (...) {                        // the other workers must not wait on this task
          std::lock_guard<std::mutex> lk(mu);
          --busy;
          cv.notify_all();
          throw;
        }
        std::lock_guard<std::mutex> lk(mu);
        for (auto& sd : subdirs) todo.push_back(std::move(sd));
        --busy;
        cv.notify_all();
      }
      std::lock_guard<std::mutex> lk(mu);
      for (auto& f : local) files.push_back(std::move(f));
    };
    run_threads(threads, worker);
    std::sort(files.begin(), files.end(), [](const FsFile& a, const FsFile& b) { return walk_order_less(a.rel, b.rel); });
  }
};

}  // namespace

std::string go_filepath_clean(const std::string& p) { return go_path_clean(p); }

// Go's WalkDir order is a pre-order DFS with every directory's entries in
// name order; with '/' ranked below every other byte, a plain comparison of
// the relative paths gives the same order (names hold no '/' or NUL).
bool walk_order_less(const std::string& a, const std::string& b) {
  const size_t n = std::min(a.size(), b.size());
  for (size_t i = 0; i < n; ++i) {
    const unsigned char x = a[i] == '/' ? 0 : static_cast<unsigned char>(a[i]);
    const unsigned char y = b[i] == '/' ? 0 : static_cast<unsigned char>(b[i]);
    if (x != y) return x < y;
  }
  return a.size() < b.size();
}

void FsWalk::fail_at(const std::string& key, const std::string& msg) {
  if (failed && !walk_order_less(key, err_key)) return;
  failed = true;
  err = msg;
  err_key = key;
}

std::vector<std::string> build_skip_paths(const std::string& base, const std::vector<std::string>& paths) {
  std::vector<std::string> out;
  const std::string abs_base = go_abs(base);
  for (const std::string& path : paths) {
    const std::string rel = go_rel(abs_base, go_abs(path));
    const bool is_abs = !path.empty() && path[0] == '/';
    std::string r;
    if (!is_abs && rel.compare(0, 2, "..") == 0) r = path;        // #1: relative to the root already
    else r = rel;                                                 // #2 / #3
    // utils.CleanSkipPaths
    r = go_filepath_clean(r);
    size_t i = 0;
    while (i < r.size() && r[i] == '/') ++i;
    out.push_back(r.substr(i));
  }
  return out;
}

bool walk_fs_tree(const std::string& root, const std::vector<std::string>& skip_files_in,
                  const std::vector<std::string>& skip_dirs_in, int threads, FsWalk* out, std::string* err) {
  const std::vector<std::string> skip_files = build_skip_paths(root, skip_files_in);
  std::vector<std::string> skip_dirs = build_skip_paths(root, skip_dirs_in);
  for (const char* d : {"**/.git", "proc", "sys", "dev"}) skip_dirs.emplace_back(d);   // defaultSkipDirs
  out->files.clear();
  struct stat sb;
  if (::lstat(root.c_str(), &sb) != 0) {
    if (is_permission(errno)) return true;
    out->fail_at("", "walk dir error: unknown error with " + root + ": lstat " + root + ": " + go_errno(errno));
    *err = out->err;
    return false;
  }
  if (S_ISREG(sb.st_mode)) {
    if (!skip_path(".", skip_files)) out->files.push_back(FsFile{".", root, 0});
    return true;
  }
  if (!S_ISDIR(sb.st_mode) || skip_path(".", skip_dirs)) return true;
  Walker w{skip_files, skip_dirs};
  w.todo.emplace_back(root, ".");
  w.run(std::max(1, threads));
  out->files = std::move(w.files);
  if (w.failed) {
    // Go stops at the first error in walk order; files after it are not walked
    out->fail_at(w.err_key, w.err);
    *err = out->err;
    return false;
  }
  return true;
}

bool stat_fs_files(FsWalk* walk, int threads) {
  const uint32_t n = static_cast<uint32_t>(walk->files.size());
  std::atomic<uint32_t> next{0};
  std::vector<int> errs(n, 0);
  auto run = [&]() {
    for (;;) {
      const uint32_t b = next.fetch_add(64);
      if (b >= n) break;
      for (uint32_t i = b; i < std::min(n, b + 64); ++i) {
        struct stat sb;
        FsFile& f = walk->files[i];
        if (::lstat(f.path.c_str(), &sb) == 0) {
          f.size = static_cast<uint64_t>(sb.st_size);
        } else {
          f.size = UINT64_MAX;
          errs[i] = errno;
        }
      }
    }
  };
  const int nt = std::max(1, std::min<int>(threads, static_cast<int>(std::max<uint32_t>(n / 64, 1))));
  run_threads(nt, run);
  for (uint32_t i = 0; i < n; ++i) {
    if (!errs[i]) continue;
    // d.Info() (fs.go:67-70): xerrors-wrapped, so not even a permission error
    // is ignored by onError -- the walk halts here
    const FsFile& f = walk->files[i];
    walk->fail_at(f.rel, "walk dir error: unknown error with " + f.path + ": file info error: lstat " + f.path + ": " +
                             go_errno(errs[i]));
    break;                                                        // files are in walk order: the first is the earliest
  }
  return !walk->failed;
}

bool read_fs_files(const FsWalk& walk, const std::vector<uint32_t>& idx, const std::vector<uint64_t>& starts,
                   uint8_t* buf, int threads, std::vector<uint64_t>* got, std::string* err) {
  const uint32_t n = static_cast<uint32_t>(idx.size());
  got->assign(n, 0);
  std::atomic<uint32_t> next{0};
  std::atomic<uint32_t> first_bad{UINT32_MAX};                   // earliest failing position in idx
  std::vector<int> errs(n, 0);
  auto run = [&]() {
    for (;;) {
      const uint32_t k = next.fetch_add(1);
      if (k >= n || k > first_bad.load(std::memory_order_relaxed)) break;
      const FsFile& f = walk.files[idx[k]];
      const int fd = ::open(f.path.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) {
        if (is_permission(errno)) { (*got)[k] = UINT64_MAX; continue; }   // AnalyzeFile: ErrPermission -> skip
        errs[k] = errno;
        uint32_t cur = first_bad.load();
        while (k < cur && !first_bad.compare_exchange_weak(cur, k)) {}
        continue;
      }
      uint64_t done = 0;
      bool rerr = false;
      while (done < f.size) {
        const ssize_t r = ::pread(fd, buf + starts[k] + done, f.size - done, static_cast<off_t>(done));
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) { rerr = true; break; }                        // Analyze's read error: no result
        if (r == 0) break;                                        // shrunk since the walk: what is there
        done += static_cast<uint64_t>(r);
      }
      ::close(fd);
      (*got)[k] = rerr ? UINT64_MAX : done;
    }
  };
  const int nt = std::max(1, std::min<int>(threads, static_cast<int>(std::max<uint32_t>(n, 1))));
  run_threads(nt, run);
  const uint32_t k = first_bad.load();
  if (k != UINT32_MAX) {
    const FsFile& f = walk.files[idx[k]];
    *err = "walk dir error: unknown error with " + f.path + ": failed to analyze file: unable to open " + f.rel +
           ": open " + f.path + ": " + go_errno(errs[k]);
    return false;
  }
  return true;
}

}  // namespace tsg
