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
#include <cstring>
#include <mutex>
#include <thread>

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

struct Walker {
  const std::vector<std::string>& skip_files;
  const std::vector<std::string>& skip_dirs;
  FsWalk* out;
  std::string* err;

  bool fail(const std::string& path, const std::string& what) {
    *err = "walk dir error: unknown error with " + path + ": " + what;
    return false;
  }

  // the WalkDirFunc for a regular file (fs.go:57-75)
  bool file(const std::string& path, const std::string& rel) {
    if (skip_path(rel, skip_files)) return true;
    struct stat sb;
    if (::lstat(path.c_str(), &sb) != 0) {                        // d.Info()
      if (is_permission(errno)) return true;
      return fail(path, "file info error: lstat " + path + ": " + go_errno(errno));
    }
    out->files.push_back(FsFile{rel, path, static_cast<uint64_t>(sb.st_size)});
    return true;
  }

  // walkDir after the WalkDirFunc accepted directory `path` (io/fs walkDir:
  // entries in os.ReadDir's name order, each visited before the next)
  bool dir(const std::string& path, const std::string& rel) {
    DIR* dp = ::opendir(path.c_str());
    if (!dp) {
      if (is_permission(errno)) return true;                      // onError: permission errors ignored
      return fail(path, "open " + path + ": " + go_errno(errno));
    }
    std::vector<std::pair<std::string, unsigned char>> ents;
    errno = 0;
    while (struct dirent* e = ::readdir(dp)) {
      if (!std::strcmp(e->d_name, ".") || !std::strcmp(e->d_name, "..")) continue;
      ents.emplace_back(e->d_name, e->d_type);
    }
    const int rerr = errno;
    ::closedir(dp);
    if (rerr != 0 && !is_permission(rerr)) return fail(path, "readdirent " + path + ": " + go_errno(rerr));
    std::sort(ents.begin(), ents.end());
    for (auto& [name, type] : ents) {
      const std::string child = join(path, name);
      const std::string crel = rel == "." ? name : rel + "/" + name;
      if (type == DT_UNKNOWN) {
        struct stat sb;
        if (::lstat(child.c_str(), &sb) != 0) {
          if (is_permission(errno)) continue;
          return fail(child, "lstat " + child + ": " + go_errno(errno));
        }
        type = S_ISDIR(sb.st_mode) ? DT_DIR : S_ISREG(sb.st_mode) ? DT_REG : DT_LNK;
      }
      if (type == DT_DIR) {
        if (skip_path(crel, skip_dirs)) continue;                 // filepath.SkipDir
        if (!dir(child, crel)) return false;
      } else if (type == DT_REG) {
        if (!file(child, crel)) return false;
      }                                                           // symlinks, devices, ...: not regular
    }
    return true;
  }
};

}  // namespace

std::string go_filepath_clean(const std::string& p) { return go_path_clean(p); }

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
                  const std::vector<std::string>& skip_dirs_in, FsWalk* out, std::string* err) {
  const std::vector<std::string> skip_files = build_skip_paths(root, skip_files_in);
  std::vector<std::string> skip_dirs = build_skip_paths(root, skip_dirs_in);
  for (const char* d : {"**/.git", "proc", "sys", "dev"}) skip_dirs.emplace_back(d);   // defaultSkipDirs
  out->files.clear();
  Walker w{skip_files, skip_dirs, out, err};
  struct stat sb;
  if (::lstat(root.c_str(), &sb) != 0) {
    if (is_permission(errno)) return true;
    return w.fail(root, "lstat " + root + ": " + go_errno(errno));
  }
  if (S_ISDIR(sb.st_mode)) {
    if (skip_path(".", skip_dirs)) return true;
    return w.dir(root, ".");
  }
  if (S_ISREG(sb.st_mode)) return w.file(root, ".");
  return true;
}

bool read_fs_files(const FsWalk& walk, const std::vector<uint8_t>& want, const std::vector<uint64_t>& starts,
                   uint8_t* buf, int threads, std::vector<uint64_t>* got, std::string* err) {
  const uint32_t n = static_cast<uint32_t>(walk.files.size());
  got->assign(n, 0);
  std::atomic<uint32_t> next{0};
  std::atomic<bool> failed{false};
  std::string first_err;
  std::mutex mu;
  auto run = [&]() {
    for (;;) {
      const uint32_t i = next.fetch_add(1);
      if (i >= n || failed.load(std::memory_order_relaxed)) break;
      if (!want[i]) continue;
      const FsFile& f = walk.files[i];
      const int fd = ::open(f.path.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) {
        if (is_permission(errno)) { (*got)[i] = UINT64_MAX; continue; }   // AnalyzeFile: ErrPermission -> skip
        std::lock_guard<std::mutex> lk(mu);
        if (!failed.exchange(true))
          first_err = "walk dir error: unknown error with " + f.path + ": failed to analyze file: unable to open " +
                      f.rel + ": open " + f.path + ": " + go_errno(errno);
        break;
      }
      uint64_t done = 0;
      bool rerr = false;
      while (done < f.size) {
        const ssize_t r = ::pread(fd, buf + starts[i] + done, f.size - done, static_cast<off_t>(done));
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) { rerr = true; break; }                        // Analyze's read error: no result
        if (r == 0) break;                                        // shrunk since the walk: what is there
        done += static_cast<uint64_t>(r);
      }
      ::close(fd);
      (*got)[i] = rerr ? UINT64_MAX : done;
    }
  };
  const int nt = std::max(1, std::min<int>(threads, static_cast<int>(std::max<uint32_t>(n, 1))));
  std::vector<std::thread> ts;
  for (int t = 1; t < nt; ++t) ts.emplace_back(run);
  run();
  for (auto& th : ts) th.join();
  if (failed) { *err = first_err; return false; }
  return true;
}

}  // namespace tsg
