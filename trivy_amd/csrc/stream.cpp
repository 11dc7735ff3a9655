// Streamed feed -> scan pipeline (stream.h).  Two stages on two threads:
//   producer (the calling thread): walk -> gate -> read the kept files into a
//     raw batch -> prepare (Required / IsBinary / CR strip / .pyc printable
//     runs) into a prepared-batch buffer;
//   consumer: the scan stage on each prepared batch, in order.
// Two prepared-batch buffers circulate (one scanned while the next is
// prepared); the raw batch is reused.  Results come back in walk order.
#include "stream.h"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>

#include "guard.h"
#include "tar.h"

extern "C" int tsg_alloc_pinned(size_t bytes, void** out);
extern "C" void tsg_free_pinned(void* p);

namespace tsg {
namespace {

using Clock = std::chrono::steady_clock;
double ms_between(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

// Pinned buffers outlive one stream: hipHostMalloc of a stream's two batch
// buffers took ~45 ms per call (profiles/rd4l_bench_c1.json, tree
// pinned_alloc_ms), paid again by every layer of an image and every call.
// Streams return theirs here (up to 4 GiB) and take the smallest that fits.
// Never freed at exit (the HIP runtime may be gone by then).
class PinnedCache {
 public:
  static PinnedCache& get() {
    static PinnedCache* c = new PinnedCache();
    return *c;
  }
  uint8_t* take(size_t want, size_t* cap) {
    std::lock_guard<std::mutex> lk(mu_);
    size_t best = free_.size();
    for (size_t i = 0; i < free_.size(); ++i)
      if (free_[i].second >= want && (best == free_.size() || free_[i].second < free_[best].second)) best = i;
    if (best == free_.size()) return nullptr;
    uint8_t* p = free_[best].first;
    *cap = free_[best].second;
    bytes_ -= *cap;
    free_.erase(free_.begin() + static_cast<long>(best));
    return p;
  }
  void give(uint8_t* p, size_t cap) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (bytes_ + cap <= kMax) {
        free_.push_back({p, cap});
        bytes_ += cap;
        return;
      }
    }
    tsg_free_pinned(p);
  }

 private:
  static constexpr size_t kMax = 4ull << 30;
  std::mutex mu_;
  std::vector<std::pair<uint8_t*, size_t>> free_;
  size_t bytes_ = 0;
};

// Raw batch buffers (the windows) likewise outlive one stream: a fresh
// 256 MiB window is backed page by page as the reader first fills it, on
// every call and every layer.  Up to 2 GiB are kept.
class RawCache {
 public:
  static RawCache& get() {
    static RawCache* c = new RawCache();
    return *c;
  }
  // a buffer of at least `want` bytes; *cap = its real size
  std::unique_ptr<uint8_t[]> take(uint64_t want, uint64_t* cap) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      size_t best = free_.size();
      for (size_t i = 0; i < free_.size(); ++i)
        if (free_[i].second >= want && (best == free_.size() || free_[i].second < free_[best].second)) best = i;
      if (best != free_.size()) {
        uint8_t* p = free_[best].first;
        *cap = free_[best].second;
        bytes_ -= *cap;
        free_.erase(free_.begin() + static_cast<long>(best));
        return std::unique_ptr<uint8_t[]>(p);
      }
    }
    *cap = want;
    return std::unique_ptr<uint8_t[]>(new uint8_t[want]);
  }
  void give(std::unique_ptr<uint8_t[]> p, uint64_t cap) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu_);
    if (bytes_ + cap > kMax) return;            // freed by the unique_ptr
    free_.push_back({p.release(), cap});
    bytes_ += cap;
  }

 private:
  static constexpr uint64_t kMax = 2ull << 30;
  std::mutex mu_;
  std::vector<std::pair<uint8_t*, uint64_t>> free_;
  uint64_t bytes_ = 0;
};

// The prepared-batch buffers: `n` of them in circulation, grown on demand.
class BufPool {
 public:
  BufPool(bool pinned, size_t n) : pinned_(pinned), n_(n) {}
  ~BufPool() {
    for (auto& b : bufs_) release(b.p, b.cap);
  }
  // a buffer of >= bytes (blocks while all are in use); nullptr if allocation failed
  uint8_t* get(size_t bytes, double* wait_ms) {
    std::unique_lock<std::mutex> lk(mu_);
    const auto t0 = Clock::now();
    cv_.wait(lk, [&] {
      return cancelled_ || bufs_.size() < n_ || std::any_of(bufs_.begin(), bufs_.end(), [](const B& b) { return !b.used; });
    });
    *wait_ms += ms_between(t0, Clock::now());
    if (cancelled_) return nullptr;
    for (auto& b : bufs_) {
      if (b.used) continue;
      if (b.cap < bytes) {
        release(b.p, b.cap);
        b.p = alloc(bytes, &b.cap);
      }
      if (!b.p) return nullptr;
      b.used = true;
      return b.p;
    }
    B b;
    b.p = alloc(bytes, &b.cap);
    if (!b.p) return nullptr;
    b.used = true;
    bufs_.push_back(b);
    return b.p;
  }
  void put(uint8_t* p) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& b : bufs_) if (b.p == p) b.used = false;
    cv_.notify_all();
  }
  // the pipeline failed: waiters give up (the scan stage may have stopped
  // returning buffers)
  void cancel() {
    std::lock_guard<std::mutex> lk(mu_);
    cancelled_ = true;
    cv_.notify_all();
  }

 private:
  struct B { uint8_t* p = nullptr; size_t cap = 0; bool used = false; };
  uint8_t* alloc(size_t bytes, size_t* cap) {
    *cap = 0;
    if (!pinned_) {
      uint8_t* p = static_cast<uint8_t*>(std::malloc(bytes));
      if (p) *cap = bytes;
      return p;
    }
    if (uint8_t* p = PinnedCache::get().take(bytes, cap)) return p;
    void* p = nullptr;
    if (tsg_alloc_pinned(bytes, &p) != 0) return nullptr;
    *cap = bytes;
    return static_cast<uint8_t*>(p);
  }
  void release(uint8_t* p, size_t cap) {
    if (!p) return;
    if (pinned_) PinnedCache::get().give(p, cap);
    else std::free(p);
  }
  bool pinned_;
  size_t n_;
  bool cancelled_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<B> bufs_;
};

// One prepared batch on its way to the scan stage.
struct Job {
  PreparedBatch b;
  std::vector<std::string> scan_paths;
};

// Producer -> prepare -> scan.  The producer (walk + reads) fills one of two
// raw batch buffers while a prepare thread turns the other (filled) one into
// a prepared pinned batch and the consumer thread scans the batch before it:
// the prepare of batch k overlaps the reads of batch k+1 (round 4: a
// synchronous prepare stopped the walk for ~9 ms per 256 MiB batch).
class Pipeline {
 public:
  Pipeline(const Ruleset& rs, const StreamOpts& o, const BatchScanFn& scan, const char* prefix, StreamResult* out)
      : rs_(rs), o_(o), scan_(scan), prefix_(prefix), out_(out), pool_(o.pinned, 2) {
    fo_ = o.feed;
    fo_.assume_required = true;                 // the producer gates each file before reading it
    limit_ = std::max<uint64_t>(o.batch_bytes, 1);
    // the whole batch limit at once: its pages are only backed as a batch
    // fills (no growth copies); a file larger than a batch grows it
    raw_cap_[0] = limit_;
    raw_[0] = RawCache::get().take(limit_, &raw_real_[0]);
    prep_ = std::thread([this] { prepare_loop(); });
    consumer_ = std::thread([this] { consume(); });
  }
  ~Pipeline() {
    finish();
    for (int i = 0; i < 2; ++i) RawCache::get().give(std::move(raw_[i]), raw_real_[i]);
  }

  // room for a file of n raw bytes in the current batch (flushing it first
  // if it does not fit); returns where to put it, nullptr on failure
  uint8_t* reserve(uint64_t n) {
    if (!paths_.empty() && used_ + n > limit_ && !flush()) return nullptr;
    if (used_ + n > raw_cap_[cur_]) {           // grow (a file larger than a batch: a buffer of its size)
      const uint64_t cap = std::max<uint64_t>(used_ + n, std::min<uint64_t>(limit_, 2 * raw_cap_[cur_]));
      grow_window(cap, 0, used_);
    }
    return raw_[cur_].get() + used_;
  }
  // the file just written at reserve()'s pointer: n bytes
  void commit(const std::string& path, uint64_t n) {
    starts_.push_back(used_);
    sizes_.push_back(n);
    paths_.push_back(path);
    used_ += n;
    out_->st.read_bytes += n;
  }
  // Window mode (stream_layer): the tar reader fills the raw buffer itself
  // and the kept files are committed where they lie, so file data is copied
  // once (reader -> window) on its way to the prepared batch.
  uint8_t* window() { return raw_[cur_].get(); }
  uint64_t window_cap() const { return raw_cap_[cur_]; }
  bool has_files() const { return !paths_.empty(); }
  double flush_wall_ms() const { return flush_wall_ms_; }   // producer wall time inside flush() so far
  void commit_at(const std::string& path, uint64_t off, uint64_t n) {
    starts_.push_back(off);
    sizes_.push_back(n);
    paths_.push_back(path);
    used_ += n;
    out_->st.read_bytes += n;
  }
  // a larger current buffer holding its bytes [from, to) at its start
  // (no file committed in it)
  void grow_window(uint64_t cap, uint64_t from, uint64_t to) {
    uint64_t real = 0;
    std::unique_ptr<uint8_t[]> nb = RawCache::get().take(cap, &real);
    if (to > from) std::memcpy(nb.get(), raw_[cur_].get() + from, to - from);
    RawCache::get().give(std::move(raw_[cur_]), raw_real_[cur_]);
    raw_[cur_] = std::move(nb);
    raw_cap_[cur_] = cap;
    raw_real_[cur_] = real;
  }
  // the window is full: hand its committed files to the prepare thread and
  // continue in the other buffer with the unconsumed bytes [from, to) of
  // this one at its start (or, with no file committed, move them down in place)
  bool next_window(uint64_t from, uint64_t to) {
    const uint64_t keep = to - from;
    if (paths_.empty()) {
      if (from) std::memmove(raw_[cur_].get(), raw_[cur_].get() + from, keep);
      return ok();
    }
    const int old = cur_;
    if (!flush()) return false;                 // switches cur_ (the prepare reads [0, from) of `old`)
    if (raw_cap_[cur_] < keep) {
      RawCache::get().give(std::move(raw_[cur_]), raw_real_[cur_]);
      raw_[cur_] = RawCache::get().take(keep, &raw_real_[cur_]);
      raw_cap_[cur_] = keep;
    }
    if (keep) std::memcpy(raw_[cur_].get(), raw_[old].get() + from, keep);
    return ok();
  }
  // hand the current batch to the prepare thread and switch buffers
  bool flush() {
    if (paths_.empty()) return ok();
    const auto t0 = Clock::now();
    auto task = std::make_unique<PrepTask>();
    task->buf = cur_;
    task->used = used_;
    task->starts.swap(starts_);
    task->sizes.swap(sizes_);
    task->paths.swap(paths_);
    used_ = 0;
    {
      std::unique_lock<std::mutex> lk(mu_);
      busy_[cur_] = true;
      prep_q_.push_back(std::move(task));
      cv_.notify_all();
      cur_ ^= 1;
      // the other buffer is free once its previous batch has been prepared
      cv_.wait(lk, [&] { return !busy_[cur_] || !err_.empty(); });
    }
    if (!raw_[cur_]) { raw_cap_[cur_] = limit_; raw_[cur_] = RawCache::get().take(limit_, &raw_real_[cur_]); }
    flush_wall_ms_ += ms_between(t0, Clock::now());
    return ok();
  }
  // drain: the last batch, then wait for the prepare and scan stages; true if no error
  bool finish() {
    if (finished_) return ok();
    finished_ = true;
    if (ok()) flush();
    {
      std::lock_guard<std::mutex> lk(mu_);
      prep_done_ = true;
    }
    cv_.notify_all();
    if (prep_.joinable()) prep_.join();
    {
      std::lock_guard<std::mutex> lk(mu_);
      done_ = true;
    }
    cv_.notify_all();
    if (consumer_.joinable()) consumer_.join();
    out_->st.feed_ms += prep_ms_;
    out_->st.wait_ms += prep_wait_ms_;
    return ok();
  }
  bool ok() {
    std::lock_guard<std::mutex> lk(mu_);
    return err_.empty();
  }
  std::string error() {
    std::lock_guard<std::mutex> lk(mu_);
    return err_;
  }
  void set_error(const std::string& e) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (err_.empty()) err_ = e;
      cv_.notify_all();
    }
    pool_.cancel();
  }

 private:
  struct PrepTask {
    int buf = 0;
    uint64_t used = 0;
    std::vector<uint64_t> starts, sizes;
    std::vector<std::string> paths;
  };
  void prepare_loop() {
    for (;;) {
      std::unique_ptr<PrepTask> task;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !prep_q_.empty() || prep_done_; });
        if (prep_q_.empty()) return;
        task = std::move(prep_q_.front());
        prep_q_.pop_front();
      }
      const auto t0 = Clock::now();
      std::unique_ptr<Job> job;
      std::string err;
      double wait = 0;
      bool good = false;
      // (a host exception -- bad_alloc in the prepare -- fails the stream; it
      // must not escape this thread)
      try {
        job = std::make_unique<Job>();
        BufPool* pool = &pool_;
        FeedAlloc alloc = [pool, &wait](size_t bytes, FeedFree* free_fn) -> uint8_t* {
          uint8_t* p = pool->get(bytes, &wait);
          if (p) *free_fn = [pool](uint8_t* q) { pool->put(q); };
          return p;
        };
        good = ok() && prepare_files(rs_, fo_, raw_[task->buf].get(), task->starts.data(), task->sizes.data(),
                                     task->paths, o_.threads, &job->b, &err, alloc);
        if (good && !job->b.data) { good = false; err = "out of memory for a prepared batch"; }
        if (good) for (uint32_t i : job->b.index) job->scan_paths.push_back(prefix_ + task->paths[i]);
      } catch (const std::exception& x) {
        good = false;
        err = std::string("host exception in the prepare stage: ") + x.what();
      } catch (...) {
        good = false;
        err = "host exception in the prepare stage";
      }
      std::lock_guard<std::mutex> lk(mu_);
      busy_[task->buf] = false;
      if (!good) {
        if (err_.empty()) err_ = err.empty() ? std::string("prepare failed") : err;
        pool_.cancel();
      } else {
        peak_batch_ = std::max<uint64_t>(peak_batch_, task->used);
        out_->st.peak_batch_bytes = peak_batch_;
        prep_ms_ += ms_between(t0, Clock::now()) - wait;   // blocked on a buffer: not feed work
        prep_wait_ms_ += wait;
        q_.push_back(std::move(job));
      }
      cv_.notify_all();
    }
  }
  void consume() {
    for (;;) {
      std::unique_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty() || done_ || !err_.empty(); });
        if (!err_.empty() || q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      const auto t0 = Clock::now();
      // (a host exception in the scan stage or while the results are moved
      // fails the stream; it must not escape this thread)
      try {
        const uint32_t nk = static_cast<uint32_t>(job->b.index.size());
        std::vector<const char*> pp(nk);
        std::vector<uint32_t> pl(nk);
        for (uint32_t k = 0; k < nk; ++k) {
          pp[k] = job->scan_paths[k].c_str();
          pl[k] = static_cast<uint32_t>(job->scan_paths[k].size());
        }
        BatchInput in;
        in.h_data = job->b.data.get();
        in.offsets = job->b.offsets.data();
        in.nfiles = nk;
        in.paths = pp.data();
        in.path_lens = pl.data();
        in.binary = job->b.binary.data();
        SecretVec res;
        std::string err;
        if (!scan_(in, &res, &err)) { set_error(err); return; }
        out_->st.scanned_bytes += job->b.offsets[nk];
        out_->st.files += nk;
        out_->st.batches += 1;
        for (auto& r : res) out_->files.push_back(std::move(r));
      } catch (const std::exception& x) {
        set_error(std::string("host exception in the scan stage: ") + x.what());
        return;
      } catch (...) {
        set_error("host exception in the scan stage");
        return;
      }
      job.reset();                                // the prepared buffer goes back to the pool
      out_->st.scan_ms += ms_between(t0, Clock::now());
    }
  }

  const Ruleset& rs_;
  const StreamOpts& o_;
  const BatchScanFn& scan_;
  std::string prefix_;
  StreamResult* out_;
  FeedOpts fo_;
  BufPool pool_;
  std::unique_ptr<uint8_t[]> raw_[2];
  uint64_t raw_cap_[2] = {0, 0};           // the size a window / batch may use
  uint64_t raw_real_[2] = {0, 0};          // the buffer's real size (a cached one may be larger)
  int cur_ = 0;
  bool busy_[2] = {false, false};
  uint64_t limit_ = 0, used_ = 0, peak_batch_ = 0;
  std::vector<uint64_t> starts_, sizes_;
  std::vector<std::string> paths_;
  double flush_wall_ms_ = 0, prep_ms_ = 0, prep_wait_ms_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::unique_ptr<PrepTask>> prep_q_;
  std::deque<std::unique_ptr<Job>> q_;
  bool prep_done_ = false, done_ = false, finished_ = false;
  std::string err_;
  std::thread prep_, consumer_;
};

// a layer from a reader callback
// The tar pulled from the reader callback straight into the pipeline's raw
// batch (the window): one callback per window fill instead of one per header
// and per file (a ctypes / cgo call each: 2.4 GB/s end to end against 10.5
// GB/s for the in-memory walk, profiles/rd4l_bench_c3.json), and a kept
// file's data is committed in place (`view`) instead of being copied out of a
// read buffer.  Headers, padding and skipped files pass through the window
// too.  The window is compacted -- its unconsumed tail moved to the start --
// only after the files committed in it have been prepared (flush).  A read
// error is reported once the bytes read before it have been consumed, where
// the unbuffered walk would have met it.
class WindowTarInput : public TarInput {
 public:
  WindowTarInput(StreamReadFn fn, void* user, Pipeline* pl) : fn_(fn), user_(user), pl_(pl) {}
  bool read(uint8_t* dst, size_t n, size_t* got, std::string* err) override {
    *got = 0;
    while (*got < n) {
      if (rpos_ < wlen_) {
        const size_t take = std::min<size_t>(n - *got, wlen_ - rpos_);
        std::memcpy(dst + *got, pl_->window() + rpos_, take);
        rpos_ += take;
        *got += take;
        continue;
      }
      if (!fill(1, err)) return false;
      if (rpos_ >= wlen_) break;                 // end of the data
    }
    pos += *got;
    return true;
  }
  bool skip(uint64_t n, uint64_t* got, std::string* err) override {
    *got = 0;
    while (*got < n) {
      if (rpos_ < wlen_) {
        const uint64_t take = std::min<uint64_t>(n - *got, wlen_ - rpos_);
        rpos_ += take;
        *got += take;
        continue;
      }
      if (!fill(1, err)) return false;
      if (rpos_ >= wlen_) break;
    }
    pos += *got;
    return true;
  }
  // the next n bytes in place, consumed: their window offset in *off, *got < n
  // only at the end of the data
  bool view(uint64_t n, uint64_t* off, uint64_t* got, std::string* err) {
    if (!fill(n, err)) return false;
    *got = std::min<uint64_t>(n, wlen_ - rpos_);
    *off = rpos_;
    rpos_ += *got;
    pos += *got;
    return true;
  }

 private:
  // at least `need` unconsumed bytes contiguous in the window (fewer only at
  // the end of the data); false: a read error before them, or a failed flush
  bool fill(uint64_t need, std::string* err) {
    while (wlen_ - rpos_ < need && !eof_ && !failed_) {
      if (rpos_ + need > pl_->window_cap() || wlen_ == pl_->window_cap()) {
        // make room: hand the files committed in the window to the prepare
        // stage and continue in the other buffer with the unconsumed tail at
        // its start; a window still full holds part of a file larger than a
        // batch: double it (by the bytes actually read, so a hostile size
        // field ends in "unexpected EOF", not an allocation)
        const uint64_t keep = wlen_ - rpos_;
        if (!pl_->next_window(rpos_, wlen_)) { *err = pl_->error(); return false; }
        rpos_ = 0;
        wlen_ = keep;
        if (wlen_ == pl_->window_cap()) pl_->grow_window(2 * pl_->window_cap(), 0, wlen_);
      }
      const int64_t r = fn_(user_, pl_->window() + wlen_, pl_->window_cap() - wlen_);
      if (r < 0) failed_ = true;
      else if (r == 0) eof_ = true;
      else wlen_ += static_cast<uint64_t>(std::min<int64_t>(r, static_cast<int64_t>(pl_->window_cap() - wlen_)));
    }
    if (failed_ && wlen_ - rpos_ < need) {
      *err = "failed to extract the archive: read error";
      return false;
    }
    return true;
  }

  StreamReadFn fn_;
  void* user_;
  Pipeline* pl_;
  uint64_t rpos_ = 0, wlen_ = 0;
  bool eof_ = false, failed_ = false;
};

}  // namespace

bool stream_layer(const Ruleset& rs, const StreamOpts& o, StreamReadFn read, void* user, const BatchScanFn& scan,
                  StreamResult* out, std::string* err) {
  *out = StreamResult();
  const auto t0 = Clock::now();
  LayerWalk walk;
  const std::string cfg_base = o.feed.config_path;
  Pipeline pl(rs, o, scan, "/", out);
  WindowTarInput in(read, user, &pl);
  auto t_feed = Clock::now();
  // processFile (tar.go:94-105) -> AnalyzeFile's gate -> read the content
  auto on_file = [&](const std::string& path, uint64_t size, TarInput& tin, std::string* e) {
    out->walked.push_back(path);
    out->st.walked_bytes += size;
    if (!secret_analyzer_wants(rs, o.feed, path, size)) return true;     // the walker skips the data
    (void)tin;                                                          // (tin is `in`)
    uint64_t off = 0, got = 0;
    if (!in.view(size, &off, &got, e)) return false;
    if (got < size) {
      *e = "failed to process the file: failed to analyze file: failed to open: unable to read the file: unexpected EOF";
      return false;
    }
    pl.commit_at(path, off, size);
    return true;
  };
  std::string werr;
  const bool wok = walk_layer(in, o.skip_files, o.skip_dirs, &walk, on_file, &werr);
  // the walk's own time: the batches it flushed (window full) count themselves
  out->st.feed_ms += ms_between(t_feed, Clock::now()) - pl.flush_wall_ms();
  if (!wok) {
    pl.set_error(werr);
    pl.finish();
    *err = werr;
    return false;
  }
  pl.flush();
  if (!pl.finish()) { *err = pl.error(); return false; }
  out->opq_dirs = std::move(walk.opq_dirs);
  out->wh_files = std::move(walk.wh_files);
  out->st.wall_ms = ms_between(t0, Clock::now());
  return true;
}

bool plan_fs_tree(const Ruleset& rs, const FeedOpts& fo, const std::string& root,
                  const std::vector<std::string>& skip_files, const std::vector<std::string>& skip_dirs, int threads,
                  FsWalk* walk, std::vector<uint32_t>* keep, std::string* err) {
  keep->clear();
  walk_fs_tree(root, skip_files, skip_dirs, threads, walk, err);   // an error is kept in walk->err
  stat_fs_files(walk, threads);                                     // d.Info() of every walked file
  // AnalyzeFile's gate before the file is opened (analyzer.go:417-419): the
  // path part first (in parallel), then Required's size check on info.Size()
  const uint32_t n = static_cast<uint32_t>(walk->files.size());
  std::vector<uint8_t> want(n, 0);
  {
    std::atomic<uint32_t> next{0};
    auto run = [&]() {
      for (;;) {
        const uint32_t b = next.fetch_add(256);
        if (b >= n) break;
        for (uint32_t i = b; i < std::min(n, b + 256); ++i)
          want[i] = static_cast<uint8_t>(secret_analyzer_wants_path(rs, fo, walk->files[i].rel));
      }
    };
    run_threads(std::min<int>(threads, static_cast<int>(n / 256) + 1), run);
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (!want[i]) continue;
    const FsFile& f = walk->files[i];
    // files at or after the walk's first error are never reached in Go
    if (walk->failed && !walk_order_less(f.rel, walk->err_key)) break;
    if (f.size == UINT64_MAX || (want[i] == 2 && f.size < 10)) continue;   // secret.go:154-156
    keep->push_back(i);
  }
  if (walk->failed) *err = walk->err;
  return !walk->failed;
}

bool stream_fs_tree(const Ruleset& rs, const StreamOpts& o, const std::string& root, const BatchScanFn& scan,
                    StreamResult* out, std::string* err) {
  *out = StreamResult();
  const auto t0 = Clock::now();
  FsWalk walk;
  std::vector<uint32_t> keep;
  std::string perr;
  const bool planned = plan_fs_tree(rs, o.feed, root, o.skip_files, o.skip_dirs, o.threads, &walk, &keep, &perr);
  for (const FsFile& f : walk.files) {
    if (walk.failed && !walk_order_less(f.rel, walk.err_key)) break;
    out->walked.push_back(f.rel);
    if (f.size != UINT64_MAX) out->st.walked_bytes += f.size;
  }
  Pipeline pl(rs, o, scan, "", out);
  out->st.feed_ms += ms_between(t0, Clock::now());
  // batches of consecutive kept files (walk order), each read by the reader
  // threads straight into the raw batch, then prepared and handed on
  size_t k = 0;
  while (k < keep.size()) {
    const auto t1 = Clock::now();
    size_t e = k;
    uint64_t bytes = 0;
    while (e < keep.size() && (e == k || bytes + walk.files[keep[e]].size <= o.batch_bytes)) bytes += walk.files[keep[e++]].size;
    uint8_t* dst = pl.reserve(bytes);
    if (!dst) break;
    std::vector<uint32_t> idx(keep.begin() + static_cast<long>(k), keep.begin() + static_cast<long>(e));
    std::vector<uint64_t> starts(idx.size()), got;
    uint64_t at = 0;
    for (size_t j = 0; j < idx.size(); ++j) { starts[j] = at; at += walk.files[idx[j]].size; }
    std::string rerr;
    if (!read_fs_files(walk, idx, starts, dst, o.threads, &got, &rerr)) {
      // an open error halts the walk there, unless an earlier walk error did
      pl.set_error(rerr);
      pl.finish();
      *err = rerr;
      return false;
    }
    // commit in order, packing out the files that vanished / shrank
    uint64_t wpos = 0;
    for (size_t j = 0; j < idx.size(); ++j) {
      if (got[j] == UINT64_MAX) continue;
      if (wpos != starts[j]) std::memmove(dst + wpos, dst + starts[j], got[j]);
      pl.commit(walk.files[idx[j]].rel, got[j]);
      wpos += got[j];
    }
    out->st.feed_ms += ms_between(t1, Clock::now());
    if (!pl.flush()) break;
    k = e;
  }
  if (!pl.finish()) { *err = pl.error(); return false; }
  if (!planned) { *err = perr; return false; }
  out->st.wall_ms = ms_between(t0, Clock::now());
  return true;
}

}  // namespace tsg
