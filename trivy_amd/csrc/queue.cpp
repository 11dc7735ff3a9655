// Per-file Scan through shared engine batches (queue.h).
#include "queue.h"

#include <algorithm>
#include <chrono>
#include <cstring>

extern "C" int tsg_alloc_pinned(size_t bytes, void** out);
extern "C" void tsg_free_pinned(void* p);

namespace tsg {

ScanQueue::ScanQueue(Engine* eng, uint32_t max_files, uint64_t max_bytes, uint32_t max_wait_us, uint32_t max_inflight)
    : eng_(eng),
      max_files_(std::max<uint32_t>(1, max_files)),
      max_wait_us_(max_wait_us),
      max_inflight_(std::max<uint32_t>(1, max_inflight)),
      max_bytes_(std::max<uint64_t>(1, max_bytes)) {}

ScanQueue::~ScanQueue() {
  for (Staging& s : free_staging_) tsg_free_pinned(s.p);
}

QueueStats ScanQueue::stats() {
  std::lock_guard<std::mutex> lk(mu_);
  return st_;
}

ScanQueue::Staging ScanQueue::take_staging(size_t bytes) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < free_staging_.size(); ++i) {
      if (free_staging_[i].cap >= bytes) {
        Staging s = free_staging_[i];
        free_staging_.erase(free_staging_.begin() + static_cast<long>(i));
        return s;
      }
    }
  }
  Staging s;
  s.cap = std::max<size_t>(bytes, 1 << 20);
  if (tsg_alloc_pinned(s.cap, &s.p) != 0) s = Staging();
  return s;
}

void ScanQueue::give_staging(Staging s) {
  if (!s.p) return;
  std::lock_guard<std::mutex> lk(mu_);
  free_staging_.push_back(s);
}

void ScanQueue::run_batch(std::vector<Req*>& batch) {
  const size_t n = batch.size();
  uint64_t total = 0;
  for (Req* r : batch) total += r->len;
  Staging stg = take_staging(total + 64);
  std::vector<uint8_t> heap;
  uint8_t* data = static_cast<uint8_t*>(stg.p);
  if (!data) {                                    // no pinned memory: pageable (slower upload, same results)
    heap.resize(total + 64);
    data = heap.data();
  }
  std::vector<uint64_t> off(n + 1, 0);
  std::vector<const char*> paths(n);
  std::vector<uint32_t> lens(n);
  std::vector<uint8_t> bin(n);
  for (size_t i = 0; i < n; ++i) {
    off[i + 1] = off[i] + batch[i]->len;
    if (batch[i]->len) std::memcpy(data + off[i], batch[i]->data, batch[i]->len);   // Scan never mutates Content
    paths[i] = batch[i]->path;
    lens[i] = static_cast<uint32_t>(batch[i]->path_len);
    bin[i] = batch[i]->binary;
  }
  std::memset(data + total, 0, 64);
  BatchInput in;
  in.h_data = data;
  in.offsets = off.data();
  in.nfiles = static_cast<uint32_t>(n);
  in.paths = paths.data();
  in.path_lens = lens.data();
  in.binary = bin.data();
  SecretVec res;
  ScanStats st;
  std::string err;
  const bool ok = eng_->scan(in, &res, &st, &err);
  give_staging(stg);
  std::lock_guard<std::mutex> lk(mu_);
  for (size_t i = 0; i < n; ++i) {
    if (ok) batch[i]->result = std::move(res[i]);
    else batch[i]->err = err;
    batch[i]->done = true;
  }
  st_.batches += 1;
  st_.files += n;
  st_.bytes += total;
  st_.max_batch = std::max<uint32_t>(st_.max_batch, static_cast<uint32_t>(n));
  in_batches_ -= static_cast<uint32_t>(n);
  --inflight_;
  cv_.notify_all();
}

bool ScanQueue::scan(const char* path, size_t path_len, const uint8_t* content, size_t len, bool binary, Secret* out,
                     std::string* err) {
  Req r{path, path_len, content, len, binary, Secret(), std::string()};
  std::unique_lock<std::mutex> lk(mu_);
  ++callers_;
  peak_callers_ = std::max(peak_callers_, callers_);
  ++st_.calls;
  pending_.push_back(&r);
  pending_bytes_ += len;
  cv_.notify_all();
  using Clock = std::chrono::steady_clock;
  while (!r.done) {
    const bool mine_pending = std::find(pending_.begin(), pending_.end(), &r) != pending_.end();
    if (mine_pending && !forming_ && inflight_ < max_inflight_) {
      // lead a batch: gather until every caller not in a running batch has
      // joined, the batch is full, or max_wait has passed
      forming_ = true;
      const auto deadline = Clock::now() + std::chrono::microseconds(max_wait_us_);
      // every caller not busy in a running batch: the most callers ever seen
      // at once (the --parallel goroutines come back one by one after their
      // previous batch, so the callers inside scan() right now undercount)
      cv_.wait_until(lk, deadline, [&] {
        return pending_.size() >= max_files_ || pending_bytes_ >= max_bytes_ ||
               pending_.size() + in_batches_ >= peak_callers_;
      });
      std::vector<Req*> batch;
      uint64_t bytes = 0;
      size_t k = 0;
      while (k < pending_.size() && batch.size() < max_files_ && (batch.empty() || bytes + pending_[k]->len <= max_bytes_)) {
        bytes += pending_[k]->len;
        batch.push_back(pending_[k++]);
      }
      pending_.erase(pending_.begin(), pending_.begin() + static_cast<long>(k));
      pending_bytes_ -= bytes;
      in_batches_ += static_cast<uint32_t>(batch.size());
      ++inflight_;
      forming_ = false;
      cv_.notify_all();                         // the next leader may start gathering
      lk.unlock();
      run_batch(batch);
      lk.lock();
      continue;
    }
    cv_.wait(lk);
  }
  --callers_;
  cv_.notify_all();
  if (!r.err.empty()) { *err = r.err; return false; }
  *out = std::move(r.result);
  return true;
}

}  // namespace tsg
