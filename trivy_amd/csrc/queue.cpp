// Per-file Scan through shared engine batches (queue.h).
#include "queue.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

extern "C" int tsg_alloc_pinned(size_t bytes, void** out);
extern "C" void tsg_free_pinned(void* p);

namespace tsg {

ScanQueue::ScanQueue(BatchScanFn scan, uint32_t max_files, uint64_t max_bytes, uint32_t max_wait_us,
                     uint32_t max_inflight)
    : scan_(std::move(scan)),
      max_files_(std::max<uint32_t>(1, max_files)),
      max_wait_us_(max_wait_us),
      max_inflight_(std::max<uint32_t>(1, max_inflight)),
      max_bytes_(std::max<uint64_t>(1, max_bytes)) {
  if (const char* v = std::getenv("TSG_QUEUE_SPREAD")) spread_ = std::atoi(v) != 0;
}

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
  try {
    free_staging_.push_back(s);
  } catch (...) {
    tsg_free_pinned(s.p);
  }
}

// Scans one gathered batch and hands every caller in it its result or the
// error.  Whatever happens -- a failed scan, or a host exception (bad_alloc
// of the staging copy or of the results, a thread the engine could not
// start) -- every request is completed and the batch's slots are released,
// so no caller is left waiting and no later leader is starved.
void ScanQueue::run_batch(std::vector<Req*>& batch) {
  const size_t n = batch.size();
  uint64_t total = 0;
  for (Req* r : batch) total += r->len;
  Staging stg;
  SecretVec res;
  std::string err;
  bool ok = false;
  try {
    stg = take_staging(total + 64);
    std::vector<uint8_t> heap;
    uint8_t* data = static_cast<uint8_t*>(stg.p);
    if (!data) {                                  // no pinned memory: pageable (slower upload, same results)
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
    ok = scan_(in, &res, &err);
    if (ok && res.size() != n) { ok = false; err = "scan returned a wrong result count"; }
  } catch (const std::bad_alloc&) {
    ok = false;
    err = "out of memory";
  } catch (const std::exception& x) {
    ok = false;
    err = std::string("internal error: ") + x.what();
  } catch (...) {
    ok = false;
    err = "internal error";
  }
  if (!ok && err.empty()) err = "scan failed";
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
  pending_.push_back(&r);
  pending_bytes_ += len;
  ++callers_;
  const auto now = Clock::now();
  if (callers_ >= expect_) {
    expect_ = callers_;
    expect_at_ = now;
  }
  ++st_.calls;
  cv_.notify_all();
  while (!r.done) {
    const bool mine_pending = std::find(pending_.begin(), pending_.end(), &r) != pending_.end();
    if (mine_pending && !forming_ && inflight_ < max_inflight_) {
      // lead a batch: gather until every caller expected and not in a
      // running batch has joined, the batch is full, or max_wait has passed
      forming_ = true;
      const auto t_lead = Clock::now();
      // a peak not reached again for kPeakHold is over: expect the callers
      // inside the queue now (a lone caller after a burst waits for nobody)
      if (t_lead - expect_at_ > kPeakHold) {
        expect_ = callers_;
        expect_at_ = t_lead;
      }
      // spread: the expected callers are split over the batch slots, so a
      // batch waits for its share only (ceil(expected / slots) files) and
      // few callers run as concurrent batches of one file each: a small
      // batch's time is fixed costs (launches, one sync, the inline confirm)
      // that concurrent batches on their own lanes overlap, where one batch
      // of all callers serialises them (5 callers, config-1 files: 1.10-1.19
      // -> 1.55-1.67 GB/s; 16 callers 1.33-1.56 -> 2.11-2.18 with 8 slots,
      // profiles/r6g_queue_probe.log)
      const size_t share = spread_ ? std::max<size_t>(1, (expect_ + max_inflight_ - 1) / max_inflight_) : max_files_;
      const size_t cap = std::min<size_t>(max_files_, share);
      auto gathered = [&] {
        return pending_.size() >= cap || pending_bytes_ >= max_bytes_ ||
               pending_.size() + in_batches_ >= expect_;
      };
#if defined(__SANITIZE_THREAD__)
      // (ThreadSanitizer of GCC 11 does not intercept pthread_cond_clockwait,
      // which a steady_clock wait uses, and reports the relock as a double
      // lock: sanitized builds wait on the system clock, pthread_cond_timedwait)
      const auto deadline = std::chrono::system_clock::now() + std::chrono::microseconds(max_wait_us_);
#else
      const auto deadline = t_lead + std::chrono::microseconds(max_wait_us_);
#endif
      if (!cv_.wait_until(lk, deadline, gathered)) {
        // the expected callers did not come: expect the ones that did (the
        // next leader does not wait for them again)
        expect_ = std::max<uint32_t>(1, static_cast<uint32_t>(pending_.size()) + in_batches_);
        expect_at_ = Clock::now();
        ++st_.timeouts;
      }
      std::vector<Req*> batch;
      try {
        batch.reserve(std::min<size_t>(pending_.size(), max_files_));   // (the only allocation while gathering)
      } catch (...) {
        forming_ = false;
        pending_.erase(std::find(pending_.begin(), pending_.end(), &r));
        pending_bytes_ -= len;
        --callers_;
        cv_.notify_all();
        throw;
      }
      uint64_t bytes = 0;
      size_t k = 0;
      while (k < pending_.size() && batch.size() < cap && (batch.empty() || bytes + pending_[k]->len <= max_bytes_)) {
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
      run_batch(batch);                         // completes every request, whatever happens
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
