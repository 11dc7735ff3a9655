// The multi-driver segment pipeline of Engine::scan, device-independent:
// the shared segment counter, the blocking hand-off of finished segments from
// the device drivers to the confirming thread (JobQueue) and the fan-out /
// fan-in around them (DriverPipeline::run).  The engine instantiates it with its HIP
// device drivers; tsg_test_multi_driver_model (pipeline_model.cpp) with
// simulated devices, so the failure behaviour is tested without a GPU.
//
// Replaces the reference's per-file goroutine fan-out
// (pkg/fanal/analyzer/analyzer.go:429-451: a semaphore of --parallel
// goroutines, errors logged per file): here whole segments go to one driver
// per device, and a driver that fails fails the call.
//
// Failure contract:
//  * a driver that returns false (or throws) records the first error and
//    aborts the queue: every other driver stops before its next segment (at
//    most the segment it is running completes), a driver blocked on a full
//    queue wakes, and the confirming thread stops popping;
//  * the confirming thread's own failure (consume throws) aborts the queue
//    the same way;
//  * DriverPipeline::run returns only after every driver thread has returned (each
//    driver releases its own lane before it returns), with the first error:
//    a failed call never returns a partial result.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tsg {

// Blocking hand-off of finished segments from the device drivers to the confirmer.
template <typename T>
class JobQueue {
 public:
  JobQueue(int producers, size_t cap) : producers_(producers), cap_(cap) {}
  // false once the queue is aborted (the job is dropped: the call fails)
  bool push(std::unique_ptr<T> j) {
    std::unique_lock<std::mutex> lk(mu_);
    space_.wait(lk, [&] { return q_.size() < cap_ || aborted_; });
    if (aborted_) return false;
    q_.push_back(std::move(j));
    ready_.notify_one();
    return true;
  }
  void producer_done() {
    std::lock_guard<std::mutex> lk(mu_);
    --producers_;
    ready_.notify_all();
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu_);
    aborted_ = true;
    q_.clear();                              // (queued segments are not confirmed: the call fails)
    space_.notify_all();
    ready_.notify_all();
  }
  bool aborted() {
    std::lock_guard<std::mutex> lk(mu_);
    return aborted_;
  }
  // nullptr once every producer is done and the queue is drained, or at
  // once when aborted; with spin_us > 0 the caller first polls that long
  // (yielding) before it sleeps on the condition variable (a futex wake-up
  // under a busy pool took ~0.1 ms)
  std::unique_ptr<T> pop(int* producers_left, int spin_us = 0) {
    std::unique_lock<std::mutex> lk(mu_);
    if (spin_us > 0) {
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
      while (q_.empty() && producers_ != 0 && !aborted_ && std::chrono::steady_clock::now() < until) {
        lk.unlock();
        std::this_thread::yield();
        lk.lock();
      }
    }
    ready_.wait(lk, [&] { return !q_.empty() || producers_ == 0 || aborted_; });
    *producers_left = producers_;
    if (aborted_ || q_.empty()) return nullptr;
    std::unique_ptr<T> j = std::move(q_.front());
    q_.pop_front();
    space_.notify_one();
    return j;
  }

 private:
  std::mutex mu_;
  std::condition_variable ready_, space_;
  std::deque<std::unique_ptr<T>> q_;
  int producers_;
  size_t cap_;
  bool aborted_ = false;
};

// One call's driver fan-out.  drive(d, &err) runs driver d: it takes segment
// indexes from next_segment() until they run out or the queue is aborted,
// pushes each finished segment, releases what it acquired, and returns false
// (err set) on failure.  consume(job, producers_left) confirms one job on the
// calling thread.  before_consume() runs on the calling thread after the
// drivers started (the engine sets up the per-file result slots there).  With
// inline_driver (one driver, one segment) the driver runs on this thread first.
template <typename Job>
class DriverPipeline {
 public:
  DriverPipeline(int ndrivers, size_t nsegments)
      : q_(ndrivers, 2 * static_cast<size_t>(ndrivers) + 2), ndrivers_(ndrivers), nseg_(nsegments) {}

  JobQueue<Job>& queue() { return q_; }
  // the next segment for a driver, or nsegments when none is left (or the call failed)
  size_t next_segment() {
    if (q_.aborted()) return nseg_;
    const size_t s = next_.fetch_add(1);
    return s < nseg_ ? s : nseg_;
  }
  size_t nsegments() const { return nseg_; }

  template <typename Drive, typename Consume>
  bool run(bool inline_driver, Drive&& drive, const std::function<void()>& before_consume, Consume&& consume,
           int pop_spin_us, std::string* err) {
    auto driver = [&](int d) {
      std::string e;
      bool ok = false;
      try {
        ok = drive(d, &e);
      } catch (const std::exception& x) {
        ok = false;
        e = std::string("host exception in the device driver: ") + x.what();
      } catch (...) {
        ok = false;
        e = "host exception in the device driver";
      }
      if (!ok) {
        {
          std::lock_guard<std::mutex> lk(mu_);
          if (drv_err_.empty()) drv_err_ = e.empty() ? "device driver failed" : e;
        }
        q_.abort();
      }
      q_.producer_done();
    };
    std::vector<std::thread> threads;
    std::string host_err;
    try {
      if (!inline_driver) for (int d = 0; d < ndrivers_; ++d) threads.emplace_back(driver, d);
      if (before_consume) before_consume();
      if (inline_driver) driver(0);
      for (;;) {
        int left = 0;
        std::unique_ptr<Job> job = q_.pop(&left, pop_spin_us);
        if (!job) break;
        consume(*job, left);
      }
    } catch (const std::exception& x) {
      // (bad_alloc in the confirmation, or a driver thread that could not be
      // started): stop the drivers, join them, fail the call
      host_err = std::string("host exception: ") + x.what();
    } catch (...) {
      host_err = "host exception";
    }
    if (!host_err.empty()) q_.abort();
    for (auto& t : threads) t.join();
    if (!host_err.empty()) { *err = host_err; return false; }
    std::lock_guard<std::mutex> lk(mu_);
    if (!drv_err_.empty()) { *err = drv_err_; return false; }
    return true;
  }

 private:
  JobQueue<Job> q_;
  int ndrivers_;
  size_t nseg_;
  std::atomic<size_t> next_{0};
  std::mutex mu_;
  std::string drv_err_;
};

}  // namespace tsg
