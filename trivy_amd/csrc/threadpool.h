// Persistent worker pool for the host confirm phase (no thread creation per batch).
#pragma once
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace tsg {

class ThreadPool {
 public:
  explicit ThreadPool(int n) {
    for (int i = 1; i < n; ++i) workers_.emplace_back([this, i] { loop(i); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return static_cast<int>(workers_.size()) + 1; }
  // Runs fn(worker_index) on every worker and the calling thread; returns when
  // all are done.  An exception thrown by fn on any thread is rethrown here,
  // on the calling thread, once every worker has finished (one escaping a
  // worker thread would call std::terminate).
  void run(const std::function<void(int)>& fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      pending_ = static_cast<int>(workers_.size());
      err_ = nullptr;
      ++gen_;
    }
    cv_.notify_all();
    std::exception_ptr mine;
    try {
      fn(0);
    } catch (...) {
      mine = std::current_exception();
    }
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
    if (!mine) mine = err_;
    err_ = nullptr;
    lk.unlock();
    if (mine) std::rethrow_exception(mine);
  }

 private:
  void loop(int idx) {
    unsigned long seen = 0;
    for (;;) {
      const std::function<void(int)>* fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        fn = fn_;
      }
      std::exception_ptr e;
      try {
        (*fn)(idx);
      } catch (...) {
        e = std::current_exception();
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (e && !err_) err_ = e;
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  std::exception_ptr err_;                 // the first exception a worker threw in this run
  int pending_ = 0;
  unsigned long gen_ = 0;
  bool stop_ = false;
};

}  // namespace tsg
