// Exception-safe fan-out for host threads.  No C++ exception may cross the
// C ABI (TSG_API_TRY catches on the calling thread only), and one escaping a
// std::thread's function calls std::terminate: every helper thread here
// catches what its work throws, the threads are joined, and the first
// exception is rethrown on the calling thread (inside TSG_API_TRY).
#pragma once
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tsg {

class ThreadErrors {
 public:
  void capture() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!first_) first_ = std::current_exception();
  }
  bool any() {
    std::lock_guard<std::mutex> lk(mu_);
    return static_cast<bool>(first_);
  }
  void rethrow() {
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> lk(mu_);
      e = first_;
    }
    if (e) std::rethrow_exception(e);
  }
  // the first exception as an error message ("" if none)
  std::string message() {
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> lk(mu_);
      e = first_;
    }
    if (!e) return std::string();
    try {
      std::rethrow_exception(e);
    } catch (const std::exception& x) {
      return std::string("host exception: ") + x.what();
    } catch (...) {
      return "host exception";
    }
  }

 private:
  std::mutex mu_;
  std::exception_ptr first_;
};

// Runs fn() on the calling thread and on nthreads - 1 helper threads (fewer if
// the system refuses to create more), joins them all, then rethrows the first
// exception any of them threw.
template <typename F>
void run_threads(int nthreads, F&& fn) {
  ThreadErrors te;
  auto body = [&]() {
    try {
      fn();
    } catch (...) {
      te.capture();
    }
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < nthreads; ++t) {
    try {
      ts.emplace_back(body);
    } catch (...) {
      break;                                  // run with the threads that started
    }
  }
  body();
  for (auto& th : ts) th.join();
  te.rethrow();
}

}  // namespace tsg
