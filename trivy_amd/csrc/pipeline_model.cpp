// CPU model of Engine::scan's multi-device segment pipeline (pipeline.h) for
// tests and sanitizer runs without a GPU: `ndevices` simulated device drivers
// pull segments from the shared counter, each holding a lane from its
// device's pool while it runs, and hand finished segments to the confirming
// thread -- the engine's driver loop with the HIP work replaced by sleeps.
// One driver can be made to fail at its k-th segment (an error return, as a
// HIP error; or a thrown bad_alloc, as a host allocation failure), or the
// confirming thread can throw.  The statistics tell a test whether the call
// failed as a whole, the other drivers stopped, and every lane came back.
//
// What it models: cgo NewScanner's default engine over every GPU
// (device_mask 0), the replacement of the reference's
// goroutine fan-out pkg/fanal/analyzer/analyzer.go:429-451.
#include <atomic>
#include <chrono>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "pipeline.h"
#include "trivy_secret.h"
#include "trivy_secret_test.h"

namespace tsg {
int capi_fail(int code, const std::string& m);   // capi.cpp: sets tsg_last_error
}

namespace {

using Clock = std::chrono::steady_clock;

struct SimLanes {                      // a device's lane pool
  std::mutex mu;
  uint32_t created = 0, out = 0;
};

struct SimJob {
  size_t seg = 0;
  uint32_t device = 0;
};

}  // namespace

extern "C" int tsg_test_multi_driver_model(uint32_t ndevices, uint32_t nsegments, int32_t fail_device,
                                           uint32_t fail_at, uint32_t fail_mode, uint32_t seg_us,
                                           uint32_t confirm_us, tsg_model_pipeline_stats* out) {
  using namespace tsg;
  if (!out || ndevices == 0 || ndevices > 64) return capi_fail(TSG_ERR_INVALID, "bad argument");
  *out = tsg_model_pipeline_stats();
  try {
    // the process's first C++ throw builds the unwinder's frame tables for
    // every loaded library (~0.2 s beside the HIP runtime): done up front so
    // the statistics time the pipeline's reaction to a failure, not that
    try {
      throw std::bad_alloc();
    } catch (const std::bad_alloc&) {
    }
    std::vector<SimLanes> pools(ndevices);
    std::vector<std::atomic<uint32_t>> confirmed(nsegments);
    for (auto& c : confirmed) c.store(0);
    std::atomic<uint64_t> started{0}, pushed{0}, after_fail{0}, nconf{0};
    std::atomic<int> alive{0};
    std::atomic<int64_t> fail_ns{-1};
    const auto t0 = Clock::now();
    auto now_ns = [&] { return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count(); };
    DriverPipeline<SimJob> pipe(static_cast<int>(ndevices), nsegments);
    auto drive = [&](int d, std::string* e) -> bool {
      alive.fetch_add(1);
      SimLanes& pool = pools[d];
      {
        std::lock_guard<std::mutex> lk(pool.mu);
        ++pool.out;
        pool.created = std::max(pool.created, pool.out);
      }
      struct Release {                  // the lane goes back on every exit, a throw included
        SimLanes& p;
        std::atomic<int>& a;
        ~Release() {
          { std::lock_guard<std::mutex> lk(p.mu); --p.out; }
          a.fetch_sub(1);
        }
      } rel{pool, alive};
      uint32_t mine = 0;
      for (size_t cur = pipe.next_segment(); cur < pipe.nsegments(); cur = pipe.next_segment()) {
        started.fetch_add(1);
        if (fail_ns.load() >= 0) after_fail.fetch_add(1);
        std::this_thread::sleep_for(std::chrono::microseconds(seg_us));     // upload + K1 + K2 + readback
        if (static_cast<int32_t>(d) == fail_device && mine == fail_at && (fail_mode == 1 || fail_mode == 2)) {
          int64_t expect = -1;
          fail_ns.compare_exchange_strong(expect, now_ns());
          if (fail_mode == 2) throw std::bad_alloc();
          *e = "injected device failure (simulated device " + std::to_string(d) + ")";
          return false;
        }
        ++mine;
        std::unique_ptr<SimJob> j(new SimJob());
        j->seg = cur;
        j->device = static_cast<uint32_t>(d);
        if (pipe.queue().push(std::move(j))) pushed.fetch_add(1);
      }
      return true;
    };
    std::string err;
    const bool ok = pipe.run(ndevices == 1 && nsegments == 1, drive, nullptr,
                             [&](SimJob& j, int) {
                               if (fail_mode == 3 && nconf.load() == fail_at) {
                                 int64_t expect = -1;
                                 fail_ns.compare_exchange_strong(expect, now_ns());
                                 throw std::bad_alloc();
                               }
                               std::this_thread::sleep_for(std::chrono::microseconds(confirm_us));
                               confirmed[j.seg].fetch_add(1);
                               nconf.fetch_add(1);
                             },
                             0, &err);
    const int64_t t_end = now_ns();
    out->segments_started = started.load();
    out->segments_pushed = pushed.load();
    out->segments_confirmed = nconf.load();
    out->started_after_failure = after_fail.load();
    for (auto& p : pools) {
      out->lanes_outstanding += p.out;
      out->lanes_created += p.created;
    }
    out->drivers_alive = static_cast<uint32_t>(alive.load());
    for (auto& c : confirmed) if (c.load() > 1) ++out->segments_confirmed_twice;
    out->wall_ms = t_end / 1e6;
    out->fail_to_return_ms = fail_ns.load() >= 0 ? (t_end - fail_ns.load()) / 1e6 : 0.0;
    if (!ok) return capi_fail(TSG_ERR_HIP, err);
    return TSG_OK;
  } catch (const std::bad_alloc&) {
    return capi_fail(TSG_ERR_INTERNAL, "out of memory");
  } catch (const std::exception& x) {
    return capi_fail(TSG_ERR_INTERNAL, std::string("internal error: ") + x.what());
  }
}
