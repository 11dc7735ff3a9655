// GPU engine: device-resident rule tables on one or more MI355X devices and
// the batch pipeline (upload -> K1 -> K2 -> candidates -> exact host confirm).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "prefilter.h"
#include "scanner.h"

namespace tsg {

struct ScanStats {
  double k1_ms = 0, k2_ms = 0, h2d_ms = 0, d2h_ms = 0, host_ms = 0, total_ms = 0;
  double gpu_wall_ms = 0;               // sum over devices of the driver threads' busy time
  uint64_t bytes = 0, files = 0, hits = 0, candidates = 0, confirm_files = 0, findings = 0;
  uint32_t k1_blocks = 0, k1_threads = 0, chunk_bytes = 0, pieces = 1;
  int table_in_lds = 0;
  uint32_t k1_launches = 0;             // K1 launches (segments x scan-DFA groups)
  uint32_t devices = 1;                 // devices that took part
  double feed_ms = 0;                   // wall time from the first upload to the last segment's upload done
};

struct BatchInput {
  const uint8_t* h_data = nullptr;     // host copy (needed by the exact confirmer)
  const void* d_data = nullptr;        // device copy; nullptr -> engine uploads h_data
  const uint64_t* offsets = nullptr;   // nfiles + 1 byte offsets into data
  uint32_t nfiles = 0;
  const char* const* paths = nullptr;  // nfiles NUL-terminated paths (ScanArgs.FilePath)
  const uint32_t* path_lens = nullptr; // optional explicit lengths
  const uint8_t* binary = nullptr;     // optional ScanArgs.Binary flags
};

// A batch scan stage: results[i] = Scan(ScanArgs{paths[i], data[off[i]:off[i+1]],
// binary[i]}) -- Engine::scan, or (tests only) the CPU model of its passes.
using BatchScanFn = std::function<bool(const BatchInput& in, SecretVec* results, std::string* err)>;

struct DeviceTables;
struct Lane;
struct GpuOut;
struct CallCtx;
struct K1Chain;
struct StageIn;

// One engine = the compiled ruleset's device tables on every selected device.
// scan() is reentrant: each call takes its own lane (HIP streams + scratch
// buffers) on every device it uses and its own host confirm pool.
class Engine {
 public:
  // devices: HIP device ordinals (may repeat one ordinal: replicas on one
  // device, used to exercise the multi-device queue on a one-GPU machine).
  // Fails (nullptr, *err set) when no HIP device is available: the product
  // path has no CPU fallback.
  static std::unique_ptr<Engine> create(std::shared_ptr<const Ruleset> rs, const std::vector<int>& devices,
                                        std::string* err);
  ~Engine();

  // results[i] is Scanner.Scan(ScanArgs{paths[i], data[off[i]:off[i+1]], binary[i]}).
  bool scan(const BatchInput& in, SecretVec* results, ScanStats* stats, std::string* err);

  // Only the two GPU passes (no host confirmation): used by tests to compare
  // raw candidates.  Resident data on the engine's first device.
  bool prefilter_only(const BatchInput& in, std::vector<std::vector<std::vector<uint64_t>>>* cands,
                      ScanStats* stats, std::string* err);

  // Host-feed ceiling (no kernels): streams `bytes` of host memory through
  // the first device's upload ring in segment_ pieces, as scan() does, and
  // returns the wall time in ms.
  bool feed_probe(const uint8_t* h_data, uint64_t bytes, double* ms, std::string* err);

  // GPU-side CR strip of a device-resident batch on the first device
  // (crstrip.hip): d_dst = d_src without '\r', d_new_off = the files' new
  // starts; *out_total = stripped bytes, *ms = the kernels' time (HIP events).
  bool strip_cr(const void* d_src, const uint64_t* d_off, uint32_t nfiles, uint64_t total, void* d_dst,
                uint64_t* d_new_off, uint64_t* out_total, double* ms, std::string* err);

  // Lanes created over all devices, call contexts, and confirm-pool threads
  // started (test hook: the per-file queue's footprint).
  void footprint(uint32_t* lanes, uint32_t* calls, uint32_t* pool_threads);
  // Test hook: the next n run_segment calls fail before their first launch.
  void inject_segment_failures(uint32_t n) { inject_fail_.store(n); }

  const Prefilter& prefilter() const { return pf_; }
  std::shared_ptr<const Ruleset> ruleset() const { return rs_; }
  const std::vector<int>& devices() const { return devices_; }
  void set_threads(int n) { threads_ = n; }

 private:
  Engine() = default;
  struct Segment;
  // while_gpu (optional) runs once on the calling thread after the segment's
  // kernels are queued, before their readbacks are; chain (optional) orders
  // the K1 launches of several drivers of one device (K1Chain); defer_copy
  // leaves the readback in the lane's pinned buffers (GpuOut::finish_copy);
  // stage (optional) is a small pinned batch the segment prologue copies in
  // (used by this call only: nothing of it stays on the pooled lane)
  bool run_segment(DeviceTables& dt, Lane& ln, const Segment& sg, const void* d_data, const uint64_t* d_off_up,
                   ScanStats* st, GpuOut* out, std::string* err, const std::function<void()>* while_gpu = nullptr,
                   K1Chain* chain = nullptr, bool defer_copy = false, const StageIn* stage = nullptr);
  void plan_confirm(const Segment& sg, GpuOut* g) const;
  void confirm_segment(CallCtx& cc, const Segment& sg, GpuOut& g, Secret* results, uint64_t* nconf,
                       uint64_t* nfind, bool gpu_in_flight);
  Lane* acquire_lane(DeviceTables& dt, std::string* err);
  void release_lane(DeviceTables& dt, Lane* ln);
  CallCtx* acquire_call();
  void release_call(CallCtx* cc);

  std::shared_ptr<const Ruleset> rs_;
  Prefilter pf_;
  std::vector<int> devices_;
  std::vector<std::unique_ptr<DeviceTables>> dev_;
  int threads_ = 0;
  std::mutex call_mu_;
  std::vector<std::unique_ptr<CallCtx>> calls_;
  std::vector<CallCtx*> free_calls_;
  // tuning (TSG_* environment knobs, read once at create)
  uint32_t chunk_ = 0;                  // K1 bytes per lane chunk (TSG_K1_CHUNK); 0 = by launch size (k1_chunk_for)
  // TSG_K1_ABL: K1 build (kAbl* bits).  Default 4560 = deferred outputs +
  // rolled word loop + 64-byte lines + temporal loads + fast words in boundary
  // lines (layout bits, results valid); the other bits are measurement builds
  // whose results are invalid.
  int k1_abl_ = 4560;
  uint32_t k1_tail_rounds_ = 1;         // v3 guided schedule: grid rounds of 2- and of 1-chunk ranges (TSG_K1_TAIL_ROUNDS)
  // launches of >= 2 GiB: 1 KiB chunks with 8-chunk bulk ranges, then rounds
  // of 4-, 2- and 1-chunk ranges (TSG_K1_TOP8=1; 2: the kU = 8 level in every
  // launch, for tests), instead of 2 KiB chunks
  int k1_top8_ = 1;
  // drivers per device for resident batches (TSG_RESIDENT_DRIVERS; 2 =
  // K1Chain).  Round 4 chained the second driver's K1 behind the first's K2:
  // no gain (config 2 1530 vs 1528 GB/s).  Chained behind the first's K1
  // (TSG_CHAIN_K1, round 5) a piece's K2 runs beside the next piece's K1 and
  // leaves the critical chain: config 2 1632 -> 1862 GB/s, 1 GB of config-1
  // files 482 -> 570 (profiles/r5p_resident_variants.log).
  int resident_drivers_ = 2;
  int chain_k1_ = 1;
  uint32_t k1_reserve_cus_ = 0;         // K1Chain pieces: CUs left out of K1's grid for the previous piece's K2 / readback (TSG_K1_RESERVE_CUS)
  bool readback_dma_ = false;
  bool file_index_ = true;              // K1 range starts' files from a per-64-KiB index (TSG_K1_FILE_INDEX)           // K1Chain pieces read back by DMA copies instead of tsg_readback (TSG_READBACK_DMA)                    // K1Chain: 0 = next K1 after this K2, 1 = after this K1, 2 = no wait (TSG_CHAIN_K1)
  // K1Chain drivers poll their readback event yielding instead of sleeping
  // 10 us (TSG_POLL_YIELD), and the confirmer polls the job queue up to
  // pop_spin_us_ before it sleeps (TSG_POP_SPIN_US): a wake-up under the busy
  // confirm pool came 0.1-0.2 ms late; config 2 resident 1838 -> 1920-1945
  // GB/s, config 1 unchanged (profiles/r6a_resident_poll.log)
  bool poll_yield_ = true;
  bool confirm_prefetch_ = true;        // confirm pool: prefetch the next file's result slot and candidate text (TSG_CONFIRM_PREFETCH)
  int pop_spin_us_ = 2000;
  uint32_t k2_hits_per_thread_ = 1;     // K2 grid: hits of the fullest region per thread (TSG_K2_HITS_PER_THREAD)
  bool k2_stats_ = false;               // TSG_K2_STATS=1: per-rule K2 counters, printed to stderr at destruction
  int k2_abl_ = 0;                      // TSG_K2_ABL (probe library): K2 trace / no-walk measurement builds
  bool host_profile_ = false;           // TSG_HOST_PROFILE=1: per-segment host confirm breakdown on stderr
  std::atomic<uint32_t> inject_fail_{0};
  std::mutex k2s_mu_;
  std::vector<unsigned long long> k2s_;  // 4 per rule: hits, past the keyword gate, verify starts, bytes walked
  // resident data: pipeline pieces (TSG_PIECES; r3za config 2: 4 pieces,
  // first 10%: 1286 GB/s, 2 at 70/30: 919), the first piece's share
  // (TSG_FIRST_PIECE) and a short last piece's (TSG_LAST_PIECE, 0: none; used
  // from 5 pieces on).  Round 5, K2 beside the next K1 (K1Chain): 5 pieces
  // with an 8% last piece 1921 GB/s vs 4 pieces 1796 on config 2 -- the last
  // piece's K2 and host confirmation are the step's tail; 1 GB of config-1
  // files gains nothing from more pieces (profiles/r5t_resident_pieces.log)
  uint32_t pieces_ = 5;
  double first_piece_ = 0.1;
  double first_piece_few_ = 0.2;        // the first piece's share when a batch makes 3 pieces (TSG_FIRST_PIECE_FEW)
  double last_piece_ = 0.08;
  uint64_t min_piece_ = 256ull << 20;   // resident data: smaller batches run as one piece (TSG_MIN_PIECE_BYTES)
  uint64_t segment_min_ = 64ull << 20;   // uploaded data: smallest segment of the geometric tail (TSG_SEGMENT_MIN; r3s: 128 MB 51.5 vs 256 MB 48.8 GB/s on config 1; r4p: 64 MB 53.2 vs 128 MB 52.5)
  bool balanced_ = true;                // uploaded large-file data: equal segments of <= segment_ (TSG_SEGMENT_BALANCED)
  uint64_t segment_tail_ = 0;           // uploaded data: a short last segment (TSG_SEGMENT_TAIL; 0 = none: the
                                        // rest after the full segments is one launch, K1 keeps its large-launch rate)
  uint64_t segment_ = 4ull << 30;       // uploaded data: bytes per pipeline segment (TSG_SEGMENT_BYTES);
                                        // 1 GB = one full K1 round (256 CUs x 1024 lanes x 4 KiB chunks)
};

int device_count();

// Test hook (tsg_test_readback): tsg_readback of min(nwords, count * per_count)
// dwords of a device buffer holding 1, 2, ... into host-mapped memory on
// device 0; *copied = the dwords that arrived.
bool readback_probe(uint32_t nwords, uint32_t count, uint32_t per_count, uint32_t* copied, std::string* err);

}  // namespace tsg
