// C-ABI (include/trivy_secret.h) over the ruleset, the GPU engine and the
// host confirmer.
#include "../../include/trivy_secret.h"
#include "../../include/trivy_secret_test.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <condition_variable>
#include <mutex>
#include <thread>

#include <malloc.h>
#include <pthread.h>

#include "engine.h"
#include "gosort.h"
#include "guard.h"
#include "feed.h"
#include "tar.h"
#include "prefilter.h"
#include "report.h"
#include "queue.h"
#include "stream.h"
#include "scanner.h"
#include "walkfs.h"
#include "wire.h"

using namespace tsg;

extern "C" const char* tsg_builtin_json_ptr();   // scanner.cpp

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& m) { g_err = m; return code; }
// No C++ exception crosses the C ABI: an allocation failure (a huge batch,
// a hostile size field) or any other escaping exception becomes an error code
// with its message in tsg_last_error().
#define TSG_API_TRY try {
#define TSG_API_CATCH                                                                          \
  } catch (const std::bad_alloc&) {                                                            \
    return fail(TSG_ERR_INTERNAL, "out of memory");                                            \
  } catch (const std::exception& ex_) {                                                        \
    return fail(TSG_ERR_INTERNAL, std::string("internal error: ") + ex_.what());                \
  } catch (...) {                                                                              \
    return fail(TSG_ERR_INTERNAL, "internal error");                                           \
  }
}  // namespace

// the C-ABI's error slot for test hooks defined in other files (pipeline_model.cpp)
namespace tsg {
int capi_fail(int code, const std::string& m);
}
int tsg::capi_fail(int code, const std::string& m) { return fail(code, m); }

struct tsg_ruleset {
  std::shared_ptr<Ruleset> rs;
};

struct tsg_engine {
  std::unique_ptr<Engine> eng;   // reentrant: every call takes its own lanes (streams + buffers)
  std::string report;
};

struct tsg_prepared {
  PreparedBatch b;
  // layer-tar batches: the kept files' ScanArgs.FilePath and the walk summary
  std::vector<std::string> scan_paths;
  std::vector<const char*> path_ptrs;
  std::vector<uint32_t> path_lens;
  std::string walk_json;
};

struct tsg_result {
  std::shared_ptr<const Ruleset> rs;     // findings point at its rules
  std::shared_ptr<std::deque<Rule>> own_rules;   // or at these (tsg_result_from_json)
  SecretVec files;
  ScanStats stats;
  std::vector<std::vector<std::vector<uint64_t>>> cands;   // optional [file][rule]
  std::vector<std::vector<LayerRef>> layers;               // optional [file][finding] (tsg_result_from_proto)
  // streamed results: the walk outcome, turned into JSON on the first
  // tsg_result_walk_json call (a layer's walked-path list runs to megabytes)
  std::unique_ptr<StreamResult> walk;
  mutable std::mutex walk_mu;
  mutable std::string walk_json;
};

extern "C" {

const char* tsg_last_error(void) { return g_err.c_str(); }
const char* tsg_version(void) { return "trivy-secret-mi355x 0.1 (gfx950)"; }

int tsg_ruleset_compile(const char* config_json, size_t config_len, tsg_ruleset** out) {
  TSG_API_TRY
  if (!out) return fail(TSG_ERR_INVALID, "out is NULL");
  std::string err;
  auto rs = std::make_shared<Ruleset>();
  if (config_json) {
    JValue cfg;
    std::string text(config_json, config_len);
    if (!json_parse(text, &cfg, &err)) return fail(TSG_ERR_CONFIG, "secrets config decode error: " + err);
    if (!build_ruleset(cfg.is_null() ? nullptr : &cfg, rs.get(), &err)) return fail(TSG_ERR_CONFIG, err);
  } else if (!build_ruleset(nullptr, rs.get(), &err)) {
    return fail(TSG_ERR_CONFIG, err);
  }
  *out = new tsg_ruleset{rs};
  return TSG_OK;
  TSG_API_CATCH
}

void tsg_ruleset_free(tsg_ruleset* rs) { delete rs; }

int tsg_ruleset_num_rules(const tsg_ruleset* rs) { return rs ? static_cast<int>(rs->rs->rules.size()) : 0; }

const char* tsg_ruleset_rule_id(const tsg_ruleset* rs, int i) {
  if (!rs || i < 0 || i >= static_cast<int>(rs->rs->rules.size())) return nullptr;
  return rs->rs->rules[i].id.c_str();
}

int tsg_ruleset_allow_path(const tsg_ruleset* rs, const char* path, size_t len) {
  TSG_API_TRY
  if (!rs) return fail(TSG_ERR_INVALID, "ruleset is NULL");
  return global_allow_path(*rs->rs, reinterpret_cast<const uint8_t*>(path), len) ? 1 : 0;
  TSG_API_CATCH
}

int tsg_device_count(void) { return device_count(); }

namespace {
// The confirmation builds each file's Secret (findings, lines, text arena) on
// the pool's threads, and the caller frees the whole result after reading
// it: with glibc's defaults the freed heap tops go back to the kernel and the
// next batch faults them in again (config 5: 19 -> 13.5 thread-ms per 3 GB
// piece in the findings phase with the heap kept, resident step 18.1 ->
// 16.6 ms; profiles/r5w_malloc_c5.log).  Once per process, at the first
// engine, and only when the embedding process asks for it (TSG_MALLOC_TUNE=1:
// the policy is process-wide, so a long-lived embedder -- a trivy server --
// keeps glibc's defaults unless it opts in; bench.py opts in): freed heap is
// kept (trim threshold 1 GiB, top pad 256 MiB) and requests below 32 MiB
// come from the heap.
void tune_malloc_once() {
  static std::once_flag once;
  std::call_once(once, [] {
    const char* v = std::getenv("TSG_MALLOC_TUNE");
    if (!v || std::atoi(v) == 0) return;
    mallopt(M_TRIM_THRESHOLD, 1 << 30);
    mallopt(M_TOP_PAD, 256 << 20);
    mallopt(M_MMAP_THRESHOLD, 32 << 20);
  });
}
}  // namespace

int tsg_engine_create(const tsg_ruleset* rs, uint64_t device_mask, tsg_engine** out) {
  TSG_API_TRY
  if (!rs || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  tune_malloc_once();
  std::string err;
  const int n = device_count();
  if (n <= 0) return fail(TSG_ERR_NO_DEVICE, "no HIP device available (the GPU engine has no CPU fallback)");
  std::vector<int> devs;
  for (int d = 0; d < n && d < 64; ++d) if (device_mask == 0 || ((device_mask >> d) & 1u)) devs.push_back(d);
  if (devs.empty()) return fail(TSG_ERR_INVALID, "device_mask selects no visible HIP device");
  // TSG_ENGINE_REPLICAS=k: each selected device appears k times (several
  // drivers share one device; exercises the multi-device queue on one GPU)
  if (const char* r = std::getenv("TSG_ENGINE_REPLICAS")) {
    const int k = std::atoi(r);
    std::vector<int> rep;
    for (int i = 0; i < std::max(1, std::min(k, 8)); ++i) rep.insert(rep.end(), devs.begin(), devs.end());
    devs = rep;
  }
  auto eng = Engine::create(rs->rs, devs, &err);
  if (!eng) return fail(device_count() <= 0 ? TSG_ERR_NO_DEVICE : TSG_ERR_HIP, err);
  auto* e = new tsg_engine();
  e->report = eng->prefilter().report;
  e->eng = std::move(eng);
  *out = e;
  return TSG_OK;
  TSG_API_CATCH
}

void tsg_engine_destroy(tsg_engine* e) { delete e; }

void tsg_engine_set_threads(tsg_engine* e, int threads) { if (e) e->eng->set_threads(threads); }

const char* tsg_engine_report(const tsg_engine* e) { return e ? e->report.c_str() : ""; }

int tsg_alloc_pinned(size_t bytes, void** out);
void tsg_free_pinned(void* p);

static int do_scan(tsg_engine* e, const void* d_data, const uint8_t* h_data, const uint64_t* offsets,
                   uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, const uint8_t* binary,
                   tsg_result** out) {
  if (!e || !out || !offsets || (nfiles && !paths) || (!h_data && nfiles)) return fail(TSG_ERR_INVALID, "NULL argument");
  BatchInput in;
  in.h_data = h_data;
  in.d_data = d_data;
  in.offsets = offsets;
  in.nfiles = nfiles;
  in.paths = paths;
  in.path_lens = path_lens;
  in.binary = binary;
  auto* r = new tsg_result();
  r->rs = e->eng->ruleset();
  std::string err;
  if (!e->eng->scan(in, &r->files, &r->stats, &err)) { delete r; return fail(TSG_ERR_HIP, err); }
  *out = r;
  return TSG_OK;
}

int tsg_scan_batch(tsg_engine* e, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                   const char* const* paths, const uint32_t* path_lens, const uint8_t* binary, tsg_result** out) {
  TSG_API_TRY
  return do_scan(e, nullptr, data, offsets, nfiles, paths, path_lens, binary, out);
  TSG_API_CATCH
}

int tsg_scan_batch_resident(tsg_engine* e, const void* d_data, const uint8_t* h_data, const uint64_t* offsets,
                            uint32_t nfiles, const char* const* paths, const uint32_t* path_lens,
                            const uint8_t* binary, tsg_result** out) {
  TSG_API_TRY
  if (!d_data) return fail(TSG_ERR_INVALID, "d_data is NULL");
  return do_scan(e, d_data, h_data, offsets, nfiles, paths, path_lens, binary, out);
  TSG_API_CATCH
}

int tsg_prefilter_resident(tsg_engine* e, const void* d_data, const uint8_t* h_data, const uint64_t* offsets,
                           uint32_t nfiles, tsg_result** out) {
  TSG_API_TRY
  if (!e || !out || !offsets) return fail(TSG_ERR_INVALID, "NULL argument");
  BatchInput in;
  in.h_data = h_data;
  in.d_data = d_data;
  in.offsets = offsets;
  in.nfiles = nfiles;
  auto* r = new tsg_result();
  std::string err;
  if (!e->eng->prefilter_only(in, &r->cands, &r->stats, &err)) { delete r; return fail(TSG_ERR_HIP, err); }
  r->files.resize(nfiles);
  *out = r;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_feed_probe(tsg_engine* e, const uint8_t* data, uint64_t bytes, double* ms) {
  TSG_API_TRY
  if (!e || !ms || (bytes && !data)) return fail(TSG_ERR_INVALID, "NULL argument");
  std::string err;
  if (!e->eng->feed_probe(data, bytes, ms, &err)) return fail(TSG_ERR_HIP, err);
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_strip_cr_device(tsg_engine* e, const void* d_src, const uint64_t* d_offsets, uint32_t nfiles, uint64_t total,
                        void* d_dst, uint64_t* d_new_offsets, uint64_t* out_total, double* ms) {
  TSG_API_TRY
  if (!e || !d_offsets || !d_new_offsets || !out_total) return fail(TSG_ERR_INVALID, "NULL argument");
  std::string err;
  if (!e->eng->strip_cr(d_src, d_offsets, nfiles, total, d_dst, d_new_offsets, out_total, ms, &err))
    return fail(err.find("CR strip:") == 0 || err.find("aligned") != std::string::npos ? TSG_ERR_INVALID : TSG_ERR_HIP,
                err);
  return TSG_OK;
  TSG_API_CATCH
}

uint32_t tsg_result_num_files(const tsg_result* r) { return r ? static_cast<uint32_t>(r->files.size()) : 0; }

int tsg_result_file_path(const tsg_result* r, uint32_t f, const char** path, size_t* len) {
  TSG_API_TRY
  if (!r || f >= r->files.size()) return fail(TSG_ERR_INVALID, "file index out of range");
  *path = r->files[f].file_path().data();
  *len = r->files[f].file_path().size();
  return TSG_OK;
  TSG_API_CATCH
}

uint32_t tsg_result_num_findings(const tsg_result* r, uint32_t f) {
  if (!r || f >= r->files.size()) return 0;
  return static_cast<uint32_t>(r->files[f].findings().size());
}

int tsg_result_file_error(const tsg_result* r, uint32_t f) {
  TSG_API_TRY
  if (!r || f >= r->files.size()) return 0;
  return r->files[f].error;
  TSG_API_CATCH
}

int tsg_result_finding(const tsg_result* r, uint32_t f, uint32_t k, tsg_finding* out) {
  TSG_API_TRY
  if (!r || f >= r->files.size() || k >= r->files[f].findings().size() || !out) return fail(TSG_ERR_INVALID, "index out of range");
  const Secret& sec = r->files[f];
  const FindingRec& x = sec.findings()[k];
  const Rule& ru = *x.rule;
  const std::string& sev = Secret::severity(x);
  out->rule_id = ru.id.data(); out->rule_id_len = ru.id.size();
  out->category = ru.category.data(); out->category_len = ru.category.size();
  out->severity = sev.data(); out->severity_len = sev.size();
  out->title = ru.title.data(); out->title_len = ru.title.size();
  out->start_line = x.start_line;
  out->end_line = x.end_line;
  out->match = sec.ptr(x.match); out->match_len = x.match.len;
  out->num_lines = x.line_count;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_result_line(const tsg_result* r, uint32_t f, uint32_t k, uint32_t l, tsg_line* out) {
  TSG_API_TRY
  if (!r || f >= r->files.size() || k >= r->files[f].findings().size() || !out) return fail(TSG_ERR_INVALID, "index out of range");
  const Secret& sec = r->files[f];
  const FindingRec& x = sec.findings()[k];
  if (l >= x.line_count) return fail(TSG_ERR_INVALID, "line index out of range");
  const LineRec& ln = sec.lines()[x.line_begin + l];
  out->number = ln.number;
  out->content = sec.ptr(ln.content); out->content_len = ln.content.len;
  out->is_cause = ln.is_cause;
  out->annotation = ""; out->annotation_len = 0;
  out->truncated = 0;
  out->highlighted = sec.ptr(ln.content); out->highlighted_len = ln.content.len;
  out->first_cause = ln.first_cause;
  out->last_cause = ln.last_cause;
  return TSG_OK;
  TSG_API_CATCH
}

static void json_bytes(std::string* o, const char* data, size_t n) {
  o->push_back('"');
  const uint8_t* p = reinterpret_cast<const uint8_t*>(data);
  size_t i = 0;
  char buf[16];
  while (i < n) {
    uint8_t c = p[i];
    if (c < 0x80) {
      if (c == '"') *o += "\\\"";
      else if (c == '\\') *o += "\\\\";
      else if (c == '\n') *o += "\\n";
      else if (c == '\r') *o += "\\r";
      else if (c == '\t') *o += "\\t";
      else if (c < 0x20 || c == 0x7f) { snprintf(buf, sizeof buf, "\\u%04x", c); *o += buf; }
      else o->push_back(static_cast<char>(c));
      ++i;
      continue;
    }
    int32_t r; int w;
    re::decode_rune(p + i, n - i, &r, &w);
    if (r == 0xFFFD && w == 1) { snprintf(buf, sizeof buf, "\\udc%02x", c); *o += buf; i += 1; continue; }
    o->append(data + i, w);
    i += w;
  }
  o->push_back('"');
}

static void json_str(std::string* o, std::string_view s) { json_bytes(o, s.data(), s.size()); }

int tsg_result_json(const tsg_result* r, char** json, size_t* len) {
  TSG_API_TRY
  if (!r || !json) return fail(TSG_ERR_INVALID, "NULL argument");
  std::string o = "[";
  for (size_t f = 0; f < r->files.size(); ++f) {
    const Secret& s = r->files[f];
    if (f) o += ",";
    o += "{\"FilePath\":";
    json_str(&o, s.file_path());
    o += ",\"Findings\":[";
    const auto sf = s.findings();
    const auto sl = s.lines();
    for (size_t k = 0; k < sf.size(); ++k) {
      const FindingRec& x = sf[k];
      if (k) o += ",";
      o += "{\"RuleID\":"; json_str(&o, x.rule->id);
      o += ",\"Category\":"; json_str(&o, x.rule->category);
      o += ",\"Severity\":"; json_str(&o, Secret::severity(x));
      o += ",\"Title\":"; json_str(&o, x.rule->title);
      o += ",\"StartLine\":" + std::to_string(x.start_line);
      o += ",\"EndLine\":" + std::to_string(x.end_line);
      o += ",\"Code\":{\"Lines\":[";
      for (uint32_t l = 0; l < x.line_count; ++l) {
        const LineRec& ln = sl[x.line_begin + l];
        if (l) o += ",";
        o += "{\"Number\":" + std::to_string(ln.number);
        o += ",\"Content\":"; json_bytes(&o, s.ptr(ln.content), ln.content.len);
        o += std::string(",\"IsCause\":") + (ln.is_cause ? "true" : "false");
        o += ",\"Annotation\":\"\"";
        o += ",\"Truncated\":false";
        o += ",\"Highlighted\":"; json_bytes(&o, s.ptr(ln.content), ln.content.len);
        o += std::string(",\"FirstCause\":") + (ln.first_cause ? "true" : "false");
        o += std::string(",\"LastCause\":") + (ln.last_cause ? "true" : "false");
        o += "}";
      }
      o += "]},\"Match\":";
      json_bytes(&o, s.ptr(x.match), x.match.len);
      if (f < r->layers.size() && k < r->layers[f].size()) {
        const LayerRef& lr = r->layers[f][k];
        o += ",\"Layer\":{\"Digest\":"; json_str(&o, lr.digest);
        o += ",\"DiffID\":"; json_str(&o, lr.diff_id);
        o += ",\"CreatedBy\":"; json_str(&o, lr.created_by);
        o += "}";
      }
      o += "}";
    }
    o += "]";
    if (s.error) o += ",\"Error\":1";
    o += "}";
  }
  o += "]";
  char* buf = static_cast<char*>(malloc(o.size() + 1));
  if (!buf) return fail(TSG_ERR_INTERNAL, "out of memory");
  memcpy(buf, o.data(), o.size());
  buf[o.size()] = 0;
  *json = buf;
  if (len) *len = o.size();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_result_stats(const tsg_result* r, tsg_stats* out) {
  TSG_API_TRY
  if (!r || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  const ScanStats& s = r->stats;
  out->k1_ms = s.k1_ms; out->k2_ms = s.k2_ms; out->h2d_ms = s.h2d_ms; out->d2h_ms = s.d2h_ms;
  out->host_ms = s.host_ms; out->total_ms = s.total_ms;
  out->bytes = s.bytes; out->files = s.files; out->hits = s.hits; out->candidates = s.candidates;
  out->confirm_files = s.confirm_files; out->findings = s.findings;
  out->k1_blocks = s.k1_blocks; out->k1_threads = s.k1_threads; out->chunk_bytes = s.chunk_bytes;
  out->table_in_lds = s.table_in_lds;
  out->gpu_wall_ms = s.gpu_wall_ms;
  out->pieces = s.pieces;
  out->k1_launches = s.k1_launches;
  out->devices = s.devices;
  out->feed_ms = s.feed_ms;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_result_candidates(const tsg_result* r, uint32_t f, uint32_t rule, const uint64_t** starts, size_t* n) {
  TSG_API_TRY
  if (!r || f >= r->cands.size() || rule >= r->cands[f].size()) { *starts = nullptr; *n = 0; return TSG_OK; }
  *starts = r->cands[f][rule].data();
  *n = r->cands[f][rule].size();
  return TSG_OK;
  TSG_API_CATCH
}

// Large results are freed on a reaper thread.  A config-5 result (297k
// Secrets, 44k findings whose arenas the confirm threads allocated, so most
// frees cross malloc arenas) took 23 ms to delete: 11% of the next step when
// done inline; config 2's 18k findings 1 ms.  The reaper frees them while
// the next batch's first upload runs.
namespace {
struct Reaper {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<tsg_result*> q;
  std::thread th;
  bool stop = false;
  void loop() {
    // idle priority: the frees of one batch's result overlap the next batch,
    // whose host confirmation keeps every core of the quota busy (on the
    // resident path a normal-priority reaper took a core from it)
    sched_param sp{};
    sp.sched_priority = 0;
    pthread_setschedparam(pthread_self(), SCHED_IDLE, &sp);
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || !q.empty(); });
      if (q.empty()) return;
      tsg_result* r = q.front();
      q.pop_front();
      lk.unlock();
      delete r;
      lk.lock();
    }
  }
  ~Reaper() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    if (th.joinable()) th.join();
  }
};
Reaper* g_reaper = nullptr;       // guarded by g_reaper_mu
bool g_reaper_closed = false;      // static destruction has begun: results are deleted inline
std::mutex g_reaper_mu;
// a forked child has no reaper thread (and maybe a held mutex): leak the
// parent's state there and start afresh on first use
void reaper_atfork_child() { g_reaper = nullptr; new (&g_reaper_mu) std::mutex(); }
struct ReaperOwner {
  ReaperOwner() { pthread_atfork(nullptr, nullptr, reaper_atfork_child); }
  ~ReaperOwner() {
    Reaper* rp = nullptr;
    {
      std::lock_guard<std::mutex> lk(g_reaper_mu);
      rp = g_reaper;
      g_reaper = nullptr;
      g_reaper_closed = true;
    }
    delete rp;                     // drains its queue, then joins
  }
} g_reaper_owner;
constexpr size_t kReapInlineFiles = 4096;
constexpr size_t kReapMaxQueued = 4;
}  // namespace

void tsg_result_free(tsg_result* r) {
  if (!r) return;
  size_t weight = r->files.size();
  for (size_t i = 0; i < r->files.size() && weight < kReapInlineFiles; ++i) weight += r->files[i].findings().size();
  if (weight < kReapInlineFiles) { delete r; return; }
  {
    std::lock_guard<std::mutex> lk(g_reaper_mu);
    if (!g_reaper_closed) {
      try {
        if (!g_reaper) {
          std::unique_ptr<Reaper> rp(new Reaper());
          Reaper* raw = rp.get();
          rp->th = std::thread([raw] { raw->loop(); });
          g_reaper = rp.release();
        }
        std::lock_guard<std::mutex> lq(g_reaper->mu);
        // backpressure: an idle-priority reaper that never gets a core (a
        // saturated host) must not let freed results pile up
        g_reaper->q.push_back(r);
        if (g_reaper->q.size() > kReapMaxQueued) {
          r = g_reaper->q.front();
          g_reaper->q.pop_front();
        } else {
          r = nullptr;
        }
      } catch (...) {}             // no reaper (thread or queue allocation failed): r is deleted inline
      if (g_reaper) g_reaper->cv.notify_one();   // under g_reaper_mu: the owner cannot delete the reaper meanwhile
    }
  }
  delete r;                        // the oldest queued result (or r itself), inline and outside the locks
}
void tsg_free(void* p) { free(p); }

static std::string path_of(const char* const* paths, const uint32_t* lens, uint32_t i) {
  return lens ? std::string(paths[i], lens[i]) : std::string(paths[i]);
}

int tsg_scan_host_reference(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                            const char* const* paths, const uint32_t* path_lens, const uint8_t* binary, int threads,
                            tsg_result** out) {
  TSG_API_TRY
  if (!rs || !out || !offsets || (nfiles && (!paths || !data))) return fail(TSG_ERR_INVALID, "NULL argument");
  auto* r = new tsg_result();
  r->rs = rs->rs;
  r->files.resize(nfiles);
  std::atomic<uint32_t> next{0};
  auto worker = [&]() {
    for (;;) {
      uint32_t f = next.fetch_add(1);
      if (f >= nfiles) break;
      r->files[f] = scan_file(*rs->rs, path_of(paths, path_lens, f), data + offsets[f], offsets[f + 1] - offsets[f],
                              binary ? binary[f] != 0 : false, nullptr);
    }
  };
  std::unique_ptr<tsg_result> guard_r(r);      // freed if a worker throws
  run_threads(threads > 0 ? threads : 1, worker);
  guard_r.release();
  *out = r;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_scan_table_model(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                         const char* const* paths, const uint32_t* path_lens, const uint8_t* binary,
                         tsg_result** out) {
  TSG_API_TRY
  if (!rs || !out || !offsets || (nfiles && (!paths || !data))) return fail(TSG_ERR_INVALID, "NULL argument");
  Prefilter pf;
  std::string err;
  if (!build_prefilter(*rs->rs, &pf, &err)) return fail(TSG_ERR_INTERNAL, err);
  auto* r = new tsg_result();
  r->rs = rs->rs;
  r->files.resize(nfiles);
  r->cands.resize(nfiles);
  // per-chunk newline counts over the packed batch, as K1 produces them
  const uint32_t ch = 2048;
  const uint64_t total = nfiles ? offsets[nfiles] : 0;
  std::vector<uint16_t> chunk_nl((total + ch - 1) / ch, 0);   // exactly K1's chunk count
  // TSG_HOST_PROFILE=1: the confirmer's time per phase on stderr (the same
  // scan_file the engine runs, here on one thread, for CPU profiling)
  const bool prof = std::getenv("TSG_HOST_PROFILE") && std::atoi(std::getenv("TSG_HOST_PROFILE")) != 0;
  if (prof) { g_scan_prof_on.store(true, std::memory_order_relaxed); for (auto& a : g_scan_prof) a.store(0); }
  uint64_t conf_ns = 0;
  for (uint64_t x = 0; x < total; ++x) chunk_nl[x / ch] += data[x] == '\n';
  bool any_full = false;
  for (size_t k = 0; k < rs->rs->rules.size(); ++k) any_full |= pf.rules[k].mode == 1;
  for (uint32_t f = 0; f < nfiles; ++f) {
    const uint8_t* c = data + offsets[f];
    const size_t len = offsets[f + 1] - offsets[f];
    std::vector<uint8_t> gate;
    const bool special = prefilter_reference_file(pf, c, len, &r->cands[f], &gate);
    if (special) prefilter_variant_file(pf, c, len, &r->cands[f], &gate);
    if (!special && !any_full && std::all_of(r->cands[f].begin(), r->cands[f].end(),
                                             [](const std::vector<uint64_t>& v) { return v.empty(); })) {
      // as the engine's confirmer: no candidate, no host-evaluated rule -> only
      // the global allow-path outcome (scanner.go:381-386)
      const std::string p = path_of(paths, path_lens, f);
      if (global_allow_path(*rs->rs, p)) r->files[f] = Secret::path_only(p.data(), p.size());
      continue;
    }
    std::vector<std::vector<uint64_t>> tmp = r->cands[f];
    FilePlan plan;
    plan_from_candidates(pf, &tmp, &plan);
    NlSource nls;
    nls.chunk_nl = chunk_nl.data();
    nls.data = data;
    nls.file_off = offsets[f];
    nls.chunk = ch;
    const auto t_conf = std::chrono::steady_clock::now();
    r->files[f] = scan_file(*rs->rs, path_of(paths, path_lens, f), c, len, binary ? binary[f] != 0 : false, &plan, &nls);
    conf_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_conf).count();
  }
  if (prof) {
    std::fprintf(stderr, "[tsg model] confirm %.1f ms: keywords %.1f, find %.1f (whole-file find-alls %.1f ms in %llu "
                 "calls), blocks %.1f, findings %.1f, sort %.1f\n",
                 conf_ns / 1e6, g_scan_prof[0].load() / 1e6, g_scan_prof[1].load() / 1e6, g_scan_prof[5].load() / 1e6,
                 static_cast<unsigned long long>(g_scan_prof[7].load()),
                 g_scan_prof[2].load() / 1e6, g_scan_prof[3].load() / 1e6, g_scan_prof[4].load() / 1e6);
  }
  *out = r;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_prefilter_report(const tsg_ruleset* rs, char** out) {
  TSG_API_TRY
  if (!rs || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  Prefilter pf;
  std::string err;
  if (!build_prefilter(*rs->rs, &pf, &err)) return fail(TSG_ERR_INTERNAL, err);
  char* buf = static_cast<char*>(malloc(pf.report.size() + 1));
  memcpy(buf, pf.report.c_str(), pf.report.size() + 1);
  *out = buf;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_scan_dfa_dump(const tsg_ruleset* rs, uint32_t group, uint16_t** next, uint8_t** byte_class, uint32_t* nstates,
                      uint32_t* nclasses, uint32_t* first_out) {
  TSG_API_TRY
  if (!rs || !next || !byte_class || !nstates || !nclasses || !first_out) return fail(TSG_ERR_INVALID, "NULL argument");
  Prefilter pf;
  std::string err;
  if (!build_prefilter(*rs->rs, &pf, &err)) return fail(TSG_ERR_INTERNAL, err);
  if (group >= pf.groups.size()) return fail(TSG_ERR_INVALID, "no such scan DFA group");
  const ScanDfa& d = pf.groups[group];
  uint16_t* nx = static_cast<uint16_t*>(malloc(std::max<size_t>(d.t.next.size(), 1) * sizeof(uint16_t)));
  uint8_t* bc = static_cast<uint8_t*>(malloc(256));
  if (!nx || !bc) { free(nx); free(bc); return fail(TSG_ERR_INTERNAL, "out of memory"); }
  std::copy(d.t.next.begin(), d.t.next.end(), nx);
  memcpy(bc, d.t.byte_class, 256);
  *next = nx;
  *byte_class = bc;
  *nstates = d.t.nstates;
  *nclasses = d.t.nclasses;
  *first_out = d.first_out_state;
  return TSG_OK;
  TSG_API_CATCH
}

const char* tsg_builtin_rules_json(void) { return tsg_builtin_json_ptr(); }

// GetSecretRulesMetadata (builtin-rules.go:91-99): lo.Map(builtinRules, ...
// iacRules.Check{Name: rule.ID, Description: rule.Title}) as json.Marshal
// writes []iacRules.Check (pkg/iac/rules/providers.go:18-21 json tags).
const char* tsg_secret_rules_metadata_json(void) {
  static const std::string out = [] {
    JValue doc;
    std::string err;
    if (!json_parse(tsg_builtin_json_ptr(), &doc, &err) || !doc.get("rules")) return std::string("null");
    std::string o = "[";
    bool first = true;
    for (const auto& r : doc.get("rules")->arr) {
      if (!first) o += ",";
      first = false;
      o += "{\"name\":";
      go_json_string(&o, r.get("id") ? r.get("id")->as_string() : std::string());
      o += ",\"description\":";
      go_json_string(&o, r.get("title") ? r.get("title")->as_string() : std::string());
      o += "}";
    }
    return o + "]";
  }();
  return out.c_str();
}

int tsg_go_json_string(const uint8_t* s, size_t n, int escape_html, char** out, size_t* len) {
  TSG_API_TRY
  if ((n && !s) || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  std::string o;
  go_json_string(&o, reinterpret_cast<const char*>(s), n, escape_html != 0);
  char* buf = static_cast<char*>(malloc(o.size() + 1));
  if (!buf) return fail(TSG_ERR_INTERNAL, "out of memory");
  memcpy(buf, o.data(), o.size());
  buf[o.size()] = 0;
  *out = buf;
  if (len) *len = o.size();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_regex_match_probe(const char* pattern, const uint8_t* text, size_t len, int* gated, int* plain,
                          int* has_gate) {
  TSG_API_TRY
  if (!pattern || (len && !text) || !gated || !plain || !has_gate) return fail(TSG_ERR_INVALID, "NULL argument");
  std::string err;
  auto rx = re::Regexp::compile(pattern, &err);
  if (!rx) return fail(TSG_ERR_CONFIG, err);
  *plain = rx->match_string(text, len) ? 1 : 0;
  re::LitGate g;
  bool bounded = false;
  uint32_t dmin = 0, dmax = 0;
  *has_gate = 0;
  if (literal_gate(*rx->ast(), &g, &bounded, &dmin, &dmax)) {
    rx->set_gate(std::move(g), bounded, dmin, dmax);
    *has_gate = bounded ? 2 : 1;
  }
  *gated = rx->match_string(text, len) ? 1 : 0;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_regex_probe(const char* pattern, const uint8_t* text, size_t len, const uint64_t* pos, size_t n,
                    int64_t* dfa_end, int64_t* vm_end) {
  TSG_API_TRY
  if (!pattern || (len && !text) || (n && (!pos || !dfa_end || !vm_end))) return fail(TSG_ERR_INVALID, "NULL argument");
  std::string err;
  auto rx = re::Regexp::compile(pattern, &err);
  if (!rx) return fail(TSG_ERR_CONFIG, err);
  std::vector<re::Cap> caps(2 * (rx->num_subexp() + 1));
  for (size_t i = 0; i < n; ++i) {
    if (pos[i] > len) return fail(TSG_ERR_INVALID, "position out of range");
    dfa_end[i] = rx->match_end_dfa(text, len, pos[i]);
    vm_end[i] = rx->match_at(text, len, pos[i], true, 0, caps.data()) ? caps[1] : -1;
    // the product's dispatch (span shape / backtracker / lazy DFA) must agree
    if (rx->match_end(text, len, pos[i]) != vm_end[i]) return fail(TSG_ERR_INTERNAL, "match_end differs from the VM");
  }
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_test_go_sort(const uint32_t* keys, size_t n, uint32_t* order) {
  TSG_API_TRY
  if (n && (!keys || !order)) return fail(TSG_ERR_INVALID, "NULL argument");
  std::vector<uint32_t> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = static_cast<uint32_t>(i);
  GoSort<uint32_t>(&v, [&v, keys](size_t i, size_t j) { return keys[v[i]] < keys[v[j]]; }).run();
  std::copy(v.begin(), v.end(), order);
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_test_readback(uint32_t nwords, uint32_t count, uint32_t per_count, uint32_t* copied) {
  TSG_API_TRY
  if (!copied) return fail(TSG_ERR_INVALID, "NULL argument");
  std::string err;
  if (!tsg::readback_probe(nwords, count, per_count, copied, &err))
    return fail(tsg::device_count() > 0 ? TSG_ERR_HIP : TSG_ERR_NO_DEVICE, err);
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_test_engine_footprint(tsg_engine* e, uint32_t* lanes, uint32_t* calls, uint32_t* pool_threads) {
  TSG_API_TRY
  if (!e || !lanes || !calls || !pool_threads) return fail(TSG_ERR_INVALID, "NULL argument");
  e->eng->footprint(lanes, calls, pool_threads);
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_test_inject_segment_failures(tsg_engine* e, uint32_t n) {
  TSG_API_TRY
  if (!e) return fail(TSG_ERR_INVALID, "engine is NULL");
  e->eng->inject_segment_failures(n);
  return TSG_OK;
  TSG_API_CATCH
}

static std::string cstr(const char* p) { return p ? std::string(p) : std::string(); }

// Test hook: a result holding the types.Secret list given as JSON (Go field
// names), so report assembly can be checked against the reference's own
// types.Secret fixtures (e.g. applier/docker_test.go).
int tsg_result_from_json(const char* json, size_t len, tsg_result** out) {
  TSG_API_TRY
  if (!json || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  JValue doc;
  std::string err;
  if (!json_parse(std::string(json, len), &doc, &err) || doc.kind != JValue::Arr) return fail(TSG_ERR_INVALID, "json: " + err);
  auto* r = new tsg_result();
  r->own_rules = std::make_shared<std::deque<Rule>>();
  auto sget = [](const JValue* o, const char* k) { const JValue* v = o ? o->get(k) : nullptr; return v ? v->as_string() : std::string(); };
  auto iget = [](const JValue* o, const char* k) { const JValue* v = o ? o->get(k) : nullptr; return v && v->kind == JValue::Num ? static_cast<int>(v->num) : 0; };
  auto bget = [](const JValue* o, const char* k) { const JValue* v = o ? o->get(k) : nullptr; return v && v->kind == JValue::Bool && v->b; };
  auto put = [](SecretBuilder* s, const std::string& v) { return s->put(v.data(), v.size()); };
  for (const auto& js : doc.arr) {
    SecretBuilder s;
    s.file_path = sget(&js, "FilePath");
    const JValue* fs = js.get("Findings");
    if (fs && fs->kind == JValue::Arr) {
      for (const auto& jf : fs->arr) {
        Rule rule;
        rule.id = sget(&jf, "RuleID");
        rule.category = sget(&jf, "Category");
        rule.title = sget(&jf, "Title");
        rule.severity = sget(&jf, "Severity");
        r->own_rules->push_back(rule);
        FindingRec f;
        f.rule = &r->own_rules->back();
        f.start_line = iget(&jf, "StartLine");
        f.end_line = iget(&jf, "EndLine");
        f.match = put(&s, sget(&jf, "Match"));
        f.line_begin = static_cast<uint32_t>(s.lines.size());
        const JValue* code = jf.get("Code");
        const JValue* lines = code ? code->get("Lines") : nullptr;
        if (lines && lines->kind == JValue::Arr) {
          for (const auto& jl : lines->arr) {
            LineRec ln;
            ln.number = iget(&jl, "Number");
            ln.content = put(&s, sget(&jl, "Content"));
            ln.is_cause = bget(&jl, "IsCause");
            ln.first_cause = bget(&jl, "FirstCause");
            ln.last_cause = bget(&jl, "LastCause");
            s.lines.push_back(ln);
          }
        }
        f.line_count = static_cast<uint32_t>(s.lines.size()) - f.line_begin;
        s.findings.push_back(f);
      }
    }
    r->files.push_back(Secret::build(s));
  }
  *out = r;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_result_to_proto(const tsg_result* r, size_t file, const tsg_layer* layers, char** out, size_t* len) {
  TSG_API_TRY
  if (!r || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  if (file >= r->files.size()) return fail(TSG_ERR_INVALID, "file index out of range");
  const Secret& s = r->files[file];
  std::vector<LayerRef> refs;
  if (layers) {
    for (size_t k = 0; k < s.findings().size(); ++k)
      refs.push_back(LayerRef{cstr(layers[k].digest), cstr(layers[k].diff_id), cstr(layers[k].created_by)});
  }
  std::string msg, err;
  if (!secret_to_proto(s, layers ? &refs : nullptr, &msg, &err)) return fail(TSG_ERR_INVALID, err);
  char* buf = static_cast<char*>(malloc(msg.size() + 1));
  if (!buf) return fail(TSG_ERR_INTERNAL, "out of memory");
  memcpy(buf, msg.data(), msg.size());
  buf[msg.size()] = 0;
  *out = buf;
  if (len) *len = msg.size();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_result_from_proto(const char* const* msgs, const size_t* lens, size_t n, tsg_result** out) {
  TSG_API_TRY
  if ((n && (!msgs || !lens)) || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  auto r = std::make_unique<tsg_result>();
  r->own_rules = std::make_shared<std::deque<Rule>>();
  r->files.resize(n);
  r->layers.resize(n);
  std::string err;
  for (size_t i = 0; i < n; ++i) {
    if (!msgs[i] && lens[i]) return fail(TSG_ERR_INVALID, "NULL message");
    if (!secret_from_proto(reinterpret_cast<const uint8_t*>(msgs[i]), lens[i], r->own_rules.get(), &r->files[i],
                           &r->layers[i], &err))
      return fail(TSG_ERR_INVALID, err);
  }
  *out = r.release();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_report_json(const tsg_result* const* layers, const tsg_layer* layer_refs, uint32_t nlayers,
                    const tsg_result* image_config, const tsg_report_opts* opts, char** out, size_t* len) {
  TSG_API_TRY
  if ((nlayers && !layers) || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  std::vector<const SecretVec*> ls;
  std::vector<LayerRef> refs;
  for (uint32_t i = 0; i < nlayers; ++i) {
    if (!layers[i]) return fail(TSG_ERR_INVALID, "NULL layer result");
    ls.push_back(&layers[i]->files);
    LayerRef r;
    if (layer_refs) {
      r.digest = cstr(layer_refs[i].digest);
      r.diff_id = cstr(layer_refs[i].diff_id);
      r.created_by = cstr(layer_refs[i].created_by);
    }
    refs.push_back(r);
  }
  const Secret* cfg = image_config && !image_config->files.empty() ? &image_config->files[0] : nullptr;
  ReportOptions o;
  JValue md;
  std::string err;
  if (opts) {
    o.schema_version = opts->schema_version;
    if (opts->created_at) o.created_at = opts->created_at;
    o.artifact_name = cstr(opts->artifact_name);
    o.artifact_type = cstr(opts->artifact_type);
    if (opts->metadata_json) {
      if (!json_parse(opts->metadata_json, &md, &err)) return fail(TSG_ERR_INVALID, "metadata_json: " + err);
      o.metadata = &md;
    }
    o.layers_sorted = opts->layers_sorted != 0;
    if (opts->severities) {
      o.severities.clear();
      std::string cur;
      for (const char* q = opts->severities;; ++q) {
        if (*q == ',' || *q == 0) { if (!cur.empty()) o.severities.push_back(cur); cur.clear(); if (!*q) break; }
        else cur.push_back(*q);
      }
    }
  }
  std::string doc;
  if (!report_json(ls, refs, cfg, o, &doc, &err)) return fail(TSG_ERR_INVALID, err);
  char* buf = static_cast<char*>(malloc(doc.size() + 1));
  if (!buf) return fail(TSG_ERR_INTERNAL, "out of memory");
  memcpy(buf, doc.data(), doc.size());
  buf[doc.size()] = 0;
  *out = buf;
  if (len) *len = doc.size();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_image_config_content(const char* config_json, size_t config_len, char** out, size_t* len) {
  TSG_API_TRY
  if (!config_json || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  std::string doc, err;
  if (!image_config_content(std::string(config_json, config_len), &doc, &err)) return fail(TSG_ERR_INVALID, err);
  char* buf = static_cast<char*>(malloc(doc.size() + 1));
  if (!buf) return fail(TSG_ERR_INTERNAL, "out of memory");
  memcpy(buf, doc.data(), doc.size());
  buf[doc.size()] = 0;
  *out = buf;
  if (len) *len = doc.size();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_guess_base_layers(const char* config_json, size_t config_len, const char* const* diff_ids, uint32_t n,
                          uint8_t* is_base) {
  TSG_API_TRY
  if (!config_json || (n && (!diff_ids || !is_base))) return fail(TSG_ERR_INVALID, "NULL argument");
  std::vector<std::string> ids, base;
  for (uint32_t i = 0; i < n; ++i) ids.push_back(cstr(diff_ids[i]));
  std::string err;
  if (!guess_base_layers(std::string(config_json, config_len), ids, &base, &err)) return fail(TSG_ERR_INVALID, err);
  for (uint32_t i = 0; i < n; ++i) is_base[i] = std::find(base.begin(), base.end(), ids[i]) != base.end();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_go_time_rfc3339(const char* in, char* out, size_t cap) {
  TSG_API_TRY
  std::string t;
  if (!in || !out || !go_time_rfc3339(in, &t) || t.size() + 1 > cap) return fail(TSG_ERR_INVALID, "not an RFC 3339 time");
  memcpy(out, t.c_str(), t.size() + 1);
  return TSG_OK;
  TSG_API_CATCH
}

}  // extern "C"

int tsg_prepare_batch(const tsg_ruleset* rs, const char* config_path, const uint8_t* raw, const uint64_t* raw_offsets,
                      uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, int threads,
                      tsg_prepared** out) {
  TSG_API_TRY
  if (!rs || !out || !raw_offsets || (nfiles && (!raw || !paths))) return fail(TSG_ERR_INVALID, "NULL argument");
  auto* p = new tsg_prepared();
  std::string err;
  const int nt = threads > 0 ? threads : static_cast<int>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
  if (!prepare_batch(*rs->rs, config_path ? config_path : "", raw, raw_offsets, nfiles, paths, path_lens, nt,
                     &p->b, &err)) {
    delete p;
    return fail(TSG_ERR_INVALID, err);
  }
  *out = p;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_prepared_view(const tsg_prepared* p, const uint8_t** data, const uint64_t** offsets, const uint32_t** index,
                      const uint8_t** binary, uint32_t* nkept) {
  TSG_API_TRY
  if (!p || !data || !offsets || !index || !binary || !nkept) return fail(TSG_ERR_INVALID, "NULL argument");
  *data = p->b.data.get();
  *offsets = p->b.offsets.data();
  *index = p->b.index.data();
  *binary = p->b.binary.data();
  *nkept = static_cast<uint32_t>(p->b.index.size());
  return TSG_OK;
  TSG_API_CATCH
}

void tsg_prepared_free(tsg_prepared* p) { delete p; }

namespace {
thread_local double g_pinned_alloc_ms = 0;   // time spent in pinned_alloc on this thread (feed reports)

uint8_t* pinned_alloc(size_t bytes, FeedFree* free_fn) {
  void* p = nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = tsg_alloc_pinned(bytes, &p);
  g_pinned_alloc_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (rc != 0 || !p) return nullptr;
  *free_fn = [](uint8_t* q) { tsg_free_pinned(q); };
  return static_cast<uint8_t*>(p);
}

void json_str_array(std::string* js, const std::vector<std::string>& v) {
  *js += "[";
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) *js += ", ";
    go_json_string(js, v[i], false);
  }
  *js += "]";
}
}  // namespace

int tsg_prepare_layer_tar(const tsg_ruleset* rs, const char* config_path, const uint8_t* tar, size_t len,
                          const char* const* skip_files, uint32_t nskip_files, const char* const* skip_dirs,
                          uint32_t nskip_dirs, int threads, int pinned, tsg_prepared** out) {
  TSG_API_TRY
  tsg_feed_opts o{};
  o.config_path = config_path;
  o.skip_files = skip_files;
  o.n_skip_files = nskip_files;
  o.skip_dirs = skip_dirs;
  o.n_skip_dirs = nskip_dirs;
  o.threads = threads;
  o.pinned = pinned;
  return tsg_prepare_layer_tar_opts(rs, tar, len, &o, out);
  TSG_API_CATCH
}

namespace {
int default_threads(int threads) {
  return threads > 0 ? threads : static_cast<int>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
}

std::vector<std::string> str_list(const char* const* v, uint32_t n) {
  std::vector<std::string> out;
  for (uint32_t i = 0; i < n; ++i) out.emplace_back(v[i]);
  return out;
}

// tsg_feed_opts -> FeedOpts (+ walker skip lists); NULL opts = defaults
bool feed_opts(const tsg_feed_opts* o, FeedOpts* fo, std::vector<std::string>* sf, std::vector<std::string>* sd,
               int* threads, bool* pinned, std::string* err) {
  *threads = default_threads(o ? o->threads : 0);
  *pinned = o && o->pinned;
  if (!o) return true;
  if ((o->n_file_patterns && !o->file_patterns) || (o->n_skip_files && !o->skip_files) ||
      (o->n_skip_dirs && !o->skip_dirs)) {
    *err = "NULL argument";
    return false;
  }
  fo->config_path = o->config_path ? o->config_path : "";
  *sf = str_list(o->skip_files, o->n_skip_files);
  *sd = str_list(o->skip_dirs, o->n_skip_dirs);
  return parse_file_patterns(str_list(o->file_patterns, o->n_file_patterns), fo, err);
}

void set_scan_paths(tsg_prepared* p, const std::vector<std::string>& paths, const char* prefix) {
  for (uint32_t i : p->b.index) p->scan_paths.push_back(prefix + paths[i]);
  for (const auto& sp : p->scan_paths) {
    p->path_ptrs.push_back(sp.c_str());
    p->path_lens.push_back(static_cast<uint32_t>(sp.size()));
  }
}
}  // namespace

int tsg_prepare_batch_opts(const tsg_ruleset* rs, const uint8_t* raw, const uint64_t* raw_offsets, uint32_t nfiles,
                           const char* const* paths, const uint32_t* path_lens, const tsg_feed_opts* opts,
                           tsg_prepared** out) {
  TSG_API_TRY
  if (!rs || !out || !raw_offsets || (nfiles && (!raw || !paths))) return fail(TSG_ERR_INVALID, "NULL argument");
  FeedOpts fo;
  std::vector<std::string> sf, sd;
  int nt;
  bool pinned;
  std::string err;
  if (!feed_opts(opts, &fo, &sf, &sd, &nt, &pinned, &err)) return fail(TSG_ERR_INVALID, err);
  auto* p = new tsg_prepared();
  if (!prepare_batch(*rs->rs, fo, raw, raw_offsets, nfiles, paths, path_lens, nt, &p->b, &err,
                     pinned ? FeedAlloc(pinned_alloc) : FeedAlloc())) {
    delete p;
    return fail(TSG_ERR_INVALID, err);
  }
  *out = p;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_prepare_layer_tar_opts(const tsg_ruleset* rs, const uint8_t* tar, size_t len, const tsg_feed_opts* opts,
                               tsg_prepared** out) {
  TSG_API_TRY
  if (!rs || !out || (len && !tar)) return fail(TSG_ERR_INVALID, "NULL argument");
  FeedOpts fo;
  std::vector<std::string> sf, sd;
  int nt;
  bool pinned;
  std::string err;
  if (!feed_opts(opts, &fo, &sf, &sd, &nt, &pinned, &err)) return fail(TSG_ERR_INVALID, err);
  LayerWalk walk;
  if (!walk_layer_tar(tar, len, sf, sd, &walk, &err)) return fail(TSG_ERR_INVALID, err);
  std::vector<uint64_t> starts, sizes;
  std::vector<std::string> paths;
  for (const TarFile& f : walk.files) {
    starts.push_back(f.offset);
    sizes.push_back(f.size);
    paths.push_back(f.path);
  }
  auto* p = new tsg_prepared();
  if (!prepare_files(*rs->rs, fo, tar, starts.data(), sizes.data(), paths, nt, &p->b, &err,
                     pinned ? FeedAlloc(pinned_alloc) : FeedAlloc())) {
    delete p;
    return fail(TSG_ERR_INVALID, err);
  }
  set_scan_paths(p, paths, "/");
  std::string& js = p->walk_json;
  js = "{\"files\": ";
  json_str_array(&js, paths);
  js += ", \"opq_dirs\": ";
  json_str_array(&js, walk.opq_dirs);
  js += ", \"wh_files\": ";
  json_str_array(&js, walk.wh_files);
  js += ", \"pinned\": ";
  js += p->b.pinned ? "true" : "false";
  js += "}";
  *out = p;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_prepare_fs_tree(const tsg_ruleset* rs, const char* root, const tsg_feed_opts* opts, tsg_prepared** out) {
  TSG_API_TRY
  if (!rs || !out || !root) return fail(TSG_ERR_INVALID, "NULL argument");
  FeedOpts fo;
  std::vector<std::string> sf, sd;
  int nt;
  bool pinned;
  std::string err;
  if (!feed_opts(opts, &fo, &sf, &sd, &nt, &pinned, &err)) return fail(TSG_ERR_INVALID, err);
  const auto t0 = std::chrono::steady_clock::now();
  FsWalk walk;
  std::vector<uint32_t> keep;
  // walk, d.Info() of every walked file, AnalyzeFile's gate (stream.cpp)
  if (!plan_fs_tree(*rs->rs, fo, root, sf, sd, nt, &walk, &keep, &err)) return fail(TSG_ERR_INVALID, err);
  const auto t1 = std::chrono::steady_clock::now();
  std::vector<uint64_t> starts(keep.size(), 0);
  uint64_t total = 0;
  for (size_t k = 0; k < keep.size(); ++k) {
    starts[k] = total;
    total += walk.files[keep[k]].size;
  }
  // the whole tree's kept files at once (tsg_scan_fs_tree streams them in bounded batches)
  std::unique_ptr<uint8_t[]> raw(new uint8_t[std::max<uint64_t>(total, 1)]);
  std::vector<uint64_t> got;
  if (!read_fs_files(walk, keep, starts, raw.get(), nt, &got, &err)) return fail(TSG_ERR_INVALID, err);
  const auto t2 = std::chrono::steady_clock::now();
  std::vector<uint64_t> rstarts, rsizes;
  std::vector<std::string> paths;
  for (size_t k = 0; k < keep.size(); ++k) {
    if (got[k] == UINT64_MAX) continue;
    rstarts.push_back(starts[k]);
    rsizes.push_back(got[k]);
    paths.push_back(walk.files[keep[k]].rel);
  }
  fo.assume_required = true;
  g_pinned_alloc_ms = 0;
  auto* p = new tsg_prepared();
  if (!prepare_files(*rs->rs, fo, raw.get(), rstarts.data(), rsizes.data(), paths, nt, &p->b, &err,
                     pinned ? FeedAlloc(pinned_alloc) : FeedAlloc())) {
    delete p;
    return fail(TSG_ERR_INVALID, err);
  }
  const auto t3 = std::chrono::steady_clock::now();
  set_scan_paths(p, paths, "");                 // fs scans: input.Dir is the root, no "/" prefix (secret.go:131-135)
  std::vector<std::string> all;
  for (const FsFile& f : walk.files) all.push_back(f.rel);
  auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  std::string& js = p->walk_json;
  js = "{\"files\": ";
  json_str_array(&js, all);
  js += ", \"read_bytes\": " + std::to_string(total);
  js += ", \"walk_ms\": " + std::to_string(ms(t0, t1)) + ", \"read_ms\": " + std::to_string(ms(t1, t2)) +
        ", \"prep_ms\": " + std::to_string(ms(t2, t3)) + ", \"alloc_ms\": " + std::to_string(g_pinned_alloc_ms);
  js += ", \"pinned\": ";
  js += p->b.pinned ? "true" : "false";
  js += "}";
  *out = p;
  return TSG_OK;
  TSG_API_CATCH
}

namespace {
// CPU model of the engine's scan stage for one batch (tsg_scan_table_model's
// per-file work): tests of the stream pipelines without a GPU.
bool model_scan_batch(const Ruleset& rs, const Prefilter& pf, const BatchInput& in, SecretVec* res) {
  const uint32_t ch = 2048;
  const uint64_t total = in.nfiles ? in.offsets[in.nfiles] : 0;
  std::vector<uint16_t> chunk_nl((total + ch - 1) / ch, 0);
  for (uint64_t x = 0; x < total; ++x) chunk_nl[x / ch] += in.h_data[x] == '\n';
  res->clear();
  res->resize(in.nfiles);
  for (uint32_t f = 0; f < in.nfiles; ++f) {
    const uint8_t* c = in.h_data + in.offsets[f];
    const size_t len = in.offsets[f + 1] - in.offsets[f];
    std::vector<std::vector<uint64_t>> cand;
    std::vector<uint8_t> gate;
    if (prefilter_reference_file(pf, c, len, &cand, &gate)) prefilter_variant_file(pf, c, len, &cand, &gate);
    FilePlan plan;
    plan_from_candidates(pf, &cand, &plan);
    NlSource nls;
    nls.chunk_nl = chunk_nl.data();
    nls.data = in.h_data;
    nls.file_off = in.offsets[f];
    nls.chunk = ch;
    (*res)[f] = scan_file(rs, path_of(in.paths, in.path_lens, f), c, len, in.binary ? in.binary[f] != 0 : false,
                          &plan, &nls);
  }
  return true;
}

bool stream_opts(const tsg_feed_opts* opts, uint64_t batch_bytes, bool pinned, StreamOpts* so, std::string* err) {
  int nt;
  bool pin_unused;
  if (!feed_opts(opts, &so->feed, &so->skip_files, &so->skip_dirs, &nt, &pin_unused, err)) return false;
  so->threads = nt;
  so->pinned = pinned;
  if (batch_bytes) so->batch_bytes = batch_bytes;
  return true;
}

void build_walk_json(const StreamResult& sr, std::string* out) {
  std::string& js = *out;
  js = "{\"files\": ";
  json_str_array(&js, sr.walked);
  js += ", \"opq_dirs\": ";
  json_str_array(&js, sr.opq_dirs);
  js += ", \"wh_files\": ";
  json_str_array(&js, sr.wh_files);
  const StreamStats& st = sr.st;
  char buf[512];
  std::snprintf(buf, sizeof buf,
                ", \"stats\": {\"wall_ms\": %.3f, \"feed_ms\": %.3f, \"scan_ms\": %.3f, \"wait_ms\": %.3f, "
                "\"walked_bytes\": %llu, \"read_bytes\": %llu, \"scanned_bytes\": %llu, \"batches\": %llu, "
                "\"files\": %llu, \"peak_batch_bytes\": %llu}}",
                st.wall_ms, st.feed_ms, st.scan_ms, st.wait_ms, static_cast<unsigned long long>(st.walked_bytes),
                static_cast<unsigned long long>(st.read_bytes), static_cast<unsigned long long>(st.scanned_bytes),
                static_cast<unsigned long long>(st.batches), static_cast<unsigned long long>(st.files),
                static_cast<unsigned long long>(st.peak_batch_bytes));
  js += buf;
}

tsg_result* stream_result(std::shared_ptr<const Ruleset> rs, StreamResult&& sr) {
  auto* r = new tsg_result();
  r->rs = std::move(rs);
  r->files = std::move(sr.files);
  r->stats.bytes = sr.st.scanned_bytes;
  r->stats.files = sr.st.files;
  r->stats.total_ms = sr.st.wall_ms;
  r->walk.reset(new StreamResult(std::move(sr)));
  return r;
}

BatchScanFn engine_stage(tsg_engine* e) {
  return [e](const BatchInput& in, SecretVec* res, std::string* err) {
    ScanStats st;
    return e->eng->scan(in, res, &st, err);
  };
}

BatchScanFn model_stage(const Ruleset& rs, const Prefilter& pf) {
  return [&rs, &pf](const BatchInput& in, SecretVec* res, std::string*) {
    return model_scan_batch(rs, pf, in, res);
  };
}
}  // namespace

int tsg_scan_layer_stream(tsg_engine* e, tsg_read_fn read, void* user, const tsg_feed_opts* opts,
                          uint64_t batch_bytes, tsg_result** out) {
  TSG_API_TRY
  if (!e || !read || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  StreamOpts so;
  std::string err;
  if (!stream_opts(opts, batch_bytes, true, &so, &err)) return fail(TSG_ERR_INVALID, err);
  StreamResult sr;
  if (!stream_layer(*e->eng->ruleset(), so, read, user, engine_stage(e), &sr, &err)) return fail(TSG_ERR_INVALID, err);
  *out = stream_result(e->eng->ruleset(), std::move(sr));
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_scan_fs_tree(tsg_engine* e, const char* root, const tsg_feed_opts* opts, uint64_t batch_bytes,
                     tsg_result** out) {
  TSG_API_TRY
  if (!e || !root || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  StreamOpts so;
  std::string err;
  if (!stream_opts(opts, batch_bytes, true, &so, &err)) return fail(TSG_ERR_INVALID, err);
  StreamResult sr;
  if (!stream_fs_tree(*e->eng->ruleset(), so, root, engine_stage(e), &sr, &err)) return fail(TSG_ERR_INVALID, err);
  *out = stream_result(e->eng->ruleset(), std::move(sr));
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_scan_layer_stream_model(const tsg_ruleset* rs, tsg_read_fn read, void* user, const tsg_feed_opts* opts,
                                uint64_t batch_bytes, tsg_result** out) {
  TSG_API_TRY
  if (!rs || !read || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  StreamOpts so;
  std::string err;
  if (!stream_opts(opts, batch_bytes, false, &so, &err)) return fail(TSG_ERR_INVALID, err);
  Prefilter pf;
  if (!build_prefilter(*rs->rs, &pf, &err)) return fail(TSG_ERR_INTERNAL, err);
  StreamResult sr;
  if (!stream_layer(*rs->rs, so, read, user, model_stage(*rs->rs, pf), &sr, &err)) return fail(TSG_ERR_INVALID, err);
  *out = stream_result(rs->rs, std::move(sr));
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_scan_fs_tree_model(const tsg_ruleset* rs, const char* root, const tsg_feed_opts* opts, uint64_t batch_bytes,
                           tsg_result** out) {
  TSG_API_TRY
  if (!rs || !root || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  StreamOpts so;
  std::string err;
  if (!stream_opts(opts, batch_bytes, false, &so, &err)) return fail(TSG_ERR_INVALID, err);
  Prefilter pf;
  if (!build_prefilter(*rs->rs, &pf, &err)) return fail(TSG_ERR_INTERNAL, err);
  StreamResult sr;
  if (!stream_fs_tree(*rs->rs, so, root, model_stage(*rs->rs, pf), &sr, &err)) return fail(TSG_ERR_INVALID, err);
  *out = stream_result(rs->rs, std::move(sr));
  return TSG_OK;
  TSG_API_CATCH
}

struct tsg_queue {
  std::unique_ptr<Prefilter> pf;          // (model queues) the CPU model's tables
  std::string fail_path;                  // (model queues) a batch holding this path throws bad_alloc
  std::unique_ptr<ScanQueue> q;
  std::shared_ptr<const Ruleset> rs;
};

int tsg_queue_create(tsg_engine* e, uint32_t max_files, uint64_t max_bytes, uint32_t max_wait_us,
                     uint32_t max_inflight, tsg_queue** out) {
  TSG_API_TRY
  if (!e || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  std::unique_ptr<tsg_queue> q(new tsg_queue());
  q->q.reset(new ScanQueue(engine_stage(e), max_files ? max_files : 4096, max_bytes ? max_bytes : (256ull << 20),
                           max_wait_us, max_inflight ? max_inflight : 8));
  q->rs = e->eng->ruleset();
  *out = q.release();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_queue_create_model(const tsg_ruleset* rs, uint32_t max_files, uint64_t max_bytes, uint32_t max_wait_us,
                           uint32_t max_inflight, const char* fail_path, tsg_queue** out) {
  TSG_API_TRY
  if (!rs || !out) return fail(TSG_ERR_INVALID, "NULL argument");
  std::unique_ptr<tsg_queue> q(new tsg_queue());
  q->pf.reset(new Prefilter());
  std::string err;
  if (!build_prefilter(*rs->rs, q->pf.get(), &err)) return fail(TSG_ERR_INTERNAL, err);
  q->rs = rs->rs;
  q->fail_path = fail_path ? fail_path : "";
  tsg_queue* qp = q.get();
  BatchScanFn model = [qp](const BatchInput& in, SecretVec* res, std::string* e2) {
    if (!qp->fail_path.empty()) {
      for (uint32_t f = 0; f < in.nfiles; ++f)
        if (path_of(in.paths, in.path_lens, f) == qp->fail_path) throw std::bad_alloc();   // injected host failure
    }
    return model_stage(*qp->rs, *qp->pf)(in, res, e2);
  };
  q->q.reset(new ScanQueue(std::move(model), max_files ? max_files : 4096, max_bytes ? max_bytes : (256ull << 20),
                           max_wait_us, max_inflight ? max_inflight : 8));
  *out = q.release();
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_queue_timeouts(tsg_queue* q, uint64_t* timeouts) {
  TSG_API_TRY
  if (!q || !timeouts) return fail(TSG_ERR_INVALID, "NULL argument");
  *timeouts = q->q->stats().timeouts;
  return TSG_OK;
  TSG_API_CATCH
}

void tsg_queue_destroy(tsg_queue* q) { delete q; }

int tsg_queue_scan(tsg_queue* q, const char* path, size_t path_len, const uint8_t* content, size_t len, int binary,
                   tsg_result** out) {
  TSG_API_TRY
  if (!q || !out || (len && !content) || (path_len && !path)) return fail(TSG_ERR_INVALID, "NULL argument");
  Secret sec;
  std::string err;
  if (!q->q->scan(path ? path : "", path_len, content, len, binary != 0, &sec, &err)) return fail(TSG_ERR_HIP, err);
  auto* r = new tsg_result();
  r->rs = q->rs;
  r->files.push_back(std::move(sec));
  *out = r;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_queue_stats(tsg_queue* q, uint64_t* calls, uint64_t* batches, uint64_t* files, uint32_t* max_batch) {
  TSG_API_TRY
  if (!q || !calls || !batches || !files || !max_batch) return fail(TSG_ERR_INVALID, "NULL argument");
  const QueueStats st = q->q->stats();
  *calls = st.calls;
  *batches = st.batches;
  *files = st.files;
  *max_batch = st.max_batch;
  return TSG_OK;
  TSG_API_CATCH
}

int tsg_queue_probe(tsg_queue* q, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                    const char* const* paths, const uint32_t* path_lens, uint32_t callers, double* seconds,
                    uint64_t* findings) {
  TSG_API_TRY
  if (!q || !offsets || !seconds || !findings || (nfiles && (!data || !paths)) || callers == 0)
    return fail(TSG_ERR_INVALID, "NULL argument");
  std::atomic<uint32_t> next{0};
  std::atomic<uint64_t> nf{0};
  std::atomic<bool> bad{false};
  std::string first_err;
  std::mutex emu;
  auto worker = [&]() {
    for (;;) {
      const uint32_t i = next.fetch_add(1);
      if (i >= nfiles || bad.load()) break;
      Secret sec;
      std::string err;
      const size_t pl = path_lens ? path_lens[i] : std::strlen(paths[i]);
      if (!q->q->scan(paths[i], pl, data + offsets[i], offsets[i + 1] - offsets[i], false, &sec, &err)) {
        std::lock_guard<std::mutex> lk(emu);
        if (!bad.exchange(true)) first_err = err;
        break;
      }
      nf += sec.findings().size();
    }
  };
  const auto t0 = std::chrono::steady_clock::now();
  run_threads(static_cast<int>(callers), worker);
  *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *findings = nf.load();
  if (bad) return fail(TSG_ERR_HIP, first_err);
  return TSG_OK;
  TSG_API_CATCH
}

const char* tsg_result_walk_json(const tsg_result* r) {
  if (!r || !r->walk) return nullptr;
  try {
    std::lock_guard<std::mutex> lk(r->walk_mu);
    if (r->walk_json.empty()) build_walk_json(*r->walk, &r->walk_json);
    return r->walk_json.c_str();
  } catch (...) {                                // (bad_alloc) NULL, the reason in tsg_last_error
    fail(TSG_ERR_INTERNAL, "out of memory");
    return nullptr;
  }
}

int tsg_prepared_paths(const tsg_prepared* p, const char* const** paths, const uint32_t** lens) {
  TSG_API_TRY
  if (!p || !paths || !lens) return fail(TSG_ERR_INVALID, "NULL argument");
  if (p->path_ptrs.size() != p->b.index.size()) return fail(TSG_ERR_INVALID, "not a layer-tar or fs-tree batch");
  *paths = p->path_ptrs.data();
  *lens = p->path_lens.data();
  return TSG_OK;
  TSG_API_CATCH
}

const char* tsg_prepared_walk_json(const tsg_prepared* p) { return p ? p->walk_json.c_str() : nullptr; }
