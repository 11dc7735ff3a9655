// Host-code sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer).
//
// Built by tools/asan_check.py from the host sources (g++ -fsanitize=...)
// linked with the unsanitized HIP objects; runs only CPU entry points of the
// C-ABI (no GPU is touched):
//   tsg_ruleset_compile, tsg_prepare_batch, tsg_scan_host_reference (threaded),
//   tsg_scan_table_model, tsg_result_json, tsg_prefilter_report;
// with --parsers <dir>: the parsers of untrusted input over fixtures and
// their truncated / mutated copies -- tsg_prepare_layer_tar_opts (tars/),
// tsg_prepare_fs_tree (tree/), tsg_image_config_content and
// tsg_guess_base_layers (configs/), tsg_result_to_proto /
// tsg_result_from_proto round trips with truncations and bit flips, and
// tsg_report_json over the results;
// with --concurrency <case dir> <parsers dir>: the concurrent host code --
// the per-file queue (tsg_queue_create_model: 16 callers through
// tsg_queue_probe, then 8 caller threads with a batch stage that throws,
// then a lone caller), the streamed layer and tree pipelines
// (tsg_scan_layer_stream_model / tsg_scan_fs_tree_model: producer, prepare
// and scan threads, small batches), large results freed from several
// threads at once (the idle-priority reaper) and a table-model result of
// 70k files (threaded SecretVec construction).
// The two scan paths must give byte-identical JSON (the superset argument of
// DESIGN.md §2).  Usage: asan_driver <dir> where <dir> holds config.json
// (may be empty = builtin rules), data.bin, offsets.bin (uint64 nfiles+1),
// paths.txt (one path per line).
#include <pthread.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <atomic>
#include <thread>

#include "trivy_secret.h"
#include "trivy_secret_test.h"

static std::string slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static int fail(const char* what) {
  std::fprintf(stderr, "asan_driver: %s failed: %s\n", what, tsg_last_error());
  return 1;
}

static int run(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: asan_driver <dir>\n");
    return 2;
  }
  const std::string dir = argv[1];
  const std::string cfg = slurp(dir + "/config.json");
  const std::string data = slurp(dir + "/data.bin");
  const std::string offs_raw = slurp(dir + "/offsets.bin");
  std::vector<uint64_t> offs(offs_raw.size() / 8);
  std::memcpy(offs.data(), offs_raw.data(), offs.size() * 8);
  std::vector<std::string> paths;
  {
    std::istringstream in(slurp(dir + "/paths.txt"));
    for (std::string l; std::getline(in, l);) paths.push_back(l);
  }
  const uint32_t n = static_cast<uint32_t>(offs.size() - 1);
  if (paths.size() != n || offs.back() != data.size()) {
    std::fprintf(stderr, "asan_driver: inconsistent inputs\n");
    return 2;
  }
  std::vector<const char*> pp(n);
  std::vector<uint32_t> pl(n);
  for (uint32_t i = 0; i < n; ++i) {
    pp[i] = paths[i].c_str();
    pl[i] = static_cast<uint32_t>(paths[i].size());
  }

  tsg_ruleset* rs = nullptr;
  if (tsg_ruleset_compile(cfg.empty() ? nullptr : cfg.c_str(), cfg.size(), &rs) != 0) return fail("ruleset_compile");
  char* rep = nullptr;
  if (tsg_prefilter_report(rs, &rep) != 0) return fail("prefilter_report");
  tsg_free(rep);

  // analyzer content preparation (Required + CR strip / binary handling)
  tsg_prepared* prep = nullptr;
  if (tsg_prepare_batch(rs, "", reinterpret_cast<const uint8_t*>(data.data()), offs.data(), n, pp.data(), pl.data(), 4,
                        &prep) != 0)
    return fail("prepare_batch");
  const uint8_t* pdata = nullptr;
  const uint64_t* poffs = nullptr;
  const uint32_t* pidx = nullptr;
  const uint8_t* pbin = nullptr;
  uint32_t nkept = 0;
  if (tsg_prepared_view(prep, &pdata, &poffs, &pidx, &pbin, &nkept) != 0) return fail("prepared_view");
  std::vector<const char*> kp(nkept);
  std::vector<uint32_t> kl(nkept);
  for (uint32_t k = 0; k < nkept; ++k) {
    kp[k] = pp[pidx[k]];
    kl[k] = pl[pidx[k]];
  }

  tsg_result* host = nullptr;
  tsg_result* model = nullptr;
  if (tsg_scan_host_reference(rs, pdata, poffs, nkept, kp.data(), kl.data(), pbin, 4, &host) != 0)
    return fail("scan_host_reference");
  if (tsg_scan_table_model(rs, pdata, poffs, nkept, kp.data(), kl.data(), pbin, &model) != 0)
    return fail("scan_table_model");
  char* jh = nullptr;
  char* jm = nullptr;
  size_t lh = 0, lm = 0;
  if (tsg_result_json(host, &jh, &lh) != 0 || tsg_result_json(model, &jm, &lm) != 0) return fail("result_json");
  size_t nfind = 0;
  for (uint32_t k = 0; k < nkept; ++k) nfind += tsg_result_num_findings(host, k);
  const bool same = lh == lm && std::memcmp(jh, jm, lh) == 0;
  std::printf("files %u kept %u findings %zu json %zu bytes host==model %s\n", n, nkept, nfind, lh,
              same ? "yes" : "NO");
  tsg_free(jh);
  tsg_free(jm);
  tsg_result_free(host);
  tsg_result_free(model);
  tsg_prepared_free(prep);
  tsg_ruleset_free(rs);
  return same ? 0 : 3;
}

static std::vector<std::string> list_dir(const std::string& d) {
  std::vector<std::string> out;
  std::istringstream in(slurp(d + "/index.txt"));
  for (std::string l; std::getline(in, l);) if (!l.empty()) out.push_back(d + "/" + l);
  return out;
}

// Parsers of untrusted input: layer tars, image-config JSON,
// client/server protobuf, the fs-tree walk.  Malformed inputs may fail with an
// error; only a sanitizer report (or a crash) fails the run.
static int run_parsers(const std::string& dir) {
  tsg_ruleset* rs = nullptr;
  if (tsg_ruleset_compile(nullptr, 0, &rs) != 0) return fail("ruleset_compile");
  size_t ok = 0, bad = 0;
  // layer tars (walker.LayerTar.Walk + Go archive/tar header parsing)
  const char* skip_files[] = {"**/*.md", "app/src/*.{py,js}"};
  const char* skip_dirs[] = {"node_modules", "usr/**"};
  const char* pats[] = {"secret:go\\.sum$", "secret:^etc/"};
  tsg_feed_opts o{};
  o.skip_files = skip_files;
  o.n_skip_files = 2;
  o.skip_dirs = skip_dirs;
  o.n_skip_dirs = 2;
  o.file_patterns = pats;
  o.n_file_patterns = 2;
  o.threads = 4;
  std::vector<tsg_result*> layer_results;
  for (const std::string& f : list_dir(dir + "/tars")) {
    const std::string tar = slurp(f);
    tsg_prepared* p = nullptr;
    if (tsg_prepare_layer_tar_opts(rs, reinterpret_cast<const uint8_t*>(tar.data()), tar.size(), &o, &p) != 0) {
      ++bad;
      continue;
    }
    ++ok;
    const char* js = tsg_prepared_walk_json(p);
    (void)js;
    const uint8_t* d = nullptr;
    const uint64_t* off = nullptr;
    const uint32_t* idx = nullptr;
    const uint8_t* bin = nullptr;
    uint32_t n = 0;
    const char* const* paths = nullptr;
    const uint32_t* lens = nullptr;
    if (tsg_prepared_view(p, &d, &off, &idx, &bin, &n) == 0 && tsg_prepared_paths(p, &paths, &lens) == 0) {
      tsg_result* r = nullptr;
      if (tsg_scan_host_reference(rs, d, off, n, paths, lens, bin, 2, &r) == 0)
        layer_results.push_back(r);
    }
    tsg_prepared_free(p);
  }
  std::printf("tars: %zu walked, %zu rejected\n", ok, bad);
  // the fs tree
  {
    tsg_prepared* p = nullptr;
    const std::string root = dir + "/tree";
    if (tsg_prepare_fs_tree(rs, root.c_str(), &o, &p) == 0) {
      const uint8_t* d = nullptr;
      const uint64_t* off = nullptr;
      const uint32_t* idx = nullptr;
      const uint8_t* bin = nullptr;
      uint32_t n = 0;
      if (tsg_prepared_view(p, &d, &off, &idx, &bin, &n) != 0) return fail("prepared_view");
      std::printf("fs tree: %u files kept\n", n);
      tsg_prepared_free(p);
    } else {
      std::printf("fs tree: %s\n", tsg_last_error());
    }
  }
  // image configs (json.MarshalIndent restatement, guessBaseLayers)
  ok = bad = 0;
  for (const std::string& f : list_dir(dir + "/configs")) {
    const std::string js = slurp(f);
    char* out = nullptr;
    size_t len = 0;
    if (tsg_image_config_content(js.data(), js.size(), &out, &len) == 0) {
      ++ok;
      tsg_free(out);
    } else {
      ++bad;
    }
    const char* ids[] = {"sha256:a", "sha256:b", "sha256:c"};
    uint8_t base[3] = {0, 0, 0};
    (void)tsg_guess_base_layers(js.data(), js.size(), ids, 3, base);
  }
  std::printf("image configs: %zu decoded, %zu rejected\n", ok, bad);
  // protobuf: every layer result's files -> Secret messages, then truncated
  // and bit-flipped copies through proto.Unmarshal + ConvertFromRPCSecrets
  ok = bad = 0;
  size_t nmsg = 0;
  std::vector<tsg_result*> wire_results;
  uint32_t seed = 12345;
  auto rnd = [&]() { seed = seed * 1103515245u + 12345u; return seed >> 8; };
  for (tsg_result* r : layer_results) {
    for (uint32_t f = 0; f < tsg_result_num_files(r); ++f) {
      char* msg = nullptr;
      size_t len = 0;
      if (tsg_result_to_proto(r, f, nullptr, &msg, &len) != 0) continue;
      const std::string m(msg, len);
      tsg_free(msg);
      std::vector<std::string> vars{m};
      for (int k = 0; k < 8 && !m.empty(); ++k) vars.push_back(m.substr(0, rnd() % m.size()));
      for (int k = 0; k < 16 && !m.empty(); ++k) {
        std::string x = m;
        x[rnd() % x.size()] ^= static_cast<char>(1u << (rnd() % 8));
        vars.push_back(x);
      }
      for (const std::string& v : vars) {
        ++nmsg;
        const char* mp = v.data();
        const size_t ml = v.size();
        tsg_result* back = nullptr;
        if (tsg_result_from_proto(&mp, &ml, 1, &back) == 0) {
          ++ok;
          char* js = nullptr;
          size_t jl = 0;
          if (tsg_result_json(back, &js, &jl) == 0) tsg_free(js);
          wire_results.push_back(back);
        } else {
          ++bad;
        }
      }
    }
  }
  std::printf("proto: %zu messages, %zu decoded, %zu rejected\n", nmsg, ok, bad);
  // reports over the layer results and the decoded wire results
  {
    std::vector<const tsg_result*> ls(layer_results.begin(), layer_results.end());
    std::vector<tsg_layer> refs(ls.size(), tsg_layer{"sha256:d", "sha256:diff", "RUN x > y"});
    tsg_report_opts ro{};
    ro.schema_version = 2;
    ro.created_at = "2024-02-03T04:05:06.5Z";
    ro.artifact_name = "img:latest";
    ro.artifact_type = "container_image";
    ro.severities = "CRITICAL,HIGH";
    char* out = nullptr;
    size_t len = 0;
    if (tsg_report_json(ls.data(), refs.data(), static_cast<uint32_t>(ls.size()), nullptr, &ro, &out, &len) != 0)
      return fail("report_json");
    tsg_free(out);
    for (tsg_result* w : wire_results) {
      const tsg_result* one = w;
      if (tsg_report_json(&one, nullptr, 1, nullptr, &ro, &out, &len) == 0) tsg_free(out);
    }
    std::printf("reports: %zu layers, %zu wire results\n", ls.size(), wire_results.size());
  }
  for (tsg_result* r : layer_results) tsg_result_free(r);
  for (tsg_result* r : wire_results) tsg_result_free(r);
  tsg_ruleset_free(rs);
  return 0;
}

struct MemReader {
  const std::string* buf;
  size_t pos;
  size_t step;
};

static int64_t mem_read(void* user, uint8_t* out, size_t cap) {
  auto* r = static_cast<MemReader*>(user);
  const size_t n = std::min({cap, r->step, r->buf->size() - r->pos});
  std::memcpy(out, r->buf->data() + r->pos, n);
  r->pos += n;
  return static_cast<int64_t>(n);
}

static int run_concurrency(const std::string& dir, const std::string& pdir) {
  const std::string data = slurp(dir + "/data.bin");
  const std::string offs_raw = slurp(dir + "/offsets.bin");
  std::vector<uint64_t> offs(offs_raw.size() / 8);
  std::memcpy(offs.data(), offs_raw.data(), offs.size() * 8);
  std::vector<std::string> paths;
  {
    std::istringstream in(slurp(dir + "/paths.txt"));
    for (std::string l; std::getline(in, l);) paths.push_back(l);
  }
  const uint32_t n = static_cast<uint32_t>(offs.size() - 1);
  std::vector<const char*> pp(n);
  std::vector<uint32_t> pl(n);
  for (uint32_t i = 0; i < n; ++i) {
    pp[i] = paths[i].c_str();
    pl[i] = static_cast<uint32_t>(paths[i].size());
  }
  const uint8_t* d = reinterpret_cast<const uint8_t*>(data.data());
  tsg_ruleset* rs = nullptr;
  if (tsg_ruleset_compile(nullptr, 0, &rs) != 0) return fail("ruleset_compile");
  // 1. the per-file queue: 16 callers sharing batches
  tsg_queue* q = nullptr;
  if (tsg_queue_create_model(rs, 0, 0, 200, 4, nullptr, &q) != 0) return fail("queue_create_model");
  double sec = 0;
  uint64_t nf = 0;
  if (tsg_queue_probe(q, d, offs.data(), n, pp.data(), pl.data(), 16, &sec, &nf) != 0) return fail("queue_probe");
  uint64_t calls = 0, batches = 0, files = 0;
  uint32_t maxb = 0;
  if (tsg_queue_stats(q, &calls, &batches, &files, &maxb) != 0) return fail("queue_stats");
  std::printf("queue: %u files, 16 callers, %llu batches (max %u files), %llu findings\n", n,
              static_cast<unsigned long long>(batches), maxb, static_cast<unsigned long long>(nf));
  tsg_queue_destroy(q);
  // 2. the queue with a batch stage that throws (a file named as fail_path)
  if (tsg_queue_create_model(rs, 0, 0, 200, 2, pp[n / 2], &q) != 0) return fail("queue_create_model");
  std::atomic<uint32_t> next{0}, errs{0};
  auto caller = [&]() {
    for (uint32_t i; (i = next.fetch_add(1)) < std::min<uint32_t>(n, 400);) {
      tsg_result* r = nullptr;
      if (tsg_queue_scan(q, pp[i], pl[i], d + offs[i], offs[i + 1] - offs[i], 0, &r) != 0) ++errs;
      else tsg_result_free(r);
    }
  };
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t) ts.emplace_back(caller);
  for (auto& t : ts) t.join();
  ts.clear();
  tsg_result* lone = nullptr;
  if (tsg_queue_scan(q, pp[0], pl[0], d + offs[0], offs[1] - offs[0], 0, &lone) != 0) return fail("queue_scan after failure");
  tsg_result_free(lone);
  std::printf("queue with an injected failure: %u calls failed, the queue went on\n", errs.load());
  if (errs.load() == 0) { std::fprintf(stderr, "asan_driver: injected failure not seen\n"); return 1; }
  tsg_queue_destroy(q);
  // 3. streamed layer tars and an fs tree through the pipelines (small batches)
  {
    std::istringstream idx(slurp(pdir + "/tars/index.txt"));
    int done = 0;
    for (std::string name; std::getline(idx, name) && done < 4; ++done) {
      const std::string tar = slurp(pdir + "/tars/" + name);
      MemReader mr{&tar, 0, 777};
      tsg_feed_opts o{};
      o.threads = 4;
      tsg_result* r = nullptr;
      if (tsg_scan_layer_stream_model(rs, mem_read, &mr, &o, 4096, &r) == 0) {
        const char* js = tsg_result_walk_json(r);
        if (!js) return fail("walk_json");
        tsg_result_free(r);
      }
    }
    tsg_feed_opts o{};
    o.threads = 4;
    tsg_result* r = nullptr;
    if (tsg_scan_fs_tree_model(rs, (pdir + "/tree").c_str(), &o, 8192, &r) != 0) return fail("scan_fs_tree_model");
    std::printf("fs tree streamed: %u files\n", tsg_result_num_files(r));
    tsg_result_free(r);
  }
  // 4. large results (>= 4096 files) freed from several threads at once: the reaper
  {
    const uint32_t m = 70000;                       // > 65536: SecretVec constructs its slots on threads
    std::vector<uint64_t> o2(m + 1);
    std::string body;
    for (uint32_t i = 0; i < m; ++i) {
      o2[i] = body.size();
      body += (i % 97 == 0) ? "key = AKIAIOSFODNN7EXAMPL" + std::to_string(i % 10) + "\n" : "x = 1\n";
    }
    o2[m] = body.size();
    std::vector<std::string> names(m);
    std::vector<const char*> np(m);
    for (uint32_t i = 0; i < m; ++i) {
      names[i] = "f" + std::to_string(i) + ".txt";
      np[i] = names[i].c_str();
    }
    std::vector<tsg_result*> rs_out(6, nullptr);
    for (auto& r : rs_out)
      if (tsg_scan_table_model(rs, reinterpret_cast<const uint8_t*>(body.data()), o2.data(), m, np.data(), nullptr,
                               nullptr, &r) != 0) return fail("scan_table_model");
    for (auto* r : rs_out) ts.emplace_back([r] { tsg_result_free(r); });
    for (auto& t : ts) t.join();
    std::printf("reaper: 6 results of %u files freed from 6 threads\n", m);
  }
  // 5. the engine's multi-device segment pipeline (pipeline.h) on 8 simulated
  // devices: no failure, a driver's error, a driver's throw, the confirmer's throw
  for (uint32_t mode = 0; mode < 4; ++mode) {
    tsg_model_pipeline_stats ms{};
    const int rc = tsg_test_multi_driver_model(8, 600, mode ? 5 : -1, 4, mode, 200, 100, &ms);
    if ((rc == 0) != (mode == 0)) return fail("multi_driver_model outcome");
    if (ms.lanes_outstanding || ms.drivers_alive || ms.segments_confirmed_twice) return fail("multi_driver_model state");
    if (mode == 0 && ms.segments_confirmed != 600) return fail("multi_driver_model confirmed");
    std::printf("multi-driver model, mode %u: rc %d, %llu started, %llu confirmed, %llu started after the failure, "
                "%.1f ms failure -> return\n", mode, rc, static_cast<unsigned long long>(ms.segments_started),
                static_cast<unsigned long long>(ms.segments_confirmed),
                static_cast<unsigned long long>(ms.started_after_failure), ms.fail_to_return_ms);
  }
  tsg_ruleset_free(rs);
  return 0;
}

// Regexp compile recurses once per nesting level, and simplify turns x{0,N}
// into N nested quests (Go's regexp/syntax does the same; its goroutine
// stacks grow).  ASan's redzones make each frame several times larger than
// at -O3, so the sanitized run gets a 1 GiB stack.
struct Args {
  int argc;
  char** argv;
  int rc;
};

static void* run_thread(void* p) {
  auto* a = static_cast<Args*>(p);
  if (a->argc == 3 && std::string(a->argv[1]) == "--parsers") a->rc = run_parsers(a->argv[2]);
  else if (a->argc == 4 && std::string(a->argv[1]) == "--concurrency") a->rc = run_concurrency(a->argv[2], a->argv[3]);
  else a->rc = run(a->argc, a->argv);
  return nullptr;
}

int main(int argc, char** argv) {
  Args a{argc, argv, 1};
  pthread_attr_t at;
  pthread_attr_init(&at);
  pthread_attr_setstacksize(&at, size_t(1) << 30);
  pthread_t t;
  if (pthread_create(&t, &at, run_thread, &a) != 0) return 2;
  pthread_join(t, nullptr);
  return a.rc;
}
