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
// tsg_report_json over the results.
// The two scan paths must give byte-identical JSON (the superset argument of
// DESIGN.md §2).  Usage: asan_driver <dir> where <dir> holds config.json
// (may be empty = builtin rules), data.bin, offsets.bin (uint64 nfiles+1),
// paths.txt (one path per line).
#include <pthread.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "trivy_secret.h"

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
