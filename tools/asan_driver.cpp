// Host-code sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer).
//
// Built by tools/asan_check.py from the host sources (g++ -fsanitize=...)
// linked with the unsanitized HIP objects; runs only CPU entry points of the
// C-ABI (no GPU is touched):
//   tsg_ruleset_compile, tsg_prepare_batch, tsg_scan_host_reference (threaded),
//   tsg_scan_table_model, tsg_result_json, tsg_prefilter_report.
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
  a->rc = run(a->argc, a->argv);
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
