/*
 * trivy_secret_test.h -- test, measurement and tooling hooks of
 * libtrivysecret.so (the product C-ABI is trivy_secret.h).
 *
 * Nothing here has a reference analogue and no product entry point calls any
 * of it: CPU models of the GPU passes (for tests without a GPU), probes that
 * time one component, restated-Go-library probes checked against the
 * oracle, and fault injection for the per-file queue.
 */
#ifndef TRIVY_SECRET_TEST_H_
#define TRIVY_SECRET_TEST_H_

#include "trivy_secret.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Test hook: Go encoding/json string encoding of s (json.Marshal; with
 * escape_html = 0 as an Encoder with SetEscapeHTML(false)).  Free with tsg_free. */
int tsg_go_json_string(const uint8_t* s, size_t n, int escape_html, char** out, size_t* len);

/* Run only the two GPU passes; the result carries stats and candidates but no
 * findings (used to time the kernels in isolation). */
int tsg_prefilter_resident(tsg_engine* e, const void* d_data, const uint8_t* h_data,
                           const uint64_t* offsets, uint32_t nfiles, tsg_result** out);

/* Raw GPU candidates of file i for rule j (sorted starts); for tests. */
int tsg_result_candidates(const tsg_result* r, uint32_t file, uint32_t rule, const uint64_t** starts, size_t* n);

/* Host exact confirmer evaluated on every (file, rule) pair with no GPU
 * prefilter (the reference algorithm restated in C++).  For tests of the
 * confirmer; never used by tsg_scan_batch. */
int tsg_scan_host_reference(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                            uint32_t nfiles, const char* const* paths, const uint32_t* path_lens,
                            const uint8_t* binary, int threads, tsg_result** out);
/* CPU model of the GPU tables (K1+K2 semantics) feeding the confirmer; for
 * tests of the compiled prefilter without a GPU.  Never used by tsg_scan_batch. */
int tsg_scan_table_model(const tsg_ruleset* rs, const uint8_t* data, const uint64_t* offsets,
                         uint32_t nfiles, const char* const* paths, const uint32_t* path_lens,
                         const uint8_t* binary, tsg_result** out);
/* Prefilter compile report without a GPU (NUL-terminated; free with tsg_free). */
int tsg_prefilter_report(const tsg_ruleset* rs, char** out);
/* Tooling (no reference analogue): scan DFA `group` as compiled for K1 --
 * next[state * nclasses + class] (state ids), byte -> class map (256 bytes),
 * states >= first_out have outputs.  Both arrays are freed with tsg_free. */
int tsg_scan_dfa_dump(const tsg_ruleset* rs, uint32_t group, uint16_t** next, uint8_t** byte_class,
                      uint32_t* nstates, uint32_t* nclasses, uint32_t* first_out);
/* Test hook for the host regexp engine: compiles `pattern` (Go syntax) and,
 * for each of the n positions, writes the end of the leftmost-first match
 * anchored there (-1: none) as computed by the lazy DFA (dfa_end) and by
 * match_at's anchored path (vm_end: the bit-state backtracker where Go would
 * use it, else the Pike VM); fails with TSG_ERR_INTERNAL if the scanner's own
 * match_end (span shape / backtracker / lazy DFA) differs from vm_end.  Never
 * used by tsg_scan_batch. */
int tsg_regex_probe(const char* pattern, const uint8_t* text, size_t len, const uint64_t* pos, size_t n,
                    int64_t* dfa_end, int64_t* vm_end);
/* Test hook for the Go sort.Slice restatement (gosort.h, pdqsort_func of
 * go1.23 sort/zsortfunc.go as scanner.go:452-457 uses it): order[] = 0..n-1
 * sorted by keys[order[i]] < keys[order[j]] -- unstable, so ties keep Go's
 * order only if the algorithm is Go's.  Never used by tsg_scan_batch. */
int tsg_test_go_sort(const uint32_t* keys, size_t n, uint32_t* order);
/* Test hook for the engine's readback kernel (tsg_readback, engine.hip) on
 * HIP device 0: copies min(nwords, count * per_count) dwords (the product in
 * 64 bits) of a device buffer filled with 1, 2, ... into host-mapped memory;
 * *copied = the dwords that arrived.  Never used by tsg_scan_batch. */
int tsg_test_readback(uint32_t nwords, uint32_t count, uint32_t per_count, uint32_t* copied);

/* Test hook: the engine's host footprint so far -- lanes (a compute and a
 * copy stream plus device scratch each) created over all its devices, call
 * contexts, and confirm-pool threads started.  Never used by tsg_scan_batch. */
int tsg_test_engine_footprint(tsg_engine* e, uint32_t* lanes, uint32_t* calls, uint32_t* pool_threads);

/* CPU model of the engine's multi-device segment pipeline (pipeline.h:
 * DriverPipeline, the code Engine::scan runs its device drivers on) with
 * simulated devices: `ndevices` drivers, each holding a lane of its device's
 * pool, pull `nsegments` segments (seg_us of "GPU" work each) and hand them to
 * the calling thread, which confirms each (confirm_us).  fail_mode 1: driver
 * fail_device returns an error at its fail_at-th segment (a HIP error); 2: it
 * throws bad_alloc there; 3: the confirming thread throws at its fail_at-th
 * segment; 0: no failure.  Returns TSG_OK, or the failure's code and message;
 * *out tells what ran.  Tests only (tests/test_pipeline_model.py). */
typedef struct {
  uint64_t segments_started, segments_pushed, segments_confirmed, segments_confirmed_twice;
  uint64_t started_after_failure;  /* segments any driver began after the failure */
  uint32_t lanes_outstanding;      /* lanes not back in their pools when the call returned */
  uint32_t lanes_created;          /* most lanes a pool had out at once, summed over devices */
  uint32_t drivers_alive;          /* driver bodies still running when the call returned */
  double wall_ms, fail_to_return_ms;
} tsg_model_pipeline_stats;
int tsg_test_multi_driver_model(uint32_t ndevices, uint32_t nsegments, int32_t fail_device, uint32_t fail_at,
                                uint32_t fail_mode, uint32_t seg_us, uint32_t confirm_us,
                                tsg_model_pipeline_stats* out);

/* Test hook: the engine's next n segment runs fail before their first
 * launch (as a failed device allocation would), so a test can check that a
 * failed call leaves nothing behind on the engine's pooled lanes.  Never used
 * by tsg_scan_batch. */
int tsg_test_inject_segment_failures(tsg_engine* e, uint32_t n);

/* The same two pipelines with the CPU model of the GPU passes as the scan
 * stage (tsg_scan_table_model's); tests only, never the product path. */
int tsg_scan_layer_stream_model(const tsg_ruleset* rs, tsg_read_fn read, void* user, const tsg_feed_opts* opts,
                                uint64_t batch_bytes, tsg_result** out);
int tsg_scan_fs_tree_model(const tsg_ruleset* rs, const char* root, const tsg_feed_opts* opts, uint64_t batch_bytes,
                           tsg_result** out);

/* Measurement hook: `callers` threads, each calling tsg_queue_scan on the
 * next not yet scanned file of the batch until all nfiles are done (the
 * reference's goroutines calling Scan per file); *seconds = wall time,
 * *findings = findings over all files.  Never used by tsg_scan_batch. */
int tsg_queue_probe(tsg_queue* q, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                    const char* const* paths, const uint32_t* path_lens, uint32_t callers, double* seconds,
                    uint64_t* findings);

/* Test hook: Regexp.MatchString(text) for `pattern` with the required-literal
 * gate the ruleset compiler sets on path / allow regexes (*gated) and without
 * it (*plain); *has_gate = 1 if a gate was found (2: bounded). */
int tsg_regex_match_probe(const char* pattern, const uint8_t* text, size_t len, int* gated, int* plain,
                          int* has_gate);

/* Test hook: a result holding the JSON array of types.Secret given (Go field
 * names), to check report assembly against the reference's types.Secret
 * fixtures.  Never used by a scan. */
int tsg_result_from_json(const char* json, size_t len, tsg_result** out);
/* Test hook: time.Time JSON round trip (RFC 3339 in, MarshalJSON's form out). */
int tsg_go_time_rfc3339(const char* in, char* out, size_t cap);

/* The per-file queue (tsg_queue_*) with the CPU model of the GPU passes as its
 * batch stage (tsg_scan_table_model's), for tests without a GPU.  fail_path
 * (may be NULL): a batch holding a file with this path throws std::bad_alloc
 * inside the stage, as an allocation failure inside the engine would; every
 * caller in that batch gets the error, the queue goes on.  Destroy with
 * tsg_queue_destroy. */
int tsg_queue_create_model(const tsg_ruleset* rs, uint32_t max_files, uint64_t max_bytes, uint32_t max_wait_us,
                           uint32_t max_inflight, const char* fail_path, tsg_queue** out);
/* Leaders of the queue that waited the full max_wait_us for callers that did
 * not come. */
int tsg_queue_timeouts(tsg_queue* q, uint64_t* timeouts);

#ifdef __cplusplus
}
#endif

#endif /* TRIVY_SECRET_TEST_H_ */
