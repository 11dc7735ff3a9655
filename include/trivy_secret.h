/*
 * trivy_secret.h -- C-ABI of the MI355X-native secret-scanning engine
 * (drop-in for mmorel-35/trivy pkg/fanal/secret).
 *
 * Reference interface each entry point replaces (paths relative to the
 * reference repository):
 *
 *   tsg_ruleset_compile     secret.ParseConfig + secret.NewScanner
 *                           pkg/fanal/secret/scanner.go:277-307, 320-364
 *   tsg_ruleset_allow_path  (Global).AllowPath        scanner.go:56-59
 *   tsg_builtin_rules_json  secret.GetBuiltinRules     builtin-rules.go:87-89
 *   tsg_secret_rules_metadata_json
 *                           secret.GetSecretRulesMetadata builtin-rules.go:91-99
 *   tsg_engine_create       (no reference analogue: binds the compiled
 *                           rules to one GPU; the reference's regexes are
 *                           compiled inside ParseConfig/NewScanner)
 *   tsg_scan_batch          N x (*Scanner).Scan(ScanArgs) -> types.Secret
 *                           scanner.go:366-463, batched as proposed in
 *                           SURVEY.md 8(b); ScanArgs{FilePath, Content,
 *                           Binary} = (paths[i], data[off[i]:off[i+1]],
 *                           binary[i])
 *   tsg_result_*            types.Secret / SecretFinding / Code / Line
 *                           pkg/fanal/types/secret.go:5-20, misconf.go:48-61
 *
 * Test, measurement and tooling hooks (CPU models of the GPU passes, probes of
 * single components, fault injection) are declared in trivy_secret_test.h;
 * the same library exports them, and no product entry point calls them.
 *
 * Conventions
 *   - status: 0 = OK, negative = error; tsg_last_error() returns a
 *     thread-local message for the last failing call on this thread.
 *   - strings crossing the boundary are Go byte strings: pointer + length,
 *     not necessarily valid UTF-8, not NUL-terminated unless stated.
 *   - ownership: the caller owns every input buffer until the call returns;
 *     the library owns every tsg_* object until its *_free/_destroy call.
 *   - threading: a tsg_ruleset is immutable and may be shared.  A tsg_engine
 *     may be shared too: concurrent tsg_scan_batch calls each take their own
 *     lane (compute + copy HIP streams and scratch buffers) on every device
 *     and their own host confirm pool, as the reference's Scan is called
 *     concurrently from --parallel goroutines (analyzer.go:434-451).
 *   - there is no CPU fallback: tsg_engine_create fails with
 *     TSG_ERR_NO_DEVICE when no MI355X (HIP device) is visible.
 */
#ifndef TRIVY_SECRET_H_
#define TRIVY_SECRET_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSG_OK 0
#define TSG_ERR_INVALID (-1)
#define TSG_ERR_CONFIG (-2)     /* ParseConfig error: yaml/regexp compile error */
#define TSG_ERR_NO_DEVICE (-3)
#define TSG_ERR_HIP (-4)
#define TSG_ERR_INTERNAL (-5)

typedef struct tsg_ruleset tsg_ruleset;
typedef struct tsg_engine tsg_engine;
typedef struct tsg_result tsg_result;

/* One types.Line (misconf.go:51-60). */
typedef struct tsg_line {
  int64_t number;
  const char* content; size_t content_len;
  int32_t is_cause;
  const char* annotation; size_t annotation_len;
  int32_t truncated;
  const char* highlighted; size_t highlighted_len;
  int32_t first_cause;
  int32_t last_cause;
} tsg_line;

/* One types.SecretFinding (secret.go:10-20); Layer is left to the caller. */
typedef struct tsg_finding {
  const char* rule_id; size_t rule_id_len;
  const char* category; size_t category_len;
  const char* severity; size_t severity_len;
  const char* title; size_t title_len;
  int64_t start_line;
  int64_t end_line;
  const char* match; size_t match_len;
  uint32_t num_lines;
} tsg_finding;

typedef struct tsg_stats {
  double k1_ms, k2_ms, h2d_ms, d2h_ms, host_ms, total_ms;
  uint64_t bytes, files, hits, candidates, confirm_files, findings;
  uint32_t k1_blocks, k1_threads, chunk_bytes;
  int32_t table_in_lds;
  double gpu_wall_ms;   /* device driver threads' busy time (sum over devices) */
  uint32_t pieces;      /* pipeline segments the batch was cut into */
  uint32_t k1_launches; /* K1 launches (segments x scan-DFA groups) */
  uint32_t devices;     /* devices that took part */
  double feed_ms;       /* uploaded batches: wall time until the last segment's upload had landed */
} tsg_stats;

const char* tsg_last_error(void);
const char* tsg_version(void);

/* ParseConfig + NewScanner.  config_json: the trivy-secret.yaml document
 * decoded to JSON with the YAML keys (rules, allow-rules, exclude-block,
 * enable-builtin-rules, disable-rules, disable-allow-rules), or NULL for the
 * builtin rules only (ParseConfig returned nil). */
int tsg_ruleset_compile(const char* config_json, size_t config_len, tsg_ruleset** out);
void tsg_ruleset_free(tsg_ruleset* rs);
int tsg_ruleset_num_rules(const tsg_ruleset* rs);
/* rule id of rule i (NUL-terminated, owned by rs) */
const char* tsg_ruleset_rule_id(const tsg_ruleset* rs, int i);
/* Global.AllowPath(path): 1 allowed, 0 not */
int tsg_ruleset_allow_path(const tsg_ruleset* rs, const char* path, size_t path_len);
/* Compile report of the GPU prefilter (NUL-terminated, owned by the engine). */
const char* tsg_engine_report(const tsg_engine* e);
/* Builtin rule data as JSON (NUL-terminated, static).  GetBuiltinRules,
 * pkg/fanal/secret/builtin-rules.go:87-89. */
const char* tsg_builtin_rules_json(void);
/* GetSecretRulesMetadata (builtin-rules.go:91-99): json.Marshal of the
 * []iacRules.Check{Name: rule ID, Description: rule title} for the builtin
 * rules (NUL-terminated, static). */
const char* tsg_secret_rules_metadata_json(void);

int tsg_device_count(void);
/* device_mask: bit d selects HIP device d (0 = every visible device).  With
 * several devices one tsg_scan_batch call is spread over all of them: the
 * batch is cut into segments (TSG_SEGMENT_BYTES, default 4 GiB, the last one
 * TSG_SEGMENT_TAIL, default 512 MiB) that each
 * device's driver thread pulls from a shared queue. */
int tsg_engine_create(const tsg_ruleset* rs, uint64_t device_mask, tsg_engine** out);
void tsg_engine_destroy(tsg_engine* e);
/* host worker threads for exact confirmation (0 = min(16, hardware)) */
void tsg_engine_set_threads(tsg_engine* e, int threads);

/* Pinned host buffers for the PCIe feed. */
int tsg_alloc_pinned(size_t bytes, void** out);
void tsg_free_pinned(void* p);

/* Scan a batch of nfiles files packed back to back in `data`
 * (offsets[0] = 0, offsets[nfiles] = total bytes).  paths[i] has length
 * path_lens[i] (or is NUL-terminated when path_lens is NULL).  binary may be
 * NULL (all false).  The batch is streamed to HBM in segments (upload of
 * segment k+1 overlapping the kernels of segment k and the host confirmation
 * of segment k-1), scanned by the GPU kernels, and confirmed exactly on the
 * host.  result[i] == Scanner.Scan(args[i]).  `data` should be pinned
 * (tsg_alloc_pinned) for full PCIe rate; pageable memory works, slower. */
int tsg_scan_batch(tsg_engine* e, const uint8_t* data, const uint64_t* offsets, uint32_t nfiles,
                   const char* const* paths, const uint32_t* path_lens, const uint8_t* binary,
                   tsg_result** out);
/* Same, with the batch already resident in HBM at d_data (16-byte aligned,
 * readable for 16 bytes past the end); h_data is the host copy used by the
 * exact confirmer. */
int tsg_scan_batch_resident(tsg_engine* e, const void* d_data, const uint8_t* h_data,
                            const uint64_t* offsets, uint32_t nfiles, const char* const* paths,
                            const uint32_t* path_lens, const uint8_t* binary, tsg_result** out);

/* Host-feed ceiling: stream `bytes` of host memory (pinned for full rate) to
 * HBM through the engine's upload path in segments, with no kernels; *ms =
 * wall time.  Reported beside scan rates, never used by a scan. */
int tsg_feed_probe(tsg_engine* e, const uint8_t* data, uint64_t bytes, double* ms);

/* GPU-side CR strip of a device-resident batch of TEXT files: the analyzer's
 *   content = bytes.ReplaceAll(content, []byte("\r"), []byte(""))
 * (pkg/fanal/analyzer/secret/secret.go:121) for every file at once.  Replaces
 * the host-side strip of tsg_prepare_batch for a feed that uploads files as
 * read.  d_src / d_dst: 16-byte aligned device buffers of >= total bytes on
 * the engine's first device (not overlapping); d_offsets: nfiles + 1 device
 * uint64, nondecreasing, d_offsets[0] = 0, d_offsets[nfiles] = total (checked);
 * d_new_offsets: nfiles + 1 device uint64 receiving each file's start in
 * d_dst.  *out_total = stripped bytes (= d_new_offsets[nfiles]); *ms (may be
 * NULL) = kernel time.  Synchronous.  Binary files (ExtractPrintableBytes)
 * stay on the host path. */
int tsg_strip_cr_device(tsg_engine* e, const void* d_src, const uint64_t* d_offsets, uint32_t nfiles,
                        uint64_t total, void* d_dst, uint64_t* d_new_offsets, uint64_t* out_total, double* ms);

uint32_t tsg_result_num_files(const tsg_result* r);
/* types.Secret.FilePath of file i ("" for types.Secret{}) */
int tsg_result_file_path(const tsg_result* r, uint32_t file, const char** path, size_t* len);
uint32_t tsg_result_num_findings(const tsg_result* r, uint32_t file);
int tsg_result_finding(const tsg_result* r, uint32_t file, uint32_t k, tsg_finding* out);
int tsg_result_line(const tsg_result* r, uint32_t file, uint32_t k, uint32_t line, tsg_line* out);
/* nonzero when the reference would panic on this file (non-participating
 * secret group, scanner.go:155-168 + 465-473) */
int tsg_result_file_error(const tsg_result* r, uint32_t file);
/* Whole result as a JSON array of types.Secret (Go field names); invalid
 * UTF-8 bytes are written as \udcXX escapes.  Free with tsg_free. */
int tsg_result_json(const tsg_result* r, char** json, size_t* len);
int tsg_result_stats(const tsg_result* r, tsg_stats* out);
/* Frees a result; one of >= 4096 files + findings is handed to a background
   thread (its memory returns shortly after the call). */
void tsg_result_free(tsg_result* r);
void tsg_free(void* p);


/* ---- host feed ----
 * Batched SecretAnalyzer.Required + Analyze content preparation, replacing the
 * per-file analyzer calls of pkg/fanal/analyzer/secret/secret.go:103-190
 * (Required: size >= 10, skip dirs/files/exts, the config file itself,
 * global AllowPath; Analyze: utils.IsBinary on the first 300 bytes
 * (utils.go:68-86), binaries other than .pyc dropped, CR stripped from text,
 * ExtractPrintableBytes for .pyc (utils.go:111-143)).  raw/raw_offsets: the
 * files as read; paths: input.FilePath as the analyzer sees it (no "/" prefix
 * for image files: the caller adds it to the scan path, secret.go:133-135).
 * The result packs the kept files back to back (+64 B pad) ready for
 * tsg_scan_batch; index[k] = source file of kept file k. */
typedef struct tsg_prepared tsg_prepared;
int tsg_prepare_batch(const tsg_ruleset* rs, const char* config_path, const uint8_t* raw, const uint64_t* raw_offsets,
                      uint32_t nfiles, const char* const* paths, const uint32_t* path_lens, int threads,
                      tsg_prepared** out);
int tsg_prepared_view(const tsg_prepared* p, const uint8_t** data, const uint64_t** offsets, const uint32_t** index,
                      const uint8_t** binary, uint32_t* nkept);
void tsg_prepared_free(tsg_prepared* p);
/* A container layer: walker.LayerTar.Walk (pkg/fanal/walker/tar.go:35-103)
 * over an uncompressed layer tar in memory -- Go archive/tar's reading of
 * ustar / GNU / PAX headers (long names, PAX path and size), header checksum,
 * TypeRegA normalisation; opaque-directory (".wh..wh..opq") and whiteout
 * (".wh.<name>") entries recorded, not analyzed; skip_files / skip_dirs as
 * walker.Option (utils.CleanSkipPaths + doublestar.Match, utils.go:88-109),
 * files under a skipped directory dropped (underSkippedDir) -- then the same
 * preparation as tsg_prepare_batch for every regular file, with Required
 * seeing the walker's path (no leading '/', analyzer.go:407-408).  pinned != 0
 * packs the kept contents into pinned host memory (tsg_alloc_pinned; heap
 * when no device is present, reported as "pinned": false) so the batch goes
 * to tsg_scan_batch as prepared.  A malformed tar fails with Walk's
 * "failed to extract the archive: ..." error. */
int tsg_prepare_layer_tar(const tsg_ruleset* rs, const char* config_path, const uint8_t* tar, size_t len,
                          const char* const* skip_files, uint32_t nskip_files, const char* const* skip_dirs,
                          uint32_t nskip_dirs, int threads, int pinned, tsg_prepared** out);
/* Analyzer-group options of the secret feed (pkg/fanal/analyzer/analyzer.go
 * AnalyzerOptions / walker.Option):
 *   config_path      SecretAnalyzer.configPath; Required skips its base name;
 *   file_patterns    --file-patterns entries "fileType:regexPattern"
 *                    (analyzer.go:332-350: a malformed entry or regexp fails
 *                    with its error text); "secret:<re>" entries force the
 *                    secret analyzer on matching paths whatever Required says
 *                    (filePatternMatch, analyzer.go:417-419,522-530);
 *   skip_files/dirs  --skip-files / --skip-dirs (walker.Option: doublestar
 *                    patterns; for tsg_prepare_fs_tree made relative to the
 *                    root by BuildSkipPaths, fs.go:99-149);
 *   threads          host threads (0: up to 16); pinned: pack into pinned
 *                    host memory (tsg_alloc_pinned) for tsg_scan_batch. */
typedef struct tsg_feed_opts {
  const char* config_path;
  const char* const* file_patterns;
  uint32_t n_file_patterns;
  const char* const* skip_files;
  uint32_t n_skip_files;
  const char* const* skip_dirs;
  uint32_t n_skip_dirs;
  int32_t threads;
  int32_t pinned;
} tsg_feed_opts;
/* tsg_prepare_batch with feed options (skip lists unused: the files are given). */
int tsg_prepare_batch_opts(const tsg_ruleset* rs, const uint8_t* raw, const uint64_t* raw_offsets, uint32_t nfiles,
                           const char* const* paths, const uint32_t* path_lens, const tsg_feed_opts* opts,
                           tsg_prepared** out);
/* tsg_prepare_layer_tar with feed options. */
int tsg_prepare_layer_tar_opts(const tsg_ruleset* rs, const uint8_t* tar, size_t len, const tsg_feed_opts* opts,
                               tsg_prepared** out);
/* `trivy fs` over a directory tree on disk: walker.FS.Walk (pkg/fanal/walker/
 * fs.go:25-97; filepath.WalkDir order, symlinks not followed, defaultSkipDirs
 * **\/.git proc sys dev, permission errors ignored), AnalyzeFile's gate before
 * a file is opened (analyzer.go:403-419), the kept files read by `threads`
 * readers, then tsg_prepare_batch's preparation.  ScanArgs.FilePath is the
 * walker's path relative to the root (tsg_prepared_paths).  The walk JSON also
 * reports "read_bytes", "walk_ms", "read_ms", "prep_ms". */
int tsg_prepare_fs_tree(const tsg_ruleset* rs, const char* root, const tsg_feed_opts* opts, tsg_prepared** out);
/* The kept files' ScanArgs.FilePath: "/" + the walker's path for a layer tar
 * (image files, secret.go:131-135), the path relative to the root for an fs
 * tree; only for batches made by tsg_prepare_layer_tar* / tsg_prepare_fs_tree. */
int tsg_prepared_paths(const tsg_prepared* p, const char* const** paths, const uint32_t** lens);
/* {"files": [every regular file the walk hands to the analyzers], "opq_dirs":
 * [...], "wh_files": [...], "pinned": bool} (Walk's return values, tar.go:90);
 * owned by p. */
const char* tsg_prepared_walk_json(const tsg_prepared* p);

/* ---- streamed feed -> scan: bounded host memory, the
 * walk / read / prepare of batch k+1 overlapping the scan of batch k.
 * A reader (an io.Reader): > 0 bytes read into buf (at most cap), 0 at the
 * end of the data, < 0 on an error. */
typedef int64_t (*tsg_read_fn)(void* user, uint8_t* buf, size_t cap);
/* One container layer read from `read` in order: walker.LayerTar.Walk over an
 * io.Reader (pkg/fanal/walker/tar.go:35-103) -> AnalyzeFile's gate
 * (analyzer.go:403-419) before a file's content is read -> SecretAnalyzer
 * .Analyze's preparation (secret.go:103-150) -> Scan, the kept files packed
 * into batches of about batch_bytes raw bytes (0: 256 MiB; a larger file is a
 * batch of its own), each scanned on the engine while the next is read.  The
 * result holds every scanned file in walk order, ScanArgs.FilePath = "/" +
 * path; tsg_result_walk_json gives Walk's return values and the feed timing.
 * Layers may be scanned concurrently on one engine (image.go:327's pipeline). */
int tsg_scan_layer_stream(tsg_engine* e, tsg_read_fn read, void* user, const tsg_feed_opts* opts,
                          uint64_t batch_bytes, tsg_result** out);
/* `trivy fs ROOT` streamed: tsg_prepare_fs_tree's walk and gate, the kept files
 * read in walk order in batches of about batch_bytes, each scanned while the
 * next is read.  ScanArgs.FilePath = the path relative to the root. */
int tsg_scan_fs_tree(tsg_engine* e, const char* root, const tsg_feed_opts* opts, uint64_t batch_bytes,
                     tsg_result** out);
/* A streamed result's walk: {"files": [every regular file handed to the
 * analyzers], "opq_dirs": [...], "wh_files": [...], "stats": {wall_ms,
 * feed_ms, scan_ms, wait_ms, walked_bytes, read_bytes, scanned_bytes,
 * batches, files, peak_batch_bytes}}; NULL for other results.  Owned by r. */
const char* tsg_result_walk_json(const tsg_result* r);

/* ---- per-file Scan for unchanged callers ----
 * SecretAnalyzer.Analyze calls Scanner.Scan once per file (pkg/fanal/analyzer/
 * secret/secret.go:137) from --parallel goroutines (analyzer.go:434-451,
 * default 5).  A queue gathers concurrent tsg_queue_scan calls into engine
 * batches: a caller that finds no batch forming leads one, waits until its
 * share of the expected callers has joined -- the recent peak of concurrent
 * callers split over the max_inflight batch slots (default 8), so 5 callers
 * run as 5 concurrent one-file batches and 64 as batches of 8 -- (or
 * max_files / max_bytes is reached, or max_wait_us has passed), scans it,
 * and hands each caller its own result; up to max_inflight batches run at
 * once.  Thread-safe. */
typedef struct tsg_queue tsg_queue;
int tsg_queue_create(tsg_engine* e, uint32_t max_files, uint64_t max_bytes, uint32_t max_wait_us,
                     uint32_t max_inflight, tsg_queue** out);
void tsg_queue_destroy(tsg_queue* q);
/* Scanner.Scan(ScanArgs{path, content, binary}) -> a one-file result */
int tsg_queue_scan(tsg_queue* q, const char* path, size_t path_len, const uint8_t* content, size_t len, int binary,
                   tsg_result** out);
int tsg_queue_stats(tsg_queue* q, uint64_t* calls, uint64_t* batches, uint64_t* files, uint32_t* max_batch);


/* ---- report and image semantics ---- */
typedef struct tsg_layer {          /* ftypes.Layer, pkg/fanal/types/artifact.go:75-79 */
  const char* digest;
  const char* diff_id;
  const char* created_by;
} tsg_layer;

typedef struct tsg_report_opts {
  int64_t schema_version;           /* report.SchemaVersion = 2 (pkg/report/writer.go:24); 0 omits it */
  const char* created_at;           /* CreatedAt, RFC 3339; re-encoded as time.Time marshals */
  const char* artifact_name;        /* ArtifactName; also the Target of image-config secrets */
  const char* artifact_type;        /* artifact.Type: "filesystem", "repository", "container_image", ... */
  const char* metadata_json;        /* types.Metadata as JSON (re-encoded in Go's field order); NULL = zero */
  const char* severities;           /* comma-separated --severity list; NULL = all five */
  int32_t layers_sorted;            /* 1: layers are cached blobs (AnalysisResult.Sort already applied) */
} tsg_report_opts;

/* `trivy -f json` output (pkg/report/json.go:22-50) for the secret results of
 * one artifact.  layers[i] = tsg_scan_batch results of layer i, lowest layer
 * first (an fs scan is one layer, layer_refs may be NULL); per layer
 * AnalysisResult.Sort (analyzer.go:224-235), across layers ApplyLayers'
 * mergeSecrets (applier/docker.go:134-146, 297-316); image_config = the scan
 * of tsg_image_config_content's output (file "config.json"), or NULL, merged
 * as local/scan.go:487-496 does; then secretsToResults (local/scan.go:236-254),
 * the severity part of filterSecrets (result/filter.go:154-169) and
 * json.MarshalIndent(report, "", "  ") + "\n".  Go iterates the merged
 * secrets map in random order; this report lists them by FilePath.  Free
 * *out with tsg_free. */
int tsg_report_json(const tsg_result* const* layers, const tsg_layer* layer_refs, uint32_t nlayers,
                    const tsg_result* image_config, const tsg_report_opts* opts, char** out, size_t* len);
/* The image-config secret analyzer's input (imgconf/secret/secret.go:44):
 * json.MarshalIndent(v1.ConfigFile, "  ", "") of the config decoded from
 * config_json.  Scan it as ScanArgs{FilePath: "config.json"}.  Free with tsg_free. */
int tsg_image_config_content(const char* config_json, size_t config_len, char** out, size_t* len);
/* Base-layer secret skip (artifact/image/image.go:331-335, 526-554;
 * image/image.go:111-137): is_base[i] = 1 when layer diff_ids[i] belongs to
 * the base image, whose layers are analysed without the secret analyzer. */
int tsg_guess_base_layers(const char* config_json, size_t config_len, const char* const* diff_ids, uint32_t n,
                          uint8_t* is_base);

/* ---- client/server wire format ---- */
/* proto.Marshal of the trivy.common.Secret message (rpc/common/service.proto:
 * 152-156, 191-223) that ConvertToRPCSecrets (pkg/rpc/convert.go:146-175)
 * makes of file `file` of the result.  layers: NULL (every finding's Layer is
 * the empty message, as an fs scan) or one tsg_layer per finding.  Fails with
 * TSG_ERR_INVALID where proto.Marshal fails: a string that is not valid UTF-8.
 * Free *out with tsg_free. */
int tsg_result_to_proto(const tsg_result* r, size_t file, const tsg_layer* layers, char** out, size_t* len);
/* proto.Unmarshal of n Secret messages + ConvertFromRPCSecrets
 * (convert.go:504-533): a result with one types.Secret per message; the
 * findings' Layers appear in tsg_result_json as "Layer". */
int tsg_result_from_proto(const char* const* msgs, const size_t* lens, size_t n, tsg_result** out);

#ifdef __cplusplus
}
#endif

#endif /* TRIVY_SECRET_H_ */
