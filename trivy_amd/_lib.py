"""ctypes binding of libtrivysecret.so (include/trivy_secret.h).

The library is built in-tree by trivy_amd/build.py; importing this module
never builds or JIT-compiles anything and fails loudly when the .so is
missing.
"""
import ctypes
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# TSG_LIB (measurement only): an alternative in-tree build, e.g.
# trivy_amd/libtrivysecret_a.so, to compare two builds on one box
LIB_PATH = os.path.join(_HERE, os.environ.get("TSG_LIB", "libtrivysecret.so"))

c_char_pp = ctypes.POINTER(ctypes.c_char_p)


class TsgModelPipelineStats(ctypes.Structure):
    _fields_ = [("segments_started", ctypes.c_uint64), ("segments_pushed", ctypes.c_uint64),
                ("segments_confirmed", ctypes.c_uint64), ("segments_confirmed_twice", ctypes.c_uint64),
                ("started_after_failure", ctypes.c_uint64), ("lanes_outstanding", ctypes.c_uint32),
                ("lanes_created", ctypes.c_uint32), ("drivers_alive", ctypes.c_uint32),
                ("wall_ms", ctypes.c_double), ("fail_to_return_ms", ctypes.c_double)]


class TsgStats(ctypes.Structure):
    _fields_ = [("k1_ms", ctypes.c_double), ("k2_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double),
                ("d2h_ms", ctypes.c_double), ("host_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("bytes", ctypes.c_uint64), ("files", ctypes.c_uint64), ("hits", ctypes.c_uint64),
                ("candidates", ctypes.c_uint64), ("confirm_files", ctypes.c_uint64), ("findings", ctypes.c_uint64),
                ("k1_blocks", ctypes.c_uint32), ("k1_threads", ctypes.c_uint32), ("chunk_bytes", ctypes.c_uint32),
                ("table_in_lds", ctypes.c_int32), ("gpu_wall_ms", ctypes.c_double),
                ("pieces", ctypes.c_uint32), ("k1_launches", ctypes.c_uint32), ("devices", ctypes.c_uint32),
                ("feed_ms", ctypes.c_double)]


# (name, restype, argtypes) for every entry point declared in include/trivy_secret.h
SIGNATURES = [
    ("tsg_last_error", ctypes.c_char_p, []),
    ("tsg_version", ctypes.c_char_p, []),
    ("tsg_ruleset_compile", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_ruleset_free", None, [ctypes.c_void_p]),
    ("tsg_ruleset_num_rules", ctypes.c_int, [ctypes.c_void_p]),
    ("tsg_ruleset_rule_id", ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_int]),
    ("tsg_ruleset_allow_path", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]),
    ("tsg_engine_report", ctypes.c_char_p, [ctypes.c_void_p]),
    ("tsg_builtin_rules_json", ctypes.c_char_p, []),
    ("tsg_secret_rules_metadata_json", ctypes.c_char_p, []),
    ("tsg_go_json_string", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]),
    ("tsg_device_count", ctypes.c_int, []),
    ("tsg_engine_create", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_engine_destroy", None, [ctypes.c_void_p]),
    ("tsg_engine_set_threads", None, [ctypes.c_void_p, ctypes.c_int]),
    ("tsg_alloc_pinned", ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_free_pinned", None, [ctypes.c_void_p]),
    ("tsg_scan_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                       c_char_pp, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_scan_batch_resident", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_uint32, c_char_pp, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_prefilter_resident", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_feed_probe", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_double)]),
    ("tsg_strip_cr_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)]),
    ("tsg_result_num_files", ctypes.c_uint32, [ctypes.c_void_p]),
    ("tsg_result_file_path", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p),
                                             ctypes.POINTER(ctypes.c_size_t)]),
    ("tsg_result_num_findings", ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_uint32]),
    ("tsg_result_finding", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]),
    ("tsg_result_line", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p]),
    ("tsg_result_file_error", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    ("tsg_result_json", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_size_t)]),
    ("tsg_result_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TsgStats)]),
    ("tsg_result_candidates", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                              ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]),
    ("tsg_result_free", None, [ctypes.c_void_p]),
    ("tsg_free", None, [ctypes.c_void_p]),
    ("tsg_test_go_sort", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    ("tsg_test_readback", ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint32)]),
    ("tsg_test_multi_driver_model", ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32,
                                                    ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                    ctypes.POINTER(TsgModelPipelineStats)]),
    ("tsg_test_engine_footprint", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                                  ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    ("tsg_test_inject_segment_failures", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    ("tsg_scan_host_reference", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                c_char_pp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_scan_table_model", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             c_char_pp, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_prefilter_report", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_scan_dfa_dump", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint16)),
                                         ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    ("tsg_prepare_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_prepared_view", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint32)]),
    ("tsg_prepared_free", None, [ctypes.c_void_p]),
    ("tsg_prepare_layer_tar", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t,
                                             c_char_pp, ctypes.c_uint32, c_char_pp, ctypes.c_uint32, ctypes.c_int,
                                             ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_prepared_paths", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.POINTER(ctypes.c_char_p)),
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32))]),
    ("tsg_prepared_walk_json", ctypes.c_char_p, [ctypes.c_void_p]),
    ("tsg_regex_match_probe", ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                             ctypes.POINTER(ctypes.c_int)]),
    ("tsg_regex_probe", ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
]

class TsgFeedOpts(ctypes.Structure):
    _fields_ = [("config_path", ctypes.c_char_p), ("file_patterns", c_char_pp), ("n_file_patterns", ctypes.c_uint32),
                ("skip_files", c_char_pp), ("n_skip_files", ctypes.c_uint32), ("skip_dirs", c_char_pp),
                ("n_skip_dirs", ctypes.c_uint32), ("threads", ctypes.c_int32), ("pinned", ctypes.c_int32)]


SIGNATURES += [
    ("tsg_prepare_batch_opts", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(TsgFeedOpts),
                                              ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_prepare_layer_tar_opts", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                  ctypes.POINTER(TsgFeedOpts), ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_prepare_fs_tree", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(TsgFeedOpts),
                                           ctypes.POINTER(ctypes.c_void_p)]),
]

# tsg_read_fn: int64_t (*)(void* user, uint8_t* buf, size_t cap)
READ_FN = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)

SIGNATURES += [
    ("tsg_scan_layer_stream", ctypes.c_int, [ctypes.c_void_p, READ_FN, ctypes.c_void_p, ctypes.POINTER(TsgFeedOpts),
                                             ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_scan_fs_tree", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(TsgFeedOpts),
                                        ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_scan_layer_stream_model", ctypes.c_int, [ctypes.c_void_p, READ_FN, ctypes.c_void_p,
                                                   ctypes.POINTER(TsgFeedOpts), ctypes.c_uint64,
                                                   ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_scan_fs_tree_model", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(TsgFeedOpts),
                                              ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_result_walk_json", ctypes.c_char_p, [ctypes.c_void_p]),
    ("tsg_queue_create", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_queue_destroy", None, [ctypes.c_void_p]),
    ("tsg_queue_scan", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_queue_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint32)]),
    ("tsg_queue_probe", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                       c_char_pp, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_uint64)]),
    ("tsg_queue_create_model", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                              ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_queue_timeouts", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
]


def feed_opts(config_path="", file_patterns=(), skip_files=(), skip_dirs=(), threads=0, pinned=False):
    """A TsgFeedOpts plus the objects its pointers refer to (keep both alive)."""
    keep = []

    def arr(v):
        b = [x.encode("utf-8", "surrogateescape") if isinstance(x, str) else x for x in v]
        a = (ctypes.c_char_p * max(1, len(b)))(*b)
        keep.extend([b, a])
        return ctypes.cast(a, c_char_pp), len(b)
    o = TsgFeedOpts()
    o.config_path = (config_path or "").encode("utf-8", "surrogateescape")
    o.file_patterns, o.n_file_patterns = arr(file_patterns)
    o.skip_files, o.n_skip_files = arr(skip_files)
    o.skip_dirs, o.n_skip_dirs = arr(skip_dirs)
    o.threads = threads
    o.pinned = 1 if pinned else 0
    return o, keep


class TsgLayer(ctypes.Structure):
    _fields_ = [("digest", ctypes.c_char_p), ("diff_id", ctypes.c_char_p), ("created_by", ctypes.c_char_p)]


class TsgReportOpts(ctypes.Structure):
    _fields_ = [("schema_version", ctypes.c_int64), ("created_at", ctypes.c_char_p),
                ("artifact_name", ctypes.c_char_p), ("artifact_type", ctypes.c_char_p),
                ("metadata_json", ctypes.c_char_p), ("severities", ctypes.c_char_p),
                ("layers_sorted", ctypes.c_int32)]


SIGNATURES += [
    ("tsg_report_json", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.POINTER(TsgReportOpts), ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_size_t)]),
    ("tsg_image_config_content", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_size_t)]),
    ("tsg_guess_base_layers", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, c_char_pp, ctypes.c_uint32,
                                              ctypes.c_void_p]),
    ("tsg_go_time_rfc3339", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]),
    ("tsg_result_from_json", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("tsg_result_to_proto", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]),
    ("tsg_result_from_proto", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.POINTER(ctypes.c_void_p)]),
]

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libtrivysecret.so is not built (run __graft_entry__.build() or "
                               "python -m trivy_amd.build); there is no fallback")
        # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
        # libamdhip64.so.7, loaded by file name), so load it first and the
        # library's libamdhip64.so.7 dependency binds to that copy.  Loading
        # /opt/rocm's copy first leaves torch a second runtime that finds no
        # device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class TsgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("tsg error %d: %s" % (code, msg))
        self.code = code


def check(rc):
    if rc != 0:
        raise TsgError(rc, lib().tsg_last_error().decode("utf-8", "replace"))


def result_json(res):
    """tsg_result -> list of types.Secret dicts (strings: surrogateescape'd)."""
    L = lib()
    buf = ctypes.c_void_p()
    n = ctypes.c_size_t()
    check(L.tsg_result_json(res, ctypes.byref(buf), ctypes.byref(n)))
    try:
        raw = ctypes.string_at(buf, n.value)
    finally:
        L.tsg_free(buf)
    return json.loads(raw.decode("utf-8"))


def result_stats(res):
    st = TsgStats()
    check(lib().tsg_result_stats(res, ctypes.byref(st)))
    return {k: getattr(st, k) for k, _ in TsgStats._fields_}


def pack_paths(paths):
    enc = [p.encode("utf-8", "surrogateescape") if isinstance(p, str) else bytes(p) for p in paths]
    arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
    lens = (ctypes.c_uint32 * max(len(enc), 1))(*[len(e) for e in enc])
    return arr, lens, enc


def go_json_string(b, escape_html=True):
    """Go encoding/json encoding of the byte string b (test hook)."""
    L = lib()
    buf = ctypes.c_void_p()
    n = ctypes.c_size_t()
    check(L.tsg_go_json_string(b, len(b), 1 if escape_html else 0, ctypes.byref(buf), ctypes.byref(n)))
    try:
        return ctypes.string_at(buf, n.value)
    finally:
        L.tsg_free(buf)
