"""Host-side mirror of github.com/aquasecurity/trivy/pkg/fanal/secret.

Same names, argument meaning and error behaviour as the reference package
(pkg/fanal/secret/scanner.go), backed by the MI355X engine behind the C-ABI in
include/trivy_secret.h:

  ParseConfig(config_path) -> Config | None     scanner.go:277-307
  NewScanner(config)       -> Scanner           scanner.go:320-364
  Scanner.Scan(ScanArgs)   -> types.Secret      scanner.go:377-463
  Scanner.ScanBatch([ScanArgs]) -> [types.Secret]   (batched entry)
  GetBuiltinRules()                             builtin-rules.go:87-89
  GetSecretRulesMetadata()                      builtin-rules.go:91-99

types.Secret is returned as a dict with the Go field names
({"FilePath", "Findings": [{"RuleID", ..., "Code": {"Lines": [...]}, "Match"}]});
Go byte strings are decoded with 'surrogateescape'.  Scan runs on the GPU; a
machine without a HIP device raises instead of silently scanning on the CPU.
"""
import collections.abc
import ctypes
import json
import os
from dataclasses import dataclass

import numpy as np
import yaml

from . import _lib


class ConfigError(Exception):
    """ParseConfig failure (file open, YAML decode, regexp compile)."""


class _GoStringLoader(yaml.SafeLoader):
    """yaml.SafeLoader that keeps every plain scalar a string (yaml.v3 decoding
    into the string fields of secret.Config), except null."""


_GoStringLoader.yaml_implicit_resolvers = {
    k: [(tag, rx) for tag, rx in v if tag == "tag:yaml.org,2002:null"]
    for k, v in yaml.SafeLoader.yaml_implicit_resolvers.items()
}


def load_yaml(path):
    """yaml.v3 Decoder.Decode of the file's FIRST document.  An input with no
    document at all (empty, or only comments) is io.EOF, which ParseConfig
    reports as "secrets config decode error: EOF" (scanner.go:296-298); an
    explicit null document decodes to the zero Config."""
    with open(path, "rb") as f:
        text = f.read()
    docs = yaml.load_all(text, Loader=_GoStringLoader)  # noqa: S506 (SafeLoader subclass)
    try:
        return next(docs)
    except StopIteration:
        raise ConfigError("secrets config decode error: EOF") from None


@dataclass
class ScanArgs:                       # scanner.go:366-370
    FilePath: str
    Content: bytes
    Binary: bool = False


def ParseConfig(config_path):
    """nil for an empty path or a missing file (builtin rules only)."""
    if not config_path:
        return None
    if not os.path.exists(config_path):
        return None
    try:
        doc = load_yaml(config_path)
    except yaml.YAMLError as e:
        raise ConfigError("secrets config decode error: %s" % e)
    if doc is None:                    # explicit null document: zero Config
        doc = {}
    if not isinstance(doc, dict):
        raise ConfigError("secrets config decode error: not a mapping")
    return doc


def GetBuiltinRules():
    return json.loads(_lib.lib().tsg_builtin_rules_json().decode("utf-8"))["rules"]


def GetSecretRulesMetadata():
    """builtin-rules.go:91-99: [{"name": rule ID, "description": rule title}]
    (iacRules.Check's json form) for the builtin rules."""
    return json.loads(_lib.lib().tsg_secret_rules_metadata_json().decode("utf-8"))


def _device_default():
    v = os.environ.get("TSG_DEVICE") or os.environ.get("LOCAL_RANK") or "0"
    return int(v)


class Scanner:
    """NewScanner(config) + Scan.  The ruleset is compiled once; the GPU
    engine is created on first use on `device` (default LOCAL_RANK or 0)."""

    def __init__(self, config=None, device=None, threads=0):
        L = _lib.lib()
        rs = ctypes.c_void_p()
        if config is None:
            _lib.check(L.tsg_ruleset_compile(None, 0, ctypes.byref(rs)))
        else:
            js = json.dumps(config, ensure_ascii=True).encode("utf-8")
            rc = L.tsg_ruleset_compile(js, len(js), ctypes.byref(rs))
            if rc != 0:
                raise ConfigError(L.tsg_last_error().decode("utf-8", "replace"))
        self._rs = rs
        self._engine = None
        self._device = _device_default() if device is None else device
        self._threads = threads

    def __del__(self):
        try:
            L = _lib.lib()
            if self._engine:
                L.tsg_engine_destroy(self._engine)
            if self._rs:
                L.tsg_ruleset_free(self._rs)
        except Exception:
            pass

    @property
    def rule_ids(self):
        L = _lib.lib()
        return [L.tsg_ruleset_rule_id(self._rs, i).decode("utf-8", "surrogateescape")
                for i in range(L.tsg_ruleset_num_rules(self._rs))]

    def AllowPath(self, path):          # scanner.go:56-59
        b = path.encode("utf-8", "surrogateescape")
        return _lib.lib().tsg_ruleset_allow_path(self._rs, b, len(b)) == 1

    def engine(self):
        if self._engine is None:
            L = _lib.lib()
            e = ctypes.c_void_p()
            mask = 0 if self._device == "all" else (1 << int(self._device))
            _lib.check(L.tsg_engine_create(self._rs, mask, ctypes.byref(e)))
            if self._threads:
                L.tsg_engine_set_threads(e, self._threads)
            self._engine = e
        return self._engine

    def report(self):
        return _lib.lib().tsg_engine_report(self.engine()).decode("utf-8", "replace")

    def StripCR(self, d_src, d_offsets, nfiles, total):
        """GPU-side CR strip (tsg_strip_cr_device) of a device-resident batch of
        text files: every file's bytes.ReplaceAll(content, "\r", "")
        (pkg/fanal/analyzer/secret/secret.go:121) in one pass.

        d_src: uint8 device tensor holding >= total bytes (16-byte aligned);
        d_offsets: int64 device tensor of nfiles + 1 file starts (0 ... total).
        Returns (d_dst, d_new_offsets, stripped_total, kernel_ms); d_dst holds
        stripped_total bytes (plus 64 bytes of padding for the resident scan).
        """
        import torch
        dev = d_src.device
        dst = torch.empty(int(total) + 64, dtype=torch.uint8, device=dev)
        new_off = torch.empty(int(nfiles) + 1, dtype=torch.int64, device=dev)
        torch.cuda.current_stream(dev).synchronize()     # the engine runs on its own stream
        out_total, ms = ctypes.c_uint64(), ctypes.c_double()
        _lib.check(_lib.lib().tsg_strip_cr_device(self.engine(), ctypes.c_void_p(d_src.data_ptr()),
                                                   ctypes.c_void_p(d_offsets.data_ptr()), int(nfiles), int(total),
                                                   ctypes.c_void_p(dst.data_ptr()),
                                                   ctypes.c_void_p(new_off.data_ptr()), ctypes.byref(out_total),
                                                   ctypes.byref(ms)))
        return dst, new_off, out_total.value, ms.value

    def Scan(self, args):
        return self.ScanBatch([args])[0]

    def ScanBatchResult(self, args_list):
        """ScanBatch keeping the C result object (trivy_amd.report.ScanResult),
        for report assembly (trivy_amd.report.JSONReport)."""
        from .report import ScanResult
        data, offsets = pack(args_list)
        paths, lens, _keep = _lib.pack_paths([a.FilePath for a in args_list])
        binary = np.array([1 if a.Binary else 0 for a in args_list] or [0], dtype=np.uint8)
        res = ctypes.c_void_p()
        _lib.check(_lib.lib().tsg_scan_batch(self.engine(), data.ctypes.data, offsets.ctypes.data,
                                             len(args_list), paths, lens, binary.ctypes.data,
                                             ctypes.byref(res)))
        return ScanResult(res)

    def ScanBatch(self, args_list, with_stats=False):
        data, offsets = pack(args_list)
        paths, lens, _keep = _lib.pack_paths([a.FilePath for a in args_list])
        binary = np.array([1 if a.Binary else 0 for a in args_list] or [0], dtype=np.uint8)
        res = ctypes.c_void_p()
        _lib.check(_lib.lib().tsg_scan_batch(self.engine(), data.ctypes.data, offsets.ctypes.data,
                                             len(args_list), paths, lens, binary.ctypes.data,
                                             ctypes.byref(res)))
        try:
            out = _lib.result_json(res)
            stats = _lib.result_stats(res)
        finally:
            _lib.lib().tsg_result_free(res)
        for s in out:
            s.pop("Error", None)
        return (out, stats) if with_stats else out


NewScanner = Scanner


def pack(args_list):
    """Pack contents back to back: (uint8 data padded by 64 B, uint64 offsets)."""
    lens = np.fromiter((len(a.Content) for a in args_list), dtype=np.uint64, count=len(args_list))
    offsets = np.zeros(len(args_list) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    data = np.zeros(int(offsets[-1]) + 64, dtype=np.uint8)
    for a, o in zip(args_list, offsets[:-1]):
        if len(a.Content):
            data[int(o):int(o) + len(a.Content)] = np.frombuffer(a.Content, dtype=np.uint8)
    return data, offsets


def PrepareBatch(scanner, files, config_path="", image=False, threads=0, file_patterns=()):
    """Batched SecretAnalyzer.Required + Analyze content prep (tsg_prepare_batch;
    pkg/fanal/analyzer/secret/secret.go:103-190).  files: [(input.FilePath, raw
    bytes)].  Returns (ScanArgs list, source index list) for the kept files;
    image=True adds the "/" prefix image files get (secret.go:133-135).
    file_patterns: --file-patterns entries (tsg_prepare_batch_opts): a
    "secret:<re>" match bypasses Required (analyzer.go:417-419)."""
    L = _lib.lib()
    raw, offsets = pack([ScanArgs(p, c) for p, c in files])
    paths, lens, _keep = _lib.pack_paths([p for p, _ in files])
    h = ctypes.c_void_p()
    if file_patterns:
        o, keep = _lib.feed_opts(config_path, file_patterns, threads=threads)
        rc = L.tsg_prepare_batch_opts(scanner._rs, raw.ctypes.data, offsets.ctypes.data, len(files), paths, lens,
                                      ctypes.byref(o), ctypes.byref(h))
        if rc != 0:
            raise ConfigError(L.tsg_last_error().decode("utf-8", "replace"))
    else:
        _lib.check(L.tsg_prepare_batch(scanner._rs, (config_path or "").encode(), raw.ctypes.data,
                                       offsets.ctypes.data, len(files), paths, lens, threads, ctypes.byref(h)))
    try:
        d, o, ix, b = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        nk = ctypes.c_uint32()
        _lib.check(L.tsg_prepared_view(h, ctypes.byref(d), ctypes.byref(o), ctypes.byref(ix), ctypes.byref(b),
                                       ctypes.byref(nk)))
        n = nk.value
        offs = np.ctypeslib.as_array(ctypes.cast(o, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,)).copy() \
            if n else np.zeros(1, np.uint64)
        idx = np.ctypeslib.as_array(ctypes.cast(ix, ctypes.POINTER(ctypes.c_uint32)), shape=(n,)).tolist() if n else []
        binf = np.ctypeslib.as_array(ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)), shape=(n,)).tolist() if n else []
        data = ctypes.string_at(d, int(offs[-1])) if n else b""
    finally:
        L.tsg_prepared_free(h)
    out = []
    for k, i in enumerate(idx):
        p = files[i][0]
        out.append(ScanArgs("/" + p if image else p, data[int(offs[k]):int(offs[k + 1])], bool(binf[k])))
    return out, idx


class WalkError(Exception):
    """walker.LayerTar.Walk's error ("failed to extract the archive: ...")."""


def PrepareLayerTar(scanner, tar, skip_files=(), skip_dirs=(), config_path="", threads=0, pinned=False,
                    scan=False):
    """One container layer: walker.LayerTar.Walk (pkg/fanal/walker/tar.go:35-103)
    over the uncompressed layer tar `tar` (bytes), then SecretAnalyzer.Required
    + Analyze content prep for every regular file (tsg_prepare_layer_tar).
    Returns (ScanArgs list with "/"-prefixed image paths, walk dict with
    "files", "opq_dirs", "wh_files").  scan=True also runs the prepared batch
    through tsg_scan_batch straight from the prepared (pinned when `pinned`)
    buffer and returns (ScanArgs list, walk dict, [types.Secret]); scan="result"
    returns a report.ScanResult in place of the list."""
    L = _lib.lib()
    buf = np.frombuffer(tar, dtype=np.uint8) if len(tar) else np.zeros(1, np.uint8)
    sf = [s.encode() for s in skip_files]
    sd = [s.encode() for s in skip_dirs]
    sfa = (ctypes.c_char_p * max(1, len(sf)))(*sf)
    sda = (ctypes.c_char_p * max(1, len(sd)))(*sd)
    h = ctypes.c_void_p()
    rc = L.tsg_prepare_layer_tar(scanner._rs, (config_path or "").encode(), buf.ctypes.data, len(tar), sfa, len(sf),
                                 sda, len(sd), threads, 1 if pinned else 0, ctypes.byref(h))
    if rc != 0:
        raise WalkError(L.tsg_last_error().decode("utf-8", "replace"))
    try:
        walk = json.loads(L.tsg_prepared_walk_json(h).decode("utf-8", "surrogateescape"))
        d, o, ix, b = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        nk = ctypes.c_uint32()
        _lib.check(L.tsg_prepared_view(h, ctypes.byref(d), ctypes.byref(o), ctypes.byref(ix), ctypes.byref(b),
                                       ctypes.byref(nk)))
        n = nk.value
        pp, pl = ctypes.POINTER(ctypes.c_char_p)(), ctypes.POINTER(ctypes.c_uint32)()
        _lib.check(L.tsg_prepared_paths(h, ctypes.byref(pp), ctypes.byref(pl)))
        offs = np.ctypeslib.as_array(ctypes.cast(o, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,)).copy() \
            if n else np.zeros(1, np.uint64)
        binf = np.ctypeslib.as_array(ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)), shape=(n,)).tolist() if n else []
        data = ctypes.string_at(d, int(offs[-1])) if n else b""
        out = [ScanArgs(ctypes.string_at(pp[k], pl[k]).decode("utf-8", "surrogateescape"),
                        data[int(offs[k]):int(offs[k + 1])], bool(binf[k])) for k in range(n)]
        if not scan:
            return out, walk
        res = ctypes.c_void_p()
        _lib.check(L.tsg_scan_batch(scanner.engine(), d, o, n, pp, ctypes.cast(pl, ctypes.c_void_p), b, ctypes.byref(res)))
        if scan == "result":                 # the C result object, for report assembly
            from .report import ScanResult
            return out, walk, ScanResult(res)
        try:
            secrets = _lib.result_json(res)
        finally:
            L.tsg_result_free(res)
        return out, walk, secrets
    finally:
        L.tsg_prepared_free(h)


def _prepared_args(L, h, with_paths, paths_in=None):
    """(ScanArgs list, walk dict or None) of a tsg_prepared handle."""
    d, o, ix, b = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    nk = ctypes.c_uint32()
    _lib.check(L.tsg_prepared_view(h, ctypes.byref(d), ctypes.byref(o), ctypes.byref(ix), ctypes.byref(b),
                                   ctypes.byref(nk)))
    n = nk.value
    offs = np.ctypeslib.as_array(ctypes.cast(o, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,)).copy() \
        if n else np.zeros(1, np.uint64)
    binf = np.ctypeslib.as_array(ctypes.cast(b, ctypes.POINTER(ctypes.c_uint8)), shape=(n,)).tolist() if n else []
    index = np.ctypeslib.as_array(ctypes.cast(ix, ctypes.POINTER(ctypes.c_uint32)), shape=(n,)).tolist() if n else []
    data = ctypes.string_at(d, int(offs[-1])) if n else b""
    if with_paths:
        pp, pl = ctypes.POINTER(ctypes.c_char_p)(), ctypes.POINTER(ctypes.c_uint32)()
        _lib.check(L.tsg_prepared_paths(h, ctypes.byref(pp), ctypes.byref(pl)))
        names = [ctypes.string_at(pp[k], pl[k]).decode("utf-8", "surrogateescape") for k in range(n)]
    else:
        names = [paths_in[i] for i in index]
    return [ScanArgs(names[k], data[int(offs[k]):int(offs[k + 1])], bool(binf[k])) for k in range(n)], (d, o, b, n)


def PrepareFsTree(scanner, root, skip_files=(), skip_dirs=(), file_patterns=(), config_path="", threads=0,
                  pinned=False, scan=False):
    """`trivy fs ROOT` feed: walker.FS.Walk + AnalyzeFile's gate + reads + content
    prep (tsg_prepare_fs_tree).  Returns (ScanArgs list, walk dict); scan=True
    also scans the prepared batch through tsg_scan_batch and returns
    (ScanArgs list, walk dict, [types.Secret])."""
    L = _lib.lib()
    o, keep = _lib.feed_opts(config_path, file_patterns, skip_files, skip_dirs, threads, pinned)
    h = ctypes.c_void_p()
    rc = L.tsg_prepare_fs_tree(scanner._rs, os.fsencode(root), ctypes.byref(o), ctypes.byref(h))
    if rc != 0:
        raise WalkError(L.tsg_last_error().decode("utf-8", "replace"))
    try:
        walk = json.loads(L.tsg_prepared_walk_json(h).decode("utf-8", "surrogateescape"))
        args, (d, off, b, n) = _prepared_args(L, h, True)
        if not scan:
            return args, walk
        pp, pl = ctypes.POINTER(ctypes.c_char_p)(), ctypes.POINTER(ctypes.c_uint32)()
        _lib.check(L.tsg_prepared_paths(h, ctypes.byref(pp), ctypes.byref(pl)))
        res = ctypes.c_void_p()
        _lib.check(L.tsg_scan_batch(scanner.engine(), d, off, n, pp, ctypes.cast(pl, ctypes.c_void_p), b,
                                    ctypes.byref(res)))
        try:
            secrets = _lib.result_json(res)
        finally:
            L.tsg_result_free(res)
        return args, walk, secrets
    finally:
        L.tsg_prepared_free(h)


def _reader(fileobj):
    """A tsg_read_fn over a Python binary file object (io.Reader): readinto()
    straight into the engine's buffer where the object has it (one copy),
    else read() + memmove."""
    into = [getattr(fileobj, "readinto", None)]

    def read(_user, buf, cap):
        try:
            if into[0] is not None:
                try:
                    n = into[0](memoryview((ctypes.c_char * cap).from_address(buf)).cast("B"))
                    return n or 0
                except NotImplementedError:    # io.RawIOBase subclasses with read() only
                    into[0] = None
            b = fileobj.read(cap)
        except Exception:                      # noqa: BLE001 -- a reader error ends the walk
            return -1
        if not b:
            return 0
        ctypes.memmove(buf, b, len(b))
        return len(b)
    return _lib.READ_FN(read)


class _Walk(collections.abc.Mapping):
    """Walk's outcome ("files", "opq_dirs", "wh_files", "stats"), decoded from
    the engine's JSON on first use (a layer's walked-path list runs to
    megabytes; most callers only want the findings)."""

    def __init__(self, raw):
        self._raw, self._d = raw, None

    def _get(self):
        if self._d is None:
            self._d = json.loads(self._raw.decode("utf-8", "surrogateescape")) if self._raw else {}
            self._raw = None
        return self._d

    def __getitem__(self, k):
        return self._get()[k]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(self._get())


def _stream_result(L, rc, res, as_result):
    if rc != 0:
        raise WalkError(L.tsg_last_error().decode("utf-8", "replace"))
    walk = _Walk(L.tsg_result_walk_json(res))
    if as_result:
        from .report import ScanResult
        return ScanResult(res), walk
    try:
        secrets = _lib.result_json(res)
    finally:
        L.tsg_result_free(res)
    for sec in secrets:
        sec.pop("Error", None)
    return secrets, walk


def ScanLayerStream(scanner, fileobj, skip_files=(), skip_dirs=(), file_patterns=(), config_path="", threads=0,
                    batch_bytes=0, as_result=False, model=False):
    """One container layer read from a binary file object in order (an
    io.Reader): walker.LayerTar.Walk -> AnalyzeFile's gate -> Analyze's prep ->
    Scan, in bounded batches scanned while the next one is read
    (tsg_scan_layer_stream).  Returns ([types.Secret] of every scanned file in
    walk order, walk dict with "files", "opq_dirs", "wh_files", "stats");
    as_result=True gives a report.ScanResult in place of the list.
    model=True runs the CPU model of the GPU passes (tests)."""
    L = _lib.lib()
    o, keep = _lib.feed_opts(config_path, file_patterns, skip_files, skip_dirs, threads)
    cb = _reader(fileobj)
    res = ctypes.c_void_p()
    if model:
        rc = L.tsg_scan_layer_stream_model(scanner._rs, cb, None, ctypes.byref(o), batch_bytes, ctypes.byref(res))
    else:
        rc = L.tsg_scan_layer_stream(scanner.engine(), cb, None, ctypes.byref(o), batch_bytes, ctypes.byref(res))
    return _stream_result(L, rc, res, as_result)


def ScanFsTree(scanner, root, skip_files=(), skip_dirs=(), file_patterns=(), config_path="", threads=0,
               batch_bytes=0, as_result=False, model=False):
    """`trivy fs ROOT` streamed (tsg_scan_fs_tree): the walk and gate of
    PrepareFsTree, the kept files read in walk order in bounded batches, each
    scanned while the next is read.  Returns ([types.Secret], walk dict)."""
    L = _lib.lib()
    o, keep = _lib.feed_opts(config_path, file_patterns, skip_files, skip_dirs, threads)
    res = ctypes.c_void_p()
    if model:
        rc = L.tsg_scan_fs_tree_model(scanner._rs, os.fsencode(root), ctypes.byref(o), batch_bytes, ctypes.byref(res))
    else:
        rc = L.tsg_scan_fs_tree(scanner.engine(), os.fsencode(root), ctypes.byref(o), batch_bytes, ctypes.byref(res))
    return _stream_result(L, rc, res, as_result)


# ScanQueue::kPeakHold (queue.h): a peak of concurrent callers not seen
# again for this long is over
QUEUE_PEAK_HOLD_S = 0.010


class ScanQueue:
    """Per-file Scanner.Scan for unchanged callers (tsg_queue_*): concurrent
    Scan calls (SecretAnalyzer.Analyze, secret.go:137, from --parallel
    goroutines) share one engine batch."""

    def __init__(self, scanner, max_files=0, max_bytes=0, max_wait_us=200, max_inflight=0, model=False,
                 fail_path=None):
        """model=True (tests only): the CPU model of the GPU passes as the
        batch stage (tsg_queue_create_model), no GPU needed; a batch holding
        `fail_path` then fails with an injected bad_alloc."""
        self._sc = scanner
        self._q = ctypes.c_void_p()
        if model:
            fp = fail_path.encode("utf-8", "surrogateescape") if fail_path else None
            _lib.check(_lib.lib().tsg_queue_create_model(scanner._rs, max_files, max_bytes, max_wait_us,
                                                         max_inflight, fp, ctypes.byref(self._q)))
        else:
            _lib.check(_lib.lib().tsg_queue_create(scanner.engine(), max_files, max_bytes, max_wait_us,
                                                   max_inflight, ctypes.byref(self._q)))

    def Scan(self, args):
        L = _lib.lib()
        p = args.FilePath.encode("utf-8", "surrogateescape")
        c = args.Content
        buf = (ctypes.c_char * max(1, len(c))).from_buffer_copy(c) if c else None
        res = ctypes.c_void_p()
        _lib.check(L.tsg_queue_scan(self._q, p, len(p), buf, len(c), 1 if args.Binary else 0, ctypes.byref(res)))
        try:
            out = _lib.result_json(res)[0]
        finally:
            L.tsg_result_free(res)
        out.pop("Error", None)
        return out

    def stats(self):
        v = [ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()]
        _lib.check(_lib.lib().tsg_queue_stats(self._q, *[ctypes.byref(x) for x in v]))
        t = ctypes.c_uint64()
        _lib.check(_lib.lib().tsg_queue_timeouts(self._q, ctypes.byref(t)))
        return {"calls": v[0].value, "batches": v[1].value, "files": v[2].value, "max_batch": v[3].value,
                "timeouts": t.value}

    def probe(self, args_list, callers):
        """callers threads scanning args_list file by file through the queue
        (tsg_queue_probe); returns (seconds, findings)."""
        data, offsets = pack(args_list)
        paths, lens, _keep = _lib.pack_paths([a.FilePath for a in args_list])
        sec, nf = ctypes.c_double(), ctypes.c_uint64()
        _lib.check(_lib.lib().tsg_queue_probe(self._q, data.ctypes.data, offsets.ctypes.data, len(args_list), paths,
                                              lens, callers, ctypes.byref(sec), ctypes.byref(nf)))
        return sec.value, nf.value

    def close(self):
        if self._q:
            _lib.lib().tsg_queue_destroy(self._q)
            self._q = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- test hooks
def scan_host_reference(scanner, args_list, threads=1):
    """The C++ confirmer on every (file, rule) pair, no prefilter (tests only)."""
    data, offsets = pack(args_list)
    paths, lens, _keep = _lib.pack_paths([a.FilePath for a in args_list])
    binary = np.array([1 if a.Binary else 0 for a in args_list] or [0], dtype=np.uint8)
    res = ctypes.c_void_p()
    _lib.check(_lib.lib().tsg_scan_host_reference(scanner._rs, data.ctypes.data, offsets.ctypes.data,
                                                  len(args_list), paths, lens, binary.ctypes.data, threads,
                                                  ctypes.byref(res)))
    try:
        out = _lib.result_json(res)
    finally:
        _lib.lib().tsg_result_free(res)
    for s in out:
        s.pop("Error", None)
    return out


def scan_host_reference_result(scanner, args_list, threads=1):
    """scan_host_reference keeping the C result object (tests only)."""
    from .report import ScanResult
    data, offsets = pack(args_list)
    paths, lens, _keep = _lib.pack_paths([a.FilePath for a in args_list])
    binary = np.array([1 if a.Binary else 0 for a in args_list] or [0], dtype=np.uint8)
    res = ctypes.c_void_p()
    _lib.check(_lib.lib().tsg_scan_host_reference(scanner._rs, data.ctypes.data, offsets.ctypes.data,
                                                  len(args_list), paths, lens, binary.ctypes.data, threads,
                                                  ctypes.byref(res)))
    return ScanResult(res)


def scan_table_model(scanner, args_list):
    """CPU model of the compiled GPU tables feeding the confirmer (tests only)."""
    data, offsets = pack(args_list)
    paths, lens, _keep = _lib.pack_paths([a.FilePath for a in args_list])
    binary = np.array([1 if a.Binary else 0 for a in args_list] or [0], dtype=np.uint8)
    res = ctypes.c_void_p()
    _lib.check(_lib.lib().tsg_scan_table_model(scanner._rs, data.ctypes.data, offsets.ctypes.data,
                                               len(args_list), paths, lens, binary.ctypes.data,
                                               ctypes.byref(res)))
    try:
        out = _lib.result_json(res)
    finally:
        _lib.lib().tsg_result_free(res)
    for s in out:
        s.pop("Error", None)
    return out


def prefilter_report(scanner):
    buf = ctypes.c_void_p()
    _lib.check(_lib.lib().tsg_prefilter_report(scanner._rs, ctypes.byref(buf)))
    try:
        return ctypes.string_at(buf).decode("utf-8", "replace")
    finally:
        _lib.lib().tsg_free(buf)
