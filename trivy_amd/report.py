"""Host-side mirror of what Trivy does with secret scan results after
Scanner.Scan, backed by the C-ABI (include/trivy_secret.h, csrc/report.cpp):

  JSONReport(...)        pkg/report/json.go:22-50 over the secrets of
                         pkg/scanner/local/scan.go:236-254 (secretsToResults),
                         pkg/fanal/applier/docker.go:134-146,297-316
                         (mergeSecrets across layers), analyzer.go:224-235
                         (AnalysisResult.Sort), result/filter.go:154-169
  ImageConfigContent()   pkg/fanal/analyzer/imgconf/secret/secret.go:39-62
  GuessBaseLayers()      pkg/fanal/artifact/image/image.go:331-335,526-554

A ScanResult owns one tsg_result (from Scanner.ScanBatchResult); reports are
built from those handles, so the report bytes come from the same C++ result
objects the scan produced.
"""
import ctypes
import json

from . import _lib


class ScanResult:
    """One tsg_result (types.Secret per file of a batch)."""

    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self):
        return self._h

    def secrets(self):
        out = _lib.result_json(self._h)
        for s in out:
            s.pop("Error", None)
        return out

    def stats(self):
        return _lib.result_stats(self._h)

    def __del__(self):
        try:
            if self._h:
                _lib.lib().tsg_result_free(self._h)
                self._h = None
        except Exception:
            pass

    def to_proto(self, file=0, layers=None):
        """proto.Marshal of the trivy.common.Secret message of file `file`
        (pkg/rpc/convert.go:146-175); layers: one {"Digest", "DiffID",
        "CreatedBy"} per finding, or None."""
        L = _lib.lib()
        refs = None
        keep = []
        if layers is not None:
            refs = (_lib.TsgLayer * max(len(layers), 1))()
            for i, r in enumerate(layers):
                vals = [_b(r.get(k, "")) for k in ("Digest", "DiffID", "CreatedBy")]
                keep.extend(vals)
                refs[i].digest, refs[i].diff_id, refs[i].created_by = vals
        buf = ctypes.c_void_p()
        ln = ctypes.c_size_t()
        _lib.check(L.tsg_result_to_proto(self._h, file, refs, ctypes.byref(buf), ctypes.byref(ln)))
        try:
            return ctypes.string_at(buf, ln.value)
        finally:
            L.tsg_free(buf)

    @classmethod
    def from_proto(cls, messages):
        """proto.Unmarshal + ConvertFromRPCSecrets (convert.go:526-533) of
        Secret messages, one types.Secret per message."""
        n = len(messages)
        bufs = [ctypes.create_string_buffer(bytes(m), max(len(m), 1)) for m in messages]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(b) for b in bufs])
        lens = (ctypes.c_size_t * max(n, 1))(*[len(m) for m in messages])
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().tsg_result_from_proto(ptrs, lens, n, ctypes.byref(h)))
        return cls(h)

    @classmethod
    def from_secrets(cls, secrets):
        """Test hook: a result holding the given types.Secret dicts."""
        js = json.dumps(secrets).encode("utf-8")
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().tsg_result_from_json(js, len(js), ctypes.byref(h)))
        return cls(h)


def _b(s):
    if s is None:
        return None
    return s if isinstance(s, bytes) else s.encode("utf-8", "surrogateescape")


def JSONReport(layers, layer_refs=None, image_config=None, artifact_name="", artifact_type="",
               created_at="0001-01-01T00:00:00Z", metadata=None, severities=None, schema_version=2,
               layers_sorted=False):
    """`trivy -f json` bytes for the secret results of one artifact.

    layers: [ScanResult] in layer order (an fs scan: one); layer_refs:
    [{"Digest", "DiffID", "CreatedBy"}] per layer or None; image_config: the
    ScanResult of ImageConfigContent scanned as "config.json", or None;
    metadata: types.Metadata as a dict (None = the zero Metadata);
    layers_sorted: the layers are cached blobs already through
    AnalysisResult.Sort (ApplyLayers' input as is)."""
    L = _lib.lib()
    n = len(layers)
    arr = (ctypes.c_void_p * max(n, 1))(*[x.handle for x in layers])
    refs = None
    keep = []
    if layer_refs is not None:
        refs = (_lib.TsgLayer * max(n, 1))()
        for i, r in enumerate(layer_refs):
            vals = [_b(r.get(k, "")) for k in ("Digest", "DiffID", "CreatedBy")]
            keep.extend(vals)
            refs[i].digest, refs[i].diff_id, refs[i].created_by = vals
    opts = _lib.TsgReportOpts()
    opts.schema_version = schema_version
    opts.created_at = _b(created_at)
    opts.artifact_name = _b(artifact_name)
    opts.artifact_type = _b(artifact_type)
    opts.metadata_json = _b(json.dumps(metadata)) if metadata is not None else None
    opts.severities = _b(",".join(severities)) if severities is not None else None
    opts.layers_sorted = 1 if layers_sorted else 0
    buf = ctypes.c_void_p()
    ln = ctypes.c_size_t()
    _lib.check(L.tsg_report_json(arr, refs, n, image_config.handle if image_config else None, ctypes.byref(opts),
                                 ctypes.byref(buf), ctypes.byref(ln)))
    try:
        return ctypes.string_at(buf, ln.value)
    finally:
        L.tsg_free(buf)


def ImageConfigContent(config_json):
    """json.MarshalIndent(v1.ConfigFile, "  ", "") of the decoded image config."""
    L = _lib.lib()
    b = _b(config_json)
    buf = ctypes.c_void_p()
    ln = ctypes.c_size_t()
    _lib.check(L.tsg_image_config_content(b, len(b), ctypes.byref(buf), ctypes.byref(ln)))
    try:
        return ctypes.string_at(buf, ln.value)
    finally:
        L.tsg_free(buf)


def GuessBaseLayers(config_json, diff_ids):
    """Diff IDs of the base-image layers (their secrets are not scanned)."""
    L = _lib.lib()
    b = _b(config_json)
    ids, _lens, _keep = _lib.pack_paths(diff_ids)
    flags = (ctypes.c_uint8 * max(len(diff_ids), 1))()
    _lib.check(L.tsg_guess_base_layers(b, len(b), ids, len(diff_ids), flags))
    return [d for d, f in zip(diff_ids, flags) if f]


def go_time(s):
    """time.Time JSON round trip (test hook)."""
    out = ctypes.create_string_buffer(64)
    _lib.check(_lib.lib().tsg_go_time_rfc3339(_b(s), out, 64))
    return out.value.decode()
