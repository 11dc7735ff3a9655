"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Python restatement of what Trivy does with types.Secret results after
Scanner.Scan, used to check trivy_amd/csrc/report.cpp:

  AnalysisResult.Sort (secrets)     pkg/fanal/analyzer/analyzer.go:224-235
  mergeSecrets / ApplyLayers        pkg/fanal/applier/docker.go:134-146,186-188,297-325
  image-config secret merge         pkg/scanner/local/scan.go:487-496
  secretsToResults                  pkg/scanner/local/scan.go:236-254
  filterSecrets (severity)          pkg/result/filter.go:154-169
  JSONWriter                        pkg/report/json.go:22-50
  GuessBaseImageIndex / guessBase   pkg/fanal/image/image.go:111-137,
                                    pkg/fanal/artifact/image/image.go:526-554

Go encoding/json is restated as: fields in struct order with omitempty,
HTML-escaping string encoder, json.Indent layout.  Pinned by the reference's
integration/testdata/secrets.json.golden (byte-identical) and the applier's
"removed and updated secret" case (applier/docker_test.go:548-700).
"""
import json

from .secret_oracle import go_sort_slice


def go_json_str(s):
    """encoding/json appendString (escapeHTML = true) of a Go string given as
    a surrogateescape'd str (each lone surrogate = one invalid byte)."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif o < 0x20:
            out.append({8: "\\b", 12: "\\f", 10: "\\n", 13: "\\r", 9: "\\t"}.get(o, "\\u%04x" % o))
        elif ch in "<>&":
            out.append("\\u%04x" % o)
        elif 0xDC80 <= o <= 0xDCFF:
            out.append("\\ufffd")
        elif o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def go_marshal_indent(v, prefix="", indent="  ", depth=0):
    """json.MarshalIndent of a value built from dict (ordered) / list / str /
    bool / int / None; str values are Go strings (surrogateescape'd)."""
    nl = "\n" + prefix + indent * (depth + 1)
    end = "\n" + prefix + indent * depth
    if isinstance(v, dict):
        if not v:
            return "{}"
        items = [go_json_str(k) + ": " + go_marshal_indent(x, prefix, indent, depth + 1) for k, x in v.items()]
        return "{" + nl + ("," + nl).join(items) + end + "}"
    if isinstance(v, list):
        if not v:
            return "[]"
        return "[" + nl + ("," + nl).join(go_marshal_indent(x, prefix, indent, depth + 1) for x in v) + end + "]"
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, int):
        return str(v)
    return go_json_str(v)


ZERO_METADATA = {"ImageConfig": {"architecture": "", "created": "0001-01-01T00:00:00Z", "os": "",
                                 "rootfs": {"type": "", "diff_ids": None}, "config": {}}}


def _detected(f, layer):
    lines = f["Code"]["Lines"]
    code_lines = None if not lines else [
        dict([("Number", ln["Number"]), ("Content", ln["Content"]), ("IsCause", ln["IsCause"]),
              ("Annotation", ln["Annotation"]), ("Truncated", ln["Truncated"])]
             + ([("Highlighted", ln["Highlighted"])] if ln["Highlighted"] else [])
             + [("FirstCause", ln["FirstCause"]), ("LastCause", ln["LastCause"])])
        for ln in lines]
    lay = {}
    for k in ("Digest", "DiffID", "CreatedBy"):
        if layer.get(k):
            lay[k] = layer[k]
    return dict([("RuleID", f["RuleID"]), ("Category", f["Category"]), ("Severity", f["Severity"]),
                 ("Title", f["Title"]), ("StartLine", f["StartLine"]), ("EndLine", f["EndLine"]),
                 ("Code", {"Lines": code_lines}), ("Match", f["Match"]), ("Layer", lay)])


def _b(s):
    return s.encode("utf-8", "surrogateescape")


def report(layers, layer_refs=None, image_config=None, artifact_name="", artifact_type="",
           created_at="0001-01-01T00:00:00Z", severities=None, schema_version=2, layers_sorted=False):
    """layers: per layer a list of types.Secret dicts (Scan results, any
    order, empty ones included); returns the JSON report text."""
    severities = severities or ["UNKNOWN", "LOW", "MEDIUM", "HIGH", "CRITICAL"]
    merged = {}
    for li, secrets in enumerate(layers):
        ref = (layer_refs or [{}] * len(layers))[li]
        secs = [s for s in secrets if s["Findings"]]
        if not layers_sorted:
            go_sort_slice(secs, lambda a, b: _b(a["FilePath"]) < _b(b["FilePath"]))
        for s in secs:
            fs = [(f, ref) for f in s["Findings"]]
            if not layers_sorted:
                go_sort_slice(fs, lambda a, b: _b(a[0]["RuleID"]) < _b(b[0]["RuleID"])
                              if a[0]["RuleID"] != b[0]["RuleID"] else a[0]["StartLine"] < b[0]["StartLine"])
            if s["FilePath"] in merged:
                # secretFindingsContains checks the growing new list
                # (docker.go:306-311): one older finding per absent RuleID
                for p in merged[s["FilePath"]]:
                    if all(f["RuleID"] != p[0]["RuleID"] for f, _ in fs):
                        fs.append(p)
            merged[s["FilePath"]] = fs
    ordered = [(p, merged[p]) for p in sorted(merged, key=_b)]
    if image_config and image_config["Findings"]:
        ordered.append((artifact_name, [(f, {}) for f in image_config["Findings"]]))
    results = []
    for target, fs in ordered:
        kept = [_detected(f, ref) for f, ref in fs if f["Severity"] in severities]
        if not target and not kept:
            continue
        r = {"Target": target, "Class": "secret"}
        if kept:
            r["Secrets"] = kept
        results.append(r)
    doc = {}
    if schema_version:
        doc["SchemaVersion"] = schema_version
    doc["CreatedAt"] = created_at
    if artifact_name:
        doc["ArtifactName"] = artifact_name
    if artifact_type:
        doc["ArtifactType"] = artifact_type
    doc["Metadata"] = json.loads(json.dumps(ZERO_METADATA))
    if results:
        doc["Results"] = results
    return go_marshal_indent(doc) + "\n"


def guess_base_layers(history, diff_ids):
    """history: [{"created_by", "empty_layer"}]; returns the base diff IDs."""
    base_idx = -1
    found_non_empty = False
    for i in range(len(history) - 1, -1, -1):
        h = history[i]
        if not found_non_empty:
            if h.get("empty_layer"):
                continue
            found_non_empty = True
        if not h.get("empty_layer"):
            continue
        cb = h.get("created_by", "")
        if cb.startswith("/bin/sh -c #(nop)  CMD") or cb.startswith("CMD"):
            base_idx = i
            break
    out, di = [], 0
    for i, h in enumerate(history):
        if i > base_idx:
            break
        if h.get("empty_layer"):
            continue
        if di >= len(diff_ids):
            return []
        out.append(diff_ids[di])
        di += 1
    return out
