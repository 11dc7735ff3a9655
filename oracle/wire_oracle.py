"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

The client/server wire form of the secret results, restated with the Python
protobuf runtime (an independent proto3 implementation) over a descriptor
built here from rpc/common/service.proto:152-156 (Layer), 191-204 (Line,
Code), 206-218 (SecretFinding; field 9 is reserved) and 220-223 (Secret),
filled exactly as pkg/rpc/convert.go does:

  ConvertToRPCSecrets / ConvertToRPCSecretFindings   convert.go:146-175
  ConvertToRPCCode (Code always set, Highlighted)    convert.go:127-144
  ConvertToRPCLayer (Layer always set)               convert.go:370-376
  ConvertFromRPCSecrets / ...SecretFindings          convert.go:504-533

Parity is pinned by the protobuf runtime's own serializer (Go's
proto.Marshal and it both write fields in number order and skip proto3
defaults); the reference ships no serialized Secret fixture.
"""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto

_MESSAGES = {
    "Layer": [("digest", 1, "string"), ("diff_id", 2, "string"), ("created_by", 3, "string")],
    "Line": [("number", 1, "int32"), ("content", 2, "string"), ("is_cause", 3, "bool"),
             ("annotation", 4, "string"), ("truncated", 5, "bool"), ("highlighted", 6, "string"),
             ("first_cause", 7, "bool"), ("last_cause", 8, "bool")],
    "Code": [("lines", 1, "repeated Line")],
    "SecretFinding": [("rule_id", 1, "string"), ("category", 2, "string"), ("severity", 3, "string"),
                      ("title", 4, "string"), ("start_line", 5, "int32"), ("end_line", 6, "int32"),
                      ("code", 7, "Code"), ("match", 8, "string"), ("layer", 10, "Layer")],
    "Secret": [("filepath", 1, "string"), ("findings", 2, "repeated SecretFinding")],
}

_SCALAR = {"string": _F.TYPE_STRING, "int32": _F.TYPE_INT32, "bool": _F.TYPE_BOOL}


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="tsg_oracle/common.proto", package="trivy.common",
                                            syntax="proto3")
    for name, fields in _MESSAGES.items():
        m = fd.message_type.add(name=name)
        for fname, num, typ in fields:
            label = _F.LABEL_OPTIONAL
            if typ.startswith("repeated "):
                label, typ = _F.LABEL_REPEATED, typ.split()[1]
            f = m.field.add(name=fname, number=num, label=label)
            if typ in _SCALAR:
                f.type = _SCALAR[typ]
            else:
                f.type = _F.TYPE_MESSAGE
                f.type_name = ".trivy.common." + typ
        if name == "SecretFinding":
            m.reserved_range.add(start=9, end=10)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return {n: message_factory.GetMessageClass(pool.FindMessageTypeByName("trivy.common." + n)) for n in _MESSAGES}


_CLS = _build()


def secret_to_proto(secret, layers=None):
    """secret: a types.Secret dict (Go field names); layers: per finding a
    {"Digest", "DiffID", "CreatedBy"} dict or None.  Returns the bytes."""
    m = _CLS["Secret"](filepath=secret["FilePath"])
    for k, f in enumerate(secret["Findings"]):
        fm = m.findings.add(rule_id=f["RuleID"], category=f["Category"], severity=f["Severity"],
                            title=f["Title"], start_line=f["StartLine"], end_line=f["EndLine"], match=f["Match"])
        fm.code.SetInParent()
        for ln in f["Code"]["Lines"] or []:
            fm.code.lines.add(number=ln["Number"], content=ln["Content"], is_cause=ln["IsCause"],
                              annotation=ln["Annotation"], truncated=ln["Truncated"],
                              highlighted=ln["Highlighted"], first_cause=ln["FirstCause"],
                              last_cause=ln["LastCause"])
        fm.layer.SetInParent()
        if layers is not None:
            lay = layers[k]
            fm.layer.digest, fm.layer.diff_id, fm.layer.created_by = (
                lay.get("Digest", ""), lay.get("DiffID", ""), lay.get("CreatedBy", ""))
    return m.SerializeToString(deterministic=True)


def secret_from_proto(data):
    """ConvertFromRPCSecrets of one message: (types.Secret dict, layers)."""
    m = _CLS["Secret"].FromString(data)
    findings, layers = [], []
    for fm in m.findings:
        findings.append({
            "RuleID": fm.rule_id, "Category": fm.category, "Severity": fm.severity, "Title": fm.title,
            "StartLine": fm.start_line, "EndLine": fm.end_line,
            "Code": {"Lines": [{"Number": ln.number, "Content": ln.content, "IsCause": ln.is_cause,
                                "Annotation": ln.annotation, "Truncated": ln.truncated,
                                "Highlighted": ln.highlighted, "FirstCause": ln.first_cause,
                                "LastCause": ln.last_cause} for ln in fm.code.lines]},
            "Match": fm.match})
        layers.append({"Digest": fm.layer.digest, "DiffID": fm.layer.diff_id, "CreatedBy": fm.layer.created_by})
    return {"FilePath": m.filepath, "Findings": findings}, layers


def message_class(name):
    return _CLS[name]
