"""Client/server wire format of the secret results:
tsg_result_to_proto / tsg_result_from_proto against the Python protobuf
runtime over the trivy.common descriptor (oracle/wire_oracle.py), filled as
pkg/rpc/convert.go:127-175, 370-376, 504-533 fill it."""
import json
import os
import random

import pytest

from oracle import secret_oracle as so
from oracle import wire_oracle as wo
from trivy_amd import _lib
from trivy_amd import report as R
from trivy_amd import secret as S

INTEG = os.path.join(os.path.dirname(__file__), "golden", "integration")


def _line(n, content, cause):
    return {"Number": n, "Content": content, "IsCause": cause, "Annotation": "", "Truncated": False,
            "Highlighted": content, "FirstCause": cause, "LastCause": cause}


def _random_secret(rng, path):
    fs = []
    for _ in range(rng.randint(0, 12)):
        rule = rng.choice(["aws-access-key-id", "github-pat", "slack<token>", "", "jwt"])
        line = rng.choice([0, 1, 7, 300, 2 ** 31 - 5, -1])
        text = rng.choice(["x=<secret> & y", "plain", "tab\there", "", "quote\"q", "été ✓ \U0001F600"])
        binary = rng.random() < 0.2
        lines = [] if binary else [_line(line + k - 1, text if k else "", k == 1) for k in range(rng.randint(1, 3))]
        fs.append({"RuleID": rule, "Category": rng.choice(["AWS", ""]),
                   "Severity": rng.choice(["CRITICAL", "HIGH", "LOW", "UNKNOWN"]),
                   "Title": "T " + rule, "StartLine": line, "EndLine": line + rng.randint(0, 2),
                   "Code": {"Lines": lines}, "Match": "Binary file matches" if binary else text})
    return {"FilePath": path, "Findings": fs}


def _layers(rng, n):
    return [{"Digest": rng.choice(["", "sha256:%d" % k]), "DiffID": rng.choice(["", "sha256:d%d" % k]),
             "CreatedBy": rng.choice(["", "RUN echo %d > /x" % k])} for k in range(n)]


@pytest.mark.parametrize("seed", range(8))
def test_encode_equals_protobuf_runtime(seed):
    rng = random.Random(seed)
    secrets = [_random_secret(rng, p) for p in ["a.txt", "", "dir/été", "b/c.py"]]
    res = R.ScanResult.from_secrets(secrets)
    for i, s in enumerate(secrets):
        lay = _layers(rng, len(s["Findings"])) if seed % 2 else None
        got = res.to_proto(i, lay)
        assert got == wo.secret_to_proto(s, lay), (seed, i)
        # decode: ours and the runtime's agree with the input
        back = R.ScanResult.from_proto([got]).secrets()[0]
        want_layers = lay or [{"Digest": "", "DiffID": "", "CreatedBy": ""}] * len(s["Findings"])
        assert back == {"FilePath": s["FilePath"],
                        "Findings": [dict(f, Layer=l) for f, l in zip(s["Findings"], want_layers)]}
        assert wo.secret_from_proto(got) == (s, want_layers)


def test_golden_scan_result_cpu():
    sc = S.Scanner(S.ParseConfig(os.path.join(INTEG, "trivy-secret.yaml")))
    content = open(os.path.join(INTEG, "deploy.sh"), "rb").read().replace(b"\r", b"")
    res = S.scan_host_reference_result(sc, [S.ScanArgs("deploy.sh", content)])
    oracle_secret = so.Scanner(so.parse_config(os.path.join(INTEG, "trivy-secret.yaml"))).scan("deploy.sh", content)
    got = res.to_proto(0)
    assert got == wo.secret_to_proto(oracle_secret)
    assert len(oracle_secret["Findings"]) == 2


@pytest.mark.gpu
def test_golden_scan_result_gpu():
    sc = S.Scanner(S.ParseConfig(os.path.join(INTEG, "trivy-secret.yaml")))
    content = open(os.path.join(INTEG, "deploy.sh"), "rb").read().replace(b"\r", b"")
    res = sc.ScanBatchResult([S.ScanArgs("deploy.sh", content)])
    oracle_secret = so.Scanner(so.parse_config(os.path.join(INTEG, "trivy-secret.yaml"))).scan("deploy.sh", content)
    assert res.to_proto(0) == wo.secret_to_proto(oracle_secret)


def test_empty_secret_is_empty_message():
    res = R.ScanResult.from_secrets([{"FilePath": "", "Findings": []}, {"FilePath": "x", "Findings": []}])
    assert res.to_proto(0) == b""
    assert res.to_proto(1) == b"\x0a\x01x"
    assert R.ScanResult.from_proto([b""]).secrets() == [{"FilePath": "", "Findings": []}]


def test_invalid_utf8_fails_like_marshal():
    s = {"FilePath": "f", "Findings": [{"RuleID": "r", "Category": "", "Severity": "HIGH", "Title": "t",
                                        "StartLine": 1, "EndLine": 1, "Code": {"Lines": [_line(1, "a\udcffb", True)]},
                                        "Match": "a\udcffb"}]}
    res = R.ScanResult.from_secrets([s])
    with pytest.raises(_lib.TsgError, match="invalid UTF-8"):
        res.to_proto(0)
    with pytest.raises(_lib.TsgError):
        res.to_proto(1)


def test_decode_skips_unknown_fields_and_rejects_garbage():
    s = _random_secret(random.Random(3), "p")
    msg = wo.secret_to_proto(s)
    # unknown fields of every wire type, at the top level
    extra = b"\x98\x06\x05" + b"\xa1\x06" + b"\x00" * 8 + b"\xaa\x06\x02hi" + b"\xad\x06" + b"\x00" * 4
    back = R.ScanResult.from_proto([extra + msg + extra]).secrets()[0]
    assert back["FilePath"] == "p" and len(back["Findings"]) == len(s["Findings"])
    for bad in [msg[:-1] if msg else b"\x0a", b"\x0a\x05ab", b"\x0f", b"\x0a\x02\xff\xfe"]:
        with pytest.raises(_lib.TsgError):
            R.ScanResult.from_proto([bad])


def test_decode_runtime_message_with_repeated_fields_merged():
    """proto3 semantics the converter sees: a repeated Secret field split over
    the stream; last-wins for a scalar given twice."""
    cls = wo.message_class("Secret")
    a = cls(filepath="first")
    a.findings.add(rule_id="r1", start_line=3).code.lines.add(number=3, content="c", highlighted="c")
    b = cls(filepath="second")
    b.findings.add(rule_id="r2", severity="LOW")
    data = a.SerializeToString() + b.SerializeToString()
    got = R.ScanResult.from_proto([data]).secrets()[0]
    want = cls.FromString(data)
    assert got["FilePath"] == want.filepath == "second"
    assert [f["RuleID"] for f in got["Findings"]] == [f.rule_id for f in want.findings] == ["r1", "r2"]
    assert got["Findings"][0]["Code"]["Lines"][0]["Number"] == 3
    # ConvertFromRPCSecretFindings keeps Severity as sent
    assert got["Findings"][1]["Severity"] == "LOW"
