"""The C-ABI library loads and exports every entry point include/trivy_secret.h declares."""
import ctypes
import os
import re

from trivy_amd import _lib

INC = os.path.join(os.path.dirname(__file__), "..", "include")
HDR = os.path.join(INC, "trivy_secret.h")             # the product C-ABI
TEST_HDR = os.path.join(INC, "trivy_secret_test.h")   # test / measurement / tooling hooks


def declared_functions(paths=(HDR, TEST_HDR)):
    names = set()
    for p in paths:
        text = open(p).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names.update(re.findall(r"\b(tsg_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_product_header_holds_no_test_hooks():
    product = declared_functions((HDR,))
    hooks = declared_functions((TEST_HDR,))
    assert not set(product) & set(hooks)
    for n in ("tsg_scan_host_reference", "tsg_scan_table_model", "tsg_test_go_sort", "tsg_test_readback",
              "tsg_regex_probe", "tsg_queue_create_model"):
        assert n in hooks and n not in product


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), n
    # and the ctypes signature table covers the header exactly
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == names


def test_version_and_builtins():
    L = _lib.lib()
    assert b"gfx950" in L.tsg_version()
    import json
    rules = json.loads(L.tsg_builtin_rules_json().decode())["rules"]
    assert len(rules) == 87


def test_ruleset_compile_errors_are_reported():
    L = _lib.lib()
    rs = ctypes.c_void_p()
    bad = b'{"rules": [{"id": "x", "regex": "a(b"}]}'
    rc = L.tsg_ruleset_compile(bad, len(bad), ctypes.byref(rs))
    assert rc == -2
    assert b"regexp compile error" in L.tsg_last_error()


def test_engine_create_without_gpu_fails_loudly():
    L = _lib.lib()
    if L.tsg_device_count() > 0:
        return
    rs = ctypes.c_void_p()
    _lib.check(L.tsg_ruleset_compile(None, 0, ctypes.byref(rs)))
    e = ctypes.c_void_p()
    rc = L.tsg_engine_create(rs, 0, ctypes.byref(e))
    assert rc == -3
    assert b"no HIP device" in L.tsg_last_error()
    L.tsg_ruleset_free(rs)


def test_parse_config_document_rules(tmp_path):
    # yaml.v3 Decoder.Decode (scanner.go:296-298): no document -> io.EOF error;
    # an explicit null document -> the zero Config; only the first document counts
    import pytest

    from oracle import secret_oracle as so
    from trivy_amd import secret as S
    cases = {"empty.yaml": b"", "comments.yaml": b"# nothing here\n\n", "null.yaml": b"---\n",
             "tilde.yaml": b"~\n", "two.yaml": b"disable-rules: [aws-access-key-id]\n---\nrules: 3\n"}
    for name, body in cases.items():
        p = tmp_path / name
        p.write_bytes(body)
        if name in ("empty.yaml", "comments.yaml"):
            with pytest.raises(S.ConfigError, match="secrets config decode error: EOF"):
                S.ParseConfig(str(p))
            with pytest.raises(so.ConfigError, match="secrets config decode error: EOF"):
                so.parse_config(str(p))
        else:
            cfg = S.ParseConfig(str(p))
            assert isinstance(cfg, dict)
            ids = S.Scanner(cfg).rule_ids
            want = [r.id for r in so.Scanner(so.parse_config(str(p))).rules]
            assert ids == want
    assert "aws-access-key-id" not in S.Scanner(S.ParseConfig(str(tmp_path / "two.yaml"))).rule_ids


def test_get_secret_rules_metadata():
    # builtin-rules.go:91-99: one iacRules.Check{Name: ID, Description: Title} per builtin rule, in order
    from trivy_amd import secret as S
    md = S.GetSecretRulesMetadata()
    rules = S.GetBuiltinRules()
    assert md == [{"name": r["id"], "description": r["title"]} for r in rules]
    assert len(md) == 87
