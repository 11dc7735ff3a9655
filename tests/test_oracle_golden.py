"""Pin the oracle (oracle/secret_oracle.py) to the reference's own expectations:
all 40 cases of pkg/fanal/secret/scanner_test.go:964-1329, the analyzer tests
(pkg/fanal/analyzer/secret/secret_test.go:16-258) and the integration golden
(integration/testdata/secrets.json.golden)."""
import json
import os

import pytest

from oracle import secret_oracle as so

G = os.path.join(os.path.dirname(__file__), "golden")
SCANNER = json.load(open(os.path.join(G, "scanner_cases.json")))
ANALYZER = json.load(open(os.path.join(G, "analyzer_cases.json")))
INTEG = json.load(open(os.path.join(G, "integration_cases.json")))


def _scan_case(base, case):
    cwd = os.getcwd()
    os.chdir(base)   # the reference tests use relative testdata/ paths
    try:
        cfg = so.parse_config(case["config"])
        content = open(case["input"], "rb").read().replace(b"\r", b"")
        return so.Scanner(cfg).scan(case["path"], content)
    finally:
        os.chdir(cwd)


@pytest.mark.parametrize("case", SCANNER, ids=[c["name"] for c in SCANNER])
def test_scanner_case(case):
    got = _scan_case(os.path.join(G, "scanner"), case)
    assert got == case["want"]


@pytest.mark.parametrize("case", INTEG, ids=[c["name"] for c in INTEG])
def test_integration_golden(case):
    got = _scan_case(os.path.join(G, "integration"), case)
    assert got == case["want"]


@pytest.mark.parametrize("case", ANALYZER["analyze"], ids=[c["name"] for c in ANALYZER["analyze"]])
def test_analyzer_case(case):
    cwd = os.getcwd()
    os.chdir(os.path.join(G, "analyzer"))
    try:
        a = so.SecretAnalyzer(case["config"])
        raw = open(case["input"], "rb").read()
        got = a.analyze(case["path"], raw, case["dir"])
    finally:
        os.chdir(cwd)
    assert (got or []) == case["want"]


@pytest.mark.parametrize("case", ANALYZER["required"], ids=[c["name"] for c in ANALYZER["required"]])
def test_required_case(case):
    cwd = os.getcwd()
    os.chdir(os.path.join(G, "analyzer"))
    try:
        a = so.SecretAnalyzer("testdata/skip-tests-config.yaml")
        got = a.required(case["path"], os.path.getsize(case["path"]))
    finally:
        os.chdir(cwd)
    assert got == case["want"]
