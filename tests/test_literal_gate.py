"""Required-literal gate on Regexp.MatchString (path / allow regexes): the
gated answer equals the plain Pike-VM answer (scanner.go:150-153,170-172,
205-221 evaluate MatchString per file path and per match; the gate only skips
the VM where no match can exist).  Patterns: every builtin rule regex, allow
path / allow regex, and config 5's generated rules; texts: paths and match
strings built to hit the gate literals in every case form, with the fold
runes U+212A / U+017F / U+0130, invalid UTF-8 and boundary positions."""
import ctypes
import json
import os

import numpy as np
import pytest

from trivy_amd import _lib
from workload import synth

DATA = os.path.join(os.path.dirname(__file__), "..", "trivy_amd", "data", "builtin_rules.json")


def _patterns():
    d = json.load(open(DATA))
    pats = []
    for r in d["rules"]:
        pats += [p for p in (r.get("regex"), r.get("path")) if p]
    for a in d["allow_rules"]:
        pats += [p for p in (a.get("regex"), a.get("path")) if p]
    cfg, _ = synth.config5(40, seed=5)
    for r in cfg.get("rules", []):
        pats += [p for p in (r.get("regex"), r.get("path")) if p]
        for a in r.get("allow-rules", []) or []:
            pats += [p for p in (a.get("regex"), a.get("path")) if p]
    for a in cfg.get("allow-rules", []) or []:
        pats += [p for p in (a.get("regex"), a.get("path")) if p]
    return sorted(set(pats))


def _probe(p, text):
    g, pl, h = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    buf = ctypes.create_string_buffer(text, len(text) + 1)
    _lib.check(_lib.lib().tsg_regex_match_probe(p.encode(), buf, len(text), ctypes.byref(g), ctypes.byref(pl),
                                                ctypes.byref(h)))
    return g.value, pl.value, h.value


PATHS = [b"", b"a", b"usr/share/doc/x", b"/usr/share/doc/x", b"USR/share/x", b"usr/lib/gems/x.rb",
         b"opt/yarn-v1.22.0/lib/cli.js", b"opt/yarn-v/x", b"usr/local/lib/python3.11/site.py",
         b"src/Test/a.go", b"src/a_test.go", b"TEST/x", b"te\xe2\x84\xaast", b"src/Example.java",
         b"x/vendor/y", b"x/locales/en.json", b"x/locale/de.po", b"README.md", b"README.md.bak",
         b"var/log/anaconda/x.log", b"usr/src/wordpress/wp-config.php", b"usr/local/go/src/x.go",
         b"\xff\xfeusr/share/", b"a/\xc4\xb0test", b"a/\xc5\xbftest", b"exampl", b"xexamplex"]


def _texts(rng):
    out = list(PATHS)
    alphabet = b"aAeEkKsStTxX0189_-./:=\"' \n" + b"usrhaedploncigvymwbjfqz"
    for _ in range(40):
        n = int(rng.integers(0, 48))
        out.append(bytes(rng.choice(list(alphabet), size=n).astype(np.uint8)))
    return out


def test_gate_matches_plain_vm():
    rng = np.random.default_rng(7)
    pats = _patterns()
    assert len(pats) > 150
    gated_patterns = 0
    for p in pats:
        texts = _texts(rng)
        # texts built from the pattern's own rune-level content: literal runs
        # of the pattern (gate literals) embedded at the start, middle and end
        lits = [s.encode() for s in p.replace("\\", " ").replace("(", " ").replace(")", " ").split() if len(s) >= 2]
        for lit in lits[:6]:
            texts += [lit, b"/" + lit, b"x" + lit + b"y", lit.upper(), lit.lower(), b"a/" + lit + b"/b"]
        seen_gate = 0
        for t in texts:
            g, pl, h = _probe(p, t)
            assert g == pl, (p, t)
            seen_gate = max(seen_gate, h)
        gated_patterns += seen_gate > 0
    assert gated_patterns > len(pats) // 2


@pytest.mark.parametrize("p", [r"(^(?i)test|\/test|-test|_test|\.test)", r"^usr\/(?:share|include|lib)\/",
                               r"\.md$", r"(?i)example", r"^opt\/yarn-v[\d.]+\/"])
def test_builtin_allow_paths_gated(p):
    for t in PATHS:
        g, pl, h = _probe(p, t)
        assert h > 0 and g == pl, (p, t)


@pytest.mark.parametrize("cfg", ["builtin", "config5"])
def test_indexed_allow_path_equals_oracle(tmp_path, cfg):
    # Scanner.AllowPath through the first-byte index of the global allow
    # rules' gate literals (global_allow_path) equals the oracle's loop over
    # every allow rule, on image / source paths built around each rule's
    # literals, with case variants and near misses
    import random

    from oracle import secret_oracle as so
    from trivy_amd import secret as S
    from workload import synth
    cfg_path = None
    if cfg == "config5":
        c5, _ = synth.config5(500, seed=3)
        cfg_path = str(tmp_path / "c5.yaml")
        synth.write_yaml(c5, cfg_path)
    sc = S.Scanner(S.ParseConfig(cfg_path) if cfg_path else None)
    ref = so.Scanner(so.parse_config(cfg_path) if cfg_path else None)
    rng = random.Random(9)
    parts = ["usr", "share", "include", "lib", "local", "go", "python3.11", "gems", "src", "wordpress", "var", "log",
             "anaconda", "opt", "yarn-v1.22.19", "vendor", "locale", "locales", "test", "Test", "TEST", "example",
             "EXAMPLE", "app", "a_test", "x-test", "y.test", "README.md", "doc.MD", "main.go", "node_modules", "tmp"]
    paths = []
    for _ in range(4000):
        p = "/".join(rng.choice(parts) for _ in range(rng.randrange(1, 6)))
        if rng.random() < 0.5:
            p = "/" + p
        paths.append(p)
    paths += ["usr/share/x", "/usr/share/x", "opt/yarn-v1.2/x", "usr/local/lib/python3.11/x", "a.md", "a.mdx", "",
              "test", "atest", "/test", "examplE", "x/vendor/y", "x/vendorz/y"]
    for p in paths:
        assert sc.AllowPath(p) == ref.allow_path(p), p
    # the index is built for the builtins-only ruleset (NewScanner(nil)) too,
    # not only when a config is given
    rep = S.prefilter_report(sc)
    assert "global allow-path index: " in rep and "unused" not in rep.split("global allow-path index: ")[1], rep
