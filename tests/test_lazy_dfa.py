"""Host regexp engine: the lazy DFA that finds anchored match ends
(goregexp.cpp LazyDfa, used by find_all_from_candidates) must agree with
the Pike VM (Go's machine restated) at every position -- empty-width
assertions, leftmost-first priority (lazy/greedy), invalid UTF-8 and
non-ASCII included.  The rule patterns are the builtin rules
(builtin-rules.go:101-849), the builtin allow rules and the config-5 custom
rules and exclude blocks (scanner.go:223-275)."""
import ctypes
import random

import numpy as np
import pytest

from trivy_amd import _lib
from workload import synth
from trivy_amd import secret as S

EDGE = [
    r"\bfoo\b", r"\Boo", r"(?m)^abc$", r"^", r"$", r"(?m)^", r"(?m)$", r"a*", r"a*?", r"(a|ab)(c|bcd)(d*)",
    r"(?s).*?END", r"(?s)BEGIN.*END", r"(?i)straße", r"(?i)k", r"\Aabc", r"abc\z", r"[^\n]*$", r"(?U)a+",
    r"(?U)a+?", r"x{2,5}", r"(x|xy){3}", r"é+", r"[à-ÿ]{2}", r"\pL+", r"\PL", r".", r"(?s).",
    r"--- ignore block start ---(.|\s)*--- ignore block stop ---", r"(^|[^0-9a-zA-Z])(tok_[A-Za-z0-9]{4})($|[^0-9a-zA-Z])",
    r"(?m)^# vault: .*$", r"#\s*nosec-block-\d+[^\n]*", r"\b(a|b)+\b", r"(?i)(?P<key>ab[a-z0-9_ .\-,]{0,5})(=|:).{0,3}['\"]",
]


def _texts(rng):
    alpha = ["a", "b", "c", "d", "x", "y", "o", "f", "E", "N", "D", "K", " ", "\n", "_", "-", "=", ":", "'", '"',
             "#", "tok_", "abc", "foo", "END", "BEGIN", "ß", "é", "K", "ſ", "ab12", "--- ignore block start ---",
             "--- ignore block stop ---", "# vault: ", "nosec-block-7", "\t"]
    out = []
    for _ in range(6):
        s = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 120))).encode()
        if rng.random() < 0.5:                        # invalid UTF-8 bytes
            b = bytearray(s)
            for _ in range(rng.randint(1, 4)):
                b.insert(rng.randint(0, len(b)), rng.choice([0x80, 0xC3, 0xE2, 0xFF, 0xBF]))
            s = bytes(b)
        out.append(s)
    return out


def _probe(pattern, text):
    L = _lib.lib()
    n = len(text) + 1
    buf = np.frombuffer(text + b"\0", dtype=np.uint8)
    pos = np.arange(n, dtype=np.uint64)
    d = np.zeros(n, dtype=np.int64)
    v = np.zeros(n, dtype=np.int64)
    _lib.check(L.tsg_regex_probe(pattern.encode(), buf.ctypes.data, len(text), pos.ctypes.data, n,
                                 d.ctypes.data, v.ctypes.data))
    return d, v


def _patterns():
    pats = list(EDGE)
    pats += [r["regex"] for r in S.GetBuiltinRules() if r.get("regex")]
    cfg, _ = synth.config5(60, seed=3)
    pats += [r["regex"] for r in cfg["rules"]]
    pats += [r["regexes"][0] for r in [cfg["exclude-block"]]] + list(synth.EXCLUDE_BLOCKS)
    return pats


@pytest.mark.parametrize("chunk", range(4))
def test_lazy_dfa_matches_vm(chunk):
    rng = random.Random(1234 + chunk)
    pats = _patterns()
    pats = pats[chunk::4]
    checked = 0
    for p in pats:
        for t in _texts(rng):
            d, v = _probe(p, t)
            bad = np.nonzero(d != v)[0]
            assert len(bad) == 0, (p, t, int(bad[0]), int(d[bad[0]]), int(v[bad[0]]))
            checked += len(t) + 1
    assert checked > 1000


def test_lazy_dfa_planted_rule_samples():
    # the builtin rules' own sampled secrets, embedded in text: real matches
    rng = random.Random(7)
    samples = synth.load_samples()
    rules = [r for r in S.GetBuiltinRules() if r.get("regex")]
    hits = 0
    for r in rules:
        ss = samples.get(r["id"], [])[:3]
        for smp in ss:
            t = ("x = 1\n" + "key: '" + smp + "'\n").encode()
            d, v = _probe(r["regex"], t)
            assert (d == v).all(), r["id"]
            hits += int((d >= 0).sum())
    assert hits > 50


SPAN_PATTERNS = [r"--- ignore block start ---(.|\s)*--- ignore block stop ---",
                 r"(?s)BEGIN NOSCAN.*?END NOSCAN", r"(?s)<x-ignore>.*?</x-ignore>", r"AB(?s:.)*CD",
                 r"AB(.|\n)*?CD", r"AB.*CD", r"AB[^z]*CD"]     # last two: not every rune -> the DFA path


@pytest.mark.parametrize("pattern", SPAN_PATTERNS)
def test_span_shape_end_matches_vm(pattern):
    # L1 (any rune)* L2: the fast anchored end (last / first L2 after L1) equals the VM
    rng = random.Random(99)
    parts = [b"--- ignore block start ---", b"--- ignore block stop ---", b"BEGIN NOSCAN", b"END NOSCAN",
             b"<x-ignore>", b"</x-ignore>", b"AB", b"CD", b"C", b"\n", b"\xe2\x84\xaa", b"\xff", b"\xc3", b"z",
             b"x", b" ", b"--- ignore block st"]
    for _ in range(40):
        t = b"".join(rng.choice(parts) for _ in range(rng.randint(0, 30)))
        d, v = _probe(pattern, t)
        assert (d == v).all(), (pattern, t, d, v)


def test_nesting_depth_limit():
    # Go regexp/syntax ErrNestingDepth (maxHeight 1000): 999 nested captures
    # around an atom parse, 1000 do not; a hostile 100k-deep group nest is an
    # error, not a stack overflow of the host process.
    d, v = _probe("(" * 999 + "a" + ")" * 999, b"xa")
    assert list(d[:2]) == [-1, 2] and list(v[:2]) == [-1, 2]
    for pat in ("(" * 1000 + "a" + ")" * 1000, "(?:" * 100000 + "a" + ")" * 100000):
        with pytest.raises(Exception, match="expression nests too deeply"):
            _probe(pat, b"a")


def test_nested_repeat_product_limit():
    # Go regexp/syntax repeatIsValid(re, 1000): counted repeats nested inside
    # counted repeats may not multiply past 1000 ("invalid repeat count");
    # without the check simplify would expand ((a{1000}){1000}){1000} into 1e9
    # nodes.  Products up to 1000, and {n,} counted by its minimum, parse.
    d, _ = _probe("(?:(?:a{10}){10}){10}", b"a" * 1000)
    assert d[0] == 1000
    for ok in ("(a{2}){500}", "(a{1000})*", "(a{0}){1000}", "(?:a{10,}){100}", "(a{2}b){2}c{1000}"):
        _probe(ok, b"ab")
    for bad in ("((a{1000}){1000}){1000}", "(a{2}){501}", "(?:a{10,}){101}", "(?:(?:a{10}){10}){11}",
                "(a{1001,})", "(x{2,3}y{3}){400}"):
        with pytest.raises(Exception, match="invalid repeat count"):
            _probe(bad, b"a")


def test_lazy_dfa_state_budget_start_state():
    # (a|b)*a(a|b){20} has ~2^21 DFA states: a walk over random a/b text adds
    # one state per byte until the 4096-state budget.  For some text length the
    # first walk (start category: begin of text) ends with the cache exactly
    # full; the next position's start state (previous rune 'a' or 'b', a word
    # character) then cannot be interned: match_end must fall back to the Pike
    # VM (goregexp.cpp LazyDfa::match_end, the budget check on the start
    # state), not read a state that was never created.  Every length around
    # the budget is probed, each position compared with the VM.
    rng = random.Random(4096)
    pattern = r"(a|b)*a(a|b){20}"
    for n in range(4080, 4112):
        text = "".join(rng.choice("ab") for _ in range(n)).encode()
        L = _lib.lib()
        buf = np.frombuffer(text + b"\0", dtype=np.uint8)
        pos = np.array([0, 1, 2, n // 2, 0, n], dtype=np.uint64)
        d = np.zeros(len(pos), dtype=np.int64)
        v = np.zeros(len(pos), dtype=np.int64)
        _lib.check(L.tsg_regex_probe(pattern.encode(), buf.ctypes.data, len(text), pos.ctypes.data, len(pos),
                                     d.ctypes.data, v.ctypes.data))
        assert (d == v).all(), (n, d, v)
        assert v[0] >= 0
