"""The oracle's regex translation (oracle/goregex.py) folds single-char
alternations such as the exclude-block idiom `(.|\\s)*` into one char class
and runs capture-free matches on a non-capturing translation.  Property test:
on random small texts both rewrites give exactly the match lists of the
literal translation (merge=False, capturing), which backtracks per char and
per recorded capture but is exact on small inputs.  Then the rewrite's point:
config 5's exclude block over a multi-MB file finishes quickly."""
import zlib

import numpy as np
import pytest

from oracle.goregex import GoRegexp

PATTERNS = [
    r"--- ignore block start ---(.|\s)*--- ignore block stop ---",
    r"start(.|\s)*?stop",
    r"(?i)(a|k|[0-9])+x",
    r"(?i)x(?P<s>k|s|\n)+y",
    r"(a|b|(c))+d",                      # a capturing alternative: not merged
    r"(?s)q(.|[^a])*?z",
    r"((?i:k)|\d|[[:space:]])\w",
    r"(x|\pL|é)+!",
    r"(^|[^0-9a-zA-Z])(k|K)ey",
    r"a(?:\n|\t| )b",
]
ALPHABET = ["a", "b", "c", "d", "k", "K", "K", "s", "S", "ſ", "x", "y", "z", "q", "!", "0", "7",
            " ", "\n", "\t", "é", "\udcff", "start", "stop", "--- ignore block start ---",
            "--- ignore block stop ---", "key", "Key", "start stop"]


def _texts(seed, n=80, max_chars=20):
    # short texts: the literal translation backtracks exponentially on an
    # ambiguous alternation such as (.|[^a])*? when no match follows
    rng = np.random.default_rng(seed)
    for _ in range(n):
        parts = rng.choice(len(ALPHABET), size=int(rng.integers(0, 10)))
        t = ""
        for i in parts:
            if len(t) + len(ALPHABET[i]) <= max_chars:
                t += ALPHABET[i]
        yield t.encode("utf-8", "surrogateescape")


@pytest.mark.parametrize("pat", PATTERNS)
def test_merged_translation_equals_literal(pat):
    fast = GoRegexp(pat)
    slow = GoRegexp(pat, merge=False)
    assert fast.subexp_names == slow.subexp_names
    for t in _texts(zlib.crc32(pat.encode())):
        assert fast.find_all(t) == slow.find_all(t), (pat, t)
        assert fast.find_all(t, submatch=True) == slow.find_all(t, submatch=True), (pat, t)
        assert fast.match_string(t) == slow.match_string(t)


def test_exclude_block_large_file():
    rx = GoRegexp(r"--- ignore block start ---(.|\s)*--- ignore block stop ---")
    body = b"x = 1\nAKIA0123456789ABCDEF\n" * 300_000              # ~8 MB
    text = (b"head\n--- ignore block start ---\n" + body + b"--- ignore block stop ---\n" + body
            + b"--- ignore block stop ---\ntail\n")
    got = rx.find_all(text)
    # greedy star: one block up to the LAST stop marker
    assert got == [[5, len(text) - len(b"\ntail\n")]]


def test_find_location_indexed_equals_literal():
    # the oracle's per-file line index gives findLocation's exact values
    # (scanner.go:495-558): lines around long lines, first/last line, spans
    # over several lines, content without a trailing newline
    import random
    from oracle import secret_oracle as so
    rng = random.Random(9)
    for trial in range(60):
        parts = []
        for _ in range(rng.randint(1, 40)):
            n = rng.choice((0, 1, 5, 40, 99, 100, 101, 250))
            parts.append(bytes(rng.choice(b"abc xyz=*") for _ in range(n)))
        content = b"\n".join(parts) + (b"\n" if rng.random() < 0.5 else b"")
        if not content:
            continue
        idx = so._LineIndex(content)
        for _ in range(20):
            s = rng.randrange(len(content))
            e = min(len(content), s + rng.randint(0, 300))
            assert so.find_location_indexed(s, e, idx) == so.find_location(s, e, content), (trial, s, e)


def test_vectorised_lower_and_offsets_equal_per_char_definitions():
    # bytes.ToLower (Map(unicode.ToLower), invalid byte -> U+FFFD) and the
    # char -> byte offset map, vectorised for multi-MB files, equal their
    # per-char definitions on mixed ASCII / fold-special / invalid UTF-8 input
    import random
    from oracle import secret_oracle as so
    from oracle.goregex import GoRegexp

    def slow_lower(b):
        if b.isascii():
            return b.lower()
        return "".join("�" if 0xDC80 <= ord(ch) <= 0xDCFF else so._go_rune_lower(ch)
                       for ch in b.decode("utf-8", "surrogateescape")).encode()
    rng = random.Random(1)
    alph = [b"a", b"Z", "K".encode(), "ſ".encode(), "İ".encode(), "Σ".encode(), b"\xff",
            b"\xe2\x82", b"\xed\xa0\x80", "\U0001f600".encode(), "É".encode(), b"\n"]
    for _ in range(2000):
        b = b"".join(rng.choice(alph) for _ in range(rng.randint(0, 30)))
        assert so.go_bytes_to_lower(b) == slow_lower(b), b
        text, offs = GoRegexp.prepare(b)
        if offs is not None:
            want = [0]
            for ch in text:
                want.append(want[-1] + (1 if 0xDC80 <= ord(ch) <= 0xDCFF else len(ch.encode())))
            assert list(offs) == want, b
