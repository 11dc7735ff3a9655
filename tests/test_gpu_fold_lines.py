"""K1's fold-special line check on lines that take the fast word steps.

U+0130 (C4 B0), U+017F (C5 BF) and U+212A (E2 84 AA) lower or fold onto ASCII
letters (scanner.go:174-186 lowers the content with bytes.ToLower before the
keyword test; Go's (?i) folds U+017F onto 's'), so K1 flags every file that
holds one and the host runs that file's passes with the variant scan DFA.
Since round 6 a fast line is checked from the registers it was loaded into
(engine.hip k1_line_special_regs, was a byte-by-byte re-read from memory).
Here every sequence sits at every phase of a 64-byte line -- inside a line,
straddling two lines, its lead byte the last byte of a line -- once per 64 KiB
file, inside a keyword or regex literal that matches only after lowering or
folding, so a file K1 fails to flag loses its finding; files with stray lead
bytes and with the sequences' bytes out of order must not gain any.  Every
file equals the oracle.
"""
import pytest

from _oracle_pool import oracle_scan_many
from trivy_amd import secret as S

pytestmark = pytest.mark.gpu

_CFG = (
    "rules:\n"
    "  - id: fold-kelvin\n    category: general\n    title: kelvin\n    severity: HIGH\n"
    "    regex: 'tok_[a-z0-9]{8}'\n    keywords: [kitten]\n"
    "  - id: fold-dotted-i\n    category: general\n    title: dotted\n    severity: HIGH\n"
    "    regex: 'iso_[a-z0-9]{8}'\n    keywords: [isotope]\n"
    "  - id: fold-long-s\n    category: general\n    title: long s\n    severity: HIGH\n"
    "    regex: '(?i)vault_sec_[a-z0-9]{8}'\n    keywords: [vault]\n"
)

_FILLER = b"lorem ipsum dolor sit amet, consectetur adipiscing elit\n"
_SIZE = 64 << 10

# (sequence, text around it): the special rune's lead byte is placed at a
# chosen phase of a 64-byte line
_CASES = [
    ("K".encode(), b"ITTEN tok_%08d\n"),          # "KITTEN" with a Kelvin sign
    ("İ".encode(), b"SOTOPE iso_%08d\n"),         # "ISOTOPE" with a dotted capital I
    (b"vault_", "ſec_%08d\n".encode()),           # "vault_sec_" with a long s
]


def _file(pos, payload, strays=b""):
    body = bytearray((_FILLER * (_SIZE // len(_FILLER) + 1))[:_SIZE])
    body[pos:pos + len(payload)] = payload
    for k, b in enumerate(strays):                     # stray bytes every ~1.5 KB
        body[700 + 1531 * k] = b
    return bytes(body)


def _corpus():
    files = []
    for ci, (pre, post) in enumerate(_CASES):
        for phase in range(64):
            n = 1000 * ci + phase
            if ci < 2:
                payload = pre + post % n
                lead = 0                                   # the rune's lead byte
            else:
                payload = pre + post % n                   # the long s follows "vault_"
                lead = len(pre)
            pos = 32768 + phase - lead
            files.append(("src/fold_%d/f%02d.txt" % (ci, phase), _file(pos, payload)))
    # stray lead bytes (C4 / C5 / E2 with other successors) and the sequences'
    # bytes out of order: no fold-special file, the ASCII findings only
    for k in range(16):
        strays = bytes([0xE2, 0xC4, 0xC5, 0x84, 0xAA, 0xB0, 0xBF][(k + j) % 7] for j in range(40))
        payload = b"kitten tok_%08d\n" % (5000 + k)
        files.append(("src/stray/s%02d.txt" % k, _file(20000 + 7 * k, payload, strays)))
        files.append(("src/order/o%02d.txt" % k,
                      _file(30000 + 5 * k, b"\x84\xe2\xaaITTEN tok_%08d \xb0\xc4SOTOPE iso_%08d\n" % (k, k))))
    return files


def test_fold_special_sequences_at_every_line_phase_gpu(tmp_path):
    from oracle import secret_oracle as so
    cfg = tmp_path / "fold.yaml"
    cfg.write_text(_CFG)
    files = _corpus()
    want = oracle_scan_many([(p, c, False) for p, c in files], procs=16, cfg=so.parse_config(str(cfg)))
    by_rule = {}
    for w in want:
        for f in w["Findings"]:
            by_rule[f["RuleID"]] = by_rule.get(f["RuleID"], 0) + 1
    # the Kelvin-sign and dotted-I files are found only through the fold
    # flag (the 16 stray files' ASCII "kitten" adds 16 Kelvin-rule findings)
    assert by_rule.get("fold-kelvin", 0) >= 64 + 16, by_rule
    assert by_rule.get("fold-dotted-i", 0) >= 64, by_rule
    sc = S.Scanner(S.ParseConfig(str(cfg)))
    got = sc.ScanBatch([S.ScanArgs(p, c) for p, c in files])
    for (p, _), g, w in zip(files, got, want):
        assert g == w, p
