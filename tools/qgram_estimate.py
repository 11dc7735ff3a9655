"""Hit rate of a q-gram prefilter over the builtin rules (round-4 dead-end estimate).

Every scan literal (anchor literals from the prefilter report, keywords) cut
to its first 4 bytes in all its case variants; a position "hits" when the 2-, 3- or
4-byte string starting there is one of them.  Run on a 200 MB
config-2 synthetic corpus:  python tools/qgram_estimate.py
"""
import sys, re, json, itertools
import numpy as np
sys.path.insert(0, "/root/repo")
from trivy_amd import secret as S
from workload import synth
rep = S.prefilter_report(S.Scanner())
lits = set()
for ln in rep.splitlines():
    m = re.search(r"\{(.*)\}\s*$", ln)
    if not m or ": anchored" not in ln: continue
    for tok in m.group(1).split(" "):
        units = re.findall(r"\(([^)]*)\)|(.)", tok)
        alts = [u[0].split("|") if u[0] else [u[1]] for u in units]
        for combo in itertools.product(*alts[:4]):
            lits.add("".join(combo))
rules = json.load(open("/root/repo/trivy_amd/data/builtin_rules.json"))
rl = rules["rules"] if isinstance(rules, dict) else rules
for r in rl:
    for k in r.get("keywords") or []:
        k = k.lower()[:4]
        for combo in itertools.product(*[(c.lower(), c.upper()) if c.isalpha() else (c,) for c in k]):
            lits.add("".join(combo))
print("literal prefixes (<=4 B, case variants):", len(lits), "by length", {q: sum(len(l) == q for l in lits) for q in (1,2,3,4)})
c = synth.generate(int(2e8), seed=3, sizes="loguniform", layout="src")
d = np.asarray(c.data[:c.nbytes], dtype=np.uint8).astype(np.uint32)
n = len(d)
g2 = d[:-3] | (d[1:-2] << 8)
g3 = g2 | (d[2:-1] << 16)
g4 = g3 | (d[3:] << 24)
hits = np.zeros(n - 3, dtype=bool)
for q, g in ((2, g2), (3, g3), (4, g4)):
    vals = np.array([sum(ord(ch) << (8 * i) for i, ch in enumerate(l)) for l in lits if len(l) == q], dtype=np.uint32)
    h = np.isin(g, vals)
    print("q=%d: %d literals, %.3e of positions" % (q, len(vals), h.mean()))
    hits |= h
print("any: %.3e of positions -> %.0f M hits per 10 GB" % (hits.mean(), hits.mean() * 1e10 / 1e6))
