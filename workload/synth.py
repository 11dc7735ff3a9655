"""Deterministic synthetic corpora for the BASELINE.json configs.

Source-like ASCII lines (mean ~40 B, 1% long lines), keyword decoys (~1 per
2 KB: key, sk, pk., live_, lob, dapi, hf_, SG., .eyJ, -----), planted secrets
in ~0.01% of lines drawn uniformly over the builtin rules (strings sampled from
each rule's own regex, never containing "example"), 10% near-miss plants,
0.1% of files with UTF-8 including U+212A/U+017F/U+0130, 0.05% with invalid
UTF-8.  Paths avoid the builtin allow-paths.  Everything is seeded (default
seed 0x71215EC7; shard k uses seed + k) so CPU and GPU runs see the same bytes.

Large corpora are assembled with numpy from a base text of generated lines
(segments copied at random offsets), then plants overwrite whole lines in place
so file sizes are exact.
"""
import json
import os
import random
import re

import numpy as np

DEFAULT_SEED = 0x71215EC7
_HERE = os.path.dirname(os.path.abspath(__file__))

WORDS = ("return value index count buffer result error config client server request response handler "
         "update delete create select insert string number object array module import export const let var "
         "func def class struct interface public private static void int float double bool true false null "
         "self this new try catch finally throw if else for while switch case break continue data user name "
         "path file line open close read write size length format parse token hash map list set get put "
         "append range items values keys print log debug info warn trace context timeout retry status").split()
DECOYS = ["key", "sk", "pk.", "live_", "lob", "dapi", "hf_", "SG.", ".eyJ", "-----", "api_key", "secret",
          "KEY", "token", "aws", "ghp", "password", "xoxb"]
EXTS = ["go", "py", "js", "ts", "java", "c", "h", "cc", "rb", "rs", "yaml", "json", "sh", "txt", "env",
        "conf", "ini", "xml", "sql", "tf"]


# ------------------------------------------------------------ regex sampler
class _Sampler:
    """Random string generator for the Go regexp syntax used by secret rules."""

    def __init__(self, pattern, rng):
        self.p = pattern
        self.i = 0
        self.rng = rng

    def sample(self):
        self.i = 0
        out = self._alt({"i": False})
        return out

    def _peek(self, k=0):
        j = self.i + k
        return self.p[j] if j < len(self.p) else ""

    def _alt(self, flags):
        branches = []
        start = self.i
        depth = 0
        # split at top-level '|'
        cuts = [start]
        j = start
        in_cls = False
        while j < len(self.p):
            c = self.p[j]
            if c == "\\":
                j += 2
                continue
            if in_cls:
                if c == "]":
                    in_cls = False
                j += 1
                continue
            if c == "[":
                in_cls = True
                if j + 1 < len(self.p) and self.p[j + 1] == "]":
                    j += 1
                elif j + 2 < len(self.p) and self.p[j + 1] == "^" and self.p[j + 2] == "]":
                    j += 2
            elif c == "(":
                depth += 1
            elif c == ")":
                if depth == 0:
                    break
                depth -= 1
            elif c == "|" and depth == 0:
                cuts.append(j + 1)
            j += 1
        end = j
        cuts.append(end + 1)
        segs = [(cuts[k], cuts[k + 1] - 1) for k in range(len(cuts) - 1)]
        a, b = segs[self.rng.randrange(len(segs))]
        # flags set inside earlier branches persist; approximate by scanning all
        self.i = a
        out = self._concat(flags, b)
        self.i = end
        for s_, _ in segs:
            branches.append(s_)
        return out

    def _concat(self, flags, end):
        out = []
        while self.i < end:
            atom = self._atom(flags)
            if atom is None:
                continue
            gen, ok = atom
            lo, hi = 1, 1
            c = self._peek()
            if c and c in "*+?":
                self.i += 1
                lo, hi = {"*": (0, 3), "+": (1, 4), "?": (0, 1)}[c]
                if self._peek() == "?":
                    self.i += 1
            elif c == "{":
                m = re.match(r"\{(\d+)(,(\d*))?\}", self.p[self.i:])
                if m:
                    self.i += m.end()
                    lo = int(m.group(1))
                    if m.group(2) is None:
                        hi = lo
                    elif m.group(3):
                        hi = int(m.group(3))
                    else:
                        hi = lo + 3
                    if self._peek() == "?":
                        self.i += 1
            n = self.rng.randint(lo, min(hi, lo + 6))
            for _ in range(n):
                out.append(gen())
        return "".join(out)

    def _class_chars(self, body, neg):
        chars = set()
        k = 0
        while k < len(body):
            c = body[k]
            if c == "\\" and k + 1 < len(body):
                e = body[k + 1]
                k += 2
                if e == "d":
                    chars.update("0123456789")
                elif e == "s":
                    chars.update(" \t")
                elif e == "w":
                    chars.update("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_")
                else:
                    lit = {"n": "\n", "r": "\r", "t": "\t"}.get(e, e)
                    if k < len(body) - 1 and body[k] == "-" and body[k + 1] != "]":
                        hi = body[k + 1]
                        chars.update(chr(x) for x in range(ord(lit), ord(hi) + 1))
                        k += 2
                    else:
                        chars.add(lit)
                continue
            if k + 2 < len(body) and body[k + 1] == "-":
                chars.update(chr(x) for x in range(ord(c), ord(body[k + 2]) + 1))
                k += 3
                continue
            chars.add(c)
            k += 1
        if neg:
            universe = set(" !#$%&()*+,-./:;<=>?@[]^_{|}~")
            chars = sorted(universe - chars) or [" "]
        chars = sorted(c for c in chars if c not in "\r\n")
        return chars or [" "]

    def _atom(self, flags):
        c = self._peek()
        rng = self.rng
        if c == "(":
            self.i += 1
            if self._peek() == "?":
                m = re.match(r"\?(P?<[A-Za-z0-9_]+>|[imsU-]*:|[imsU-]*\))", self.p[self.i:])
                tok = m.group(1)
                self.i += m.end()
                if tok.endswith(")"):
                    if "i" in tok.split("-")[0]:
                        flags["i"] = True
                    return None
            save_flags = dict(flags)
            if self.i >= 1 and self.p[self.i - 1] == ":" and "i" in self.p[:self.i].rsplit("(?", 1)[-1].split("-")[0]:
                save_flags["i"] = True
            start = self.i
            self._alt(dict(flags))   # advance to matching ')'
            end = self.i
            self.i = end + 1
            sub = self.p[start:end]

            def gen(sub=sub, fl=save_flags):
                s = _Sampler(sub, rng)
                s.i = 0
                return s._alt(dict(fl))
            return gen, True
        if c == "[":
            j = self.i + 1
            neg = False
            if self._peek(1) == "^":
                neg = True
                j += 1
            k = j
            if k < len(self.p) and self.p[k] == "]":
                k += 1
            while self.p[k] != "]":
                k += 2 if self.p[k] == "\\" else 1
            body = self.p[j:k]
            self.i = k + 1
            chars = self._class_chars(body, neg)
            fold = flags["i"]
            return (lambda: self._fold(rng.choice(chars), fold)), True
        if c == "\\":
            e = self._peek(1)
            self.i += 2
            if e == "s":
                return (lambda: rng.choice(" ")), True
            if e == "d":
                return (lambda: rng.choice("0123456789")), True
            if e == "w":
                return (lambda: rng.choice("abcdefXYZ019_")), True
            lit = {"n": "\n", "t": "\t"}.get(e, e)
            fold = flags["i"]
            return (lambda: self._fold(lit, fold)), True
        if c and c in "^$":
            self.i += 1
            return (lambda: ""), True
        if c == ".":
            self.i += 1
            return (lambda: rng.choice("abc=:_- ")), True
        self.i += 1
        fold = flags["i"]
        return (lambda: self._fold(c, fold)), True

    def _fold(self, ch, fold):
        if fold and ch.isalpha() and self.rng.random() < 0.3:
            return ch.swapcase()
        return ch


def rule_samples(rules, rng, per_rule=24):
    """For each builtin rule: strings sampled from its regex that the Go
    regexp (oracle) matches, and never containing 'example'."""
    from oracle.goregex import GoRegexp  # sampling validation only (generator)
    out = {}
    for r in rules:
        rx = GoRegexp(r["regex"])
        got = []
        tries = 0
        while len(got) < per_rule and tries < per_rule * 40:
            tries += 1
            s = _Sampler(r["regex"], rng).sample()
            if "example" in s.lower() or "\n" in s:
                continue
            b = s.encode("utf-8", "surrogateescape")
            if rx.find_all(b):
                # make sure the rule's keyword gate is true for the plant itself
                kws = [k.lower() for k in r["keywords"]]
                if kws and not any(k in s.lower() for k in kws):
                    s = s + " " + r["keywords"][0]
                got.append(s)
        out[r["id"]] = got
    return out


_SAMPLES_CACHE = os.path.join(_HERE, "rule_samples.json")
_BUILTIN_JSON = os.path.join(_HERE, "..", "trivy_amd", "data", "builtin_rules.json")


def load_samples(seed=DEFAULT_SEED):
    """Cached plant strings (workload/rule_samples.json, generated here
    once with the oracle so the GPU box needs no oracle import to build a corpus)."""
    if os.path.exists(_SAMPLES_CACHE):
        return json.load(open(_SAMPLES_CACHE))
    rules = json.load(open(_BUILTIN_JSON))["rules"]
    s = rule_samples(rules, random.Random(seed))
    with open(_SAMPLES_CACHE, "w") as f:
        json.dump(s, f, indent=0, ensure_ascii=False)
    return s


# ------------------------------------------------------------- base text
def _source_line(rng):
    r = rng.random()
    ind = " " * rng.choice((0, 0, 2, 4, 4, 8))
    w = rng.choice
    if r < 0.25:
        s = "%s%s = %s(%s, %d)" % (ind, w(WORDS), w(WORDS), w(WORDS), rng.randint(0, 9999))
    elif r < 0.45:
        s = "%s%s %s.%s(%s)" % (ind, w(WORDS), w(WORDS), w(WORDS), ", ".join(w(WORDS) for _ in range(rng.randint(0, 3))))
    elif r < 0.6:
        s = "%s# %s" % (ind, " ".join(w(WORDS) for _ in range(rng.randint(2, 9))))
    elif r < 0.7:
        s = '%s"%s": "%s",' % (ind, w(WORDS), w(WORDS))
    elif r < 0.8:
        s = "%sif %s %s %d {" % (ind, w(WORDS), rng.choice(("==", "!=", "<", ">=")), rng.randint(0, 100))
    elif r < 0.9:
        s = "%s}" % ind
    else:
        s = ""
    if rng.random() < 0.01:   # long line (0.1-8 KB)
        n = rng.randint(100, 8000)
        s = ind + "".join(rng.choice("abcdefghijklmnopqrstuvwxyz0123456789 ,.;()=+-") for _ in range(n))
    return s


def base_text(nbytes, seed):
    """~nbytes of newline-terminated source-like text with decoys."""
    rng = random.Random(seed)
    parts = []
    total = 0
    since_decoy = 0
    while total < nbytes:
        line = _source_line(rng)
        since_decoy += len(line) + 1
        if since_decoy > 2048 or rng.random() < 0.02:
            since_decoy = 0
            d = rng.choice(DECOYS)
            pos = rng.randint(0, len(line))
            line = line[:pos] + d + ("_" + rng.choice(WORDS) if rng.random() < 0.5 else "") + line[pos:]
        parts.append(line)
        total += len(line) + 1
    return ("\n".join(parts) + "\n").encode()


# ---------------------------------------------------------------- corpus
class Corpus:
    """A packed corpus: data (uint8, padded by 64 bytes), offsets (uint64),
    paths (list of str), plus what was planted (for reporting only)."""

    def __init__(self, data, offsets, paths, planted, near_miss):
        self.data, self.offsets, self.paths = data, offsets, paths
        self.planted, self.near_miss = planted, near_miss

    @property
    def nbytes(self):
        return int(self.offsets[-1])

    def file(self, i):
        return bytes(self.data[int(self.offsets[i]):int(self.offsets[i + 1])])

    def subset(self, idx):
        """A new Corpus with files idx (copies)."""
        lens = [int(self.offsets[i + 1] - self.offsets[i]) for i in idx]
        off = np.zeros(len(idx) + 1, dtype=np.uint64)
        np.cumsum(np.array(lens, dtype=np.uint64), out=off[1:])
        data = np.zeros(int(off[-1]) + 64, dtype=np.uint8)
        for j, i in enumerate(idx):
            data[int(off[j]):int(off[j + 1])] = self.data[int(self.offsets[i]):int(self.offsets[i + 1])]
        return Corpus(data, off, [self.paths[i] for i in idx], 0, 0)


def _sizes(kind, n_or_bytes, rng):
    sizes = []
    total = 0
    while total < n_or_bytes:
        if kind == "lognormal":          # config 1: median 16 KB, sigma 1.2, clip [16 B, 8 MB]
            s = int(min(max(rng.lognormvariate(np.log(16384), 1.2), 16), 8 << 20))
        elif kind == "loguniform":       # config 2: [64 B, 64 MB]
            s = int(np.exp(rng.uniform(np.log(64), np.log(64 << 20))))
        elif kind == "tiny":             # offset-table stress: ~300 B files
            s = int(min(max(rng.lognormvariate(np.log(200), 1.0), 1), 64 << 10))
        elif kind == "one":              # K1 probes: the whole batch as one file (no file boundaries)
            s = n_or_bytes
        else:                            # small files (config 3): mean ~25 KB
            s = int(min(max(rng.lognormvariate(np.log(9000), 1.3), 16), 4 << 20))
        s = min(s, n_or_bytes - total) if n_or_bytes - total > 16 else s
        sizes.append(max(s, 1))
        total += sizes[-1]
    return sizes


IMAGE_DIRS = ("usr/share/doc/pkg%d", "usr/lib/python3.%d/site-packages/mod", "usr/local/lib/python3.%d/dist",
              "usr/local/go/src/p%d", "etc/app%d", "opt/app%d/src", "var/lib/app%d", "home/user%d/app",
              "srv/www%d", "root/.config/tool%d", "usr/src/wordpress/wp%d", "opt/yarn-v1.%d/lib")


def generate(total_bytes, seed=DEFAULT_SEED, sizes="lognormal", plant_rate=1e-4, near_miss=0.1,
             base_bytes=32 << 20, max_files=None, layout="src", alloc=None, progress=None):
    """A seeded Corpus of ~total_bytes.  `alloc(n)` (optional) returns the
    uint8 array of n bytes the corpus is written into -- e.g. a view of pinned
    host memory, so a bench holds one copy of its batch instead of two.
    `progress(i, nfiles)` (optional) is called every 200k files."""
    rng = random.Random(seed)
    samples = load_samples()
    rule_ids = sorted(k for k, v in samples.items() if v)
    base = np.frombuffer(base_text(min(base_bytes, max(total_bytes, 1 << 20)), seed ^ 0x5EED), dtype=np.uint8)
    nl_pos = np.flatnonzero(base == 10)
    sz = _sizes(sizes, total_bytes, rng)
    if max_files:
        sz = sz[:max_files]
    n = len(sz)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(np.array(sz, dtype=np.uint64), out=offsets[1:])
    total = int(offsets[-1])
    if alloc is None:
        data = np.zeros(total + 64, dtype=np.uint8)
    else:
        data = alloc(total + 64)
        data[total:] = 0
    paths = []
    seg = 1 << 16
    B = len(base)
    for i, s in enumerate(sz):
        if progress is not None and i and i % 200000 == 0:
            progress(i, n)
        o = int(offsets[i])
        filled = 0
        while filled < s:
            take = min(seg, s - filled)
            # start just after a random newline so files begin at a line
            st = int(nl_pos[rng.randrange(len(nl_pos))]) + 1
            take = min(take, B - st)
            if take <= 0:
                continue
            data[o + filled:o + filled + take] = base[st:st + take]
            filled += take
        if layout == "image":
            # extracted-layer layout (config 3): rootfs dirs, some under the
            # builtin allow-paths; image scans prefix "/" (analyzer secret.go:133-135)
            d1 = rng.choice(IMAGE_DIRS) % rng.randrange(10)
            paths.append("%s%s/%s_%d.%s" % ("/" if rng.random() < 0.5 else "", d1, rng.choice(WORDS), i,
                                            rng.choice(EXTS)))
        else:
            d1 = rng.choice(("src", "lib", "pkg", "app", "internal", "cmd", "deploy", "config", "scripts"))
            paths.append("%s/%s_%d/%s_%d.%s" % (d1, rng.choice(WORDS), rng.randrange(100), rng.choice(WORDS), i,
                                                rng.choice(EXTS)))
    # plants: ~plant_rate of lines (40 B mean line) -> one per 40/plant_rate bytes
    n_plants = max(1, int(total / 40 * plant_rate))
    planted = nmiss = 0
    for _ in range(n_plants):
        f = rng.randrange(n)
        fo, fs = int(offsets[f]), int(offsets[f + 1] - offsets[f])
        rid = rule_ids[rng.randrange(len(rule_ids))]
        sec = rng.choice(samples[rid])
        if rng.random() < near_miss:
            cut = max(1, len(sec) - rng.randint(1, 4))
            sec = sec[:cut]
            nmiss += 1
        else:
            planted += 1
        ctx = rng.choice(("%s", "export X=%s", "  token: %s", 'val = "%s"', "%s ;", "cfg[\"k\"] = '%s'"))
        line = ("\n" + (ctx % sec) + "\n").encode()
        if len(line) >= fs:
            continue
        p = fo + rng.randrange(fs - len(line) + 1)
        data[p:p + len(line)] = np.frombuffer(line, dtype=np.uint8)
    # non-ASCII files: 0.1% with UTF-8 incl. fold-special runes, 0.05% invalid UTF-8
    specials = ["K", "ſ", "İ", "é", "—", "日本語", "ß", "Ω"]
    for f in range(n):
        r = rng.random()
        fo, fs = int(offsets[f]), int(offsets[f + 1] - offsets[f])
        if r < 0.001 and fs > 32:
            for _ in range(1 + fs // 4096):
                t = rng.choice(specials).encode()
                p = fo + rng.randrange(fs - len(t) + 1)
                data[p:p + len(t)] = np.frombuffer(t, dtype=np.uint8)
        elif r < 0.0015 and fs > 8:
            for _ in range(1 + fs // 8192):
                p = fo + rng.randrange(fs)
                data[p] = rng.choice((0x80, 0xC3, 0xE2, 0xFF, 0xED))
    return Corpus(data, offsets, paths, planted, nmiss)


# ------------------------------------------------------------ config 5
EXCLUDE_BLOCKS = [
    r"--- ignore block start ---(.|\s)*--- ignore block stop ---",   # scanner_test exclude-block.yaml
    r"(?s)BEGIN NOSCAN.*?END NOSCAN",
    r"#\s*nosec-block-\d+[^\n]*",
    r"<<<SKIP>>>[^<]*<<<ENDSKIP>>>",
    r"(?m)^# vault: .*$",
]


def _vendor_names(n, rng):
    cons, vows = "bcdfghjklmnprstvwxz", "aeiou"
    out, seen = [], set()
    while len(out) < n:
        k = rng.randint(3, 5)
        v = "".join(rng.choice(cons) + rng.choice(vows) for _ in range(k))[:rng.randint(5, 9)]
        if v in seen or "example" in v:
            continue
        seen.add(v)
        out.append(v)
    return out


def config5(n_rules=500, seed=DEFAULT_SEED, n_allow=20):
    """trivy-secret.yaml of BASELINE.json configs[4]:
    n_rules custom rules from the builtin templates (vendor key=value form and
    prefix-token form), 10% without keywords, severities needing
    normalisation, some per-rule allow-rules / exclude-blocks / paths; plus
    n_allow global allow rules (path and regex) and 5 global exclude blocks.
    Builtins stay enabled.  Returns (config dict in the YAML schema of
    scanner.go:29-43, plant descriptors for plant_custom)."""
    rng = random.Random(seed ^ 0xC0F5)
    names = _vendor_names(n_rules, rng)
    sev = ["HIGH", "critical", "Medium", "low", "UNKNOWN", "severe", ""]
    rules, plants = [], []
    for i, v in enumerate(names):
        n = rng.randint(16, 40)
        r = {"id": "custom-%s" % v, "category": "Custom%d" % (i % 7), "title": "%s secret" % v.capitalize(),
             "severity": rng.choice(sev)}
        if i % 10 < 6:
            r["regex"] = (r"(?i)(?P<key>%s[a-z0-9_ .\-,]{0,25})(=|>|:=|\|\|:|<=|=>|:).{0,5}['\"]"
                          r"(?P<secret>[a-z0-9]{%d})['\"]" % (v, n))
            r["secret-group-name"] = "secret"
            kind = "kv"
        else:
            p = v[:4] + "_" + rng.choice(("pat", "tok", "live", "sk"))
            if i % 3 == 0:
                r["regex"] = r"(^|[^0-9a-zA-Z])(?P<secret>%s_[A-Za-z0-9]{%d})($|[^0-9a-zA-Z])" % (p, n)
                r["secret-group-name"] = "secret"
            else:
                r["regex"] = r"%s_[A-Za-z0-9]{%d}" % (p, n)
            kind = "tok"
            v = p
        if i % 10 != 9:                                  # 10% have no keywords: gate always true
            r["keywords"] = [v if i % 4 else v.upper()]
        if i % 25 == 3:
            r["allow-rules"] = [{"id": "allow-%d" % i, "description": "dummy values", "regex": "(?i)dummy"}]
        if i % 40 == 5:
            r["exclude-block"] = {"description": "rule block", "regexes": [r"(?s)<%s-ignore>.*?</%s-ignore>" % (v, v)]}
        if i % 50 == 7:
            r["path"] = r"\.(env|conf|ini|yaml)$"
        rules.append(r)
        plants.append((kind, v, n))
    allow = []
    for k in range(n_allow):
        if k % 2 == 0:
            allow.append({"id": "global-path-%d" % k, "description": "fixture dirs", "path": r"/fixtures_%d/" % k})
        else:
            allow.append({"id": "global-rx-%d" % k, "description": "placeholders", "regex": r"(?i)notasecret%02d" % k})
    cfg = {"rules": rules, "allow-rules": allow,
           "exclude-block": {"description": "global exclude blocks", "regexes": list(EXCLUDE_BLOCKS)}}
    return cfg, plants


def plant_custom(corpus, plants, seed=DEFAULT_SEED, rate=1e-4):
    """Overwrite whole lines of `corpus` (in place) with strings matching the
    config5() rules, some inside exclude blocks or carrying allow-rule text;
    moves ~1% of files under allow-listed fixtures_k/ dirs and ~2% to .env."""
    rng = random.Random(seed ^ 0x9A47)
    n = len(corpus.paths)
    alnum_lo = "abcdefghijklmnopqrstuvwxyz0123456789"
    alnum = alnum_lo + "ABCDEFGHIJKLMNOPQRSTUVWXYZ"
    n_plants = max(1, int(corpus.nbytes / 40 * rate))
    placed = 0
    for _ in range(n_plants):
        kind, v, nlen = plants[rng.randrange(len(plants))]
        if kind == "kv":
            name = "".join(c.upper() if rng.random() < 0.3 else c for c in v)
            sec = "".join(rng.choice(alnum_lo) for _ in range(nlen))
            op = rng.choice(("=", ": ", ":=", "=>", None))
            if op is None:
                s = '%s_api_key = "%s"' % (name, sec)
            else:
                s = "%s%s%s'%s'" % (name, rng.choice(("_key", "_token", " secret", "")), op, sec)
        else:
            s = "%s_%s" % (v, "".join(rng.choice(alnum) for _ in range(nlen)))
        r = rng.random()
        if r < 0.05:
            s = s + " # dummy"                                   # per-rule allow (some rules)
        elif r < 0.10:
            s = s + " notasecret%02d" % rng.choice((1, 3, 5))   # global allow regex
        elif r < 0.15:
            s = "--- ignore block start ---\n%s\n--- ignore block stop ---" % s
        elif r < 0.18:
            s = "BEGIN NOSCAN %s END NOSCAN" % s
        elif r < 0.20:
            s = "<%s-ignore>\n%s\n</%s-ignore>" % (v, s, v)
        elif r < 0.22:
            s = "# vault: " + s
        line = ("\n" + s + "\n").encode()
        f = rng.randrange(n)
        fo, fs = int(corpus.offsets[f]), int(corpus.offsets[f + 1] - corpus.offsets[f])
        if len(line) >= fs:
            continue
        p = fo + rng.randrange(fs - len(line) + 1)
        corpus.data[p:p + len(line)] = np.frombuffer(line, dtype=np.uint8)
        placed += 1
    for f in range(n):
        r = rng.random()
        if r < 0.01:
            corpus.paths[f] = "repo/fixtures_%d/%s" % (2 * rng.randrange(10), corpus.paths[f])
        elif r < 0.03:
            corpus.paths[f] = corpus.paths[f].rsplit(".", 1)[0] + ".env"
    return placed


def write_yaml(cfg, path):
    import yaml
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False, allow_unicode=False, width=1 << 20)
