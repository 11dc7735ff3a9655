"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Go `regexp` (RE2 syntax, Perl flags, leftmost-first) restated on top of the
third-party Python `regex` module.  The reference compiles every secret rule
with Go's `regexp.Compile` / `regexp.MustCompile`
(/root/reference/pkg/fanal/secret/scanner.go:66-87), i.e. go1.23.4
`regexp/syntax` with flags `syntax.Perl` (ClassNL|OneLine|PerlX|UnicodeGroups).
Go is absent from this image, so this module translates a Go pattern into an
equivalent `regex` pattern with every flag resolved per atom, so none of the
two libraries' flag-scoping differences can leak in:

  * literal / class under (?i)  -> (?i:...)  (regex's simple case folding folds
    k/K/U+212A and s/S/U+017F exactly like Go's unicode.SimpleFold orbits)
  * .      -> [^\\n]   ( (?s) -> (?s:.) )
  * ^ / $  -> \\A / \\Z     ( (?m) -> (?:(?<=\\n)|\\A) / (?=\\n|\\Z) )
  * \\b \\B  -> ASCII word-boundary lookarounds (Go: \\w = [0-9A-Za-z_])
  * \\d \\s \\w (and negations, [[:posix:]]) -> explicit ASCII classes
    (Go \\s = [\\t\\n\\f\\r ], no \\v)
  * named groups (?P<n>..) / (?<n>..) -> plain groups; names kept in
    `subexp_names` (Go allows duplicate names, scanner.go:155-168 relies on it)
  * an alternation whose alternatives each match exactly one char and hold no
    capture (e.g. `(.|\\s)` of the exclude-block idiom) -> one char class, the
    union of the alternatives' char sets (computed by running each over every
    code point).  Each alternative consumes the same single char, so the union
    matches exactly what the alternation matches; without the rewrite the
    `regex` module backtracks per char and exhausts memory on MB-sized inputs.
    `_Translator(pattern, merge=False)` keeps the literal alternation
    (tests/test_oracle_regex.py checks both translations agree).

Matches that need no submatches (MatchString, FindAllIndex) run on a second
translation with every group non-capturing: the `regex` module records every
iteration of a repeated capturing group, which is what made config 5's
`(.|\\s)*` block scan run out of memory.

Matching runs on `bytes.decode('utf-8', 'surrogateescape')`, so each invalid
byte is one char, like Go's utf8.DecodeRune (RuneError, width 1).  Offsets are
mapped back to bytes.  `find_all` restates Go's `Regexp.allMatches`
(empty match right after the previous match is dropped; an empty match
advances one rune).
"""
import numpy as np
import regex

WORD = "0-9A-Za-z_"
POSIX = {
    "alnum": "0-9A-Za-z", "alpha": "A-Za-z", "ascii": "\\x00-\\x7f", "blank": "\\t ",
    "cntrl": "\\x00-\\x1f\\x7f", "digit": "0-9", "graph": "!-~", "lower": "a-z",
    "print": " -~", "punct": "!-/:-@\\[-`{-~", "space": "\\t\\n\\x0b\\f\\r ",
    "upper": "A-Z", "word": WORD, "xdigit": "0-9A-Fa-f",
}
PERL = {"d": "0-9", "s": "\\t\\n\\f\\r ", "w": WORD}


class GoSyntaxError(ValueError):
    pass


def _lit(cp):
    c = chr(cp)
    if c.isalnum() and cp < 128:
        return c
    return "\\U%08x" % cp


def _cls_lit(cp):
    return "\\U%08x" % cp


_ALL_CHARS = None


def _all_chars():
    """Every char a scanned text can hold: all code points except surrogates,
    plus U+DC80..U+DCFF (invalid bytes under 'surrogateescape')."""
    global _ALL_CHARS
    if _ALL_CHARS is None:
        cps = list(range(0xD800)) + list(range(0xDC80, 0xDD00)) + list(range(0xE000, 0x110000))
        _ALL_CHARS = "".join(map(chr, cps))
    return _ALL_CHARS


_UNION_CACHE = {}


def _char_set(pat):
    """Code points matched by a one-char pattern, or None if it can match
    anything but exactly one char."""
    if pat not in _UNION_CACHE:
        rx = regex.compile(pat, regex.VERSION0)
        if rx.match("") is not None:
            _UNION_CACHE[pat] = None
        else:
            text = _all_chars()
            pts = []
            ok = True
            for m in rx.finditer(text):
                if m.end() - m.start() != 1:
                    ok = False
                    break
                pts.append(ord(text[m.start()]))
            _UNION_CACHE[pat] = set(pts) if ok else None
    return _UNION_CACHE[pat]


def _union_class(alts):
    sets = [_char_set(a) for a in alts]
    if any(x is None for x in sets):
        return None
    cps = sorted(set().union(*sets))
    if not cps:
        return "[^\\x00-\\U0010ffff]"
    ranges = []
    lo = prev = cps[0]
    for c in cps[1:]:
        if c != prev + 1:
            ranges.append((lo, prev))
            lo = c
        prev = c
    ranges.append((lo, prev))
    return "[%s]" % "".join(_cls_lit(a) if a == b else "%s-%s" % (_cls_lit(a), _cls_lit(b)) for a, b in ranges)


class _Translator:
    def __init__(self, pat, merge=True, capture=True):
        self.p = pat
        self.i = 0
        self.names = [""]   # index 0 = whole match
        self.depth = 0
        self.merge = merge       # single-char alternations -> one class
        self.capture = capture   # False: every group non-capturing
        self._single = False     # the last atom / concat / alternation matches exactly one char, no capture

    # ------------------------------------------------------------------ lexing
    def peek(self, k=0):
        j = self.i + k
        return self.p[j] if j < len(self.p) else ""

    def eof(self):
        return self.i >= len(self.p)

    # ---------------------------------------------------------------- grammar
    def parse(self):
        flags = {"i": False, "m": False, "s": False, "U": False}
        out = self.alternation(flags)
        if not self.eof():
            raise GoSyntaxError("unexpected ) at %d in %r" % (self.i, self.p))
        return out

    def alternation(self, flags):
        # Flags set by (?x) persist to the end of the enclosing group,
        # across '|' (Go regexp/syntax parse.go semantics).
        alts = [self.concat(flags)]
        singles = [self._single]
        while self.peek() == "|":
            self.i += 1
            alts.append(self.concat(flags))
            singles.append(self._single)
        if self.merge and len(alts) > 1 and all(singles):
            u = _union_class(alts)
            if u is not None:
                self._single = True
                return u
        self._single = len(alts) == 1 and singles[0]
        return "|".join(alts)

    def concat(self, flags):
        items = []
        single = False
        while not self.eof() and self.peek() not in "|)":
            self._single = False
            atom = self.atom(flags)
            if atom is None:
                continue
            single = self._single
            rep = self.repeat(atom, flags)
            if rep is not atom:
                single = False
            items.append(rep)
        self._single = len(items) == 1 and single
        return "".join(items)

    def repeat(self, atom, flags):
        seen = False
        while True:
            c = self.peek()
            if c in ("*", "+", "?"):
                op = c
                self.i += 1
            elif c == "{":
                save = self.i
                r = self.try_brace()
                if r is None:
                    self.i = save
                    return atom
                lo, hi = r
                if lo > 1000 or (hi is not None and (hi > 1000 or hi < lo)):
                    raise GoSyntaxError("invalid repeat count in %r" % self.p)
                op = "{%d,%s}" % (lo, "" if hi is None else hi) if hi != lo else "{%d}" % lo
            else:
                return atom
            if seen:
                raise GoSyntaxError("invalid nested repetition operator in %r" % self.p)
            seen = True
            lazy = False
            if self.peek() == "?":
                self.i += 1
                lazy = True
            if flags["U"]:
                lazy = not lazy
            atom = "(?:%s)%s%s" % (atom, op, "?" if lazy else "")

    def try_brace(self):
        # '{' digits [ ',' [digits] ] '}'  -- else literal '{'
        j = self.i + 1
        p = self.p
        k = j
        while k < len(p) and p[k].isdigit():
            k += 1
        if k == j:
            return None
        lo = int(p[j:k])
        hi = lo
        if k < len(p) and p[k] == ",":
            k += 1
            m = k
            while m < len(p) and p[m].isdigit():
                m += 1
            hi = int(p[k:m]) if m > k else None
            k = m
        if k >= len(p) or p[k] != "}":
            return None
        self.i = k + 1
        return lo, hi

    def atom(self, flags):
        c = self.peek()
        if c == "(":
            return self.group(flags)
        if c == "[":
            self._single = True
            return self.char_class(flags)
        if c in ("*", "+", "?"):
            raise GoSyntaxError("missing argument to repetition operator in %r" % self.p)
        if c == "{":
            save = self.i
            if self.try_brace() is not None:
                raise GoSyntaxError("missing argument to repetition operator in %r" % self.p)
            self.i = save + 1
            self._single = True
            return self.fold_wrap(_lit(ord("{")), flags)
        self.i += 1
        self._single = c not in "^$"
        if c == ".":
            return "(?s:.)" if flags["s"] else "[^\\n]"
        if c == "^":
            return "(?:(?<=\\n)|\\A)" if flags["m"] else "\\A"
        if c == "$":
            return "(?=\\n|\\Z)" if flags["m"] else "\\Z"
        if c == "\\":
            return self.escape(flags)
        return self.fold_wrap(_lit(ord(c)), flags)

    def fold_wrap(self, s, flags):
        return "(?i:%s)" % s if flags["i"] else s

    def group(self, flags):
        assert self.peek() == "("
        self.i += 1
        name = None
        if self.peek() == "?":
            if self.p.startswith("?P<", self.i) or (self.p.startswith("?<", self.i)
                                                   and self.peek(2) not in ("=", "!")):
                start = self.i + (3 if self.peek(1) == "P" else 2)
                end = self.p.index(">", start)
                name = self.p[start:end]
                if not name or not all(ch.isalnum() or ch == "_" for ch in name):
                    raise GoSyntaxError("invalid named capture in %r" % self.p)
                self.i = end + 1
            else:
                # flags: (?flags) or (?flags:re)
                self.i += 1
                neg = False
                newf = dict(flags)
                while True:
                    ch = self.peek()
                    if ch == "":
                        raise GoSyntaxError("missing closing ) in %r" % self.p)
                    self.i += 1
                    if ch in "imsU":
                        newf[ch] = not neg
                    elif ch == "-":
                        if neg:
                            raise GoSyntaxError("invalid flags in %r" % self.p)
                        neg = True
                    elif ch == ")":
                        flags.update(newf)     # persists to end of group
                        return None
                    elif ch == ":":
                        inner = self.alternation(newf)
                        if self.peek() != ")":
                            raise GoSyntaxError("missing closing ) in %r" % self.p)
                        self.i += 1
                        return "(?:%s)" % inner     # keeps self._single of `inner`
                    else:
                        raise GoSyntaxError("invalid or unsupported Perl syntax in %r" % self.p)
        # capturing group
        self.names.append(name or "")
        inner = self.alternation(dict(flags))
        if self.peek() != ")":
            raise GoSyntaxError("missing closing ) in %r" % self.p)
        self.i += 1
        if not self.capture:
            return "(?:%s)" % inner         # keeps self._single of `inner`
        self._single = False
        return "(%s)" % inner

    # ---------------------------------------------------------------- escapes
    def escape_char(self):
        """Parse a char escape after the backslash; return a code point."""
        c = self.peek()
        if c == "":
            raise GoSyntaxError("trailing backslash in %r" % self.p)
        self.i += 1
        if c in "1234567" and not ("0" <= self.peek() <= "7"):
            # a single non-zero digit is a backreference: unsupported in Go
            raise GoSyntaxError("invalid escape (backreference) in %r" % self.p)
        if c in "01234567":
            digits = c
            while len(digits) < 3 and "0" <= self.peek() <= "7":
                digits += self.peek()
                self.i += 1
            return int(digits, 8)
        if c == "x":
            if self.peek() == "{":
                end = self.p.index("}", self.i)
                v = int(self.p[self.i + 1:end], 16)
                self.i = end + 1
                if v > 0x10FFFF:
                    raise GoSyntaxError("invalid escape in %r" % self.p)
                return v
            h = self.p[self.i:self.i + 2]
            if len(h) != 2:
                raise GoSyntaxError("invalid escape in %r" % self.p)
            self.i += 2
            return int(h, 16)
        simple = {"a": 7, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11}
        if c in simple:
            return simple[c]
        if ord(c) < 128 and not c.isalnum():
            return ord(c)
        raise GoSyntaxError("invalid escape \\%s in %r" % (c, self.p))

    def unicode_class(self, c):
        """\\pX / \\p{Name} / \\PX -> regex syntax (already consumed 'p'/'P')."""
        if self.peek() == "{":
            end = self.p.index("}", self.i)
            name = self.p[self.i + 1:end]
            self.i = end + 1
        else:
            name = self.peek()
            self.i += 1
        neg = c == "P"
        if name.startswith("^"):
            neg = not neg
            name = name[1:]
        if name == "Any":
            body = "\\x00-\\U0010ffff"
            return body, neg
        return ("\\p{%s}" % name), neg

    def escape(self, flags):
        c = self.peek()
        self._single = c not in "AzbBQ"
        if c in "dswDSW":
            self.i += 1
            body = PERL[c.lower()]
            return ("[^%s]" if c.isupper() else "[%s]") % body
        if c in "pP":
            self.i += 1
            body, neg = self.unicode_class(c)
            s = ("[^%s]" if neg else "[%s]") % body
            return self.fold_wrap(s, flags)
        if c == "A":
            self.i += 1
            return "\\A"
        if c == "z":
            self.i += 1
            return "\\Z"
        if c == "b":
            self.i += 1
            return "(?:(?<=[%s])(?![%s])|(?<![%s])(?=[%s]))" % (WORD, WORD, WORD, WORD)
        if c == "B":
            self.i += 1
            return "(?:(?<=[%s])(?=[%s])|(?<![%s])(?![%s]))" % (WORD, WORD, WORD, WORD)
        if c == "Q":
            self.i += 1
            end = self.p.find("\\E", self.i)
            lit = self.p[self.i:] if end < 0 else self.p[self.i:end]
            self.i = len(self.p) if end < 0 else end + 2
            self._single = len(lit) == 1
            return "".join(self.fold_wrap(_lit(ord(ch)), flags) for ch in lit)
        if c == "C":
            raise GoSyntaxError("invalid escape \\C in %r" % self.p)
        return self.fold_wrap(_lit(self.escape_char()), flags)

    def char_class(self, flags):
        assert self.peek() == "["
        self.i += 1
        neg = False
        if self.peek() == "^":
            neg = True
            self.i += 1
        parts = []
        first = True
        while first or self.peek() != "]":
            if self.eof():
                raise GoSyntaxError("missing closing ] in %r" % self.p)
            first = False
            c = self.peek()
            if c == "[" and self.peek(1) == ":":
                end = self.p.find(":]", self.i + 2)
                if end >= 0:
                    name = self.p[self.i + 2:end]
                    pneg = name.startswith("^")
                    if pneg:
                        name = name[1:]
                    if name not in POSIX:
                        raise GoSyntaxError("invalid character class range in %r" % self.p)
                    self.i = end + 2
                    if pneg:
                        parts.append(("neg", POSIX[name]))
                    else:
                        parts.append(("raw", POSIX[name]))
                    continue
            if c == "\\" and self.peek(1) in "dswDSW":
                self.i += 2
                k = self.p[self.i - 1]
                parts.append(("neg" if k.isupper() else "raw", PERL[k.lower()]))
                continue
            if c == "\\" and self.peek(1) in "pP":
                self.i += 2
                body, pneg = self.unicode_class(self.p[self.i - 1])
                parts.append(("neg" if pneg else "raw", body))
                continue
            lo = self.class_char()
            if self.peek() == "-" and self.peek(1) not in ("]", ""):
                self.i += 1
                hi = self.class_char()
                if hi < lo:
                    raise GoSyntaxError("invalid character class range in %r" % self.p)
                parts.append(("raw", "%s-%s" % (_cls_lit(lo), _cls_lit(hi))))
            else:
                parts.append(("raw", _cls_lit(lo)))
        self.i += 1  # ']'
        pos = "".join(b for k, b in parts if k == "raw")
        negs = [b for k, b in parts if k == "neg"]
        # union of positive items and negated sub-classes
        alts = []
        if pos:
            alts.append("[%s]" % pos)
        for b in negs:
            alts.append("[^%s]" % b)
        if not alts:
            s = "[^\\x00-\\U0010ffff]" if not neg else "(?s:.)"
            return s
        union = alts[0] if len(alts) == 1 else "(?:%s)" % "|".join(alts)
        if neg:
            # any char (incl. \n: Go ClassNL) that is not in the union
            s = "(?:(?!%s)(?s:.))" % union
        else:
            s = union
        return self.fold_wrap(s, flags)

    def class_char(self):
        c = self.peek()
        if c == "\\":
            self.i += 1
            return self.escape_char()
        self.i += 1
        return ord(c)


class GoRegexp:
    """A compiled Go regexp (oracle restatement)."""

    def __init__(self, pattern, merge=True):
        self.pattern = pattern
        t = _Translator(pattern, merge=merge)
        self.py_pattern = t.parse()
        self.subexp_names = t.names
        self.rx = regex.compile(self.py_pattern, regex.VERSION0)
        # no-capture translation for matches whose submatches are not wanted
        self.py_pattern_nocap = _Translator(pattern, merge=merge, capture=False).parse()
        self.rx_nocap = regex.compile(self.py_pattern_nocap, regex.VERSION0)

    # -- helpers on (text, byte-offset map)
    @staticmethod
    def prepare(content):
        """bytes -> (str, char->byte offset array or None if ASCII)."""
        try:
            text = content.decode("ascii")
            return text, None
        except UnicodeDecodeError:
            pass
        text = content.decode("utf-8", "surrogateescape")
        # UTF-8 length of each char; an escaped invalid byte (U+DC80-U+DCFF) is 1
        cp = np.frombuffer(text.encode("utf-32-le", "surrogatepass"), dtype=np.uint32)
        lens = np.where(cp < 0x80, 1, np.where(cp < 0x800, 2, np.where(cp < 0x10000, 3, 4))).astype(np.int64)
        lens[(cp >= 0xDC80) & (cp <= 0xDCFF)] = 1
        offs = np.zeros(len(text) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        return text, offs

    def match_string(self, s):
        if isinstance(s, bytes):
            s = s.decode("utf-8", "surrogateescape")
        return self.rx_nocap.search(s) is not None

    def find_all(self, content, prepared=None, submatch=False):
        """Go Regexp.FindAll(Submatch)Index(content, -1) (regexp.go allMatches)."""
        text, offs = prepared if prepared is not None else self.prepare(content)
        end = len(text)
        out = []
        pos, prev_end = 0, -1
        rx = self.rx if submatch else self.rx_nocap
        while pos <= end:
            m = rx.search(text, pos)
            if m is None:
                break
            accept = True
            if m.end() == pos:
                if m.start() == prev_end:
                    accept = False
                pos = pos + 1 if pos < end else end + 1
            else:
                pos = m.end()
            prev_end = m.end()
            if accept:
                if submatch:
                    spans = []
                    for g in range(len(self.subexp_names)):
                        a, b = m.span(g)
                        spans += [a, b]
                else:
                    spans = [m.start(), m.end()]
                if offs is not None:
                    spans = [int(offs[x]) if x >= 0 else -1 for x in spans]
                out.append(spans)
        return out
