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


class _Translator:
    def __init__(self, pat):
        self.p = pat
        self.i = 0
        self.names = [""]   # index 0 = whole match
        self.depth = 0

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
        while self.peek() == "|":
            self.i += 1
            alts.append(self.concat(flags))
        return "|".join(alts)

    def concat(self, flags):
        items = []
        while not self.eof() and self.peek() not in "|)":
            atom = self.atom(flags)
            if atom is None:
                continue
            atom = self.repeat(atom, flags)
            items.append(atom)
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
            return self.char_class(flags)
        if c in ("*", "+", "?"):
            raise GoSyntaxError("missing argument to repetition operator in %r" % self.p)
        if c == "{":
            save = self.i
            if self.try_brace() is not None:
                raise GoSyntaxError("missing argument to repetition operator in %r" % self.p)
            self.i = save + 1
            return self.fold_wrap(_lit(ord("{")), flags)
        self.i += 1
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
                        return "(?:%s)" % inner
                    else:
                        raise GoSyntaxError("invalid or unsupported Perl syntax in %r" % self.p)
        # capturing group
        self.names.append(name or "")
        inner = self.alternation(dict(flags))
        if self.peek() != ")":
            raise GoSyntaxError("missing closing ) in %r" % self.p)
        self.i += 1
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

    def __init__(self, pattern):
        self.pattern = pattern
        t = _Translator(pattern)
        self.py_pattern = t.parse()
        self.subexp_names = t.names
        self.rx = regex.compile(self.py_pattern, regex.VERSION0)

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
        lens = np.fromiter((1 if 0xDC80 <= ord(ch) <= 0xDCFF else len(ch.encode("utf-8"))
                            for ch in text), dtype=np.int64, count=len(text))
        offs = np.zeros(len(text) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        return text, offs

    def match_string(self, s):
        if isinstance(s, bytes):
            s = s.decode("utf-8", "surrogateescape")
        return self.rx.search(s) is not None

    def find_all(self, content, prepared=None, submatch=False):
        """Go Regexp.FindAll(Submatch)Index(content, -1) (regexp.go allMatches)."""
        text, offs = prepared if prepared is not None else self.prepare(content)
        end = len(text)
        out = []
        pos, prev_end = 0, -1
        while pos <= end:
            m = self.rx.search(text, pos)
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
