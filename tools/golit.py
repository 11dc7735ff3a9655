"""Tiny reader for the Go composite literals that hold the reference's rule data
and unit-test expectations.

Dev-time only: the generators in tools/ and tests/golden/ use it to turn
`/root/reference/pkg/fanal/secret/builtin-rules.go` (rule DATA) and
`scanner_test.go` (expected findings) into JSON committed in this repo.  Nothing
at run time imports it, and nothing on the GPU box reads /root/reference.

Supported: identifiers (dotted), interpreted "..." and raw `...` strings, ints,
true/false/nil, `T{...}` composite literals (keyed or positional), function
calls `f(a, b)`, and `+` string concatenation.
"""
import re

_TOKEN = re.compile(r"""
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/)
  | (?P<raw>`[^`]*`)
  | (?P<str>"(?:\\.|[^"\\\n])*")
  | (?P<chr>'(?:\\.|[^'\\\n])+')
  | (?P<num>-?\d+)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z_][A-Za-z0-9_]*)*)
  | (?P<op>:=|\[\]|[{}()\[\],:+*&=])
  | (?P<other>.)
""", re.X | re.S)


def tokenize(src):
    out = []
    pos = 0
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m:
            raise ValueError("golit: cannot tokenize at %r" % src[pos:pos + 40])
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        if kind == "other":
            kind = "op"
        out.append((kind, m.group(kind)))
    return out


def go_unquote(tok):
    """Decode a Go interpreted string literal body (without quotes) to str."""
    body = tok[1:-1]
    res = []
    i = 0
    simple = {"a": "\a", "b": "\b", "f": "\f", "n": "\n", "r": "\r",
              "t": "\t", "v": "\v", "\\": "\\", '"': '"', "'": "'"}
    raw = bytearray()

    def flush():
        if raw:
            res.append(raw.decode("utf-8", "surrogateescape"))
            raw.clear()
    while i < len(body):
        c = body[i]
        if c != "\\":
            flush()
            res.append(c)
            i += 1
            continue
        n = body[i + 1]
        if n in simple:
            flush()
            res.append(simple[n])
            i += 2
        elif n == "x":
            raw.append(int(body[i + 2:i + 4], 16))
            i += 4
        elif n in "01234567":
            raw.append(int(body[i + 1:i + 4], 8))
            i += 4
        elif n == "u":
            flush()
            res.append(chr(int(body[i + 2:i + 6], 16)))
            i += 6
        elif n == "U":
            flush()
            res.append(chr(int(body[i + 2:i + 10], 16)))
            i += 10
        else:
            raise ValueError("golit: bad escape \\%s" % n)
    flush()
    return "".join(res)


class Call:
    def __init__(self, fn, args):
        self.fn, self.args = fn, args

    def __repr__(self):
        return "Call(%s, %r)" % (self.fn, self.args)


class Ident:
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return "Ident(%s)" % self.name


class Composite:
    def __init__(self, typ, keyed, items):
        self.typ, self.keyed, self.items = typ, keyed, items

    def get(self, key, default=None):
        return self.keyed.get(key, default)

    def __repr__(self):
        return "Composite(%s, %r, %r)" % (self.typ, self.keyed, self.items)


class Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else (None, None)

    def take(self, val=None):
        tok = self.t[self.i]
        if val is not None and tok[1] != val:
            raise ValueError("golit: expected %r got %r" % (val, tok))
        self.i += 1
        return tok

    def parse_type(self):
        # []T, []*T, T, pkg.T
        s = ""
        while self.peek()[1] in ("[]", "*", "&"):
            s += self.take()[1]
        s += self.take()[1]
        return s

    def parse_expr(self):
        left = self.parse_unary()
        while self.peek()[1] == "+":
            self.take()
            right = self.parse_unary()
            left = ("+", left, right)
        return left

    def parse_unary(self):
        kind, val = self.peek()
        if kind == "raw":
            self.take()
            return val[1:-1]
        if kind == "str":
            self.take()
            return go_unquote(val)
        if kind == "num":
            self.take()
            return int(val)
        if val in ("[]", "&"):
            typ = self.parse_type()
            return self.parse_composite(typ)
        if val == "{":
            return self.parse_composite(None)
        if kind == "ident":
            self.take()
            if val in ("true", "false"):
                return val == "true"
            if val == "nil":
                return None
            nk = self.peek()[1]
            if nk == "(":
                self.take("(")
                args = []
                while self.peek()[1] != ")":
                    args.append(self.parse_expr())
                    if self.peek()[1] == ",":
                        self.take()
                self.take(")")
                return Call(val, args)
            if nk == "{":
                return self.parse_composite(val)
            return Ident(val)
        raise ValueError("golit: unexpected %r" % (self.peek(),))

    def parse_composite(self, typ):
        self.take("{")
        keyed, items = {}, []
        while self.peek()[1] != "}":
            if self.peek()[0] == "ident" and self.peek(1)[1] == ":":
                key = self.take()[1]
                self.take(":")
                keyed[key] = self.parse_expr()
            else:
                items.append(self.parse_expr())
            if self.peek()[1] == ",":
                self.take()
        self.take("}")
        return Composite(typ, keyed, items)


def parse_expr_at(src, start):
    """Parse one expression starting at character offset `start` of `src`."""
    p = Parser(tokenize(src[start:]))
    return p.parse_expr()


def find_block(src, header):
    """Offset just after `header` (e.g. 'var builtinRules = ')."""
    i = src.index(header)
    return i + len(header)
