"""TEST INFRASTRUCTURE ONLY (never imported by the product path): a restatement
of walker.LayerTar.Walk (pkg/fanal/walker/tar.go:35-119) on Python's own tar
reader (stdlib `tarfile`, an implementation independent of the C++ one), with
utils.CleanSkipPaths / utils.SkipPath (pkg/fanal/utils/utils.go:88-109) and
doublestar v4 Match (github.com/bmatcuk/doublestar/v4, absent here) restated
as a regex translation of its syntax: '*' (no '/'), '**' path segments, '?',
'[...]' with '!'/'^' negation, '{a,b}', '\\' escapes.

Returns what Walk returns plus the files it hands to the analyzers:
  walk(tar_bytes, skip_files, skip_dirs) -> (files [(path, content)], opq_dirs, wh_files)
"""
import io
import posixpath
import re
import tarfile


def _glob_comp(p):
    out, i = "", 0
    while i < len(p):
        c = p[i]
        if c == "*":
            while i < len(p) and p[i] == "*":
                i += 1
            out += "[^/]*"
            continue
        if c == "?":
            out += "[^/]"
        elif c == "[":
            j = i + 1
            neg = j < len(p) and p[j] in "!^"
            if neg:
                j += 1
            k = j
            if k < len(p) and p[k] == "]":
                k += 1
            while k < len(p) and p[k] != "]":
                k += 2 if p[k] == "\\" else 1
            if k >= len(p):
                raise ValueError("bad pattern")
            body = p[j:k].replace("\\", "\\\\")
            out += "[" + ("^" if neg else "") + body + "]"
            i = k
        elif c == "\\":
            i += 1
            if i >= len(p):
                raise ValueError("bad pattern")
            out += re.escape(p[i])
        else:
            out += re.escape(c)
        i += 1
    return out


def _expand(p):
    depth, start = 0, None
    i = 0
    while i < len(p):
        if p[i] == "\\":
            i += 2
            continue
        if p[i] == "{":
            if depth == 0:
                start = i
            depth += 1
        elif p[i] == "}" and depth:
            depth -= 1
            if depth == 0:
                body, alts, d, b = p[start + 1:i], [], 0, 0
                for k, ch in enumerate(body):
                    if ch == "{":
                        d += 1
                    elif ch == "}":
                        d -= 1
                    elif ch == "," and d == 0:
                        alts.append(body[b:k])
                        b = k + 1
                alts.append(body[b:])
                return [x for a in alts for x in _expand(p[:start] + a + p[i + 1:])]
        i += 1
    if depth:
        raise ValueError("bad pattern")
    return [p]


def doublestar_match(pattern, name):
    try:
        for alt in _expand(pattern):
            comps = alt.split("/")
            rx = ""
            for k, c in enumerate(comps):
                last = k == len(comps) - 1
                if c == "**":
                    rx += "(?:[^/]*(?:/[^/]*)*/)?" if not last else "(?:[^/]*(?:/[^/]*)*)?"
                    if last and rx.endswith(")?") and k > 0:
                        # "a/**" also matches "a" itself: drop the separator before it
                        rx = rx[:-len("(?:[^/]*(?:/[^/]*)*)?")]
                        rx = rx[:-1] if rx.endswith("/") else rx
                        rx += "(?:/.*)?"
                    continue
                rx += _glob_comp(c) + ("" if last else "/")
            if re.fullmatch(rx, name, re.S):
                return True
        return False
    except ValueError:
        return False


def clean_skip_paths(paths):
    return [posixpath.normpath(p).lstrip("/") if p else "." for p in paths]


def skip_path(path, patterns):
    path = path.lstrip("/")
    return any(doublestar_match(p, path) for p in patterns)


def _go_clean(p):
    if p == "":
        return "."
    c = posixpath.normpath(p)
    if c.startswith("//"):
        c = "/" + c.lstrip("/")
    return c


def walk(tar_bytes, skip_files=(), skip_dirs=()):
    skip_files, skip_dirs = clean_skip_paths(skip_files), clean_skip_paths(skip_dirs)
    files, opq, wh, skipped = [], [], [], []
    with tarfile.open(fileobj=io.BytesIO(tar_bytes), mode="r:") as tf:
        for m in tf:
            file_path = _go_clean(m.name).lstrip("/")
            d, name = posixpath.split(file_path)
            d = d + "/" if d else ""
            if name == ".wh..wh..opq":
                opq.append(d)
                continue
            if name.startswith(".wh."):
                wh.append(_go_clean(posixpath.join(d, name[4:])))
                continue
            if m.isdir():
                if skip_path(file_path, skip_dirs):
                    skipped.append(file_path)
                continue
            if not (m.isreg() and m.type in (tarfile.REGTYPE, tarfile.AREGTYPE)):
                continue
            if skip_path(file_path, skip_files):
                continue
            if any(file_path == s or file_path.startswith(s + "/") or s == "." for s in skipped):
                continue
            files.append((file_path, tf.extractfile(m).read()))
    return files, opq, wh


# ------------------------------------------------------------ walker.FS.Walk
def build_skip_paths(base, paths):
    """walker.FS.BuildSkipPaths (pkg/fanal/walker/fs.go:99-149) + CleanSkipPaths."""
    import os
    abs_base = os.path.abspath(base)
    out = []
    for p in paths:
        rel = os.path.relpath(os.path.abspath(p), abs_base)
        if not os.path.isabs(p) and rel.startswith(".."):
            r = p                                            # #1: as given
        else:
            r = rel                                          # #2, #3
        out.append(r)
    return clean_skip_paths(out)


DEFAULT_SKIP_DIRS = ["**/.git", "proc", "sys", "dev"]        # walker/walk.go:11-16


def walk_fs(root, skip_files=(), skip_dirs=()):
    """walker.FS.Walk (fs.go:25-97) on Python's os.scandir: filepath.WalkDir's
    lexical order, directories entered as met, symlinks not followed,
    permission errors ignored.  Returns [(rel_path, abs_path)] of the regular
    files handed to the WalkFunc."""
    import os
    sf = build_skip_paths(root, skip_files)
    sd = build_skip_paths(root, skip_dirs) + DEFAULT_SKIP_DIRS
    out = []

    def rec(path, rel):
        try:
            ents = sorted(os.scandir(path), key=lambda e: os.fsencode(e.name))
        except PermissionError:
            return
        for e in ents:
            crel = e.name if rel == "." else rel + "/" + e.name
            if e.is_dir(follow_symlinks=False):
                if skip_path(crel, sd):
                    continue
                rec(e.path, crel)
            elif e.is_file(follow_symlinks=False):
                if skip_path(crel, sf):
                    continue
                out.append((crel, e.path))
    if os.path.isdir(root) and not os.path.islink(root):
        if not skip_path(".", sd):
            rec(root, ".")
    elif os.path.isfile(root) and not os.path.islink(root) and not skip_path(".", sf):
        out.append((".", root))
    return out


def fs_feed(analyzer, root, skip_files=(), skip_dirs=(), file_patterns=()):
    """`trivy fs ROOT` up to Scan: walk, AnalyzeFile's gate (analyzer.go:403-419:
    a "secret:<re>" --file-patterns match or Required on the path with leading
    '/' trimmed), Analyze's binary check / CR strip / printable extraction.
    analyzer: an oracle.secret_oracle.SecretAnalyzer.  Returns
    [(FilePath, Content, Binary)] in walk order."""
    import os
    from .goregex import GoRegexp
    from . import secret_oracle as so
    pats = []
    for p in file_patterns:
        typ, sep, rx = p.partition(":")
        if not sep:
            raise ValueError("invalid file pattern (%s)" % p)
        r = GoRegexp(rx)
        if typ == "secret":
            pats.append(r)
    out = []
    for rel, path in walk_fs(root, skip_files, skip_dirs):
        clean = rel.lstrip("/")
        size = os.lstat(path).st_size
        if not any(r.match_string(clean) for r in pats) and not analyzer.required(clean, size):
            continue
        raw = open(path, "rb").read()
        binary = so.is_binary(raw[:300])
        if binary and so.go_ext(rel) != ".pyc":
            continue
        content = so.extract_printable_bytes(raw) if binary else raw.replace(b"\r", b"")
        out.append((rel, content, binary))
    return out
