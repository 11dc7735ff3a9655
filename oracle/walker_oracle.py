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
