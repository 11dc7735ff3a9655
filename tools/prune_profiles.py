#!/usr/bin/env python
"""List (or git-rm with --apply) the files under profiles/ that nothing cites.

A profile is cited when its file name, or a glob-like stem the docs use
(`rd5h_*`, `r5e_k1_trace_*`), appears in DESIGN.md, README.md,
INTEGRATION.md, bench.py, tests/ or tools/.  traffic_c*.json are read by
bench.py and always kept.

  python tools/prune_profiles.py [--apply]
"""
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cited_text():
    parts = []
    for p in ["DESIGN.md", "README.md", "INTEGRATION.md", "bench.py"] + glob.glob(os.path.join(ROOT, "tests", "*.py")) \
            + glob.glob(os.path.join(ROOT, "tools", "*.py")) + glob.glob(os.path.join(ROOT, "tools", "*.sh")):
        fp = p if os.path.isabs(p) else os.path.join(ROOT, p)
        if os.path.exists(fp):
            parts.append(open(fp, encoding="utf-8", errors="replace").read())
    return "\n".join(parts)


def main():
    text = cited_text()
    # stems written with a trailing * or _ glob in the docs: `rd5h_*`, `r5e_k1_trace_*.txt`
    stems = set(m.group(1) for m in re.finditer(r"([A-Za-z0-9_.]+?)\*", text))
    keep, drop = [], []
    for f in sorted(os.listdir(os.path.join(ROOT, "profiles"))):
        if f.startswith("traffic_c") or f in text or any(f.startswith(st) for st in stems if len(st) >= 4):
            keep.append(f)
        else:
            drop.append(f)
    print("keep %d, drop %d" % (len(keep), len(drop)))
    for f in drop:
        print("  drop", f)
    if "--apply" in sys.argv and drop:
        subprocess.check_call(["git", "rm", "-q"] + [os.path.join("profiles", f) for f in drop], cwd=ROOT)


if __name__ == "__main__":
    main()
