#!/usr/bin/env python
"""GPU timeline from a rocprofv3 database (--kernel-trace, optionally
--memory-copy-trace): every kernel dispatch and copy in start order with its
start relative to the window's first op, its duration and the gap since the
previous op ended -- to see where a small batch's wall time goes between
the GPU passes.

  python tools/prof_timeline.py <results.db> [--last N] [--from-kernel NAME]
"""
import argparse
import re
import sqlite3


def short(name):
    m = re.search(r"(tsg_[a-z0-9_]+|__amd_rocclr_[A-Za-z]+|at::native::[A-Za-z_]+)", name or "")
    return m.group(1) if m else (name or "")[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=40, help="ops shown (the last N)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ops = [(s, e, short(n), "q%s" % q) for s, e, n, q in c.execute("select start, end, name, queue_id from kernels")]
    try:
        ops += [(s, e, "copy %s %dB" % (n, sz), "copy") for s, e, n, sz in
                c.execute("select start, end, name, size from memory_copies")]
    except sqlite3.OperationalError:
        pass
    ops.sort()
    ops = ops[-a.last:]
    t0 = ops[0][0]
    prev_end = t0
    print("%10s %9s %9s  %-6s %s" % ("start_us", "dur_us", "gap_us", "queue", "op"))
    for s, e, n, q in ops:
        print("%10.1f %9.1f %9.1f  %-6s %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev_end) / 1e3, q, n))
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
