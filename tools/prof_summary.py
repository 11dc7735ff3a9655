"""Kernel-trace summary (rocprofv3 --kernel-trace --stats) from a rocpd SQLite
database or from a *_kernel_stats.csv, written as the CSV that rocprofv3's
csv output uses (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs,
MaxNs, StdDev), plus one line per K1/K2 dispatch (grid, LDS).  Register
counts are not printed: rocprofv3's vgpr_count is not the allocated count
(it read 64 for K1, whose build allocates 118-128); the compiler's figures are
in tools/kernel_resources.py's output.

  python tools/prof_summary.py gpurun_out/<run>/prof/run_results.db > profiles/<round>_kernel_stats.csv
"""
import csv
import math
import re
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, duration, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count from kernels").fetchall()
    by = {}
    for name, dur, gx, wx, lds, vgpr, sgpr in rows:
        by.setdefault(name, []).append((dur, gx, wx, lds, vgpr, sgpr))
    total = sum(d for v in by.values() for d, *_ in v)
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(by.items(), key=lambda kv: -sum(d for d, *_ in kv[1])):
        ds = [d for d, *_ in v]
        avg = sum(ds) / len(ds)
        sd = math.sqrt(sum((d - avg) ** 2 for d in ds) / len(ds))
        w.writerow([name, len(ds), sum(ds), avg, 100.0 * sum(ds) / total, min(ds), max(ds), sd])
    print()
    print("# per dispatch of the scan kernels: duration_ns, grid_x, workgroup_x, lds_bytes")
    for name, v in by.items():
        if "tsg_k" not in name:
            continue
        short = re.search(r"(tsg_k\w+(<\w+>)?)", name).group(1)
        for d in v:
            print("# %s %d %d %d %d" % ((short,) + tuple(d[:4])))


if __name__ == "__main__":
    from_db(sys.argv[1])
