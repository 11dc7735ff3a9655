"""Kernel statistics from a rocprofv3 database (rocpd .db, the default output
format of ROCm 7.2's rocprofv3): per kernel name the call count, total and
mean duration, plus every K1 dispatch's duration in launch order, so a bench
line's HIP-event K1 figures can be checked against the profiler's.

  python tools/prof_db_summary.py gpurun_out/<run>/prof/<name>_results.db > profiles/<round>_kernel_stats.txt
"""
import collections
import re
import sqlite3
import sys


def short(name):
    m = re.search(r"(tsg_[a-z0-9_]+(?:<[^>]*>)?|__amd_rocclr_[A-Za-z]+|at::native::[A-Za-z_]+)", name)
    return m.group(1) if m else name[:60]


def main(path):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count from kernels order by start"))
    agg = collections.OrderedDict()
    for name, s, e, gx, wx, lds, vg in rows:
        k = short(name)
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    print("%-40s %6s %12s %10s %6s" % ("kernel", "calls", "total_us", "mean_us", "pct"))
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-40s %6d %12.1f %10.2f %6.2f" % (k, n, t, t / n, 100 * t / tot))
    # (rocprofv3's vgpr_count is not the allocated count -- it read 64 for K1,
    # whose build allocates 118-128: tools/kernel_resources.py has the
    # compiler's figures -- so no register column here)
    print("\nK1 dispatches in launch order (us; grid x workgroup, LDS bytes):")
    for name, s, e, gx, wx, lds, vg in rows:
        if "tsg_k1_scan" in name:
            print("  %10.1f   %d x %d  lds %d" % ((e - s) / 1e3, gx // max(wx, 1), wx, lds))


if __name__ == "__main__":
    main(sys.argv[1])
