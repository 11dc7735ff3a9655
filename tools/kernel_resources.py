#!/usr/bin/env python
"""The compiler's register / scratch / occupancy report for every kernel of
the product library's HIP sources (hipcc -Rpass-analysis=kernel-resource-usage,
gfx950, the build's flags): the allocated VGPR / SGPR counts, spills, scratch
bytes per lane, occupancy and static LDS.  rocprofv3's vgpr_count column is
not the allocated count; DESIGN.md section 4 cites this table.

  python tools/kernel_resources.py [--probe] > profiles/<round>_kernel_resources.txt
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "trivy_amd", "csrc")


def demangle_short(name):
    m = re.search(r"_GLOBAL__N_1\d+(tsg_\w+?)(I.*)?E*v?P", name) or re.search(r"(tsg_\w+)", name)
    base = m.group(1) if m else name
    base = re.sub(r"ENS0_.*$", "", base)
    t = re.search(r"ILi(\d+)ELi(\d+)ELb([01])E", name)
    if t:
        base += "<%s,%s,%s>" % (t.group(1), t.group(2), "true" if t.group(3) == "1" else "false")
    t = re.search(r"verifyIL[bi](\d+)E", name)
    if t:
        base += "<%s>" % t.group(1)
    return base


def main():
    probe = "--probe" in sys.argv
    rows = []
    for src in ("engine.hip", "crstrip.hip"):
        cmd = ["hipcc", "-c", os.path.join(CSRC, src), "-o", "/dev/null", "--offload-arch=gfx950", "-x", "hip", "-O3",
               "-std=c++17", "-fPIC", "-I", CSRC, "-I", os.path.join(ROOT, "include"),
               "-Rpass-analysis=kernel-resource-usage"] + (["-DTSG_K1_PROBE"] if probe else [])
        out = subprocess.run(cmd, capture_output=True, text=True).stderr
        cur = None
        for line in out.splitlines():
            m = re.search(r"remark:\s+Function Name: (\S+)", line)
            if m:
                cur = {"kernel": demangle_short(m.group(1))}
                rows.append(cur)
                continue
            m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+)", line)
            if m and cur is not None:
                cur[m.group(1).strip()] = m.group(2)
    cols = ["VGPRs", "AGPRs", "TotalSGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize", "Occupancy", "LDS Size"]
    print("# hipcc -Rpass-analysis=kernel-resource-usage, gfx950, -O3%s" % (" -DTSG_K1_PROBE" if probe else ""))
    print("%-40s " % "kernel" + " ".join("%12s" % c for c in cols))
    for r in rows:
        if not probe or "4560" in r["kernel"] or "k1" not in r["kernel"]:
            print("%-40s " % r["kernel"][:40] + " ".join("%12s" % r.get(c, "-") for c in cols))


if __name__ == "__main__":
    main()
