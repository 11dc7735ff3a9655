"""Per-kernel PMC summary of a tools/pmc_probe.sh run: every counter summed
over the rows of a dispatch, then averaged over the kernel's dispatches, plus
derived ratios (waitcnt share of wave cycles, LDS conflict share, instructions
per content byte, FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note).

  python tools/pmc_summary.py gpurun_out/<run> BYTES_PER_K1_DISPATCH > profiles/<round>_pmc.txt
"""
import collections
import csv
import glob
import re
import sys


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, dispatch) -> counter -> sum
    for f in sorted(glob.glob(root + "/*/*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(tsg_k1_scan_v2|tsg_k1_scan|tsg_k2_verify)", r["Kernel_Name"])
            if not m:
                continue
            per[(m.group(1), f + ":" + r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            out[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}


def main():
    root = sys.argv[1]
    nbytes = float(sys.argv[2]) if len(sys.argv) > 2 else None
    data = load(root)
    for k in sorted(data):
        cs = data[k]
        print("== %s (mean per dispatch)" % k)
        for c in sorted(cs):
            print("  %-24s %16.6g" % (c, cs[c]))
        wc = cs.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in cs:
                    print("  %-24s %16.3f" % (c + "/WAVE_CYCLES", cs[c] / wc))
        if cs.get("SQ_LDS_IDX_ACTIVE"):
            print("  %-24s %16.3f" % ("LDS_BANK_CONFLICT/IDX", cs.get("SQ_LDS_BANK_CONFLICT", 0) / cs["SQ_LDS_IDX_ACTIVE"]))
        if nbytes and k.startswith("tsg_k1"):
            lane_bytes = nbytes / 64.0          # one wave instruction covers 64 lanes = 64 content bytes
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH"):
                if c in cs:
                    print("  %-24s %16.3f" % (c + " per byte", cs[c] / lane_bytes))
            if "FETCH_SIZE" in cs:
                print("  %-24s %16.3f" % ("HBM read B per byte", cs["FETCH_SIZE"] * 1024 * 2 / nbytes))
            if "WRITE_SIZE" in cs:
                print("  %-24s %16.4f" % ("HBM write B per byte", cs["WRITE_SIZE"] * 1024 / nbytes))


if __name__ == "__main__":
    main()
