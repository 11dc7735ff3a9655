"""Summarise rocprofv3 --pmc CSVs per kernel (sum over dispatches)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(root + "/*/*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        k = "K1" if "tsg_k1_scan" in name else "K2" if "tsg_k2_verify" in name else None
        if not k:
            continue
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for (k, c), v in sorted(agg.items()):
    print("%s %-24s %14.6g  (dispatches %d)" % (k, c, v, len(disp[(k, c)])))
