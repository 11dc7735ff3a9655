#!/usr/bin/env python
"""K1's L2 -> memory read requests from tools/pmc_dram.sh output: per launch
of the timed step, the requests by size (32 / 64 / 128 B), the bytes they
ask for, and the share destined for DRAM (TCC_EA0_RDREQ_DRAM: the local
memory side -- HBM or the Infinity Cache in front of it; no counter on this
ROCm separates an Infinity-Cache hit from an HBM read).

  python tools/pmc_dram.py gpurun_out/<run>/dram_c2 > profiles/<round>_dram_c2.json
"""
import collections
import csv
import glob
import json
import re
import sys

COUNTERS = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_DRAM_sum")


def main():
    run = sys.argv[1]
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(run + "/dram/*_counter_collection.csv") + glob.glob(run + "/dram/*/*_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "tsg_k1_scan" not in r["Kernel_Name"] or r["Counter_Name"] not in COUNTERS:
                continue
            vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    bench = None
    for line in open(run + "/dram.log"):
        if line.startswith("{"):
            bench = json.loads(line)
    n = bench["roofline"]["launches_per_step"]
    per = [vals[d] for d in sorted(vals)][:n]
    req = sum(v["TCC_EA0_RDREQ_sum"] for v in per)
    r64 = sum(v["TCC_EA0_RDREQ_64B_sum"] for v in per)
    r128 = sum(v["TCC_EA0_RDREQ_128B_sum"] for v in per)
    dram = sum(v["TCC_EA0_RDREQ_DRAM_sum"] for v in per)
    r32 = max(req - r64 - r128, 0.0)
    req_bytes = 128 * r128 + 64 * r64 + 32 * r32
    content = bench["roofline"]["bytes_per_launch"] * n
    out = {
        "kernel": "tsg_k1_scan", "k1_build": bench["roofline"].get("k1_build"),
        "config": bench["config"].get("config_id"), "step_launches": n, "content_bytes": content,
        "requests": req, "requests_64B": r64, "requests_128B": r128, "requests_32B": r32,
        "request_bytes": req_bytes, "request_bytes_over_content": req_bytes / content,
        "dram_requests": dram, "dram_share_of_requests": dram / req if req else None,
        "counters": list(COUNTERS),
        "note": "request bytes = 128 x RDREQ_128B + 64 x RDREQ_64B + 32 x the rest; DRAM-destined requests include "
                "Infinity-Cache hits (memory-side cache): this pass bounds K1's HBM reads from above",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
