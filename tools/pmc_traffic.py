"""Per-launch HBM traffic of the scan kernels from tools/pmc_traffic.sh output.

FETCH_SIZE (KB) is scaled by the calibration run of tools/calib_fetch, which
reads a known byte count in K1's exact access pattern (lane-owned 4 KiB
chunks, 64-byte lines of temporal 16-byte loads, as K1 v3 reads):
    scale = bytes_read / (FETCH_SIZE_KB * 1024)   of calib_k1v3
    traffic(K1) = FETCH_SIZE_KB(K1 launch) * 1024 * scale
WRITE_SIZE is reported as read (exact for streaming stores per the guide;
K1's writes are keyword bits, hit records and per-chunk counts).

  python tools/pmc_traffic.py gpurun_out/<run> > profiles/traffic_c<config>.json
(bench.py uses it only while K1's build hash -- bench.k1_build: all of K1's device code in engine.hip --
equals its k1_build; only the timed step's launches are kept)
"""
import collections
import csv
import glob
import json
import re
import sys


def per_kernel(root, counter):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(root + "/*_counter_collection.csv") + glob.glob(root + "/*/*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            m = re.search(r"(tsg_k1_scan|tsg_k2_verify|calib_coalesced|calib_k1pattern|calib_k1v3)", name)
            if m:
                vals[(m.group(1), r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    out = collections.defaultdict(list)
    for (k, d), v in sorted(vals.items(), key=lambda kv: int(kv[0][1])):
        out[k].append(sum(v))          # sum over XCD/instance rows of one dispatch, in dispatch order
    return out


def main():
    run = sys.argv[1]
    calib = per_kernel(run + "/calib", "FETCH_SIZE")
    calib_bytes = None
    for line in open(run + "/calib.log"):
        m = re.match(r"calib_k1v3 bytes (\d+)", line)
        if m:
            calib_bytes = int(m.group(1))
    k1 = per_kernel(run + "/k1", "FETCH_SIZE")
    k1w = per_kernel(run + "/k1w", "WRITE_SIZE")
    cal = sorted(calib["calib_k1v3"])[len(calib["calib_k1v3"]) // 2]
    scale = calib_bytes / (cal * 1024.0)
    coal = calib.get("calib_coalesced")
    bench = None
    for line in open(run + "/k1.log"):
        if line.startswith("{"):
            bench = json.loads(line)
    out = {
        "kernel": "tsg_k1_scan",
        "k1_build": bench["roofline"].get("k1_build") if bench else None,
        "layout": {"config": bench["config"].get("config_id") if bench else None,
                   "segment_bytes": bench["config"].get("segment_bytes") if bench else None,
                   "segment_balanced": bench["config"].get("segment_balanced", False) if bench else None,
                   "chunk_bytes": bench["breakdown_ms"].get("chunk_bytes") if bench else None},
        "source": run,
        "bytes_per_launch": bench["roofline"]["bytes_per_launch"] if bench else None,
        "workload": bench["config"]["workload"] if bench else None,
        "k1_fetch_size_kb_per_launch": k1["tsg_k1_scan"],
        "k1_write_size_kb_per_launch": k1w.get("tsg_k1_scan", []),
        "k2_fetch_size_kb_per_launch": k1.get("tsg_k2_verify", []),
        "calib_k1v3": {"bytes": calib_bytes, "fetch_size_kb": cal, "scale": scale},
        "calib_coalesced_fetch_size_kb": coal,
    }
    # the timed step's launches only: with --steps 1 --warmup 0 they are the
    # process's first launches_per_step K1 dispatches (the resident leg, the
    # parity sample and the other legs come after it with other sizes); the
    # step's bytes are bytes_per_launch x launches_per_step
    n = bench["roofline"]["launches_per_step"] if bench else len(k1["tsg_k1_scan"])
    kf = k1["tsg_k1_scan"][:n]
    kw = (k1w.get("tsg_k1_scan") or [0.0] * n)[:n]
    out["step_launches"] = n
    out["k1_fetch_size_kb_per_launch"] = k1["tsg_k1_scan"][:n]
    out["k1_write_size_kb_per_launch"] = k1w.get("tsg_k1_scan", [])[:n]
    out["k2_fetch_size_kb_per_launch"] = k1.get("tsg_k2_verify", [])[:n]
    f = sum(kf) / len(kf) * 1024.0 * scale
    w = sum(kw) / len(kw) * 1024.0
    out["traffic_bytes_per_launch"] = f + w
    out["read_bytes_per_launch"] = f
    out["write_bytes_per_launch"] = w
    if out["bytes_per_launch"]:
        out["traffic_over_algorithmic"] = (f + w) / out["bytes_per_launch"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
