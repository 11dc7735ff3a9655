#!/usr/bin/env python
"""Per-file queue probe: `callers` threads calling Scan file by file through
tsg_queue_* (the --parallel goroutines of an unchanged Trivy), over config
1's size model, for several queue settings (max files per batch, leader wait,
batches in flight).

  python tools/queue_probe.py [--mb 256] [--callers 5,16] [--variants F:W:I,...]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=256)
    ap.add_argument("--callers", default="5,16")
    ap.add_argument("--variants", default="0:200:0,1:200:0,1:200:8,2:200:8,0:0:8",
                    help="comma list of max_files:max_wait_us:max_inflight[:spread] (0 = the library default; "
                         "spread 0/1 sets TSG_QUEUE_SPREAD)")
    ap.add_argument("--seed", type=int, default=0x71215EC7)
    a = ap.parse_args()
    from trivy_amd import secret as S
    from workload import synth
    c = synth.generate(int(a.mb * 1e6), seed=a.seed, sizes="lognormal")
    args = [S.ScanArgs(c.paths[i], c.file(i)) for i in range(len(c.paths))]
    sc = S.Scanner(None, threads=16)
    for v in a.variants.split(","):
        parts = [int(x) for x in v.split(":")]
        f, w, i = parts[:3]
        if len(parts) > 3:
            os.environ["TSG_QUEUE_SPREAD"] = str(parts[3])
        else:
            os.environ.pop("TSG_QUEUE_SPREAD", None)
        for cl in (int(x) for x in a.callers.split(",")):
            q = S.ScanQueue(sc, max_files=f, max_wait_us=w, max_inflight=i)
            q.probe(args[:200], cl)                      # warm lanes and staging buffers
            q.close()
            q = S.ScanQueue(sc, max_files=f, max_wait_us=w, max_inflight=i)
            sec, nf = q.probe(args, cl)
            st = q.stats()
            q.close()
            print({"max_files": f, "max_wait_us": w, "max_inflight": i, "callers": cl,
                   "spread": os.environ.get("TSG_QUEUE_SPREAD", "default"),
                   "gbps": round(c.nbytes / sec / 1e9, 3), "files_per_s": round(len(args) / sec),
                   "findings": nf, "batches": st["batches"],
                   "mean_batch_files": round(st["files"] / max(1, st["batches"]), 2)}, flush=True)


if __name__ == "__main__":
    main()
