#!/usr/bin/env python
"""Pinned-host vs HBM-resident entry points on bench.py's workload: report the
files whose results differ, with the host reference (tsg_scan_host_reference,
no GPU prefilter) for each of them.

  python tools/diff_paths.py [--gb 10] [--config 2]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=0x71215EC7)
    ap.add_argument("--max-report", type=int, default=5)
    args = ap.parse_args()
    import torch

    import bench
    from trivy_amd import _lib
    from trivy_amd import secret as S
    from workload import synth
    L = _lib.lib()
    corpus = synth.generate(int(args.gb * 1e9), seed=args.seed, sizes="loguniform")
    sc = S.Scanner(None, threads=16)
    eng = sc.engine()
    batch = bench.PinnedBatch(L, corpus.data, corpus.offsets, corpus.paths)
    n = batch.nfiles
    res = ctypes.c_void_p()
    _lib.check(L.tsg_scan_batch(eng, batch.ptr, batch.offsets.ctypes.data, n, batch.cpaths, batch.clens, None,
                                ctypes.byref(res)))
    pinned = _lib.result_json(res)
    L.tsg_result_free(res)
    d = torch.empty(batch.nbytes + 64, dtype=torch.uint8, device="cuda:0")
    d.copy_(torch.from_numpy(batch.view))
    torch.cuda.synchronize()
    _lib.check(L.tsg_scan_batch_resident(eng, ctypes.c_void_p(d.data_ptr()), batch.ptr, batch.offsets.ctypes.data, n,
                                         batch.cpaths, batch.clens, None, ctypes.byref(res)))
    resident = _lib.result_json(res)
    st = _lib.result_stats(res)
    L.tsg_result_free(res)
    diff = [i for i in range(n) if pinned[i] != resident[i]]
    print("files %d, differing %d, resident pieces %d" % (n, len(diff), st["pieces"]), flush=True)
    for i in diff[:args.max_report]:
        a = S.ScanArgs(batch.paths[i], batch.file(i))
        ref = S.scan_host_reference(sc, [a], threads=1)[0]
        off0 = int(batch.offsets[i])
        print(json.dumps({"file": i, "path": batch.paths[i], "offset": off0, "size": len(a.Content),
                          "pinned_ok": pinned[i] == ref, "resident_ok": resident[i] == ref}), flush=True)
        for name, r in (("pinned", pinned[i]), ("resident", resident[i]), ("reference", ref)):
            fs = [(f["RuleID"], f["StartLine"], f["Match"][:40]) for f in r.get("Findings", [])]
            print("  %-9s %d findings; first differing entries:" % (name, len(fs)), flush=True)
            ref_fs = [(f["RuleID"], f["StartLine"], f["Match"][:40]) for f in ref.get("Findings", [])]
            shown = 0
            for x in fs:
                if x not in ref_fs and shown < 6:
                    print("     ", x, flush=True)
                    shown += 1
    batch.free()


if __name__ == "__main__":
    main()
