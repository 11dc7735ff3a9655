#!/usr/bin/env python
"""Latency of small tsg_scan_batch calls (the per-file drop-in's batches:
1 / 5 / 64 files of 8-32 KB in pinned host memory), with the engine's own
stats per call: where a small batch's wall time goes (the GPU passes by HIP
events, the upload, host confirm, the rest).  Run under rocprofv3
--kernel-trace --memory-copy-trace for the GPU timeline
(tools/prof_timeline.py).

  python tools/small_probe.py [--reps 200] [--counts 1,5,64]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--counts", default="1,5,64")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime, as the bench)
    from trivy_amd import _lib
    from trivy_amd import secret as S
    from workload import synth
    c = synth.generate(8_000_000, seed=5, sizes="lognormal")
    sizes = np.diff(c.offsets)
    pick = [i for i in range(len(c.paths)) if (8 << 10) <= sizes[i] <= (32 << 10)]
    L = _lib.lib()
    sc = S.Scanner(None)
    eng = sc.engine()
    for n in [int(x) for x in args.counts.split(",")]:
        files = [c.file(i) for i in pick[:n]]
        offs = np.zeros(n + 1, np.uint64)
        offs[1:] = np.cumsum([len(f) for f in files])
        p = ctypes.c_void_p()
        _lib.check(L.tsg_alloc_pinned(int(offs[-1]) + 64, ctypes.byref(p)))
        view = np.ctypeslib.as_array((ctypes.c_uint8 * (int(offs[-1]) + 64)).from_address(p.value))
        view[:int(offs[-1])] = np.frombuffer(b"".join(files), np.uint8)
        view[int(offs[-1]):] = 0
        paths, lens, _k = _lib.pack_paths([c.paths[i] for i in pick[:n]])
        rows = []
        for r in range(args.reps + 5):
            res = ctypes.c_void_p()
            t0 = time.perf_counter()
            _lib.check(L.tsg_scan_batch(eng, p, offs.ctypes.data, n, paths, lens, None, ctypes.byref(res)))
            dt = (time.perf_counter() - t0) * 1e3
            st = _lib.result_stats(res)
            L.tsg_result_free(res)
            if r >= 5:
                rows.append((dt, st["k1_ms"], st["k2_ms"], st["h2d_ms"], st["host_ms"], st["total_ms"]))
        L.tsg_free_pinned(p)
        a = np.array(rows)
        med = np.median(a, axis=0)
        print(json.dumps({"files": n, "bytes": int(offs[-1]), "wall_ms": round(med[0], 4), "k1_ms": round(med[1], 4),
                          "k2_ms": round(med[2], 4), "h2d_ms": round(med[3], 4), "host_confirm_ms": round(med[4], 4),
                          "engine_total_ms": round(med[5], 4), "wall_p90_ms": round(float(np.percentile(a[:, 0], 90)), 4)}),
              flush=True)


if __name__ == "__main__":
    main()
