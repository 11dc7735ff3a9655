#!/usr/bin/env python
"""K1/K2 probe: one HBM-resident batch through the two GPU passes only
(tsg_prefilter_resident: one K1 launch per scan-DFA group + K2), repeated.

  python tools/k1_probe.py [--gb 4] [--reps 5] [--sizes loguniform] [--config 2|5]

Prints per-launch K1 / K2 times and GB/s; used for K1 tuning and for
rocprofv3 runs (a short program with few dispatches).  Variants other than
the product build (TSG_K1_ABL != 4560) need the probe library
(python -m trivy_amd.build --probe), selected here through TSG_LIB.
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
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sizes", default="loguniform")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0x71215EC7)
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--threads", type=int, default=16, help="host confirm threads (--full)")
    ap.add_argument("--full", action="store_true",
                    help="the whole resident scan (tsg_scan_batch_resident: pieces, K1/K2, host confirmation) "
                         "instead of the two GPU passes")
    ap.add_argument("--prewarm-ms", type=float, default=0.0,
                    help="keep the GPU busy (torch elementwise kernels) this long right before each K1/K2 run")
    ap.add_argument("--variants", default="",
                    help="comma list of ABL[:CHUNK[:NAME=V+NAME=V]] (TSG_K1_ABL build bits / TSG_K1_CHUNK / extra "
                         "TSG_* settings), one engine each")
    args = ap.parse_args()
    if any(v.split(":")[0] not in ("", "4560") for v in args.variants.split(",") if v):
        os.environ.setdefault("TSG_LIB", "libtrivysecret_probe.so")
    import torch

    from trivy_amd import _lib
    from trivy_amd import secret as S
    from workload import synth
    c = synth.generate(int(args.gb * 1e9), seed=args.seed, sizes=args.sizes)
    cfg = None
    if args.config == 5:
        cfg5, plants = synth.config5(500, seed=args.seed)
        cfg = "/tmp/tsg_k1probe_c5.yaml"
        synth.write_yaml(cfg5, cfg)
        synth.plant_custom(c, plants, seed=args.seed, rate=1e-4)
    d = torch.from_numpy(c.data).to("cuda:0")
    torch.cuda.synchronize()
    L = _lib.lib()
    variants = [v for v in args.variants.split(",") if v] or [None]
    for v in variants:
        if v is not None:
            parts = v.split(":") + ["", ""]
            os.environ["TSG_K1_ABL"] = parts[0] or "4560"
            if parts[1]:
                os.environ["TSG_K1_CHUNK"] = parts[1]
            else:
                os.environ.pop("TSG_K1_CHUNK", None)
            for kv in parts[2].split("+"):                # extra NAME=VALUE settings
                if "=" in kv:
                    k, _, val = kv.partition("=")
                    os.environ[k] = val
        sc = S.Scanner(S.ParseConfig(cfg) if cfg else None, threads=args.threads)
        probe(args, sc, c, d, L)
        del sc                                    # engine destroyed here (TSG_K2_STATS prints its counters)


def probe(args, sc, c, d, L):
    from trivy_amd import _lib
    eng = sc.engine()
    rows = []
    if args.full:
        cpaths, clens, keep = _lib.pack_paths(c.paths)
    import torch
    busy = torch.ones(1 << 26, device="cuda:0") if args.prewarm_ms > 0 else None
    for r in range(args.reps + 1):
        if busy is not None:                      # clocks up: the GPU was busy until just now
            t1 = time.perf_counter()
            while (time.perf_counter() - t1) * 1e3 < args.prewarm_ms:
                for _ in range(8):
                    busy.mul_(1.0000001)
                torch.cuda.synchronize()
        res = ctypes.c_void_p()
        t0 = time.perf_counter()
        if args.full:
            _lib.check(L.tsg_scan_batch_resident(eng, ctypes.c_void_p(d.data_ptr()), c.data.ctypes.data,
                                                 c.offsets.ctypes.data, len(c.paths), cpaths, clens, None,
                                                 ctypes.byref(res)))
        else:
            _lib.check(L.tsg_prefilter_resident(eng, ctypes.c_void_p(d.data_ptr()), c.data.ctypes.data,
                                                c.offsets.ctypes.data, len(c.paths), ctypes.byref(res)))
        wall = (time.perf_counter() - t0) * 1e3
        st = _lib.result_stats(res)
        L.tsg_result_free(res)
        if r == 0:
            continue                              # warm-up (allocations)
        rows.append((st["k1_ms"], st["k2_ms"], wall, st["hits"], st["candidates"], st["k1_launches"],
                     st.get("host_ms", 0.0), st.get("pieces", 1)))
    k1 = float(np.median([x[0] for x in rows]))
    k2 = float(np.median([x[1] for x in rows]))
    out = {"bytes": c.nbytes, "files": len(c.paths), "k1_ms": round(k1, 4), "k2_ms": round(k2, 4),
           "k1_gbps": round(c.nbytes / k1 / 1e6, 1), "k1_launches": rows[-1][5], "hits": rows[-1][3],
           "candidates": rows[-1][4], "wall_ms": round(float(np.median([x[2] for x in rows])), 3),
           "wall_gbps": round(c.nbytes / float(np.median([x[2] for x in rows])) / 1e6, 1),
           "host_ms": round(float(np.median([x[6] for x in rows])), 3), "pieces": rows[-1][7],
           "env": {k: v for k, v in os.environ.items() if k.startswith("TSG_")}}
    print(json.dumps(out) if args.json else out, flush=True)


if __name__ == "__main__":
    main()
