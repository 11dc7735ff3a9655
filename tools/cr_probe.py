#!/usr/bin/env python
"""Time the GPU CR strip (tsg_strip_cr_device) on a device batch (tooling).

  python tools/cr_probe.py [--gb 10] [--density 0.025] [--files 2000] [--reps 5]
density: share of bytes that are '\\r' (0.025 ~ CRLF text; 0 = the direct-store path)."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trivy_amd import secret as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=10)
    ap.add_argument("--density", type=float, default=0.025)
    ap.add_argument("--files", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n = int(a.gb * 1e9) // 16 * 16
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1)
    src = torch.randint(32, 127, (n + 64,), dtype=torch.uint8, device="cuda:0", generator=g)
    if a.density > 0:
        # CRs every ~1/density bytes: positions from a strided pattern with jitter (no n-sized float temp)
        step = int(round(1 / a.density))
        pos = torch.arange(0, n - step, step, device="cuda:0", dtype=torch.int64)
        pos += torch.randint(0, step, pos.shape, device="cuda:0", generator=g)
        src[pos] = 13
        del pos
    rng = np.random.default_rng(2)
    cuts = np.sort(rng.choice(np.arange(1, n, 997), a.files - 1, replace=False)).astype(np.int64)
    off = torch.from_numpy(np.concatenate([[0], cuts, [n]]).astype(np.int64)).to("cuda:0")
    sc = S.Scanner(None)
    ms = []
    for _ in range(a.reps):
        dst, noff, stripped, kms = sc.StripCR(src, off, a.files, n)
        ms.append(kms)
        del dst, noff
    m = float(np.mean(ms[1:]))
    print("CR strip %.2f GB density %.3f: %s ms -> mean %.3f ms, %.0f GB/s input, %.0f GB/s N+N'" % (
        n / 1e9, a.density, " ".join("%.3f" % x for x in ms), m, n / m / 1e6, (n + stripped) / m / 1e6), flush=True)


if __name__ == "__main__":
    main()
