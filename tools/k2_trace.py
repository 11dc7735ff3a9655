#!/usr/bin/env python
"""Summarise K2 wall-clock traces (probe library, TSG_K2_ABL=2,
TSG_K2_TRACE_FILE=<file>): per launch, the waves' durations, their hits and
verify bytes, and how the slowest waves differ from the median one.

  python tools/k2_trace.py <trace file> [--launch K]
"""
import argparse

import numpy as np

TICK_US = 0.01            # s_memrealtime: 100 MHz


def launches(path):
    a = np.fromfile(path, dtype=np.uint32)
    i = 0
    while i + 4 <= len(a):
        waves = int(a[i])
        i += 4
        yield a[i:i + 8 * waves].reshape(waves, 8).astype(np.int64)
        i += 8 * waves


def summarise(k, w):
    w = w[w[:, 2] > 0]                      # waves that verified at least one hit
    if len(w) == 0:
        print("launch %d: no hits" % k)
        return
    t0 = w[:, 0].min()
    st = ((w[:, 0] - t0) % (1 << 32)) * TICK_US
    en = ((w[:, 1] - t0) % (1 << 32)) * TICK_US
    d = en - st
    print("launch %d: %d waves with hits, span %.1f us; wave duration p10 %.1f p50 %.1f p90 %.1f max %.1f us" % (
        k, len(w), en.max(), *np.percentile(d, [10, 50, 90]), d.max()))
    print("  starts: p50 %.1f max %.1f us; ends: p10 %.1f p50 %.1f p90 %.1f us" % (
        float(np.median(st)), st.max(), *np.percentile(en, [10, 50, 90])))
    print("  per wave: hits p50 %d max %d; walk bytes p50 %d max %d; most bytes of one lane p50 %d p90 %d max %d" % (
        np.median(w[:, 2]), w[:, 2].max(), np.median(w[:, 3]), w[:, 3].max(),
        np.median(w[:, 5]), np.percentile(w[:, 5], 90), w[:, 5].max()))
    slow = d >= np.percentile(d, 90)
    print("  slowest 10%% of waves: duration %.1f us, hits %.1f, bytes %.0f, lane max bytes %.0f, lane max hits %.1f "
          "(the rest: %.1f us, %.1f, %.0f, %.0f, %.1f)" % (
              d[slow].mean(), w[slow, 2].mean(), w[slow, 3].mean(), w[slow, 5].mean(), w[slow, 4].mean(),
              d[~slow].mean(), w[~slow, 2].mean(), w[~slow, 3].mean(), w[~slow, 5].mean(), w[~slow, 4].mean()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--launch", type=int, default=-1)
    a = ap.parse_args()
    for k, w in enumerate(launches(a.path)):
        if a.launch < 0 or k == a.launch:
            summarise(k, w)


if __name__ == "__main__":
    main()
