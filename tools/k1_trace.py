#!/usr/bin/env python
"""Summarise K1 wall-clock traces (probe build TSG_K1_ABL with kAblTrace,
262144 | ...; TSG_K1_TRACE_FILE=<file>): per launch, where the kernel's time
goes -- workgroup dispatch spread, LDS table load, per-item durations by
range size, the first and last item of each wave, and the busy share.

  python tools/k1_trace.py <trace file> [--launch K]
"""
import argparse

import numpy as np

TICK_US = 0.01            # s_memrealtime: 100 MHz


def launches(path):
    a = np.fromfile(path, dtype=np.uint32)
    i = 0
    while i + 4 <= len(a):
        blocks, items, nchunks, chunk = (int(v) for v in a[i:i + 4])
        i += 4
        wg = a[i:i + 4 * blocks].reshape(blocks, 4).astype(np.int64)
        i += 4 * blocks
        it = a[i:i + 8 * items].reshape(items, 8).astype(np.int64)   # kTraceItemWords (round 6)
        i += 8 * items
        yield blocks, nchunks, chunk, wg, it


def rel(v, t0):
    return ((v - t0) % (1 << 32)) * TICK_US


def summarise(k, blocks, nchunks, chunk, wg, it):
    t0 = int(wg[:, 0].min())
    entry, loaded, exit_ = rel(wg[:, 0], t0), rel(wg[:, 1], t0), rel(wg[:, 2], t0)
    used = it[(it[:, 0] != 0) | (it[:, 1] != 0)]
    st, en = rel(used[:, 0], t0), rel(used[:, 1], t0)
    dur = en - st
    span = exit_.max()
    print("launch %d: %d WGs, %d chunks of %d B (%.1f MB), %d items; span %.1f us" % (
        k, blocks, nchunks, chunk, nchunks * chunk / 1e6, len(used), span))
    print("  WG entry: spread %.1f us; table loaded after %.1f us (median), last WG ready at %.1f us" % (
        entry.max() - entry.min(), float(np.median(loaded - entry)), loaded.max()))
    kus = used[:, 2] >> 24
    setup, loop, kw = rel(used[:, 3], t0), rel(used[:, 4], t0), rel(used[:, 5], t0)
    for ku in (4, 2, 1):
        m = kus == ku
        if m.any():
            d = dur[m]
            print("  kU=%d: %6d items, duration us p10 %.1f p50 %.1f p90 %.1f max %.1f; starts %.1f-%.1f" % (
                ku, m.sum(), *np.percentile(d, [10, 50, 90]), d.max(), st[m].min(), st[m].max()))
            print("        phases (p50 us): item taken + range set up (file lookup) %.1f, line loop %.1f, outputs "
                  "drained + keyword bits flushed %.1f, hit buffer flushed %.1f" % (
                      np.median(setup[m] - st[m]), np.median(loop[m] - setup[m]), np.median(kw[m] - loop[m]),
                      np.median(en[m] - kw[m])))
    waves = used[:, 2] & 0xffffff
    first_start, last_end, busy = {}, {}, {}
    for w, s, e in zip(waves, st, en):
        first_start[w] = min(first_start.get(w, 1e18), s)
        last_end[w] = max(last_end.get(w, 0), e)
        busy[w] = busy.get(w, 0) + (e - s)
    le = np.array(list(last_end.values()))
    fs = np.array(list(first_start.values()))
    print("  waves %d: first item start p50 %.1f max %.1f us; last item end p10 %.1f p50 %.1f p90 %.1f max %.1f us" % (
        len(le), float(np.median(fs)), fs.max(), *np.percentile(le, [10, 50, 90]), le.max()))
    print("  busy share (sum of item time / waves x span): %.2f; WG exit after last item end: %.1f us" % (
        sum(busy.values()) / (len(busy) * span), span - le.max()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--launch", type=int, default=-1)
    args = ap.parse_args()
    for k, (blocks, nchunks, chunk, wg, it) in enumerate(launches(args.path)):
        if args.launch < 0 or k == args.launch:
            summarise(k, blocks, nchunks, chunk, wg, it)


if __name__ == "__main__":
    main()
