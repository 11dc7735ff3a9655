#!/usr/bin/env python
"""LDS bank-conflict model of K1's transition reads (tooling, CPU only).

K1 (v3) reads one uint16 transition per byte per lane: ds_read_u16 at byte
address 256 + 2 * row(state) + 2 * class(byte).  On gfx950 a b32-class LDS
read is served in two groups of 32 lanes, one LDS cycle per group when the
lanes touch distinct banks ((address / 4) mod 32) or the same dword
(broadcast); every further distinct dword on a busy bank costs one more cycle
(MI355X_MICROARCH.md, LDS).  This tool replays the builtin scan DFA over a
synthetic corpus with 64 lanes per wave, each lane on its own 4 KiB chunk as
K1 assigns them, and reports LDS cycles per wave-instruction for a table
layout:

  current   rows of 33 dwords (silent) / 39 dwords (output), classes as compiled
  freq      classes renumbered by their byte frequency in the corpus (most
            frequent first), rows as current
  phase     freq + every state's row start placed so its bank phase
            ((row dword) mod 32) is chosen greedily against the states that
            are live together, with padding in LDS
  rootrep   current + the root row replicated per lane in a transposed
            layout (a root-state lane always reads its own bank)
  rootskip  (round 6) lanes at the root state skip the
            transition read (EXEC-masked off: they take the root's next
            state from a widened class map instead); reported with the class
            map read that then costs more: a 16-bit map entry per byte value
            (class and root successor) has ASCII on 64 dwords instead of 32,
            so bytes 64 apart collide
  hotphase  (round 6, item 1b) current + the K hottest states' rows shifted
            by 0-31 dwords of padding, each shift chosen greedily (two sweeps,
            coordinate descent) to minimise the replayed conflict cycles;
            trained on half of the waves, reported on the other half
  qword     rows read as 8-byte units (ds_read_b64: 64 banks, a lane takes
            two; four classes per unit, so same-state lanes broadcast more)

  python tools/lds_bank_sim.py [--mb 64] [--waves 64] [--layouts current,freq,phase]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump_dfa():
    from trivy_amd import _lib
    from trivy_amd import secret as S
    L = _lib.lib()
    global _SCANNER
    _SCANNER = S.Scanner(None)                       # keeps the ruleset alive
    rs = _SCANNER._rs
    nx, bc = ctypes.POINTER(ctypes.c_uint16)(), ctypes.POINTER(ctypes.c_uint8)()
    ns, nc, fo = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(L.tsg_scan_dfa_dump(rs, 0, ctypes.byref(nx), ctypes.byref(bc), ctypes.byref(ns), ctypes.byref(nc),
                                   ctypes.byref(fo)))
    n, c = ns.value, nc.value
    nxt = np.ctypeslib.as_array(nx, shape=(n * c,)).astype(np.int64).reshape(n, c).copy()
    cls = np.ctypeslib.as_array(bc, shape=(256,)).astype(np.int64).copy()
    L.tsg_free(ctypes.cast(nx, ctypes.c_void_p))
    L.tsg_free(ctypes.cast(bc, ctypes.c_void_p))
    return nxt, cls, fo.value


def lane_states(nxt, cls, text, starts, length):
    """DFA state of each lane after each byte: (length, lanes)."""
    lanes = len(starts)
    st = np.zeros(lanes, dtype=np.int64)
    out = np.empty((length, lanes), dtype=np.int64)
    byts = np.stack([text[s:s + length] for s in starts], axis=1).astype(np.int64)   # (length, lanes)
    cl = cls[byts]
    for j in range(length):
        out[j] = st                                  # state BEFORE byte j (the row read at step j)
        st = nxt[st, cl[j]]
    return out, cl


def cycles(dwords, active=None):
    """LDS cycles per wave-instruction: dwords (steps, 64) -> mean over steps of the two half-waves' max bank load.
    active (optional, same shape): lanes taking part (EXEC); a group with no active lane costs 1 (issue)."""
    tot = 0.0
    for h in range(2):
        d = dwords[:, 32 * h:32 * h + 32]
        if active is not None:
            d = np.where(active[:, 32 * h:32 * h + 32], d, -1)
        d = np.sort(d, axis=1)
        new = np.ones_like(d, dtype=bool)
        new[:, 1:] = d[:, 1:] != d[:, :-1]
        new &= d >= 0
        bank = np.where(d >= 0, d % 32, 0)
        key = np.arange(d.shape[0])[:, None] * 32 + bank
        cnt = np.bincount(key[new], minlength=d.shape[0] * 32).reshape(d.shape[0], 32)
        tot += np.maximum(cnt.max(axis=1), 1).mean()
    return tot


def layout_rows(nstates, fo, stride, ostride, phase=None):
    """Row start (uint16 units) of each state; phase: wanted (row dword mod 32) per state or None."""
    rows = np.zeros(nstates, dtype=np.int64)
    pos = 0
    for s in range(nstates):
        if phase is not None:
            d = pos // 2
            pad = (phase[s] - d) % 32
            pos += 2 * pad
        rows[s] = pos
        pos += stride if s < fo else ostride
    return rows, pos


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=64)
    ap.add_argument("--waves", type=int, default=48)
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--layouts", default="current,freq,phase")
    ap.add_argument("--hot", type=int, default=30, help="hotphase: states whose rows are shifted")
    args = ap.parse_args()
    from workload import synth
    nxt, cls, fo = dump_dfa()
    n, C = nxt.shape
    corp = synth.generate(int(args.mb * 1e6), seed=7, sizes="loguniform")
    text = np.asarray(corp.data[:corp.nbytes])
    rng = np.random.default_rng(1)
    nchunks = corp.nbytes // args.chunk - 1
    waves, wave_bytes = [], []
    for w in range(args.waves):
        base = int(rng.integers(0, nchunks - 64))
        starts = [(base + i) * args.chunk for i in range(64)]
        waves.append(lane_states(nxt, cls, text, starts, args.chunk))
        wave_bytes.append(np.stack([text[s:s + args.chunk] for s in starts], axis=1).astype(np.int64))
    args.wave_bytes = wave_bytes
    # class frequency over the replay (bytes read) and state occupancy
    cfreq = np.bincount(np.concatenate([cl.ravel() for _, cl in waves]), minlength=C)
    sfreq = np.bincount(np.concatenate([st.ravel() for st, _ in waves]), minlength=n)
    print("scan DFA: %d states x %d classes, first output state %d; root occupancy %.3f, top-8 states %s" % (
        n, C, fo, sfreq[0] / sfreq.sum(), np.argsort(-sfreq)[:8].tolist()))
    S = (C + 2) & ~1
    if (S // 2) % 2 == 0:
        S += 2
    So = S + 10
    if (So // 2) % 2 == 0:
        So += 2
    perm_id = np.arange(C)
    order = np.argsort(-cfreq)
    perm_freq = np.empty(C, dtype=np.int64)
    perm_freq[order] = np.arange(C)                  # class c -> new index by frequency rank
    results = {}
    for name in args.layouts.split(","):
        if name in ("rootskip", "hotphase", "qword"):
            extra(name, waves, nxt, cls, fo, S, So, sfreq, args)
            continue
        perm = perm_id if name == "current" else perm_freq
        phase = None
        if name == "phase":
            # the busiest states get bank phases spread so their hot classes
            # (low new indices -> dwords 0..) land on different banks: state
            # rank r gets phase 16 * (r & 1) + 8 * ((r >> 1) & 1) + ...
            rank = np.empty(n, dtype=np.int64)
            rank[np.argsort(-sfreq)] = np.arange(n)
            phase = np.array([int('{:05b}'.format(int(r) & 31)[::-1], 2) for r in rank])
        rows, size = layout_rows(n, fo, S, So, phase)
        tot = 0.0
        for st, cl in waves:
            dw = (256 + 2 * rows[st] + 2 * perm[cl]) // 4
            if name == "rootrep":
                # the root row replicated per lane, transposed: lane l reads
                # class c of the root at dword base + (c / 2) * 32 + l % 32
                # (bank l % 32 always); other states as current
                lane = np.arange(dw.shape[1])[None, :] % 32
                rootdw = (1 << 20) + (perm[cl] // 2) * 32 + lane
                dw = np.where(st == 0, rootdw, dw)
            tot += cycles(dw)
        results[name] = (tot / len(waves), size * 2)
        print("%-8s LDS cycles per transition read (2 groups, 2.0 = conflict-free): %.3f   table %d B" % (
            name, results[name][0], results[name][1]))


def extra(name, waves, nxt, cls, fo, S, So, sfreq, args):
    """the round-6 candidates (module docstring)"""
    n, C = nxt.shape
    rows, _ = layout_rows(n, fo, S, So)
    base_dw = rows // 2                              # a state's row start in dwords
    if name == "rootskip":
        tr = cur = cl_cur = cl_wide = 0.0
        for (st, cl), b in zip(waves, args.wave_bytes):
            dw = 64 + base_dw[st] + cl // 2
            cur += cycles(dw)
            tr += cycles(dw, st != 0)
            cl_cur += cycles(b // 4)                   # class map of u8 entries: 4 byte values per dword
            cl_wide += cycles(b // 2)                  # u16 entries (class + root successor): 2 per dword
        k = len(waves)
        print("rootskip transition read %.3f (current %.3f); class map read u8 %.3f -> u16 %.3f: net %+.3f LDS "
              "cycles per byte, plus a compare and a select on the dependent chain" % (
                  tr / k, cur / k, cl_cur / k, cl_wide / k, (tr - cur + cl_wide - cl_cur) / k))
    elif name == "qword":
        tot = 0.0
        Rq, Rqo = (C + 3) // 4 | 1, ((C + 3) // 4 + 3) | 1
        qrow = np.where(np.arange(n) < fo, np.arange(n) * Rq, fo * Rq + (np.arange(n) - fo) * Rqo)
        for st, cl in waves:
            tot += cycles(qrow[st] + cl // 4)
        print("qword    LDS cycles per transition read (ds_read_b64, 8-byte units): %.3f  (+2-3 VALU per byte "
              "to pick the 16-bit entry)" % (tot / len(waves)))
    elif name == "hotphase":
        half = len(waves) // 2
        st_tr = np.concatenate([w[0] for w in waves[:half]])
        cl_tr = np.concatenate([w[1] for w in waves[:half]]) // 2
        st_te = np.concatenate([w[0] for w in waves[half:]])
        cl_te = np.concatenate([w[1] for w in waves[half:]]) // 2
        cur = base_dw.copy()
        best = cycles(64 + cur[st_tr] + cl_tr)
        base_te = cycles(64 + cur[st_te] + cl_te)
        for sweep in range(2):
            for s in np.argsort(-sfreq)[:args.hot]:
                b0, bestd = base_dw[s], cur[s] - base_dw[s]
                for d in range(32):
                    cur[s] = b0 + d
                    c = cycles(64 + cur[st_tr] + cl_tr)
                    if c < best - 1e-9:
                        best, bestd = c, d
                cur[s] = b0 + bestd
        print("hotphase %d hottest rows shifted: %.3f on held-out waves (current %.3f), padding <= %d B" % (
            args.hot, cycles(64 + cur[st_te] + cl_te), base_te, args.hot * 31 * 4))


if __name__ == "__main__":
    main()
