"""GPU-side CR strip (tsg_strip_cr_device).

The reference strips carriage returns from every text file before scanning:
    content = bytes.ReplaceAll(content, []byte("\\r"), []byte(""))
(pkg/fanal/analyzer/secret/secret.go:121).  The checker here is that same
operation on the host (Python's bytes.replace / numpy), per file:

* ragged batches: empty files, all-CR files, files starting and ending with
  CR, runs of tiny files inside one 1 KiB sub-tile, files spanning the
  kernel's 64 KiB regions, totals that are not a multiple of 16, batches
  without any CR (the aligned direct-store path) and dense CR;
* a 256 MB batch at CRLF density checked through numpy;
* end to end: raw CRLF files uploaded as read, stripped on the GPU, the
  stripped bytes brought back and scanned resident equal Scan over the
  host-stripped files (the analyzer's contract).
CPU part: argument checking at the boundary (no GPU call)."""
import ctypes

import numpy as np
import pytest

from trivy_amd import _lib
from trivy_amd import secret as S


def test_strip_cr_rejects_null_arguments_cpu():
    L = _lib.lib()
    tot, ms = ctypes.c_uint64(), ctypes.c_double()
    assert L.tsg_strip_cr_device(None, None, None, 0, 0, None, None, ctypes.byref(tot), ctypes.byref(ms)) != 0
    assert "NULL" in _lib.lib().tsg_last_error().decode()


def _files_case(rng, kind):
    if kind == "ragged":
        files = [b"", b"\r", b"\r\r\r\r", b"a\r", b"\rb", b"abc", b"x" * 15, b"\r" * 17]
        for _ in range(300):                       # tiny files, many per sub-tile
            n = int(rng.integers(0, 24))
            files.append(bytes(rng.choice(np.frombuffer(b"ab\r\n", np.uint8), n)))
        for n in (65535, 65536, 65537, 131072 + 7, 300_001):   # across 64 KiB regions
            a = rng.integers(32, 127, n, dtype=np.uint8)
            a[rng.random(n) < 0.03] = 13
            files.append(a.tobytes())
        files += [b"", b""]                        # trailing empty files end at the batch end
        return files
    if kind == "no_cr":
        return [rng.integers(32, 127, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 200_000, 40)]
    if kind == "dense":
        out = []
        for n in rng.integers(0, 70_000, 30):
            a = np.full(int(n), 13, np.uint8)
            a[rng.random(int(n)) < 0.01] = ord("k")
            out.append(a.tobytes())
        return out
    if kind == "crlf":
        out = []
        for n in rng.integers(1, 40_000, 200):
            lines = [bytes(rng.integers(97, 123, int(m), dtype=np.uint8)) for m in rng.integers(0, 80, int(n) // 40 + 1)]
            out.append(b"\r\n".join(lines) + (b"\r\n" if n % 2 else b""))
        return out
    if kind == "all_empty":
        return [b"", b"", b""]
    raise ValueError(kind)


def _pack(files):
    off = np.zeros(len(files) + 1, np.uint64)
    off[1:] = np.cumsum([len(f) for f in files])
    data = np.frombuffer(b"".join(files) + bytes(64), np.uint8)
    return data, off


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["ragged", "no_cr", "dense", "crlf", "all_empty"])
def test_strip_cr_matches_replace_gpu(kind):
    import torch
    rng = np.random.default_rng(sum(kind.encode()))
    files = _files_case(rng, kind)
    data, off = _pack(files)
    total = int(off[-1])
    sc = S.Scanner(None)
    d_src = torch.from_numpy(data.copy()).to("cuda:0")
    d_off = torch.from_numpy(off.astype(np.int64)).to("cuda:0")
    dst, new_off, stripped, ms = sc.StripCR(d_src, d_off, len(files), total)
    want = [f.replace(b"\r", b"") for f in files]
    want_off = np.zeros(len(files) + 1, np.int64)
    want_off[1:] = np.cumsum([len(w) for w in want])
    assert stripped == int(want_off[-1])
    got_off = new_off.cpu().numpy()
    assert np.array_equal(got_off, want_off)
    got = dst[:stripped].cpu().numpy().tobytes()
    assert got == b"".join(want)
    assert ms >= 0


@pytest.mark.gpu
def test_strip_cr_large_batch_gpu():
    """256 MB at CRLF density (one CR per ~40 bytes), 2000 files, against numpy."""
    import torch
    n = 256 << 20
    g = torch.Generator(device="cuda:0")
    g.manual_seed(7)
    d_src = torch.randint(32, 127, (n + 64,), dtype=torch.uint8, device="cuda:0", generator=g)
    d_src[:n][torch.rand(n, device="cuda:0", generator=g) < 1 / 40] = 13
    rng = np.random.default_rng(3)
    cuts = np.sort(rng.choice(np.arange(1, n), 1999, replace=False)).astype(np.int64)
    off = np.concatenate([[0], cuts, [n]]).astype(np.int64)
    sc = S.Scanner(None)
    dst, new_off, stripped, ms = sc.StripCR(d_src, torch.from_numpy(off).to("cuda:0"), len(off) - 1, n)
    src = d_src[:n].cpu().numpy()
    iscr = src == 13
    keep = ~iscr
    assert stripped == int(keep.sum())
    assert np.array_equal(dst[:stripped].cpu().numpy(), src[keep])
    cr_before = np.concatenate([[0], np.cumsum(iscr)])
    assert np.array_equal(new_off.cpu().numpy(), off - cr_before[off])


@pytest.mark.gpu
def test_strip_cr_then_resident_scan_gpu():
    """Raw CRLF files as read -> GPU strip -> resident scan == Scan(host-stripped)."""
    import torch
    from workload import synth
    c = synth.generate(2_000_000, seed=21, sizes="lognormal", plant_rate=3e-3, base_bytes=1 << 20)
    raw = []
    for i in range(len(c.paths)):
        f = c.file(i)
        raw.append(f.replace(b"\n", b"\r\n") if i % 2 == 0 else f)
    data, off = _pack(raw)
    sc = S.Scanner(None)
    d_src = torch.from_numpy(data.copy()).to("cuda:0")
    dst, new_off, stripped, _ms = sc.StripCR(d_src, torch.from_numpy(off.astype(np.int64)).to("cuda:0"), len(raw),
                                             int(off[-1]))
    h_off = new_off.cpu().numpy().astype(np.uint64)
    h_data = np.ascontiguousarray(dst.cpu().numpy())
    L = _lib.lib()
    paths, lens, _keep = _lib.pack_paths(c.paths)
    res = ctypes.c_void_p()
    _lib.check(L.tsg_scan_batch_resident(sc.engine(), ctypes.c_void_p(dst.data_ptr()), h_data.ctypes.data,
                                         h_off.ctypes.data, len(raw), paths, lens, None, ctypes.byref(res)))
    try:
        got = _lib.result_json(res)
    finally:
        L.tsg_result_free(res)
    want = sc.ScanBatch([S.ScanArgs(c.paths[i], raw[i].replace(b"\r", b"")) for i in range(len(raw))])
    nfind = 0
    for p, g, w in zip(c.paths, got, want):
        g.pop("Error", None)
        assert g == w, p
        nfind += len(w.get("Findings") or [])
    assert nfind > 5


@pytest.mark.gpu
def test_strip_cr_rejects_host_buffers_gpu():
    """Buffers that are not device memory of one of the engine's devices are
    refused at the boundary (no kernel gets a host or foreign pointer)."""
    import torch
    files = [b"a\r\nb", b"\r\r", b"xyz"]
    data, off = _pack(files)
    sc = S.Scanner(None)
    L = _lib.lib()
    d_src = torch.from_numpy(data.copy()).to("cuda:0")
    d_off = torch.from_numpy(off.astype(np.int64)).to("cuda:0")
    h_off = torch.from_numpy(off.astype(np.int64)).pin_memory()
    dst = torch.empty(len(data), dtype=torch.uint8, device="cuda:0")
    new_off = torch.empty(len(files) + 1, dtype=torch.int64, device="cuda:0")
    tot, ms = ctypes.c_uint64(), ctypes.c_double()
    for src, offs, out in ((d_src, h_off, dst), (data.ctypes.data, d_off, dst), (d_src, d_off, h_off)):
        p = lambda t: ctypes.c_void_p(t if isinstance(t, int) else t.data_ptr())
        rc = L.tsg_strip_cr_device(sc.engine(), p(src), p(offs), len(files), int(off[-1]), p(out), p(new_off),
                                   ctypes.byref(tot), ctypes.byref(ms))
        assert rc != 0 and "device memory" in L.tsg_last_error().decode()
    # and the same call with device buffers works
    got_dst, got_off, stripped, _ = sc.StripCR(d_src, d_off, len(files), int(off[-1]))
    assert got_dst[:stripped].cpu().numpy().tobytes() == b"".join(f.replace(b"\r", b"") for f in files)
