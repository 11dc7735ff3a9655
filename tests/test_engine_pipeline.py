"""The engine's batch pipeline and boundary threading:

* a pinned host batch streamed to HBM in many segments (upload of segment k+1
  overlapping the kernels of k and the host confirmation of k-1) gives the
  one-segment result and the HBM-resident result;
* one engine shared by concurrent tsg_scan_batch callers (the reference calls
  Scan from --parallel goroutines): every caller gets exactly its sequential
  result;
* several device drivers pulling segments from one shared queue
  (TSG_ENGINE_REPLICAS drivers on the box's one GPU stand in for an 8-GPU
  node) give the single-driver result.

CPU part: the host confirmer is reentrant (concurrent tsg_scan_host_reference
callers on one ruleset equal the sequential run)."""
import ctypes
import threading

import numpy as np
import pytest

from trivy_amd import _lib
from trivy_amd import secret as S
from workload import synth


def _corpus(nbytes, seed):
    c = synth.generate(nbytes, seed=seed, sizes="lognormal", plant_rate=3e-3, base_bytes=1 << 20)
    return c, [S.ScanArgs(c.paths[i], c.file(i)) for i in range(len(c.paths))]


def test_concurrent_host_confirm_cpu():
    sc = S.Scanner(None)
    batches = [_corpus(600_000, 40 + k)[1] for k in range(4)]
    want = [S.scan_host_reference(sc, b, threads=2) for b in batches]
    got = [None] * len(batches)

    def run(k):
        got[k] = S.scan_host_reference(sc, batches[k], threads=2)
    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(batches))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert got == want
    assert sum(len(s["Findings"]) for w in want for s in w) > 10


def _scan_pinned(sc, c):
    L = _lib.lib()
    hp = ctypes.c_void_p()
    _lib.check(L.tsg_alloc_pinned(c.nbytes + 64, ctypes.byref(hp)))
    try:
        ctypes.memmove(hp, c.data.ctypes.data, c.nbytes)
        paths, lens, _keep = _lib.pack_paths(c.paths)
        res = ctypes.c_void_p()
        _lib.check(L.tsg_scan_batch(sc.engine(), hp, c.offsets.ctypes.data, len(c.paths), paths, lens, None,
                                    ctypes.byref(res)))
        try:
            out = _lib.result_json(res)
            stats = _lib.result_stats(res)
        finally:
            L.tsg_result_free(res)
    finally:
        L.tsg_free_pinned(hp)
    for s in out:
        s.pop("Error", None)
    return out, stats


@pytest.mark.gpu
def test_pinned_segments_equal_one_segment(monkeypatch):
    c, args = _corpus(24_000_000, 41)
    want = S.Scanner(None).ScanBatch(args)                  # one segment (< 512 MB)
    monkeypatch.setenv("TSG_SEGMENT_BYTES", str(1 << 20))
    got, stats = _scan_pinned(S.Scanner(None), c)
    assert stats["pieces"] >= 16
    assert stats["h2d_ms"] > 0 and stats["feed_ms"] > 0
    assert got == want
    # and the HBM-resident entry point on the same corpus
    import torch
    d = torch.from_numpy(np.ascontiguousarray(c.data)).to("cuda:0")
    L = _lib.lib()
    paths, lens, _keep = _lib.pack_paths(c.paths)
    res = ctypes.c_void_p()
    sc = S.Scanner(None)                                    # keeps the engine alive across the call
    _lib.check(L.tsg_scan_batch_resident(sc.engine(), ctypes.c_void_p(d.data_ptr()), c.data.ctypes.data,
                                         c.offsets.ctypes.data, len(c.paths), paths, lens, None, ctypes.byref(res)))
    try:
        res_json = _lib.result_json(res)
    finally:
        L.tsg_result_free(res)
    for s in res_json:
        s.pop("Error", None)
    assert res_json == want
    assert sum(len(w["Findings"]) for w in want) > 50


@pytest.mark.gpu
def test_concurrent_callers_share_one_engine(monkeypatch):
    monkeypatch.setenv("TSG_SEGMENT_BYTES", str(2 << 20))
    batches = [_corpus(8_000_000, 50 + k)[1] for k in range(4)]
    sc = S.Scanner(None, threads=4)
    want = [sc.ScanBatch(b) for b in batches]               # sequential
    got = [None] * len(batches)
    errs = []

    def run(k):
        try:
            for _ in range(3):
                got[k] = sc.ScanBatch(batches[k])
        except Exception as e:                               # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(batches))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=150)
    assert not errs, errs
    assert got == want


@pytest.mark.gpu
def test_multi_driver_queue_equals_single(monkeypatch):
    c, args = _corpus(30_000_000, 42)
    want = S.Scanner(None).ScanBatch(args)
    monkeypatch.setenv("TSG_ENGINE_REPLICAS", "3")
    monkeypatch.setenv("TSG_SEGMENT_BYTES", str(1 << 20))
    got, stats = S.Scanner(None).ScanBatch(args, with_stats=True)
    assert stats["devices"] == 3
    assert stats["pieces"] >= 20
    assert got == want


def test_many_files_result_vector_cpu():
    # > 64k files: the per-file result vector is constructed on several
    # threads (SecretVec::resize); every file keeps its own result
    n = 70_000
    args = [S.ScanArgs("/f/%d.txt" % i, b"plain text %d\n" % i) for i in range(n)]
    args[12345] = S.ScanArgs("/f/key.txt", b"token = ghp_" + b"a1B2" * 9 + b"\n")
    got = S.scan_table_model(S.Scanner(None), args)
    assert len(got) == n
    hits = [i for i, g in enumerate(got) if g.get("Findings")]
    assert hits == [12345] and got[12345]["FilePath"] == "/f/key.txt"


@pytest.mark.gpu
def test_failed_segment_leaves_lane_clean():
    """a direct (prologue-staged) small pinned batch whose segment
    run fails before its first launch must leave nothing staged on the pooled
    lane: the same engine's next scans -- resident (prologue stages only the
    offsets) and direct again -- equal a fresh engine's results."""
    import torch
    L = _lib.lib()
    small, small_args = _corpus(200_000, 61)               # <= 1 MiB: the direct (prologue-staged) path
    big, big_args = _corpus(6_000_000, 62)
    ref = S.Scanner(None)
    want_small = ref.ScanBatch(small_args)
    want_big = ref.ScanBatch(big_args)
    sc = S.Scanner(None, threads=2)
    for _ in range(3):
        _lib.check(L.tsg_test_inject_segment_failures(sc.engine(), 1))
        with pytest.raises(Exception, match="injected segment failure"):
            _scan_pinned(sc, small)
        # resident: the prologue copies the staged offsets only
        d = torch.from_numpy(np.ascontiguousarray(np.concatenate([big.data[:big.nbytes], np.zeros(64, np.uint8)])))
        d = d.to("cuda:0")
        paths, lens, _keep = _lib.pack_paths(big.paths)
        res = ctypes.c_void_p()
        _lib.check(L.tsg_scan_batch_resident(sc.engine(), ctypes.c_void_p(d.data_ptr()), big.data.ctypes.data,
                                             big.offsets.ctypes.data, len(big.paths), paths, lens, None,
                                             ctypes.byref(res)))
        try:
            got = _lib.result_json(res)
        finally:
            L.tsg_result_free(res)
        for s in got:
            s.pop("Error", None)
        assert got == want_big
        got_small, _ = _scan_pinned(sc, small)
        assert got_small == want_small
    assert sum(len(w["Findings"]) for w in want_big) > 5
