"""Per-file Scan for unchanged callers (tsg_queue_*): Trivy's
SecretAnalyzer.Analyze calls Scanner.Scan once per file (pkg/fanal/analyzer/
secret/secret.go:137) from --parallel goroutines (analyzer.go:434-451,
default 5).  Concurrent Scan calls through the queue share engine batches and
each gets exactly Scan(its file): compared with one ScanBatch of the same
files and with the oracle, from 5 and 16 caller threads (Python threads, and
the C-level probe)."""
import threading

import pytest

from oracle import secret_oracle as so
from trivy_amd import secret as S
from workload import synth

pytestmark = pytest.mark.gpu


def _files(seed, n_bytes=6_000_000):
    c = synth.generate(n_bytes, seed=seed, sizes="lognormal", plant_rate=5e-3)
    return [S.ScanArgs(c.paths[i], c.file(i)) for i in range(len(c.paths))]


@pytest.mark.parametrize("callers", [5, 16])
def test_queue_scan_equals_batch_gpu(callers):
    sc = S.Scanner(None)
    args = _files(21 + callers)
    want = sc.ScanBatch(args)
    q = S.ScanQueue(sc, max_inflight=2)       # more callers than batch slots: calls share batches
    got = [None] * len(args)
    nxt = [0]
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(args):
                return
            got[i] = q.Scan(args[i])
    ts = [threading.Thread(target=worker) for _ in range(callers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert got == want
    st = q.stats()
    assert st["calls"] == st["files"] == len(args)
    assert st["batches"] < len(args) and st["max_batch"] > 1          # calls shared batches
    ref = so.Scanner(None)
    sample = list(range(0, len(args), 7))
    assert [got[i] for i in sample] == [ref.scan(args[i].FilePath, args[i].Content) for i in sample]
    assert sum(len(g["Findings"]) for g in got) > 0
    q.close()


def test_queue_probe_and_single_caller_gpu():
    sc = S.Scanner(None)
    args = _files(31)
    want = sc.ScanBatch(args)
    q = S.ScanQueue(sc, max_wait_us=0)
    sec, nf = q.probe(args, 8)
    assert nf == sum(len(w["Findings"]) for w in want) and sec > 0
    assert q.Scan(args[0]) == want[0]                      # one caller alone: a batch of one, no waiting
    assert q.Scan(S.ScanArgs("empty.txt", b"")) == {"FilePath": "", "Findings": []}
    q.close()


def test_queue_spread_default_gpu():
    # the default queue (8 batch slots) with Trivy's default --parallel 5:
    # every call runs as its own concurrent one-file batch on its own lane,
    # and every caller gets exactly its file's result
    sc = S.Scanner(None)
    args = _files(41)
    want = sc.ScanBatch(args)
    q = S.ScanQueue(sc)
    got = [None] * len(args)
    nxt = [0]
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(args):
                return
            got[i] = q.Scan(args[i])
    ts = [threading.Thread(target=worker) for _ in range(5)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    st = q.stats()
    q.close()
    assert got == want
    assert st["calls"] == st["files"] == st["batches"] == len(args) and st["max_batch"] == 1


def test_queue_footprint_16_callers_gpu():
    """the default queue splits callers over up to 8 concurrent
    batches, each an Engine::scan with its own lane.  16 callers on a fresh
    engine create at most max_inflight lanes and call contexts, and per-file
    batches (confirmed inline) start no confirm-pool threads."""
    import ctypes
    from trivy_amd import _lib
    sc = S.Scanner(None)
    args = _files(51, n_bytes=3_000_000)
    q = S.ScanQueue(sc)                         # default: 8 batch slots
    sec, nf = q.probe(args, 16)
    st = q.stats()
    q.close()
    assert sec > 0 and st["files"] == len(args)
    lanes, calls, threads = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(_lib.lib().tsg_test_engine_footprint(sc.engine(), ctypes.byref(lanes), ctypes.byref(calls),
                                                    ctypes.byref(threads)))
    assert 1 <= lanes.value <= 8, lanes.value
    assert 1 <= calls.value <= 8, calls.value
    # batches of <= 4 files / 512 KB confirm on the calling thread and start
    # no pool; a leader that gathered a larger batch starts one of <= 16 threads
    assert threads.value <= 16 * calls.value, (threads.value, calls.value)
    print("queue footprint, 16 callers: lanes %d, call contexts %d, pool threads %d, max batch %d"
          % (lanes.value, calls.value, threads.value, st["max_batch"]))
