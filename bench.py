#!/usr/bin/env python
"""bench.py -- GB/s secret-scanned (builtin rules) on MI355X, findings diff = 0.

Workload (BASELINE.json configs[1], the metric's config): a 10 GB synthetic
text/source corpus per GPU (log-uniform file sizes 64 B - 64 MB, ~0.01% of
lines carry planted secrets drawn from all 87 builtin rules, 10% near misses)
scanned with the builtin rules.

One step = SURVEY.md 8(d)'s wall clock: the packed batch in PINNED HOST
memory -> tsg_scan_batch -> assembled types.Secret results for every file.
Inside, the engine streams the batch to HBM in 4 GiB segments (the rest
after the last full one is one more segment; upload of segment k+1 on a copy
stream overlapping K1/K2 of segment k and the host confirmation of segment
k-1), so `value` includes PCIe.  Reported beside it,
never as `value`: the HBM-resident rate (corpus already in HBM), the
host-feed ceiling (the same segmented upload with no kernels) and the host
content-preparation rate (tsg_prepare_batch).

  python bench.py [--gpus N --steps K --warmup W --config 1|2|3|5 --gb G]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Multi-GPU: each rank scans its own file shard (seed + rank, weak scaling) on
its own GPU; there is no collective on the data path (gloo carries only the
barrier and the max-time reduction).  Rank 0 prints one JSON line.

Extra fields: roofline (K1, HBM bound: achieved = content bytes / summed K1
time from HIP events on the engine's compute stream over the timed steps;
per-launch figures from the same events), cpu_baseline (the oracle --
oracle/secret_oracle.py, a Python restatement of the reference Go scanner --
on a bounded sample of the same corpus with a process pool), parity (GPU
findings vs the oracle on that sample; the run exits 1 unless diff = 0 and
the oracle evaluated every sampled file).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# the bench owns its process: keep the confirmation's freed heap across steps
# (the library's opt-in allocator policy; TSG_MALLOC_TUNE=0 to
# measure without it)
os.environ.setdefault("TSG_MALLOC_TUNE", "1")

HBM_PEAK_GBPS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md)
PCIE_PEAK_GBPS = 63.0     # PCIe Gen5 x16 spec per direction (MI355X_MICROARCH.md "Host link")


def _oracle_worker_init(cfg_path):
    global _ORACLE
    from oracle import secret_oracle as so
    _ORACLE = so.Scanner(so.parse_config(cfg_path) if cfg_path else None)


def _oracle_scan(item):
    path, content, binary = item
    return _ORACLE.scan(path, content, binary)


def cpu_baseline(items, procs, cfg_path=None, log=None, what="oracle"):
    """Oracle over `items` [(path, content, binary)] with a process pool; a
    progress line every ~20 s through `log` (a silent multi-minute leg looks
    hung to the GPU runner)."""
    import multiprocessing as mp
    nbytes = sum(len(c) for _, c, _ in items)
    ctx = mp.get_context("fork")
    with ctx.Pool(procs, initializer=_oracle_worker_init, initargs=(cfg_path,)) as pool:
        t0 = time.perf_counter()
        # largest files first (LPT): one 64 MB file is seconds of oracle work
        order = sorted(range(len(items)), key=lambda j: -len(items[j][1]))
        res = [None] * len(items)
        t_log, done_b = t0, 0
        for j, r in zip(order, pool.imap(_oracle_scan, [items[j] for j in order], chunksize=1)):
            res[j] = r
            done_b += len(items[j][1])
            if log is not None and time.perf_counter() - t_log > 20:
                t_log = time.perf_counter()
                log("%s: %.2f of %.2f GB checked (%.0f s)" % (what, done_b / 1e9, nbytes / 1e9, t_log - t0))
        dt = time.perf_counter() - t0
    return nbytes / dt / 1e9, res, dt, nbytes


def pick_sample(offsets, target_bytes, seed, large=8 << 20, large_share=0.5):
    """A seeded sample of files of about target_bytes: files up to `large`
    bytes fill (1 - large_share) of it, files above `large` (up to the 64 MB
    maximum) the rest, so the oracle also checks the batch's largest files."""
    rng = np.random.default_rng(seed)
    n = len(offsets) - 1
    small_t, large_t = target_bytes * (1 - large_share), target_bytes * large_share
    idx, st, lt = [], 0, 0
    for i in rng.permutation(n):
        sz = int(offsets[i + 1] - offsets[i])
        if sz > large:
            if lt >= large_t:
                continue
            lt += sz
        else:
            if st >= small_t:
                continue
            st += sz
        idx.append(int(i))
        if st >= small_t and lt >= large_t:
            break
    return sorted(idx)


def pick_parity(offsets, base_idx, share, seed, large=8 << 20):
    """The parity leg's files: the CPU-baseline sample `base_idx`, every file
    above `large` bytes, then seeded small files until the set holds `share`
    of the batch's bytes (>= 50% of the step's bytes)."""
    n = len(offsets) - 1
    sizes = np.diff(np.asarray(offsets, dtype=np.int64))
    total = int(sizes.sum())
    chosen = np.zeros(n, dtype=bool)
    chosen[np.asarray(base_idx, dtype=np.int64)] = True
    chosen |= sizes > large
    have = int(sizes[chosen].sum())
    if have < share * total:
        for i in np.random.default_rng(seed + 1).permutation(n):
            if chosen[i]:
                continue
            chosen[i] = True
            have += int(sizes[i])
            if have >= share * total:
                break
    return [int(i) for i in np.nonzero(chosen)[0]]


def _alloc_pinned(L, n):
    from trivy_amd import _lib
    ptr = ctypes.c_void_p()
    _lib.check(L.tsg_alloc_pinned(n, ctypes.byref(ptr)))
    return ptr, np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(n,))


class PinnedAlloc:
    """synth.generate(alloc=...) hook: the corpus is written straight into
    pinned host memory (one host copy of the batch per rank, not three)."""

    def __init__(self, L):
        self.L, self.ptr, self.view = L, None, None

    def __call__(self, n):
        assert self.ptr is None
        self.ptr, self.view = _alloc_pinned(self.L, n)
        return self.view


class PinnedBatch:
    """A packed batch in pinned host memory (tsg_alloc_pinned) + offsets, paths, binary flags."""

    def __init__(self, L, data_u8, offsets, paths, binary=None, pinned=None, prepared=None):
        """Copies data_u8 into new pinned memory, or adopts `pinned` (a
        PinnedAlloc the data was generated into) or `prepared` (a tsg_prepared
        handle whose data is pinned) without a copy."""
        from trivy_amd import _lib
        self.L = L
        self.nbytes = int(offsets[-1])
        self.prepared = prepared
        if prepared is not None:
            d_ = ctypes.c_void_p()
            o_, i_, b_, nk = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint32()
            _lib.check(L.tsg_prepared_view(prepared, ctypes.byref(d_), ctypes.byref(o_), ctypes.byref(i_),
                                           ctypes.byref(b_), ctypes.byref(nk)))
            self.ptr = d_
            self.view = np.ctypeslib.as_array(ctypes.cast(d_, ctypes.POINTER(ctypes.c_uint8)),
                                              shape=(self.nbytes + 64,))
        elif pinned is not None:
            self.ptr, self.view = pinned.ptr, pinned.view
            pinned.ptr = None
        else:
            self.ptr, self.view = _alloc_pinned(L, self.nbytes + 64)
            self.view[:self.nbytes] = data_u8[:self.nbytes]
        self.view[self.nbytes:] = 0
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.paths = paths
        self.cpaths, self.clens, self._keep = _lib.pack_paths(paths)
        self.binary = None if binary is None else np.ascontiguousarray(binary, dtype=np.uint8)

    @property
    def nfiles(self):
        return len(self.paths)

    def file(self, i):
        return bytes(self.view[int(self.offsets[i]):int(self.offsets[i + 1])])

    def free(self):
        if self.prepared is not None:
            self.L.tsg_prepared_free(self.prepared)
            self.prepared = None
            self.ptr = ctypes.c_void_p()
        elif self.ptr:
            self.L.tsg_free_pinned(self.ptr)
            self.ptr = ctypes.c_void_p()


def layer_tar_rate(L, sc, batch, target_bytes, threads, stream_batch=256 << 20):
    """tsg_prepare_layer_tar over one PAX layer tar built from the batch's files
    (rate in tar bytes per second, pinned output), and the same layer through
    tsg_scan_layer_stream end to end (tar bytes -> findings)."""
    import io
    import tarfile
    from trivy_amd import _lib
    buf = io.BytesIO()
    nfiles, tot = 0, 0
    with tarfile.open(fileobj=buf, mode="w", format=tarfile.PAX_FORMAT) as tf:
        for i in range(batch.nfiles):
            c = batch.file(i)
            ti = tarfile.TarInfo(batch.paths[i].lstrip("/"))
            ti.size = len(c)
            tf.addfile(ti, io.BytesIO(c))
            nfiles += 1
            tot += len(c)
            if tot >= target_bytes:
                break
    tar_bytes = buf.getvalue()
    tar = np.frombuffer(tar_bytes, dtype=np.uint8)
    best, kept = None, 0
    for _ in range(3):
        h = ctypes.c_void_p()
        t0 = time.perf_counter()
        _lib.check(L.tsg_prepare_layer_tar(sc._rs, b"", tar.ctypes.data, len(tar), None, 0, None, 0, threads, 1,
                                           ctypes.byref(h)))
        dt = time.perf_counter() - t0
        d_, o_, i_, b_, nk = (ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(),
                              ctypes.c_uint32())
        _lib.check(L.tsg_prepared_view(h, ctypes.byref(d_), ctypes.byref(o_), ctypes.byref(i_), ctypes.byref(b_),
                                       ctypes.byref(nk)))
        kept = nk.value
        L.tsg_prepared_free(h)
        best = dt if best is None else min(best, dt)
    # the same layer streamed end to end (tsg_scan_layer_stream: walk + gate +
    # prep of batch k+1 overlapping the GPU scan of batch k) -> findings
    from trivy_amd import secret as S
    sbest, swalk, nfind = None, None, 0
    for _ in range(3):
        t0 = time.perf_counter()
        # results stay in the C result object (types.Secret per file), as in
        # the headline step; the walk dict (every walked path) is parsed
        res, walk = S.ScanLayerStream(sc, io.BytesIO(tar_bytes), threads=threads, batch_bytes=stream_batch,
                                      as_result=True)
        dt = time.perf_counter() - t0
        if sbest is None or dt < sbest:
            nf = L.tsg_result_num_files(res.handle)
            sbest, swalk, nfind = dt, walk, sum(L.tsg_result_num_findings(res.handle, i) for i in range(nf))
        del res
    stream = {"gbps": round(len(tar) / sbest / 1e9, 2), "s": round(sbest, 4), "findings": nfind,
              "batches": swalk["stats"]["batches"], "feed_ms": round(swalk["stats"]["feed_ms"], 1),
              "scan_ms": round(swalk["stats"]["scan_ms"], 1), "wait_ms": round(swalk["stats"]["wait_ms"], 1),
              "engine_wall_ms": round(swalk["stats"]["wall_ms"], 1),
              "batch_bytes": stream_batch, "of_walk_rate": round(best / sbest, 3),
              "note": "tsg_scan_layer_stream from an io.BytesIO reader to types.Secret results (C result object); "
                      "engine_wall_ms: the C call alone; of_walk_rate: against tsg_prepare_layer_tar over the "
                      "same tar already in memory (walk + prep, no scan)"}
    return len(tar) / best / 1e9, nfiles, kept, best, stream


def _fs_type(path):
    """Filesystem type of `path` from /proc/mounts (longest mount prefix)."""
    best, typ = "", "?"
    try:
        for line in open("/proc/mounts"):
            parts = line.split()
            mnt = parts[1]
            if (path == mnt or path.startswith(mnt.rstrip("/") + "/")) and len(mnt) > len(best):
                best, typ = mnt, parts[2]
    except OSError:
        pass
    return typ


def tree_feed(L, sc, batch, threads, base_dir):
    """`trivy fs` host feed over a real directory tree: the batch's files
    written under base_dir, then tsg_prepare_fs_tree (walker.FS.Walk +
    AnalyzeFile's gate + threaded reads + content prep into pinned memory)
    with the page cache warm and cold (every file's pages dropped with
    posix_fadvise(DONTNEED) after a sync), and the cold-read batch scanned by
    tsg_scan_batch: disk -> findings.  Checks the tree's prepared files equal
    tsg_prepare_batch over the same files in memory."""
    import shutil
    import tempfile
    from trivy_amd import _lib
    root = tempfile.mkdtemp(prefix="tsg_tree_", dir=base_dir)
    try:
        t0 = time.perf_counter()
        for i in range(batch.nfiles):
            fp = os.path.join(root, batch.paths[i])
            os.makedirs(os.path.dirname(fp), exist_ok=True)
            with open(fp, "wb") as f:
                f.write(memoryview(batch.view[int(batch.offsets[i]):int(batch.offsets[i + 1])]))
        os.sync()
        t_write = time.perf_counter() - t0

        def drop_cache():
            for i in range(batch.nfiles):
                fd = os.open(os.path.join(root, batch.paths[i]), os.O_RDONLY)
                try:
                    os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
                finally:
                    os.close(fd)

        def run(scan):
            o, _k = _lib.feed_opts(threads=threads, pinned=True)
            h = ctypes.c_void_p()
            t1 = time.perf_counter()
            _lib.check(L.tsg_prepare_fs_tree(sc._rs, os.fsencode(root), ctypes.byref(o), ctypes.byref(h)))
            dt = time.perf_counter() - t1
            walk = json.loads(L.tsg_prepared_walk_json(h).decode("utf-8", "surrogateescape"))
            d_, o_, i_, b_, nk = (ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(),
                                  ctypes.c_uint32())
            _lib.check(L.tsg_prepared_view(h, ctypes.byref(d_), ctypes.byref(o_), ctypes.byref(i_), ctypes.byref(b_),
                                           ctypes.byref(nk)))
            row = {"s": round(dt, 4), "walk_ms": round(walk["walk_ms"], 2), "read_ms": round(walk["read_ms"], 2),
                   "prep_ms": round(walk["prep_ms"], 2), "pinned_alloc_ms": round(walk["alloc_ms"], 2),
                   "read_bytes": walk["read_bytes"],
                   "gbps": round(walk["read_bytes"] / dt / 1e9, 3), "kept_files": nk.value}
            extra = None
            if scan:
                pp, pl = ctypes.POINTER(ctypes.c_char_p)(), ctypes.POINTER(ctypes.c_uint32)()
                _lib.check(L.tsg_prepared_paths(h, ctypes.byref(pp), ctypes.byref(pl)))
                res = ctypes.c_void_p()
                t2 = time.perf_counter()
                _lib.check(L.tsg_scan_batch(sc.engine(), d_, o_, nk.value, pp, ctypes.cast(pl, ctypes.c_void_p), b_,
                                            ctypes.byref(res)))
                ts = time.perf_counter() - t2
                row["scan_s"] = round(ts, 4)
                row["end_to_end_gbps"] = round(walk["read_bytes"] / (dt + ts) / 1e9, 3)
                got = _lib.result_json(res)
                L.tsg_result_free(res)
                n = nk.value
                offs = np.ctypeslib.as_array(ctypes.cast(o_, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,))
                data = np.ctypeslib.as_array(ctypes.cast(d_, ctypes.POINTER(ctypes.c_uint8)), shape=(int(offs[-1]),))
                names = [ctypes.string_at(pp[k], pl[k]).decode("utf-8", "surrogateescape") for k in range(n)]
                extra = ({names[k]: bytes(data[int(offs[k]):int(offs[k + 1])]) for k in range(n)},
                         {names[k]: got[k] for k in range(n)})
            L.tsg_prepared_free(h)
            return row, extra
        warm, _ = run(False)
        drop_cache()
        cold, (tree_files, tree_res) = run(True)
        # the same tree streamed (tsg_scan_fs_tree: reads + prep of batch k+1
        # overlapping the scan of batch k), page cache dropped again
        from trivy_amd import secret as S
        drop_cache()
        t1 = time.perf_counter()
        sresult, swalk = S.ScanFsTree(sc, root, threads=threads, batch_bytes=256 << 20, as_result=True)
        sdt = time.perf_counter() - t1
        sres = sresult.secrets()                 # (outside the timed region, as for the other legs)
        streamed = {"s": round(sdt, 4), "end_to_end_gbps": round(swalk["stats"]["read_bytes"] / sdt / 1e9, 3),
                    "engine_wall_ms": round(swalk["stats"]["wall_ms"], 1),
                    "batches": swalk["stats"]["batches"], "feed_ms": round(swalk["stats"]["feed_ms"], 1),
                    "scan_ms": round(swalk["stats"]["scan_ms"], 1),
                    "same_findings": {r["FilePath"]: r for r in sres if r["FilePath"]} ==
                                     {k: v for k, v in tree_res.items() if v["FilePath"]}}
        # parity: the tree's prepared files == tsg_prepare_batch over the same files in memory
        o, _k = _lib.feed_opts(threads=threads)
        h = ctypes.c_void_p()
        _lib.check(L.tsg_prepare_batch_opts(sc._rs, batch.ptr, batch.offsets.ctypes.data, batch.nfiles, batch.cpaths,
                                            batch.clens, ctypes.byref(o), ctypes.byref(h)))
        d_, o_, i_, b_, nk = (ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(),
                              ctypes.c_uint32())
        _lib.check(L.tsg_prepared_view(h, ctypes.byref(d_), ctypes.byref(o_), ctypes.byref(i_), ctypes.byref(b_),
                                       ctypes.byref(nk)))
        n = nk.value
        offs = np.ctypeslib.as_array(ctypes.cast(o_, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,))
        idx = np.ctypeslib.as_array(ctypes.cast(i_, ctypes.POINTER(ctypes.c_uint32)), shape=(n,))
        data = np.ctypeslib.as_array(ctypes.cast(d_, ctypes.POINTER(ctypes.c_uint8)), shape=(int(offs[-1]) + 1,))
        mem = {batch.paths[int(idx[k])]: bytes(data[int(offs[k]):int(offs[k + 1])]) for k in range(n)}
        L.tsg_prepared_free(h)
        same = mem == tree_files
        return {"files": batch.nfiles, "bytes": batch.nbytes, "dir_fs": _fs_type(os.path.realpath(root)),
                "write_s": round(t_write, 2), "warm": warm, "cold": cold, "streamed_cold": streamed,
                "prepared_equal_in_memory": same,
                "findings": sum(len(r["Findings"]) for r in tree_res.values()),
                "note": "tsg_prepare_fs_tree: walk + gate + %d reader threads + prep into pinned memory; cold = page "
                        "cache dropped per file (posix_fadvise DONTNEED after sync; no effect on tmpfs); the cold "
                        "batch then scanned by tsg_scan_batch (end_to_end = disk -> findings)" % threads}
    finally:
        shutil.rmtree(root, ignore_errors=True)


def small_batches(L, eng, batch, counts=(1, 5, 64), reps=40):
    """tsg_scan_batch latency on batches of 1 / 5 / 64 files of 8-32 KB (the
    per-file drop-in's batch sizes: unchanged Trivy calls Scan per file from
    --parallel goroutines, secret.go:137), pinned host memory, median of reps."""
    from trivy_amd import _lib
    sizes = np.diff(batch.offsets)
    pick = [i for i in range(batch.nfiles) if (8 << 10) <= sizes[i] <= (32 << 10)][:max(counts)]
    out = {}
    if len(pick) < max(counts):
        return {"note": "not enough 8-32 KB files in the batch"}
    for n in counts:
        files = [batch.file(i) for i in pick[:n]]
        offs = np.zeros(n + 1, np.uint64)
        offs[1:] = np.cumsum([len(f) for f in files])
        ptr, view = _alloc_pinned(L, int(offs[-1]) + 64)
        view[:int(offs[-1])] = np.frombuffer(b"".join(files), np.uint8)
        view[int(offs[-1]):] = 0
        paths, lens, _k = _lib.pack_paths([batch.paths[i] for i in pick[:n]])
        ts = []
        for r in range(reps + 3):
            res = ctypes.c_void_p()
            t0 = time.perf_counter()
            _lib.check(L.tsg_scan_batch(eng, ptr, offs.ctypes.data, n, paths, lens, None, ctypes.byref(res)))
            dt = time.perf_counter() - t0
            L.tsg_result_free(res)
            if r >= 3:
                ts.append(dt)
        L.tsg_free_pinned(ptr)
        med = float(np.median(ts))
        out[str(n)] = {"ms": round(med * 1e3, 3), "p90_ms": round(float(np.percentile(ts, 90)) * 1e3, 3),
                       "bytes": int(offs[-1]), "gbps": round(int(offs[-1]) / med / 1e9, 4)}
    return out


def per_file_queue(sc, batch, callers_list, max_bytes=256 << 20, target_bytes=256e6):
    """The per-file drop-in: `callers` threads (--parallel goroutines) each
    calling Scan on one file at a time through the shared queue (tsg_queue_*),
    over the batch's first files up to target_bytes."""
    from trivy_amd import secret as S
    n, tot = 0, 0
    while n < batch.nfiles and tot < target_bytes:
        tot += int(batch.offsets[n + 1] - batch.offsets[n])
        n += 1
    args = [S.ScanArgs(batch.paths[i], batch.file(i)) for i in range(n)]
    out = {"files": n, "bytes": tot}
    for c in callers_list:
        q = S.ScanQueue(sc, max_bytes=max_bytes)
        q.probe(args[:min(n, 200)], c)                       # warm (lanes, staging buffers)
        q.close()
        q = S.ScanQueue(sc, max_bytes=max_bytes)
        sec, nf = q.probe(args, c)
        st = q.stats()
        q.close()
        out["parallel_%d" % c] = {"gbps": round(tot / sec / 1e9, 4), "files_per_s": round(n / sec),
                                  "s": round(sec, 3), "findings": nf, "batches": st["batches"],
                                  "mean_batch_files": round(st["files"] / max(1, st["batches"]), 2),
                                  "max_batch_files": st["max_batch"]}
    return out


def numa_bind(device):
    """Pin this rank to the CPUs of its GPU's NUMA node (before the corpus and
    the pinned batch are allocated, so both are first-touched there and each
    GPU's DMA reads node-local memory).  Returns what was done, or None."""
    try:
        import torch
        pr = torch.cuda.get_device_properties(device)
        bdf = "%04x:%02x:%02x.0" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
        base = "/sys/bus/pci/devices/" + bdf
        node = int(open(base + "/numa_node").read().strip())
        cpus = set()
        for part in open(base + "/local_cpulist").read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        if node < 0 or len(cpus) < 8:
            return None
        os.sched_setaffinity(0, cpus)
        return {"pci": bdf, "numa_node": node, "cpus": len(cpus)}
    except Exception:
        return None


def available_cores():
    """CPUs this process may run on: the affinity set, capped by a cgroup CPU
    quota (cpu.max) when one is set.  Returns (cores, detail)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except Exception:
        pass
    cores = min(aff, quota) if quota else aff
    return cores, {"affinity": aff, "cgroup_quota_cpus": quota}


def rank_envs(n, port, base_env=None):
    """Environment of each of the n ranks `bench.py --gpus n` starts when it is
    not already running under torchrun (one process per GPU, rank r on HIP
    device r, its engine's device_mask = 1 << r)."""
    env0 = dict(os.environ if base_env is None else base_env)
    out = []
    for r in range(n):
        e = dict(env0)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "TSG_BENCH_LAUNCHED": "1"})
        out.append(e)
    return out


def launch_ranks(n, argv, dry=False):
    """`python bench.py --gpus n` without torchrun: start n rank processes
    (children, never an exec of this process) and return the worst exit code.
    Fails loudly before starting anything when fewer than n GPUs are visible
    (torch.cuda.device_count() does not initialise the GPU)."""
    import socket
    import subprocess
    if not dry:
        import torch
        have = torch.cuda.device_count()
        if have < n and not _share_devices():
            print("[bench] --gpus %d needs %d GPUs, %d visible" % (n, n, have), file=sys.stderr, flush=True)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    print("[bench] launcher: %d ranks, one per GPU, rendezvous 127.0.0.1:%d" % (n, port), file=sys.stderr, flush=True)
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e) for e in rank_envs(n, port)]
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0:
                    rc = rc or r
                    for q in pending:          # one rank failed: the others cannot finish their barriers
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def k1_build(src=None):
    """Build hash of K1's source in trivy_amd/csrc/engine.hip: the file up to
    its "==== K2 begin" line (the readback / prologue kernels, K1's stream
    state, word steps and output handling) plus "==== K2 end" .. "==== host
    side" (K1's line loop, tsg_k1_scan_v3 itself and its build table).  K2 and
    the host code are left out.  A committed traffic measurement applies only
    to the K1 build it was taken on.  src: the file's bytes (tests)."""
    import hashlib
    if src is None:
        with open(os.path.join(ROOT, "trivy_amd", "csrc", "engine.hip"), "rb") as f:
            src = f.read()
    a = src.find(b"\n// ==== K2 begin")
    b = src.find(b"\n// ==== K2 end")
    c = src.find(b"\n// ==== host side")
    if min(a, b, c) < 0 or not a < b < c:
        raise RuntimeError("engine.hip lacks the K1 build-hash markers")
    import re
    # the measurement builds listed under #ifdef TSG_K1_PROBE exist only in
    # the probe library: not part of the product's K1
    k1 = re.sub(rb"#ifdef TSG_K1_PROBE\n.*?#endif[^\n]*\n", b"", src[:a] + src[b:c], flags=re.S)
    return hashlib.sha256(k1).hexdigest()[:16]


def gather_ranks(dist, world, mine):
    """Every rank's record on every rank (gloo all_gather_object), rank order."""
    if not dist:
        return [mine]
    got = [None] * world
    dist.all_gather_object(got, mine)
    return got


def _share_devices():
    """rehearsal of the N-rank path on fewer GPUs (TSG_BENCH_SHARE_DEVICES=1): never a metric run"""
    return os.environ.get("TSG_BENCH_SHARE_DEVICES", "0") == "1"


def _segment_balanced():
    """large-file batches cut into equal segments (engine default; TSG_SEGMENT_BALANCED=0: full segments + rest)"""
    return os.environ.get("TSG_SEGMENT_BALANCED", "1") != "0"


def _segment_bytes():
    v = os.environ.get("TSG_SEGMENT_BYTES")
    return int(v) if v and int(v) >= 4096 else 4 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each); without torchrun, bench.py starts the ranks itself")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5],
                    help="BASELINE.json config: 1 = 1 GB source tree (log-normal sizes), 2 = 10 GB source "
                         "corpus (the metric's workload), 3 = extracted image layers (small files; bytes counted "
                         "after Required), 4 = 200 GB as 20 config-2 shards split over the ranks (one step streams "
                         "the rank's shards), 5 = 500 custom rules + allow rules + exclude blocks")
    ap.add_argument("--distinct-shards", type=int, default=2,
                    help="config 4: distinct generated shards per rank, cycled over its shards (generation of a "
                         "10 GB shard takes ~5 s, 20 of them would dominate the run)")
    ap.add_argument("--gb", type=float, default=None, help="corpus GB per GPU (default: 1 for config 1, else 10)")
    ap.add_argument("--seed", type=int, default=0x71215EC7)
    ap.add_argument("--threads", type=int, default=16, help="host confirm threads per rank")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="CPU baseline workers (default: every core this rank may use, SURVEY 8d's T = nproc)")
    ap.add_argument("--cpu-sample-mb", type=float, default=1200.0)
    ap.add_argument("--parity-share", type=float, default=0.5,
                    help="the oracle checks at least this share of the step's bytes (every file above 8 MB, the "
                         "CPU-baseline sample, then seeded small files); 0 = the CPU-baseline sample only")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-resident", action="store_true", help="skip the HBM-resident comparison leg")
    ap.add_argument("--resident-keep", action="store_true",
                    help="diagnostic: keep the resident leg's results until its timed steps are done (their frees "
                         "then run after the timing instead of on the reaper thread beside the next steps)")
    ap.add_argument("--tree", type=int, default=-1,
                    help="1: also measure the `trivy fs` feed over the batch written as a directory tree "
                         "(default: config 1 only)")
    ap.add_argument("--tree-dir", default=os.environ.get("TSG_TREE_DIR", "/tmp"))
    ap.add_argument("--per-file", type=int, default=-1,
                    help="1: also time the per-file drop-in (small batches, the Scan queue at --parallel 5 and at "
                         "the rank's core count); default: config 1 only")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--dry-launch", action="store_true",
                    help="ranks only report their wiring (rank, device, device_mask) and exit: the launcher's "
                         "CPU test")
    args = ap.parse_args()
    gb = args.gb if args.gb is not None else (1.0 if args.config == 1 else 10.0)

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], dry=args.dry_launch))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print("[bench] --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr, flush=True)
        sys.exit(2)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    if args.dry_launch:
        # the wiring, and the per-rank gather the real run uses for its
        # concurrent feed ceiling (a host memcpy probe stands in for the PCIe
        # upload, every rank at once after a barrier)
        wiring = {"rank": rank, "world": world, "local_rank": local_rank, "device": local_rank,
                  "device_mask": 1 << local_rank}
        if dist:
            dist.barrier()
        src = np.ones(64 << 20, np.uint8)
        dst = np.empty_like(src)
        t0 = time.perf_counter()
        for _ in range(4):
            np.copyto(dst, src)
        wiring["ceiling_gbps"] = round(4 * src.nbytes / (time.perf_counter() - t0) / 1e9, 2)
        got = gather_ranks(dist, world, wiring)
        if dist:
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"dry_launch": got, "ceiling_gbps_all_ranks": round(sum(g["ceiling_gbps"] for g in got), 2)}),
                  flush=True)
        return

    import torch
    if torch.cuda.device_count() <= local_rank and not _share_devices():
        print("[bench] rank %d needs HIP device %d, %d visible" % (rank, local_rank, torch.cuda.device_count()),
              file=sys.stderr, flush=True)
        sys.exit(2)

    from trivy_amd import _lib
    from trivy_amd import secret as S
    from workload import synth

    def log(*a):
        if rank == 0:
            print("[bench]", *a, file=sys.stderr, flush=True)

    L = _lib.lib()
    # (TSG_BENCH_SHARE_DEVICES=1, rehearsal only: ranks beyond the visible
    # devices share them round-robin, so the N-rank path runs on a 1-GPU box)
    device = local_rank % torch.cuda.device_count() if _share_devices() else local_rank
    torch.cuda.set_device(device)
    numa = numa_bind(device)
    cores, cores_detail = available_cores()

    # ---------------------------------------------------------------- workload
    t_gen = time.perf_counter()
    cfg_path = None
    sizes = {1: "lognormal", 2: "loguniform", 3: "small", 4: "loguniform", 5: "lognormal"}[args.config]
    # configs other than 3 scan the files as generated: generate them straight
    # into the pinned batch (config 3 scans tsg_prepare_batch's output)
    palloc = PinnedAlloc(L) if args.config != 3 else None
    corpus = synth.generate(int(gb * 1e9), seed=args.seed + rank, sizes=sizes,
                            layout="image" if args.config == 3 else "src", alloc=palloc,
                            progress=lambda i, n: log("generating: %d of %d files" % (i, n)))
    if args.config == 5:      # 500 custom rules + allow rules + exclude blocks (+ builtins)
        cfg5, plants = synth.config5(500, seed=args.seed)
        cfg_path = "/tmp/tsg_bench_config5_%d.yaml" % rank
        synth.write_yaml(cfg5, cfg_path)
        synth.plant_custom(corpus, plants, seed=args.seed + rank, rate=1e-4)
    raw_bytes, raw_files = corpus.nbytes, len(corpus.paths)
    log("corpus: %.2f GB, %d files, %d plants (%d near-miss), generated in %.1fs" % (
        raw_bytes / 1e9, raw_files, corpus.planted, corpus.near_miss, time.perf_counter() - t_gen))

    sc = S.Scanner(S.ParseConfig(cfg_path) if cfg_path else None, device=device, threads=args.threads)
    eng = sc.engine()

    # host content preparation over the files as read (SecretAnalyzer.Required +
    # IsBinary + CR strip + .pyc extraction, tsg_prepare_batch); for config 3
    # its output IS the scanned batch (bytes counted after gating)
    # (measured on rank 0 only for configs other than 3: its output is a second
    # copy of the batch, which every rank of an 8-GPU node need not hold)
    prep_gbps, nk = None, ctypes.c_uint32()
    hpb = ctypes.c_void_p()
    if args.config == 3 or rank == 0:
        paths, lens, _keep = _lib.pack_paths(corpus.paths)
        # config 3 prepares straight into pinned memory: its output is the batch
        fo, _fkeep = _lib.feed_opts(threads=args.threads, pinned=args.config == 3)
        t0 = time.perf_counter()
        _lib.check(L.tsg_prepare_batch_opts(sc._rs, corpus.data.ctypes.data, corpus.offsets.ctypes.data, raw_files,
                                            paths, lens, ctypes.byref(fo), ctypes.byref(hpb)))
        tprep = time.perf_counter() - t0
        d_, o_, i_, b_ = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(L.tsg_prepared_view(hpb, ctypes.byref(d_), ctypes.byref(o_), ctypes.byref(i_),
                                       ctypes.byref(b_), ctypes.byref(nk)))
        prep_gbps = raw_bytes / tprep / 1e9
        del paths, lens, _keep
        log("host feed prepare (Required + IsBinary + CR strip, %d threads): %.1f GB/s, %d of %d files kept" % (
            args.threads, prep_gbps, nk.value, raw_files))
    if args.config == 3:
        n = nk.value
        offs = np.ctypeslib.as_array(ctypes.cast(o_, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,)).copy()
        index = np.ctypeslib.as_array(ctypes.cast(i_, ctypes.POINTER(ctypes.c_uint32)), shape=(n,)).copy()
        binf = np.ctypeslib.as_array(ctypes.cast(b_, ctypes.POINTER(ctypes.c_uint8)), shape=(n,)).copy()
        # image scans prefix "/" to layer paths (analyzer secret.go:133-135)
        scan_paths = ["/" + corpus.paths[i] for i in index]
        batch = PinnedBatch(L, None, offs, scan_paths, binf, prepared=hpb)   # owns hpb now
    else:
        batch = PinnedBatch(L, None, corpus.offsets, corpus.paths, pinned=palloc)
        if hpb:
            L.tsg_prepared_free(hpb)
    del corpus
    nfiles, nbytes = batch.nfiles, batch.nbytes
    bin_ptr = batch.binary.ctypes.data if batch.binary is not None else None
    # config 4: this rank's share of 20 config-2 shards, streamed one after
    # another from pinned memory (the distinct shards cycled)
    shard_batches, nshards = [batch], 1
    if args.config == 4:
        nshards = -(-20 // world)
        for j in range(1, min(args.distinct_shards, nshards)):
            pa = PinnedAlloc(L)
            c2 = synth.generate(int(gb * 1e9), seed=args.seed + 1000 * j + rank, sizes=sizes, layout="src",
                                alloc=pa)
            shard_batches.append(PinnedBatch(L, None, c2.offsets, c2.paths, pinned=pa))
            del c2
        nbytes = sum(shard_batches[k % len(shard_batches)].nbytes for k in range(nshards))
        log("config 4: %d shards per rank (%d distinct), %.1f GB per rank per step" % (
            nshards, len(shard_batches), nbytes / 1e9))

    def scan_one(b):
        res = ctypes.c_void_p()
        _lib.check(L.tsg_scan_batch(eng, b.ptr, b.offsets.ctypes.data, b.nfiles, b.cpaths, b.clens,
                                    b.binary.ctypes.data if b.binary is not None else None, ctypes.byref(res)))
        return res

    def step():
        """One step: the rank's batch (config 4: its shards); returns the last
        result and the step's stats (summed over shards)."""
        if nshards == 1:
            res = scan_one(batch)
            return res, _lib.result_stats(res)
        agg = None
        res = None
        for k in range(nshards):
            if res is not None:
                L.tsg_result_free(res)
            res = scan_one(shard_batches[k % len(shard_batches)])
            st = _lib.result_stats(res)
            if agg is None:
                agg = dict(st)
            else:
                for key in ("k1_ms", "k2_ms", "host_ms", "h2d_ms", "feed_ms", "total_ms", "k1_launches", "pieces",
                            "hits", "candidates", "confirm_files"):
                    agg[key] += st[key]
        return res, agg

    # ------------------------------------------------------- timed (pinned host)
    for _ in range(args.warmup):
        L.tsg_result_free(step()[0])
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    stats = []
    last = None
    free_s = 0.0
    t0 = time.perf_counter()
    for k in range(args.steps):
        res, st = step()
        stats.append(st)
        if k == args.steps - 1:
            last = res
        else:
            tf = time.perf_counter()
            L.tsg_result_free(res)
            free_s += time.perf_counter() - tf
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    b = torch.tensor([float(nbytes)], dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
    elapsed_max = float(t[0])
    value = float(b[0]) * args.steps / elapsed_max / 1e9

    def mean(key):
        return float(np.mean([s[key] for s in stats]))
    k1_ms, k2_ms, host_ms, h2d_ms = mean("k1_ms"), mean("k2_ms"), mean("host_ms"), mean("h2d_ms")
    launches = max(1, int(stats[-1]["k1_launches"]))
    segments = max(1, int(stats[-1]["pieces"]))
    groups = max(1, launches // segments)
    if nshards > 1:                    # config 4: the parity legs below check the first shard's batch
        L.tsg_result_free(last)
        last = scan_one(batch)
    gpu_results = _lib.result_json(last)
    L.tsg_result_free(last)
    findings = sum(len(s["Findings"]) for s in gpu_results)
    rules_hit = sorted({f["RuleID"] for s in gpu_results for f in s["Findings"]})
    k1_gbps = nbytes / (k1_ms / 1e3) / 1e9
    log("step %.1f ms (%.1f GB/s incl. PCIe): K1 %.2f ms in %d launches (%.0f GB/s), K2 %.2f ms, H2D %.1f ms, "
        "host confirm %.1f ms; hits %d, candidates %d, findings %d over %d rules" % (
            elapsed_max / args.steps * 1e3, value, k1_ms, launches, k1_gbps, k2_ms, h2d_ms, host_ms,
            stats[-1]["hits"], stats[-1]["candidates"], findings, len(rules_hit)))

    # HBM traffic of K1 (PMC FETCH_SIZE + WRITE_SIZE, corrected as the microarch
    # guide prescribes) from a rocprofv3 run of this same layout AND this same
    # K1 build (profiles/traffic_c<config>.json carries the build hash of
    # engine.hip it was measured on; a file from another build is refused)
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "traffic_c%d.json" % args.config)
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        lay = tj.get("layout", {})
        if (tj.get("k1_build") == k1_build() and lay.get("config") == args.config
                and lay.get("segment_bytes") == _segment_bytes() and lay.get("chunk_bytes") == stats[-1]["chunk_bytes"]
                and (args.config not in (2, 4) or lay.get("segment_balanced", False) == _segment_balanced())):
            traffic = round(tj["traffic_over_algorithmic"] * nbytes / segments)
            traffic_src = "%s: %.3f HBM bytes per content byte, K1 dispatches of this layout and build %s (%s)" % (
                os.path.relpath(tpath, ROOT), tj["traffic_over_algorithmic"], tj["k1_build"], tj.get("source", ""))

    workload = {
        1: "config1: %.0f GB synthetic source tree (log-normal sizes, median 16 KB), builtin rules" % gb,
        2: "config2: %.0f GB synthetic text/source corpus per GPU, log-uniform 64 B-64 MB files, 0.01%% planted "
           "secrets (87 builtin rules), builtin rules" % gb,
        3: "config3: %.0f GB of extracted-image-layer small files per GPU (mean ~25 KB, rootfs paths), scanned "
           "after Required/IsBinary/CR strip (tsg_prepare_batch), '/'-prefixed image paths, builtin rules" % gb,
        4: "config4: 200 GB = 20 config-2 shards (%.0f GB each, log-uniform 64 B-64 MB files), %d per GPU streamed "
           "one after another from pinned memory (%d distinct generated shards cycled), builtin rules" % (
               gb, nshards, len(shard_batches)),
        5: "config5: %.0f GB synthetic source corpus per GPU, trivy-secret.yaml with 500 custom rules + 87 "
           "builtins, 20 allow rules, 5 exclude blocks" % gb,
    }[args.config]
    out = {
        "metric": "GB/s secret-scanned (builtin rules) at 1/2/4/8 MI355X; findings diff = 0",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        **({"rehearsal": "TSG_BENCH_SHARE_DEVICES=1: ranks share %d device(s); not a metric run"
                         % torch.cuda.device_count()} if _share_devices() else {}),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (workload/synth.py, seed %#x + rank)" % args.seed,
        "config": {
            "workload": workload + "; one step = packed batch in pinned host memory -> tsg_scan_batch -> "
                                   "types.Secret for every file (PCIe upload included)",
            "bytes_per_gpu": nbytes,
            "files_per_gpu": nfiles,
            "raw_bytes_per_gpu": raw_bytes,
            "raw_files_per_gpu": raw_files,
            "parallelism": "file shards per GPU, no collective (dp%d)" % world,
            "host_confirm_threads": args.threads,
            "segment_bytes": _segment_bytes(),
            "segment_balanced": _segment_balanced(),
            "config_id": args.config,
            "numa": numa,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "tsg_k1_scan",
            "k1_build": k1_build(),
            "achieved": round(k1_gbps, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(k1_gbps / HBM_PEAK_GBPS, 5),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes": "1 byte read per content byte (SURVEY 8d); scan-DFA groups: %d" % groups,
            "launches_per_step": launches,
            "bytes_per_launch": round(nbytes / launches * groups),
            "avg_launch_ms": round(k1_ms / launches, 4),
            "per_launch_gbps": round(nbytes / launches * groups / (k1_ms / launches / 1e3) / 1e9, 2),
            "note": "mean over the step's K1 launches (segments of unequal size; each segment is read once "
                    "per scan-DFA group, the bytes counted once as SURVEY 8d prescribes)",
        },
        "link": {"bound": "pcie", "achieved": round(nbytes / (h2d_ms / 1e3) / 1e9, 2), "peak": PCIE_PEAK_GBPS,
                 "unit": "GB/s", "note": "H2D copy time of the step's segments (copy-stream HIP events)"},
        "breakdown_ms": {"segments": segments, "chunk_bytes": stats[-1]["chunk_bytes"], "k1": round(k1_ms, 3), "k2": round(k2_ms, 3),
                         "h2d": round(h2d_ms, 3), "host_confirm": round(host_ms, 3),
                         "feed": round(mean("feed_ms"), 3), "engine_total": round(mean("total_ms"), 3),
                         "result_free": round(free_s / max(1, args.steps - 1) * 1e3, 3),
                         "hits": stats[-1]["hits"], "candidates": stats[-1]["candidates"],
                         "confirm_files": stats[-1]["confirm_files"], "findings": findings,
                         "rules_with_findings": len(rules_hit)},
        "host_feed": {"prepare_gbps": None if prep_gbps is None else round(prep_gbps, 2),
                      "prepare_kept_files": nk.value if prep_gbps is not None else None},
        "cpu_baseline": None,
        "parity": None,
    }

    # host-feed ceiling: the same segmented upload with no kernels, every rank
    # at once after a barrier (the ranks share host DRAM and the root
    # complexes: the concurrent sum is the node's feed ceiling)
    fms = ctypes.c_double()
    if dist:
        dist.barrier()
    _lib.check(L.tsg_feed_probe(eng, batch.ptr, batch.nbytes, ctypes.byref(fms)))
    my_ceiling = batch.nbytes / (fms.value / 1e3) / 1e9
    mine = {"rank": rank, "device": device, "numa": numa, "ceiling_gbps": round(my_ceiling, 2),
            "link_gbps": round(nbytes / (h2d_ms / 1e3) / 1e9, 2), "step_ms": round(elapsed / args.steps * 1e3, 3),
            "k1_ms": round(k1_ms, 3), "k2_ms": round(k2_ms, 3), "h2d_ms": round(h2d_ms, 3),
            "host_confirm_ms": round(host_ms, 3), "bytes": nbytes}
    ranks = gather_ranks(dist, world, mine)
    out["host_feed"]["ceiling_gbps"] = round(my_ceiling, 2)
    out["host_feed"]["ceiling_gbps_all_ranks"] = round(sum(r["ceiling_gbps"] for r in ranks), 2)
    out["per_rank"] = ranks
    out["host_feed"]["note"] = ("ceiling_gbps: tsg_feed_probe on rank 0, the step's segmented pinned upload with no "
                                "kernels; ceiling_gbps_all_ranks: the same probe on every rank at once after a "
                                "barrier, summed (the node's concurrent host-feed ceiling to set `value` against); "
                                "prepare_gbps: tsg_prepare_batch over the raw files")
    log("host-feed ceiling (segmented pinned upload, no kernels): %.1f GB/s on rank 0, %.1f GB/s over %d ranks at "
        "once" % (my_ceiling, out["host_feed"]["ceiling_gbps_all_ranks"], world))
    if args.config == 3 and rank == 0:
        # the image path's host feed from a layer tar: walker.LayerTar.Walk +
        # Required + content prep into pinned memory (tsg_prepare_layer_tar)
        tgb, tfiles, tkept, tdt, tstream = layer_tar_rate(L, sc, batch, 2e9, args.threads)
        out["host_feed"]["layer_tar_gbps"] = round(tgb, 2)
        out["host_feed"]["layer_tar_sample"] = "%d files / %.0f MB of this batch written as one PAX layer tar, %d " \
                                               "kept, best of 3: %.1f ms" % (tfiles, tgb * tdt * 1e3, tkept, tdt * 1e3)
        out["host_feed"]["layer_tar_to_findings"] = tstream
        log("layer-tar feed (walk + Required + prep into pinned memory, %d threads): %.1f GB/s; streamed end to end "
            "(tar -> findings, tsg_scan_layer_stream): %.1f GB/s = %.2f of the walk rate" % (
                args.threads, tgb, tstream["gbps"], tstream["of_walk_rate"]))

    if rank == 0 and (args.tree == 1 or (args.tree == -1 and args.config == 1)):
        tr = tree_feed(L, sc, batch, args.threads, args.tree_dir)
        out["host_feed"]["tree"] = tr
        out["host_feed"]["tree_read_gbps"] = {"warm": tr["warm"]["gbps"], "cold": tr["cold"]["gbps"]}
        out["host_feed"]["tree_to_findings_gbps"] = {"prepare_then_scan": tr["cold"]["end_to_end_gbps"],
                                                      "streamed": tr["streamed_cold"]["end_to_end_gbps"]}
        log("fs-tree feed (%d files on %s): warm %.2f GB/s, cold %.2f GB/s, disk -> findings %.2f GB/s (streamed "
            "%.2f GB/s, same findings %s); prepared == in-memory: %s" % (
                tr["files"], tr["dir_fs"], tr["warm"]["gbps"], tr["cold"]["gbps"], tr["cold"]["end_to_end_gbps"],
                tr["streamed_cold"]["end_to_end_gbps"], tr["streamed_cold"]["same_findings"],
                tr["prepared_equal_in_memory"]))
        if not tr["prepared_equal_in_memory"]:
            print("[bench] fs-tree feed differs from the in-memory preparation", file=sys.stderr, flush=True)
            sys.exit(1)

    if rank == 0 and (args.per_file == 1 or (args.per_file == -1 and args.config == 1)):
        out["small_batch"] = small_batches(L, eng, batch)
        out["per_file"] = per_file_queue(sc, batch, (5, cores))
        sb = out["small_batch"]
        log("small batches (tsg_scan_batch, 8-32 KB files): %s" % ", ".join(
            "%s files %.3f ms" % (k, v["ms"]) for k, v in sb.items() if isinstance(v, dict)))
        log("per-file Scan through the queue: %s" % ", ".join(
            "%s %.3f GB/s (%.1f files/batch)" % (k, v["gbps"], v["mean_batch_files"])
            for k, v in out["per_file"].items() if isinstance(v, dict)))

    if not args.no_resident:
        # the same batch already resident in HBM (reported, never `value`)
        d_data = torch.empty(batch.nbytes + 64, dtype=torch.uint8, device="cuda:%d" % device)
        d_data.copy_(torch.from_numpy(batch.view), non_blocking=False)
        torch.cuda.synchronize()

        def rstep():
            res = ctypes.c_void_p()
            _lib.check(L.tsg_scan_batch_resident(eng, ctypes.c_void_p(d_data.data_ptr()), batch.ptr,
                                                 batch.offsets.ctypes.data, nfiles, batch.cpaths, batch.clens,
                                                 bin_ptr, ctypes.byref(res)))
            return res
        res = rstep()
        same = _lib.result_json(res) == gpu_results
        L.tsg_result_free(res)
        # untimed warm-up of the resident layout (its pieces and K1Chain lanes
        # differ from the pinned step's; r7q: the first two timed steps ran
        # 7.0 / 6.2 ms against a 5.4 ms median)
        for _ in range(max(2, args.warmup)):
            L.tsg_result_free(rstep())
        rst, rwall, kept = [], [], []
        t0 = time.perf_counter()
        for k in range(max(8, args.steps)):
            t1 = time.perf_counter()
            res = rstep()
            rwall.append(time.perf_counter() - t1)
            rst.append(_lib.result_stats(res))
            if args.resident_keep:
                kept.append(res)           # diagnostic: results freed after the timed steps
            else:
                L.tsg_result_free(res)
        rdt = (time.perf_counter() - t0) / len(rst)
        for res in kept:
            L.tsg_result_free(res)
        rmed = float(np.median(rwall))
        rk1 = float(np.mean([s["k1_ms"] for s in rst]))
        out["resident"] = {"gbps": round(batch.nbytes / rdt / 1e9, 2), "ms_per_step": round(rdt * 1e3, 3),
                           "k1_ms": round(rk1, 3), "k1_gbps": round(batch.nbytes / (rk1 / 1e3) / 1e9, 2),
                           "k1_launches": int(rst[-1]["k1_launches"]), "pieces": int(rst[-1]["pieces"]),
                           "k2_ms": round(float(np.mean([s["k2_ms"] for s in rst])), 3),
                           "host_confirm_ms": round(float(np.mean([s["host_ms"] for s in rst])), 3),
                           "same_findings": same,
                           "median_step_ms": round(rmed * 1e3, 3),
                           "gbps_median_step": round(batch.nbytes / rmed / 1e9, 2),
                           "steps": len(rst),
                           "step_ms": [round(w * 1e3, 2) for w in rwall],
                           "results_freed_after_timing": bool(args.resident_keep),
                           "note": "the same batch already in HBM (tsg_scan_batch_resident); gbps over the mean "
                                   "step, gbps_median_step over the median one (host-bound configs vary with the "
                                   "box's CPU quota)"}
        log("HBM-resident: %.1f GB/s (%.2f ms/step; median step %.2f ms = %.1f GB/s; K1 %.2f ms = %.0f GB/s), "
            "same findings: %s" % (out["resident"]["gbps"], rdt * 1e3, rmed * 1e3, out["resident"]["gbps_median_step"],
                                   rk1, out["resident"]["k1_gbps"], same))
        # GPU-side CR strip (tsg_strip_cr_device) over a copy
        # of this batch with every '\n' turned into '\r' (CRLF density: the
        # kernel's work depends on where the CRs are, not on the other bytes);
        # reported beside the scan, never `value`
        d_cr = d_data.clone()
        d_cr.masked_fill_(d_cr == 10, 13)
        d_off = torch.from_numpy(batch.offsets.astype(np.int64)).to("cuda:%d" % device)
        cms = []
        for _ in range(4):
            d_dst, _noff, stripped, kms = sc.StripCR(d_cr, d_off, nfiles, batch.nbytes)
            cms.append(kms)
            del d_dst, _noff
        cms = float(np.mean(cms[1:]))
        algo = batch.nbytes + stripped
        out["cr_strip"] = {
            "bytes": batch.nbytes, "stripped_bytes": stripped, "ms": round(cms, 3),
            "gbps": round(batch.nbytes / (cms / 1e3) / 1e9, 1),
            "roofline": {"bound": "hbm", "achieved": round(algo / (cms / 1e3) / 1e9, 1), "peak": 8000.0,
                         "unit": "GB/s", "frac": round(algo / (cms / 1e3) / 1e9 / 8000.0, 3),
                         "design_traffic": batch.nbytes * 2 + stripped},
            "note": "four kernels (count, first-file, scan, compact), HIP events; algorithmic bytes = read N + write "
                    "N'; the count pass reads N once more (design_traffic)"}
        log("GPU CR strip: %.1f GB in %.2f ms = %.0f GB/s of input (%.2f of HBM roofline on N + N')" % (
            batch.nbytes / 1e9, cms, out["cr_strip"]["gbps"], out["cr_strip"]["roofline"]["frac"]))
        del d_cr, d_off, d_data
        torch.cuda.empty_cache()

    failed = False
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        procs = args.cpu_procs or cores
        idx = pick_sample(batch.offsets, int(args.cpu_sample_mb * 1e6), args.seed)
        items = [(batch.paths[i], batch.file(i), bool(batch.binary[i]) if batch.binary is not None else False)
                 for i in idx]
        gbps, ores, dt, nb = cpu_baseline(items, procs, cfg_path, log, "cpu baseline (oracle)")
        diff = [batch.paths[i] for j, i in enumerate(idx) if ores[j] != gpu_results[i]]
        ofind = sum(len(r["Findings"]) for r in ores)
        out["cpu_baseline"] = {
            "value": round(gbps, 5), "unit": "GB/s", "cores": procs, "kind": "port",
            "sample": "%d files / %.1f MB of the same batch (%d files > 8 MB, largest %.1f MB), "
                      "oracle/secret_oracle.py (Python restatement of pkg/fanal/secret/scanner.go) in a "
                      "%d-process pool on the %d cores this rank may use, %.1f s"
                      % (len(idx), nb / 1e6, sum(1 for _, c, _ in items if len(c) > (8 << 20)),
                         max(len(c) for _, c, _ in items) / 1e6, procs, procs, dt),
            "cores_detail": cores_detail,
        }
        # the C++ restatement of the reference algorithm (every rule's keyword
        # gate + Go-regexp find-all over every file, no GPU prefilter) on the
        # same sample: a compiled CPU scanner closer to the Go reference's speed
        sargs = [S.ScanArgs(p, c, bf) for p, c, bf in items]
        t0 = time.perf_counter()
        cres = S.scan_host_reference(sc, sargs, threads=procs)
        cdt = time.perf_counter() - t0
        cdiff = sum(1 for j in range(len(idx)) if cres[j] != ores[j])
        out["cpu_baseline_cxx"] = {
            "value": round(nb / cdt / 1e9, 5), "unit": "GB/s", "cores": procs, "kind": "port",
            "sample": "same %d files, C++ Go-regexp restatement of scanner.go on every (file, rule) pair "
                      "(tsg_scan_host_reference), %d threads, %.2f s; diff vs oracle: %d files"
                      % (len(idx), procs, cdt, cdiff),
            "note": "the one that approximates the reference's own speed: the same algorithm as Go's scanner.go "
                    "(per rule: keyword gate, then regexp find-all over the whole file) on Go's regexp engines "
                    "(Pike VM; bit-state backtracker only for small inputs, as Go), compiled; cpu_baseline "
                    "(the oracle) runs the third-party `regex` module's backtracking engine with Go-semantics "
                    "rewrites, faster on these patterns than a Pike VM but not Go's algorithm",
        }
        if "per_file" in out:
            for k, v in out["per_file"].items():
                if isinstance(v, dict):
                    v["vs_cpu_baseline_cxx"] = round(v["gbps"] / (nb / cdt / 1e9), 2)
        # parity beyond the baseline sample: every file above 8 MB and seeded
        # small files up to --parity-share of the step's bytes, through the
        # same oracle pool (not part of the baseline timing)
        pidx = idx
        pfind, pnb, pdt, pall = ofind, nb, 0.0, set(idx)
        if args.parity_share > 0 and nb < args.parity_share * batch.nbytes:
            pidx = pick_parity(batch.offsets, idx, args.parity_share, args.seed)
            base = set(idx)
            rest = [i for i in pidx if i not in base]
            ritems = [(batch.paths[i], batch.file(i), bool(batch.binary[i]) if batch.binary is not None else False)
                      for i in rest]
            log("parity: the oracle on %d more files (%.2f GB) to reach %.0f%% of the batch" % (
                len(rest), sum(len(c) for _, c, _ in ritems) / 1e9, 100 * args.parity_share))
            _, rres, pdt, rnb = cpu_baseline(ritems, procs, cfg_path, log, "parity (oracle)")
            del ritems
            diff += [batch.paths[i] for j, i in enumerate(rest) if rres[j] != gpu_results[i]]
            pfind += sum(len(r["Findings"]) for r in rres)
            pnb += rnb
            pall = set(pidx)
        sizes = np.diff(batch.offsets.astype(np.int64))
        out["parity"] = {"sample_files": len(pidx), "sample_bytes": pnb, "sample_findings": pfind,
                         "sample_share": round(pnb / max(batch.nbytes, 1), 4),
                         "sample_files_share": round(len(pidx) / max(batch.nfiles, 1), 4),
                         "files_over_8mb_checked": sum(1 for i in pall if sizes[i] > (8 << 20)),
                         "files_over_8mb": int((sizes > (8 << 20)).sum()),
                         "oracle_s": round(dt + pdt, 1),
                         "diff_files": len(diff), "diff_examples": diff[:5], "cxx_diff_files": cdiff,
                         "note": "the oracle (oracle/secret_oracle.py) checks these files of the step's batch: the "
                                 "CPU-baseline sample, every file above 8 MB and seeded small files up to "
                                 "--parity-share of the bytes; cxx_diff_files compares the C++ restatement on the "
                                 "baseline sample only"}
        failed = bool(diff) or cdiff > 0
        log("cpu baseline %.4f GB/s (oracle, %d procs), %.4f GB/s (C++ restatement, %d threads); "
            "parity: %d files / %.2f GB (%.0f%% of the batch) checked by the oracle in %.0f s, diff files: %d "
            "(findings in sample: %d)" % (gbps, procs, nb / cdt / 1e9, procs, len(pidx), pnb / 1e9,
                                          100.0 * pnb / max(batch.nbytes, 1), dt + pdt, len(diff), pfind))

    for b in shard_batches:
        b.free()
    if os.environ.get("TSG_K2_STATS") and sc._engine:
        L.tsg_engine_destroy(sc._engine)      # prints the per-rule K2 counters
        sc._engine = None
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if failed:
        print("[bench] PARITY FAILURE: GPU findings differ from the oracle", file=sys.stderr, flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
