#!/usr/bin/env python
"""bench.py -- GB/s secret-scanned (builtin rules) on MI355X, findings diff = 0.

Workload (BASELINE.json configs[1]): a 10 GB synthetic text/source corpus per
GPU (log-uniform file sizes 64 B - 64 MB, ~0.01% of lines carry planted
secrets drawn from all 87 builtin rules, 10% near misses), scanned with the
builtin rules.  One step = one full scan of the corpus resident in HBM:
K1 (streaming scan DFA) + K2 (anchored verify) + candidate D2H + exact host
confirmation + types.Secret assembly for every file.

  python bench.py [--gpus N --steps K --warmup W --gb G]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Multi-GPU: each rank scans its own shard (seed + rank, weak scaling), no
collective on the data path; gloo carries only the barrier and the max-time
reduction.  Rank 0 prints one JSON line.

Extra fields: roofline (K1, HBM bound, achieved = content bytes / mean K1
launch time from HIP events on the engine's stream), cpu_baseline (the
oracle -- oracle/secret_oracle.py, a Python restatement of the reference Go
scanner -- on a bounded sample of the same corpus with a process pool),
parity (GPU findings vs the oracle on that sample: diff must be 0), and a
per-phase breakdown.
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

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def _oracle_worker_init(cfg_path):
    global _ORACLE
    from oracle import secret_oracle as so
    _ORACLE = so.Scanner(so.parse_config(cfg_path) if cfg_path else None)


def _oracle_scan(item):
    path, content = item
    try:
        return _ORACLE.scan(path, content)
    except MemoryError:      # the `regex` module's backtracking on a huge `(.|\s)*` block
        return None


def cpu_baseline(corpus, idx, procs, cfg_path=None):
    """Oracle over files idx with a process pool; returns (GB/s, results, seconds)."""
    import multiprocessing as mp
    items = [(corpus.paths[i], corpus.file(i)) for i in idx]
    nbytes = sum(len(c) for _, c in items)
    ctx = mp.get_context("fork")
    with ctx.Pool(procs, initializer=_oracle_worker_init, initargs=(cfg_path,)) as pool:
        t0 = time.perf_counter()
        res = pool.map(_oracle_scan, items, chunksize=1)
        dt = time.perf_counter() - t0
    return nbytes / dt / 1e9, res, dt, nbytes


def pick_sample(corpus, target_bytes, max_file, seed):
    rng = np.random.default_rng(seed)
    order = rng.permutation(len(corpus.paths))
    idx, tot = [], 0
    for i in order:
        n = int(corpus.offsets[i + 1] - corpus.offsets[i])
        if n > max_file:
            continue
        idx.append(int(i))
        tot += n
        if tot >= target_bytes:
            break
    return sorted(idx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gb", type=float, default=10.0, help="corpus GB per GPU (config 2: 10)")
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 5],
                    help="BASELINE.json config: 2 = 10 GB source corpus (the metric's workload), "
                         "3 = image-layer small files, 5 = 500 custom rules")
    ap.add_argument("--sizes", default="loguniform", choices=["loguniform", "lognormal", "small"])
    ap.add_argument("--seed", type=int, default=0x71215EC7)
    ap.add_argument("--threads", type=int, default=16, help="host confirm threads per rank")
    ap.add_argument("--cpu-procs", type=int, default=16)
    ap.add_argument("--cpu-sample-mb", type=float, default=1200.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive (host batch) measurement")
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    import torch
    from trivy_amd import _lib
    from workload import synth
    from trivy_amd import secret as S

    def log(*a):
        if rank == 0:
            print("[bench]", *a, file=sys.stderr, flush=True)

    t_gen = time.perf_counter()
    cfg_path = None
    if args.config == 3:      # extracted image layers: small files, rootfs paths
        corpus = synth.generate(int(args.gb * 1e9), seed=args.seed + rank, sizes="small", layout="image")
    else:
        corpus = synth.generate(int(args.gb * 1e9), seed=args.seed + rank, sizes=args.sizes)
    if args.config == 5:      # 500 custom rules + allow rules + exclude blocks (+ builtins)
        cfg5, plants = synth.config5(500, seed=args.seed)
        cfg_path = "/tmp/tsg_bench_config5_%d.yaml" % rank
        synth.write_yaml(cfg5, cfg_path)
        synth.plant_custom(corpus, plants, seed=args.seed + rank, rate=1e-4)
    log("corpus: %.2f GB, %d files, %d plants (%d near-miss), generated in %.1fs" % (
        corpus.nbytes / 1e9, len(corpus.paths), corpus.planted, corpus.near_miss, time.perf_counter() - t_gen))

    device = local_rank
    torch.cuda.set_device(device)
    host_t = torch.from_numpy(corpus.data)
    # host-feed ceiling: pinned -> HBM copy rate on a <= 4 GB slice (reported, never the metric)
    n_pin = min(len(corpus.data), 4 << 30)
    pinned = torch.empty(n_pin, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(host_t[:n_pin])
    d_data = torch.empty(len(corpus.data), dtype=torch.uint8, device="cuda:%d" % device)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d_data[:n_pin].copy_(pinned, non_blocking=True)
    torch.cuda.synchronize()
    h2d_gbps = n_pin / (time.perf_counter() - t0) / 1e9
    del pinned
    if n_pin < len(corpus.data):
        d_data[n_pin:].copy_(host_t[n_pin:])
        torch.cuda.synchronize()
    log("H2D (pinned) %.1f GB/s" % h2d_gbps)

    sc = S.Scanner(S.ParseConfig(cfg_path) if cfg_path else None, device=device, threads=args.threads)
    eng = sc.engine()
    L = _lib.lib()
    paths, lens, _keep = _lib.pack_paths(corpus.paths)
    nfiles = len(corpus.paths)
    h_ptr = corpus.data.ctypes.data
    off_ptr = corpus.offsets.ctypes.data

    def step():
        res = ctypes.c_void_p()
        _lib.check(L.tsg_scan_batch_resident(eng, ctypes.c_void_p(d_data.data_ptr()), h_ptr, off_ptr, nfiles,
                                             paths, lens, None, ctypes.byref(res)))
        return res

    for _ in range(args.warmup):
        L.tsg_result_free(step())
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    stats = []
    last = None
    t0 = time.perf_counter()
    for k in range(args.steps):
        res = step()
        stats.append(_lib.result_stats(res))
        if k == args.steps - 1:
            last = res
        else:
            L.tsg_result_free(res)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    b = torch.tensor([float(corpus.nbytes)], dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
    elapsed_max = float(t[0])
    total_bytes = float(b[0]) * args.steps
    value = total_bytes / elapsed_max / 1e9

    k1_ms = float(np.mean([s["k1_ms"] for s in stats]))
    k2_ms = float(np.mean([s["k2_ms"] for s in stats]))
    host_ms = float(np.mean([s["host_ms"] for s in stats]))
    d2h_ms = float(np.mean([s["d2h_ms"] for s in stats]))
    gpu_wall_ms = float(np.mean([s["gpu_wall_ms"] for s in stats]))
    eng_total_ms = float(np.mean([s["total_ms"] for s in stats]))
    k1_gbps = corpus.nbytes / (k1_ms / 1e3) / 1e9
    pieces = max(1, int(stats[-1].get("pieces", 1)))      # one K1 launch per pipeline piece
    bytes_per_launch = corpus.nbytes / pieces
    # HBM traffic per launch: PMC FETCH_SIZE + WRITE_SIZE (calibrated as the
    # microarch guide prescribes) measured by tools/pmc_traffic.sh on this
    # workload, committed under profiles/; scaled to this launch's bytes
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "r1j_traffic.json")
    if args.config == 2 and os.path.exists(tpath):
        tj = json.load(open(tpath))
        traffic = round(tj["traffic_over_algorithmic"] * bytes_per_launch)
        traffic_src = "profiles/r1j_traffic.json: %.3f HBM bytes per content byte (rocprofv3 --pmc)" % (
            tj["traffic_over_algorithmic"])
    gpu_results = _lib.result_json(last)
    L.tsg_result_free(last)
    findings = sum(len(s["Findings"]) for s in gpu_results)
    rules_hit = sorted({f["RuleID"] for s in gpu_results for f in s["Findings"]})
    log("step %.1f ms: K1 %.1f ms (%.0f GB/s), K2 %.1f ms, D2H %.1f ms, host %.1f ms; hits %d, candidates %d, "
        "findings %d over %d rules" % (elapsed_max / args.steps * 1e3, k1_ms, k1_gbps, k2_ms, d2h_ms, host_ms,
                                        stats[-1]["hits"], stats[-1]["candidates"], findings, len(rules_hit)))

    out = {
        "metric": "GB/s secret-scanned (builtin rules) at 1/2/4/8 MI355X; findings diff = 0",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (trivy_amd/synth.py, seed %#x + rank)" % args.seed,
        "config": {
            "workload": {
                2: "config2: %.0f GB synthetic text/source corpus per GPU, %s file sizes, 0.01%% planted "
                   "secrets (87 builtin rules), builtin rules, corpus resident in HBM" % (args.gb, args.sizes),
                3: "config3: %.0f GB of extracted-image-layer small files per GPU (mean ~25 KB, rootfs paths), "
                   "builtin rules, corpus resident in HBM" % args.gb,
                5: "config5: %.0f GB synthetic source corpus per GPU, trivy-secret.yaml with 500 custom rules "
                   "+ 87 builtins, 20 allow rules, 5 exclude blocks, corpus resident in HBM" % args.gb,
            }[args.config],
            "bytes_per_gpu": corpus.nbytes,
            "files_per_gpu": nfiles,
            "parallelism": "file shards per GPU, no collective (dp%d)" % world,
            "host_confirm_threads": args.threads,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "tsg_k1_scan",
            "achieved": round(k1_gbps, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(k1_gbps / HBM_PEAK_GBPS, 5),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "bytes_per_launch": round(bytes_per_launch),
            "avg_launch_ms": round(k1_ms / pieces, 4),
            "launches_per_step": pieces,
        },
        "breakdown_ms": {"pipeline_pieces": pieces, "gpu_phase_wall": round(gpu_wall_ms, 3), "engine_total": round(eng_total_ms, 3),
                         "k1": round(k1_ms, 3), "k2": round(k2_ms, 3), "d2h": round(d2h_ms, 3),
                         "host_confirm": round(host_ms, 3), "hits": stats[-1]["hits"],
                         "candidates": stats[-1]["candidates"], "confirm_files": stats[-1]["confirm_files"],
                         "findings": findings, "rules_with_findings": len(rules_hit)},
        "host_feed": {"h2d_pinned_gbps": round(h2d_gbps, 2),
                      "note": "h2d_pinned_gbps: one torch copy of a <= 4 GB pinned slice; pcie_inclusive_gbps: the "
                              "whole batch from pinned host memory through tsg_scan_batch (uploads overlap confirmation)"},
        "cpu_baseline": None,
        "parity": None,
    }

    if rank == 0:
        # host feed: batched Required + IsBinary + CR strip (tsg_prepare_batch)
        # over the same files as read (reported beside the scan, never `value`)
        hpb = ctypes.c_void_p()
        t0 = time.perf_counter()
        _lib.check(L.tsg_prepare_batch(sc._rs, None, h_ptr, off_ptr, nfiles, paths, lens, args.threads,
                                       ctypes.byref(hpb)))
        tprep = time.perf_counter() - t0
        d_, o_, i_, b_, nk = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint32()
        _lib.check(L.tsg_prepared_view(hpb, ctypes.byref(d_), ctypes.byref(o_), ctypes.byref(i_), ctypes.byref(b_),
                                       ctypes.byref(nk)))
        L.tsg_prepared_free(hpb)
        out["host_feed"]["prepare_gbps"] = round(corpus.nbytes / tprep / 1e9, 2)
        out["host_feed"]["prepare_kept_files"] = nk.value
        log("host feed prepare (Required + IsBinary + CR strip, %d threads): %.1f GB/s, %d of %d files kept" % (
            args.threads, corpus.nbytes / tprep / 1e9, nk.value, nfiles))

    if rank == 0 and world == 1 and not args.no_pcie:
        # PCIe-inclusive rate (reported, never `value`): the same batch handed
        # over in pinned host memory through tsg_scan_batch, which uploads each
        # pipeline piece while the host confirms the previous one
        hp = ctypes.c_void_p()
        _lib.check(L.tsg_alloc_pinned(corpus.nbytes + 64, ctypes.byref(hp)))
        try:
            ctypes.memmove(hp, h_ptr, corpus.nbytes)
            times = []
            for k in range(2):
                t0 = time.perf_counter()
                res = ctypes.c_void_p()
                _lib.check(L.tsg_scan_batch(eng, hp, off_ptr, nfiles, paths, lens, None, ctypes.byref(res)))
                times.append(time.perf_counter() - t0)
                if k == 1:
                    pc = _lib.result_json(res)
                    out["host_feed"]["pcie_inclusive_same_findings"] = pc == gpu_results
                L.tsg_result_free(res)
            out["host_feed"]["pcie_inclusive_gbps"] = round(corpus.nbytes / times[-1] / 1e9, 2)
            log("PCIe-inclusive (pinned host batch -> tsg_scan_batch): %.1f GB/s" % (corpus.nbytes / times[-1] / 1e9))
        finally:
            L.tsg_free_pinned(hp)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # config 5's exclude blocks make the oracle's backtracking engine
        # blow up on multi-MB files: its sample keeps files <= 512 KB
        idx = pick_sample(corpus, int(args.cpu_sample_mb * 1e6), (512 << 10) if args.config == 5 else (8 << 20),
                          args.seed)
        gbps, ores, dt, nb = cpu_baseline(corpus, idx, args.cpu_procs, cfg_path)
        oracle_failed = [corpus.paths[i] for j, i in enumerate(idx) if ores[j] is None]
        diff = [corpus.paths[i] for j, i in enumerate(idx) if ores[j] is not None and ores[j] != gpu_results[i]]
        ofind = sum(len(r["Findings"]) for r in ores if r is not None)
        out["cpu_baseline"] = {
            "value": round(gbps, 5), "unit": "GB/s", "cores": args.cpu_procs, "kind": "port",
            "sample": "%d files / %.1f MB of the same corpus (files <= 8 MB), oracle/secret_oracle.py "
                      "(Python restatement of pkg/fanal/secret/scanner.go) in a %d-process pool, %.1f s"
                      % (len(idx), nb / 1e6, args.cpu_procs, dt),
        }
        # the C++ restatement of the reference algorithm (every rule's keyword
        # gate + Go-regexp find-all over every file, no GPU prefilter) on the
        # same sample: a compiled CPU scanner closer to the Go reference's speed
        sub = corpus.subset(idx)
        sargs = [S.ScanArgs(sub.paths[j], sub.file(j)) for j in range(len(idx))]
        t0 = time.perf_counter()
        cres = S.scan_host_reference(sc, sargs, threads=args.cpu_procs)
        cdt = time.perf_counter() - t0
        cdiff = sum(1 for j in range(len(idx)) if ores[j] is not None and cres[j] != ores[j])
        out["cpu_baseline_cxx"] = {
            "value": round(nb / cdt / 1e9, 5), "unit": "GB/s", "cores": args.cpu_procs, "kind": "port",
            "sample": "same %d files, C++ Go-regexp restatement of scanner.go on every (file, rule) pair "
                      "(tsg_scan_host_reference), %d threads, %.2f s; diff vs oracle: %d files"
                      % (len(idx), args.cpu_procs, cdt, cdiff),
        }
        out["parity"] = {"sample_files": len(idx), "sample_findings": ofind, "diff_files": len(diff),
                         "diff_examples": diff[:5], "oracle_failed_files": len(oracle_failed)}
        log("cpu baseline %.4f GB/s (oracle, %d procs), %.4f GB/s (C++ restatement, %d threads); "
            "parity diff files: %d (findings in sample: %d)" % (
                gbps, args.cpu_procs, nb / cdt / 1e9, args.cpu_procs, len(diff), ofind))

    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
