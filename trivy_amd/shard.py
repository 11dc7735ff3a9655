"""Multi-GPU sharding of a file batch.

Files are independent units for Scanner.Scan (no cross-file state), so a
batch is split by bytes across ranks with longest-processing-time (LPT)
assignment; each rank (one process per GPU, torch.distributed) scans its shard
on its own engine and HIP stream.  No collective touches file data: results
travel to rank 0 with gather_object (gloo) only when the caller asks for them,
mirroring how the reference's analyzer merges per-file results
(pkg/fanal/analyzer/analyzer.go:250-301 Merge, :188-249 Sort).
"""
import heapq

import numpy as np


def lpt_shards(sizes, world):
    """Assign files (by byte size) to `world` shards, largest first onto the
    lightest shard.  Returns a list of sorted index lists."""
    order = np.argsort(-np.asarray(sizes, dtype=np.int64), kind="stable")
    heap = [(0, r) for r in range(world)]
    out = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(int(i))
        heapq.heappush(heap, (load + int(sizes[i]), r))
    return [sorted(x) for x in out]


def scan_sharded(args_list, scan_fn, rank, world, group=None, gather=True):
    """Scan this rank's LPT shard of args_list with scan_fn (list -> list of
    types.Secret) and optionally gather every rank's results on rank 0 in the
    original order.  Returns (my_indices, my_results, all_results_or_None)."""
    import torch.distributed as dist
    shards = lpt_shards([len(a.Content) for a in args_list], world)
    mine = shards[rank]
    res = scan_fn([args_list[i] for i in mine]) if mine else []
    if not gather or world == 1:
        full = None
        if world == 1:
            full = [None] * len(args_list)
            for i, r in zip(mine, res):
                full[i] = r
        return mine, res, full
    objs = [None] * world if rank == 0 else None
    dist.gather_object((mine, res), objs, dst=0, group=group)
    full = None
    if rank == 0:
        full = [None] * len(args_list)
        for idx, rr in objs:
            for i, r in zip(idx, rr):
                full[i] = r
    return mine, res, full
