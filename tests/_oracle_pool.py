"""Oracle (oracle/secret_oracle.py) over many files in a process pool, largest
files first -- for GPU parity tests whose samples include multi-MB files (the
oracle reads ~4-10 MB/s per process on such files).  Forked workers run only
the oracle (CPU), never HIP."""
import multiprocessing as mp

_SC = None


def _init(cfg):
    global _SC
    from oracle import secret_oracle as so
    _SC = so.Scanner(cfg)


def _scan(item):
    path, content, binary = item
    return _SC.scan(path, content, binary)


def oracle_scan_many(items, procs=8, cfg=None):
    """items: [(path, content, binary)] -> oracle types.Secret dicts, in order.
    cfg: an oracle config (so.parse_config(...)) or None for the builtins."""
    order = sorted(range(len(items)), key=lambda j: -len(items[j][1]))
    # (tens of thousands of small files: a task per file is mostly IPC; the
    # largest files lead the order, so chunks of neighbours stay balanced)
    cs = max(1, min(64, len(items) // (procs * 32)))
    with mp.get_context("fork").Pool(procs, initializer=_init, initargs=(cfg,)) as pool:
        got = pool.map(_scan, [items[j] for j in order], chunksize=cs)
    out = [None] * len(items)
    for j, r in zip(order, got):
        out[j] = r
    return out
