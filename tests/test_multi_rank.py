"""N>1 path on CPU: two gloo ranks each scan an LPT shard of one synthetic
batch (CPU model of the GPU tables + exact confirmer), rank 0 gathers the
results, and they equal a single-process scan.  Mirrors bench.py's
one-process-per-GPU layout (no collective on file data)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from trivy_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, engine=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trivy_amd import secret as S
    from workload import synth
    c = synth.generate(300_000 if not engine else 8_000_000, seed=11, sizes="lognormal", plant_rate=2e-3,
                       base_bytes=1 << 20)
    args = [S.ScanArgs(c.paths[i], c.file(i)) for i in range(len(c.paths))]
    sc = S.Scanner(None, device=0) if engine else S.Scanner(None)
    scan = (lambda a: sc.ScanBatch(a)) if engine else (lambda a: S.scan_table_model(sc, a))
    mine, res, full = shard.scan_sharded(args, scan, rank, world)
    if rank == 0:
        q.put(full)
    dist.barrier()
    dist.destroy_process_group()


def test_lpt_shards_balance():
    sizes = [100, 90, 80, 10, 10, 5, 5, 1]
    sh = shard.lpt_shards(sizes, 3)
    assert sorted(i for s in sh for i in s) == list(range(len(sizes)))
    loads = [sum(sizes[i] for i in s) for s in sh]
    assert max(loads) - min(loads) <= 100


@pytest.mark.timeout(300)
def test_two_gloo_ranks_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    full = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    from trivy_amd import secret as S
    from workload import synth
    c = synth.generate(300_000, seed=11, sizes="lognormal", plant_rate=2e-3, base_bytes=1 << 20)
    args = [S.ScanArgs(c.paths[i], c.file(i)) for i in range(len(c.paths))]
    want = S.scan_table_model(S.Scanner(None), args)
    assert full == want
    assert sum(len(w["Findings"]) for w in want) > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_gloo_ranks_engines_gpu():
    # bench.py's N>1 layout on one card: two processes, each with its own
    # engine (both on device 0 here, one per GPU on a node), LPT shards, no
    # collective on file data; the gathered result equals one process's scan
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, True)) for r in range(2)]
    for p in ps:
        p.start()
    full = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    from trivy_amd import secret as S
    from workload import synth
    c = synth.generate(8_000_000, seed=11, sizes="lognormal", plant_rate=2e-3, base_bytes=1 << 20)
    args = [S.ScanArgs(c.paths[i], c.file(i)) for i in range(len(c.paths))]
    want = S.Scanner(None).ScanBatch(args)
    assert full == want
    assert sum(len(w["Findings"]) for w in want) > 20
