"""Config 4 (BASELINE.json configs[3]) reduced to one card: a corpus of
several config-2 shards (distinct seeds, log-uniform 64 B - 64 MB sizes)
streamed one after another through one engine, then split over two engines
(two processes, as bench.py runs one rank per GPU, both on device 0 here),
compared file by file with each other and with the oracle on a sample that
includes every file above 4 MB."""
import os
import random
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SHARD_BYTES = 40_000_000
SHARDS = 4
SEED = 0x71215EC7


def _shard_args(k):
    from trivy_amd import secret as S
    from workload import synth
    c = synth.generate(SHARD_BYTES, seed=SEED + 1000 * k, sizes="loguniform", plant_rate=1e-3,
                       base_bytes=4 << 20)
    return [S.ScanArgs("shard%d/%s" % (k, c.paths[i]), c.file(i)) for i in range(len(c.paths))]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    # one "GPU" rank of config 4: its shards (k % world == rank) streamed
    # through its own engine; results travel to rank 0 (no collective on data)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TSG_SEGMENT_BYTES=str(8 << 20))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trivy_amd import secret as S
    sc = S.Scanner(None, device=0)
    mine = {k: sc.ScanBatch(_shard_args(k)) for k in range(SHARDS) if k % world == rank}
    objs = [None] * world if rank == 0 else None
    dist.gather_object(mine, objs, dst=0)
    if rank == 0:
        q.put({k: v for o in objs for k, v in o.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_config4_shards_one_engine_two_engines_oracle(monkeypatch):
    from _oracle_pool import oracle_scan_many
    from trivy_amd import secret as S
    monkeypatch.setenv("TSG_SEGMENT_BYTES", str(8 << 20))    # several segments per shard
    sc = S.Scanner(None)
    shards = [_shard_args(k) for k in range(SHARDS)]
    one, pieces = [], []
    for args in shards:                                      # streamed through one engine
        got, st = sc.ScanBatch(args, with_stats=True)
        pieces.append(st["pieces"])                          # segments end at file boundaries
        one.append(got)
    assert sum(pieces) >= SHARDS + 2, pieces
    # two engines in two processes (bench.py's one-rank-per-GPU layout)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    two = q.get(timeout=400)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [two[k] for k in range(SHARDS)] == one
    # oracle on a sample of every shard: all files above 4 MB + 60 others
    rng = random.Random(4)
    items, where = [], []
    for k, args in enumerate(shards):
        large = [i for i, a in enumerate(args) if len(a.Content) > 4 << 20]
        rest = [i for i, a in enumerate(args) if len(a.Content) <= 4 << 20]
        for i in sorted(large + rng.sample(rest, min(60, len(rest)))):
            items.append((args[i].FilePath, args[i].Content, False))
            where.append((k, i))
    assert sum(1 for it in items if len(it[1]) > 4 << 20) >= 4
    want = oracle_scan_many(items, procs=16)
    assert sum(len(w["Findings"]) for w in want) > 100
    for (k, i), w in zip(where, want):
        assert one[k][i] == w, shards[k][i].FilePath
