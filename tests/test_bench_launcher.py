"""bench.py's multi-GPU wiring on the CPU (one process per GPU,
file shards, no collective).  `python bench.py --gpus N` without torchrun
starts N rank processes itself; each rank scans on HIP device LOCAL_RANK with
an engine of device_mask 1 << LOCAL_RANK."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _run(args, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_rank_envs_wiring():
    envs = bench.rank_envs(4, 29999, base_env={"X": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["LOCAL_RANK"] == e["RANK"] and e["WORLD_SIZE"] == "4" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999" and e["X"] == "1" for e in envs)


def test_launcher_dry_run_two_ranks():
    p = _run(["--gpus", "2", "--dry-launch"])
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout.strip().splitlines()[-1])["dry_launch"]
    assert [(g["rank"], g["world"], g["device"], g["device_mask"]) for g in got] == [(0, 2, 0, 1), (1, 2, 1, 2)]


def test_launcher_dry_run_four_ranks():
    p = _run(["--gpus", "4", "--dry-launch"])
    assert p.returncode == 0, p.stderr
    got = json.loads(p.stdout.strip().splitlines()[-1])["dry_launch"]
    assert [g["device_mask"] for g in got] == [1, 2, 4, 8]


def test_launcher_dry_run_eight_ranks():
    # the 8-GPU node's wiring: ranks 0-7 on devices 0-7, and the per-rank
    # gather behind the N > 1 line's concurrent feed ceiling (every rank's
    # probe after one barrier, summed on rank 0)
    p = _run(["--gpus", "8", "--dry-launch"], timeout=300)
    assert p.returncode == 0, p.stderr
    doc = json.loads(p.stdout.strip().splitlines()[-1])
    got = doc["dry_launch"]
    assert [(g["rank"], g["device"], g["device_mask"]) for g in got] == [(r, r, 1 << r) for r in range(8)]
    assert all(g["world"] == 8 and g["ceiling_gbps"] > 0 for g in got)
    assert abs(doc["ceiling_gbps_all_ranks"] - sum(g["ceiling_gbps"] for g in got)) < 0.05


def test_gpus_beyond_visible_devices_fails_loudly():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs visible")
    p = _run(["--gpus", "2"], timeout=120)
    assert p.returncode == 2
    assert "needs 2 GPUs" in p.stderr


def test_gpus_must_match_world_size():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-launch"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


def test_pick_sample_covers_large_files():
    rng = np.random.default_rng(3)
    sizes = np.exp(rng.uniform(np.log(64), np.log(64 << 20), 3000)).astype(np.uint64)
    off = np.zeros(len(sizes) + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    idx = bench.pick_sample(off, 1_200_000_000, seed=7)
    sz = np.array([int(off[i + 1] - off[i]) for i in idx])
    assert idx == sorted(set(idx))
    assert (sz > (8 << 20)).sum() >= 8                   # files above the old 8 MB cap are checked
    assert sz[sz > (8 << 20)].sum() >= 0.5 * 1.2e9
    assert sz[sz <= (8 << 20)].sum() >= 0.5 * 1.2e9


def test_available_cores():
    cores, detail = bench.available_cores()
    assert 1 <= cores <= detail["affinity"] == len(os.sched_getaffinity(0))
