"""CPU: bench.py's multi-GPU launcher. `--gpus N` without a launcher
starts N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as
torch.distributed.run sets them) before anything touches a GPU; under a launcher whose
WORLD_SIZE differs from --gpus it exits with status 2 instead of reporting a run of the
wrong size. `--dry-run` makes every rank print its environment and row slab (the
reference's outer-dimension split, backend_cpu_mt.t:716-737) without GPU work, so the
spawn path itself runs here."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("n,workload,halo", [(2, "image_warping", 2), (4, "image_warping", 2),
                                             (8, "image_warping", 2), (8, "shape_from_shading", 2),
                                             (3, "image_warping", 2)])
def test_spawns_n_ranks_with_slabs(n, workload, halo):
    p = run(["--gpus", str(n), "--dry-run", "--workload", workload])
    assert p.returncode == 0, p.stderr
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert sorted(r["rank"] for r in lines) == list(range(n))
    H = 4096
    slabs = sorted((r["slab"][0], r["slab"][1], r["mem_rows"], r) for r in lines)
    assert slabs[0][0] == 0 and slabs[-1][1] == H
    for (lo, hi, mem, r), nxt in zip(slabs, slabs[1:] + [None]):
        assert r["world"] == n and r["local_rank"] == r["rank"] and r["device"] == f"cuda:{r['rank']}"
        assert r["master"].startswith("127.0.0.1:")
        assert mem == [max(0, lo - halo), min(H, hi + halo)]
        assert hi - lo == (H // n if r["rank"] < n - 1 else H - (n - 1) * (H // n))
        if nxt:
            assert nxt[0] == hi   # contiguous, non-overlapping owned rows
    assert len({r["master"] for r in lines}) == 1   # one rendezvous for all ranks


def test_single_gpu_default_runs_in_process():
    p = run(["--dry-run"])
    assert p.returncode == 0, p.stderr
    (r,) = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert r["world"] == 1 and r["slab"] == [0, 4096]


@pytest.mark.parametrize("world,gpus", [("2", "4"), ("8", "1"), ("1", "8")])
def test_launcher_world_size_must_match_gpus(world, gpus):
    p = run(["--gpus", gpus, "--dry-run"], {"WORLD_SIZE": world, "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE" in p.stderr and not p.stdout.strip()


def test_under_torch_distributed_run_env():
    """torch.distributed.run's environment for rank 1 of 4: that rank's slab only."""
    p = run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "4", "RANK": "1", "LOCAL_RANK": "1",
                                           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29555"})
    assert p.returncode == 0, p.stderr
    (r,) = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert r["rank"] == 1 and r["slab"] == [1024, 2048] and r["master"] == "127.0.0.1:29555"


def test_failed_rank_fails_the_launch():
    p = run(["--gpus", "2", "--dry-run", "--size", "1"])   # a 1-row image cannot be split in 2
    assert p.returncode != 0


def test_bad_gpu_count():
    assert run(["--gpus", "0", "--dry-run"]).returncode == 2
