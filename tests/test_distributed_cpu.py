"""CPU, world_size 2 (gloo): the row-slab decomposition that the GPU solver uses
(halo = stencil radius 1, one owned slab per rank, global sums as all-reduces)
reproduces the undecomposed J^T J p, J^T F and cost. Runs the C oracle per slab."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from opt_amd import distributed as dd
from opt_amd import workloads


def test_slab_partition_tiles_the_image():
    for H in (1, 2, 7, 64, 4096, 4097):
        for world in (1, 2, 3, 8):
            if H < world:
                continue
            rows = []
            for r in range(world):
                s = dd.slab(H, r, world, 1)
                rows.extend(range(s.y_lo, s.y_hi))
                assert s.mem_lo == max(0, s.y_lo - 1) and s.mem_hi == min(H, s.y_hi + 1)
            assert rows == list(range(H))
    with pytest.raises(ValueError):
        dd.slab(3, 0, 8, 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch

    from oracle import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H = 50, 37
    rng = np.random.default_rng(3)
    w = workloads.image_warping(W, H, seed=3, n_handles=4, max_move=0.2)
    w["Angle"] = rng.normal(0, 0.2, W * H).astype(np.float32)
    w["Offset"] = (w["Offset"] + rng.normal(0, 0.3, 2 * W * H)).astype(np.float32)
    p = rng.normal(size=3 * W * H).astype(np.float32)
    s = dd.slab(H, rank, world, 1)
    lw = dd.local_image_warping(w, s)
    N = W * s.mem_rows
    pl = np.concatenate([dd.slice_rows(p[: 2 * W * H], W, 2, s), dd.slice_rows(p[2 * W * H:], W, 1, s)])
    act = lw["Mask"] == 0
    # the owned-row contribution to the global dot product; halo rows belong to neighbours
    own = np.zeros(s.mem_rows, bool)
    own[s.y_lo - s.mem_lo: s.y_hi - s.mem_lo] = True
    ownpx = np.repeat(own, W)
    Ap, _ = oracle.iw_apply_jtj(lw, pl)
    pAp_local = float(np.dot(pl[:2 * N][np.repeat(ownpx & act, 2)].astype(np.float64),
                             Ap[:2 * N][np.repeat(ownpx & act, 2)]) +
                      np.dot(pl[2 * N:][ownpx & act].astype(np.float64), Ap[2 * N:][ownpx & act]))
    t = torch.tensor([pAp_local], dtype=torch.float64)
    dist.all_reduce(t)
    Ap_o, Ap_t = dd.owned_vec(Ap, W, s)
    r, pre, _ = oracle.iw_eval_jtf(lw)
    r_o, r_t = dd.owned_vec(r, W, s)
    # cost over owned rows: cost of the slab minus its halo rows' own residual sums
    res = oracle.iw_residuals(lw).reshape(s.mem_rows, W, 10)
    c_local = 0.5 * float(np.sum(res[own].astype(np.float64) ** 2))
    c = torch.tensor([c_local], dtype=torch.float64)
    dist.all_reduce(c)
    gathered = [None] * world
    dist.all_gather_object(gathered, (rank, Ap_o, Ap_t, r_o, r_t))
    if rank == 0:
        Ap_g, pAp_g = oracle.iw_apply_jtj(w, p)
        r_g, _, _ = oracle.iw_eval_jtf(w)
        parts = sorted(gathered, key=lambda g: g[0])
        ApO = np.concatenate([g[1] for g in parts])
        ApT = np.concatenate([g[2] for g in parts])
        rO = np.concatenate([g[3] for g in parts])
        rT = np.concatenate([g[4] for g in parts])
        ok = (np.array_equal(ApO, Ap_g[: 2 * W * H]) and np.array_equal(ApT, Ap_g[2 * W * H:]) and
              np.array_equal(rO, r_g[: 2 * W * H]) and np.array_equal(rT, r_g[2 * W * H:]))
        q.put((ok, float(t.item()), pAp_g, float(c.item()), oracle.iw_cost(w)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_slab_decomposition_reproduces_global_operators(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    ok, pAp, pAp_g, c, c_g = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
    assert ok, "owned rows of the slab operators differ from the global operators"
    assert pAp == pytest.approx(pAp_g, rel=1e-12)
    assert c == pytest.approx(c_g, rel=1e-6)
