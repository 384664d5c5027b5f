"""GPU: the RCCL transport with two ranks — two processes, each its own RCCL communicator
rank (librccl via OptAMD_CommCreateRccl), ncclSend/Recv halo exchange and ncclAllReduce
of the PCG scalars — against the single-domain solve (the multi-rank RCCL
path had never executed).

The pool's boxes have one GPU, so both ranks share device 0. RCCL may refuse two ranks
of one communicator on one device; the test then skips with RCCL's reason (the
LocalGroup tests in test_decomposition_gpu.py still run the same solver code)."""
import ctypes
import multiprocessing as pymp
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank_main(rank, world, uid, W, H, q):
    try:
        import sys
        sys.path.insert(0, ROOT)
        import torch

        from opt_amd import api
        from opt_amd import distributed as dd
        from tests.iw_helpers import device_params, perturbed, solver

        torch.cuda.set_device(0)
        lib = api.load_library()
        raw = (ctypes.c_uint8 * 128)(*uid)
        comm = lib.OptAMD_CommCreateRccl(raw, rank, world)
        if not comm:
            q.put((rank, "refused", None))
            return
        w = perturbed(W, H, seed=31)
        s = solver(W, H)
        sl = dd.slab(H, rank, world, s.halo())
        s.set_decomposition(comm, sl.y_lo, sl.y_hi)
        prm = device_params(dd.local_image_warping(w, sl))
        s.set_solver_params({"nIterations": 3, "lIterations": 10})
        costs = s.profiled_solve(prm)
        O = dd.owned(prm[0].cpu().numpy(), W, 2, sl)
        A = dd.owned(prm[1].cpu().numpy(), W, 1, sl)
        s.close()
        lib.OptAMD_CommDestroy(comm)
        q.put((rank, "ok", (costs, O, A)))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "error", repr(e)))


def test_two_rccl_ranks_match_single_domain():
    from opt_amd import api
    from tests.iw_helpers import device_params, perturbed, solver

    W, H, world = 160, 120, 2
    uidbuf = (ctypes.c_uint8 * 128)()
    assert api.load_library().OptAMD_RcclUniqueId(uidbuf) == 0
    ctx = pymp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, list(uidbuf), W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, status, payload = q.get(timeout=180)
            out[r] = (status, payload)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join()
    if any(v[0] == "refused" for v in out.values()):
        pytest.skip("RCCL refused two ranks of one communicator on one device")
    assert all(v[0] == "ok" for v in out.values()), out
    w = perturbed(W, H, seed=31)
    s = solver(W, H)
    prm = device_params(w)
    s.set_solver_params({"nIterations": 3, "lIterations": 10})
    ref = s.profiled_solve(prm)
    c0, c1 = out[0][1][0], out[1][1][0]
    assert c0 == c1                      # both ranks report the global energy
    np.testing.assert_allclose(c0, ref, rtol=1e-5)
    O = np.concatenate([out[r][1][1] for r in range(world)])
    A = np.concatenate([out[r][1][2] for r in range(world)])
    ro, ra = prm[0].cpu().numpy(), prm[1].cpu().numpy()
    assert np.abs(O - ro).max() / np.abs(ro).max() < 1e-5
    assert np.abs(A - ra).max() < 1e-4 * max(1.0, np.abs(ra).max())
