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


# ---------------------------------------------------------------- the RCCL transport code
# RcclComm (comm.cpp) — grouped ncclSend/ncclRecv halos, the split
# halo communicator, the all-reduce of the PCG scalars — had never run with more than one
# rank: real RCCL refuses two ranks of one communicator on the pool's one-GPU boxes. Here
# each rank is a PROCESS whose RcclComm is bound (OPT_AMD_RCCL_LIB) to tests/rccl_stub, a
# stand-in exporting the same ten entry points over shared memory + HIP IPC, whose
# all-reduce sums ranks in the order OptAMD_LocalGroup does. The solve over the real
# transport code must then be BITWISE the LocalGroup solve of the same slabs (same kernels,
# same halo/interior overlap, same sums). Reference: backend_cpu_mt.t:716-737 (the
# reference's own outer-dimension split), SURVEY.md §8(e).
STUB = os.path.join(ROOT, "tests", "rccl_stub", "librccl_stub.so")


def _stub_id():
    import secrets
    name = f"/optamd_rccl_stub_{os.getpid()}_{secrets.token_hex(8)}".encode()
    return list(name + bytes(128 - len(name)))


def _stub_rank_main(rank, world, uid, family, W, H, nit, lit, q):
    try:
        import sys
        os.environ["OPT_AMD_RCCL_LIB"] = STUB
        sys.path.insert(0, ROOT)
        import torch

        from opt_amd import api
        from opt_amd import distributed as dd

        torch.cuda.set_device(0)
        lib = api.load_library()
        raw = (ctypes.c_uint8 * 128)(*uid)
        comm = lib.OptAMD_CommCreateRccl(raw, rank, world)
        assert comm, "OptAMD_CommCreateRccl failed over the stub"
        name = ctypes.create_string_buffer(16)
        if family == "image_warping":
            from tests.iw_helpers import device_params, perturbed, solver
            w = perturbed(W, H, seed=31)
            s = solver(W, H)
            sl = dd.slab(H, rank, world, s.halo())
            s.set_decomposition(comm, sl.y_lo, sl.y_hi)
            prm = device_params(dd.local_image_warping(w, sl))
            nscal, key, ch, nsc = 0, 0, 2, 2 + 5 * (lit + 2)
        else:
            from tests.test_decomposition_generic_gpu import SFS
            from opt_amd import OptSolver
            w = SFS.make(W, H)
            s = OptSolver([W, H], SFS.energy, SFS.kind)
            sl = dd.slab(H, rank, world, s.halo())
            s.set_decomposition(comm, sl.y_lo, sl.y_hi)
            prm = SFS.params(w, sl)
            nscal, ch, nsc = len(w["params"]), 1, 8 + 7 * (lit + 2)
            key = nscal
        s.set_solver_params({"nIterations": nit, "lIterations": lit})
        costs = s.profiled_solve(prm)
        X = dd.owned(prm[key].cpu().numpy(), W, ch, sl)
        sc = np.array(s.scalars(nsc))
        kind = "rccl" if lib.OptAMD_CommKind(comm, name, 16) >= 0 and name.value == b"rccl" else name.value
        s.close()
        lib.OptAMD_CommDestroy(comm)
        q.put((rank, "ok", (costs, X, sc, kind)))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "error", repr(e) + traceback.format_exc()))


def _local_group_run(family, W, H, world, nit, lit):
    import threading

    from opt_amd import OptSolver, api
    from opt_amd import distributed as dd
    from tests.iw_helpers import device_params, perturbed, solver
    from tests.test_decomposition_generic_gpu import SFS

    lib = api.load_library()
    group = lib.OptAMD_LocalGroupCreate(world)
    solvers, params, slabs = [], [], []
    w = perturbed(W, H, seed=31) if family == "image_warping" else SFS.make(W, H)
    for r in range(world):
        if family == "image_warping":
            sv = solver(W, H)
        else:
            sv = OptSolver([W, H], SFS.energy, SFS.kind)
        sl = dd.slab(H, r, world, sv.halo())
        sv.set_decomposition(lib.OptAMD_LocalGroupRank(group, r), sl.y_lo, sl.y_hi)
        sv.set_solver_params({"nIterations": nit, "lIterations": lit})
        solvers.append(sv)
        params.append(device_params(dd.local_image_warping(w, sl)) if family == "image_warping" else SFS.params(w, sl))
        slabs.append(sl)
    out = [None] * world
    th = [threading.Thread(target=lambda r=r: out.__setitem__(r, solvers[r].profiled_solve(params[r])))
          for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    key, ch = (0, 2) if family == "image_warping" else (len(w["params"]), 1)
    nsc = 2 + 5 * (lit + 2) if family == "image_warping" else 8 + 7 * (lit + 2)
    X = np.concatenate([dd.owned(params[r][key].cpu().numpy(), W, ch, slabs[r]) for r in range(world)])
    sc = np.array(solvers[0].scalars(nsc))
    for sv in solvers:
        sv.close()
    lib.OptAMD_LocalGroupDestroy(group)
    return out, X, sc


@pytest.mark.parametrize("family,world,W,H", [("image_warping", 2, 160, 120), ("image_warping", 4, 256, 200),
                                              ("shape_from_shading", 2, 128, 96),
                                              ("shape_from_shading", 4, 160, 128)])
def test_rccl_transport_is_bitwise_the_local_group(family, world, W, H):
    assert os.path.exists(STUB), "build the stub first: make rccl_stub"
    nit, lit = 3, 10
    uid = _stub_id()
    ctx = pymp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_stub_rank_main, args=(r, world, uid, family, W, H, nit, lit, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, status, payload = q.get(timeout=240)
            out[r] = (status, payload)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join()
    assert all(v[0] == "ok" for v in out.values()), out
    assert all(out[r][1][3] == "rccl" for r in range(world))    # the RcclComm transport ran
    ref, Xref, scref = _local_group_run(family, W, H, world, nit, lit)
    for r in range(world):
        assert out[r][1][0] == ref[r], (r, out[r][1][0], ref[r])   # bitwise, every rank
    X = np.concatenate([out[r][1][1] for r in range(world)])
    np.testing.assert_array_equal(X, Xref)
    np.testing.assert_array_equal(out[0][1][2], scref)          # the PCG scalar slots of rank 0
    assert ref[0][-1] < ref[0][0]
