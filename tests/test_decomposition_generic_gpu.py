"""GPU: row-slab decomposition of the generic GN/LM driver (poisson_image_editing,
shape_from_shading with its radius-2 halo and computed-array exchange, image_warping
under LM) against the single-domain solve. Ranks are threads of this process sharing
the one GPU (OptAMD_LocalGroup transport); the RCCL transport runs the same code."""
import os
import threading

import numpy as np
import pytest

from opt_amd import OptSolver, api, workloads
from opt_amd import distributed as dd
from tests.iw_helpers import ENERGY as IW_ENERGY, ROOT, device_params, perturbed

pytestmark = pytest.mark.gpu


def to_np(t):
    return t.detach().cpu().numpy()


def _cuda(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


class Family:
    def __init__(self, energy, kind, make, arrays, unknowns):
        self.energy, self.kind, self.make = energy, kind, make
        self.arrays = arrays        # [(name, channels)] in declaration order (after scalars)
        self.unknowns = unknowns    # names of the unknown arrays

    def params(self, w, s=None):
        scal = [float(v) for v in w.get("params", [])]
        out = []
        for name, ch in self.arrays:
            a = w[name] if s is None else dd.slice_rows(w[name], w["W"], ch, s)
            out.append(_cuda(a.copy()))
        return scal + out


POISSON = Family(os.path.join(ROOT, "energies", "poisson_image_editing.t"), "LMGPU",
                 lambda W, H: workloads.poisson_image_editing(W, H, seed=3), [("X", 4), ("T", 4), ("M", 1)], ["X"])
SFS = Family(os.path.join(ROOT, "energies", "shape_from_shading.t"), "LMGPU",
             lambda W, H: workloads.shape_from_shading(W, H, seed=5, valid_frac=0.7),
             [("X", 1), ("D_i", 1), ("Im", 1), ("edgeMaskR", 1), ("edgeMaskC", 1)], ["X"])


def run(fam, w, world, nit, lit, scalars=0):
    """scalars > 0: also return rank 0's first `scalars` plan scalar slots after the solve
    (its last step's PCG sums, stencil_plan.h rz / pap / identity slots)."""
    W, H = w["W"], w["H"]
    lib = api.load_library()
    group = lib.OptAMD_LocalGroupCreate(world)
    solvers, prms, slabs = [], [], []
    for r in range(world):
        sv = OptSolver([W, H], fam.energy, fam.kind)
        s = dd.slab(H, r, world, sv.halo())
        sv.set_decomposition(lib.OptAMD_LocalGroupRank(group, r), s.y_lo, s.y_hi)
        sv.set_solver_params({"nIterations": nit, "lIterations": lit})
        solvers.append(sv)
        prms.append(fam.params(w, s))
        slabs.append(s)
    results, errors = [None] * world, []

    def body(r):
        try:
            results[r] = solvers[r].profiled_solve(prms[r])
        except Exception as e:  # pragma: no cover
            errors.append(e)
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors
    nscal = len(w.get("params", []))
    X = np.concatenate([dd.owned(to_np(prms[r][nscal]), W, fam.arrays[0][1], slabs[r]) for r in range(world)])
    sc = np.array(solvers[0].scalars(scalars)) if scalars else None
    for sv in solvers:
        sv.close()
    lib.OptAMD_LocalGroupDestroy(group)
    return (results, X, sc) if scalars else (results, X)


@pytest.mark.parametrize("fam,world,W,H", [(POISSON, 1, 96, 64), (POISSON, 2, 96, 64), (POISSON, 3, 130, 77),
                                           (SFS, 1, 96, 80), (SFS, 2, 96, 80), (SFS, 4, 128, 120)])
def test_decomposed_matches_single_domain(fam, world, W, H):
    w = fam.make(W, H)
    s = OptSolver([W, H], fam.energy, fam.kind)
    prm = fam.params(w)
    s.set_solver_params({"nIterations": 4, "lIterations": 10})
    ref = s.profiled_solve(prm)
    nscal = len(w.get("params", []))
    Xref = to_np(prm[nscal])
    costs, X = run(fam, w, world, 4, 10)
    for r in range(world):
        assert costs[r] == costs[0]
    if world == 1:
        assert costs[0] == ref and np.array_equal(X, Xref)
    else:
        assert len(costs[0]) == len(ref)
        np.testing.assert_allclose(costs[0], ref, rtol=1e-5)
        act = np.abs(Xref) < 1e3
        assert np.abs(X - Xref)[act].max() <= 1e-5 * np.abs(Xref[act]).max()


def test_optical_flow_refuses_slabs():
    sv = OptSolver([64, 32], os.path.join(ROOT, "energies", "optical_flow.t"), "LMGPU")
    lib = api.load_library()
    group = lib.OptAMD_LocalGroupCreate(2)
    with pytest.raises(Exception):
        sv.set_decomposition(lib.OptAMD_LocalGroupRank(group, 0), 0, 16)
    lib.OptAMD_LocalGroupDestroy(group)


@pytest.mark.parametrize("world", [2, 3])
def test_image_warping_lm_decomposed(world):
    W, H = 120, 90
    w = perturbed(W, H, seed=31)
    s = OptSolver([W, H], IW_ENERGY, "LMGPU")
    prm = device_params(w)
    s.set_solver_params({"nIterations": 4, "lIterations": 10})
    ref = s.profiled_solve(prm)
    lib = api.load_library()
    group = lib.OptAMD_LocalGroupCreate(world)
    solvers, prms, slabs = [], [], []
    for r in range(world):
        sl = dd.slab(H, r, world, 1)
        sv = OptSolver([W, H], IW_ENERGY, "LMGPU")
        sv.set_decomposition(lib.OptAMD_LocalGroupRank(group, r), sl.y_lo, sl.y_hi)
        sv.set_solver_params({"nIterations": 4, "lIterations": 10})
        solvers.append(sv)
        prms.append(device_params(dd.local_image_warping(w, sl)))
        slabs.append(sl)
    out = [None] * world
    th = [threading.Thread(target=lambda r=r: out.__setitem__(r, solvers[r].profiled_solve(prms[r])))
          for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    np.testing.assert_allclose(out[0], ref, rtol=1e-5)
    O = np.concatenate([dd.owned(to_np(prms[r][0]), W, 2, slabs[r]) for r in range(world)])
    ro = to_np(prm[0])
    assert np.abs(O - ro).max() / np.abs(ro).max() < 1e-5
    for sv in solvers:
        sv.close()
    lib.OptAMD_LocalGroupDestroy(group)


# ----------------------------------------- the generated kernels (general front end)
def _intrinsic(W, H):
    rng = np.random.default_rng(17)
    return {"W": W, "H": H, "params": [1.5, 0.7, 0.9, 1.2],
            "r": rng.normal(size=3 * W * H).astype(np.float32), "i": rng.normal(size=3 * W * H).astype(np.float32),
            "s": rng.normal(size=W * H).astype(np.float32)}


class Intrinsic(Family):
    """energies/intrinsic_image_decomposition.t: r at slots 4 (Unknown) and 4 (its Array
    view, the same pointer), i at 5, s at 6."""

    def params(self, w, s=None):
        sl = (lambda a, ch: a) if s is None else (lambda a, ch: dd.slice_rows(a, w["W"], ch, s))
        r = _cuda(sl(w["r"], 3).copy())
        return [float(v) for v in w["params"]] + [r, _cuda(sl(w["i"], 3).copy()), _cuda(sl(w["s"], 1).copy())]


INTRINSIC = Intrinsic(os.path.join(ROOT, "energies", "intrinsic_image_decomposition.t"), "LMGPU", _intrinsic,
                      [("r", 3), ("i", 3), ("s", 1)], ["r"])


@pytest.mark.parametrize("fam,world,W,H", [(POISSON, 2, 96, 64), (SFS, 1, 96, 80), (SFS, 3, 96, 80),
                                           (INTRINSIC, 1, 64, 48), (INTRINSIC, 2, 64, 48), (INTRINSIC, 4, 70, 61)])
def test_generated_kernels_decomposed_match_single_domain(monkeypatch, fam, world, W, H):
    """Row slabs of the generated kernels: the halo from the energy's vertical reach
    (2 for shape_from_shading through its ComputedArray, 1 for the others), ComputedArray
    planes exchanged after precompute, owned-row loops with global coordinates."""
    monkeypatch.setenv("OPT_AMD_GENERIC", "1")
    w = fam.make(W, H)
    s = OptSolver([W, H], fam.energy, fam.kind)
    assert s.family() == "generic"
    assert s.halo() == (2 if fam is SFS else 1)
    prm = fam.params(w)
    s.set_solver_params({"nIterations": 4, "lIterations": 10})
    ref = s.profiled_solve(prm)
    nscal = len(w.get("params", []))
    Xref = to_np(prm[nscal])
    costs, X = run(fam, w, world, 4, 10)
    for r in range(world):
        assert costs[r] == costs[0]
    if world == 1:
        assert costs[0] == ref and np.array_equal(X, Xref)
    else:
        assert len(costs[0]) == len(ref)
        np.testing.assert_allclose(costs[0], ref, rtol=1e-5)
        act = np.abs(Xref) < 1e3
        assert np.abs(X - Xref)[act].max() <= 1e-5 * np.abs(Xref[act]).max()


def test_generated_kernels_refuse_slabs_where_reads_are_data_dependent(monkeypatch):
    monkeypatch.setenv("OPT_AMD_GENERIC", "1")
    lib = api.load_library()
    group = lib.OptAMD_LocalGroupCreate(2)
    for energy, dims in (("optical_flow", [64, 32]), ("volume_denoise", [16, 16, 8])):
        sv = OptSolver(dims, os.path.join(ROOT, "energies", energy + ".t"), "LMGPU")
        assert sv.family() == "generic"
        with pytest.raises(Exception):
            sv.set_decomposition(lib.OptAMD_LocalGroupRank(group, 0), 0, 8)
    lib.OptAMD_LocalGroupDestroy(group)


@pytest.mark.parametrize("world", [2, 3])
def test_sfs_halo_overlap_is_bitwise_the_blocking_exchange(monkeypatch, world):
    """shape_from_shading slabs: the halo refresh of p runs on a second stream beside
    the apply's interior blocks (sfs.hip apply_split, stencil_plan.h pcg_loop), the
    boundary blocks after it; bitwise the blocking exchange before a whole-slab apply."""
    W, H = 256, 240
    w = SFS.make(W, H)
    monkeypatch.setenv("OPT_AMD_HALO_OVERLAP", "0")
    c0, X0 = run(SFS, w, world, 3, 10)
    monkeypatch.setenv("OPT_AMD_HALO_OVERLAP", "1")
    c1, X1 = run(SFS, w, world, 3, 10)
    assert c1[0] == c0[0]
    assert np.array_equal(X1, X0)
