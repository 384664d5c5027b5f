"""GPU: BASELINE config 3's 8-way row split at its real shapes, on one device.

north_star tiles shape_from_shading 4096^2 (LM + PCG) across the 8 GPUs of a node with a
halo exchange and an all-reduce of the PCG scalars, and bench.py --gpus N
splits the image_warping 4096^2 headline the same way. Here the 8 ranks are threads of
this process (OptAMD_LocalGroup: host-staged halos and sums) running the same solver code
as the RCCL transport, on the per-rank shapes the driver's 8-GPU run gives them:
4096 x 512 slabs, where the plans pick their slab-specific strip heights
(image_warping.hip iw::rows_for: 8-row waves; sfs.hip: 12-row strips).

Checks: the decomposed energies against the single-domain solve within the fp32 noise
floor of the trajectory (the single-domain solve's own response to a 1-ulp input change;
1e-5 where that is larger), every rank reporting the same energy, and the halo/interior
overlap bitwise equal to the blocking exchange. Reference: backend_cpu_mt.t:716-737 (the
reference's own outer-dimension split)."""
import numpy as np
import pytest

from tests.test_decomposition_generic_gpu import SFS, run as run_generic, to_np
from tests.test_decomposition_gpu import run_decomposed
from tests.iw_helpers import device_params, solver
from opt_amd import OptSolver, workloads

pytestmark = pytest.mark.gpu

WORLD, N = 8, 4096


def _ulp(a, seed):
    rng = np.random.default_rng(seed)
    return (a * (1 + 2.0 ** -24 * rng.standard_normal(a.size))).astype(np.float32)


def _floor_bar(ref, perturbed):
    return np.maximum(4 * np.abs(perturbed - ref) / np.abs(ref), 1e-5)


@pytest.fixture(scope="module")
def sfs4096():
    return workloads.shape_from_shading(N, N, seed=3)


def test_sfs_lm_4096_split_8_ways_matches_single_domain(monkeypatch, sfs4096):
    # the same PCG loop on one domain and on the slabs: the fused PCGStep2+3 (the slabs'
    # default; its agreement with the classic loop is test_sfs_gpu.py's
    # test_fused_pcg_step_matches_classic)
    monkeypatch.setenv("OPT_AMD_FUSE23", "1")
    w = sfs4096
    nit, lit = 3, 10

    def single(X):
        s = OptSolver([N, N], SFS.energy, SFS.kind)
        s.set_solver_params({"nIterations": nit, "lIterations": lit})
        prm = SFS.params(dict(w, X=X))
        c = np.array(s.profiled_solve(prm))
        return c, to_np(prm[len(w["params"])])

    ref, Xref = single(w["X"])
    pert, _ = single(_ulp(w["X"], 1))
    costs, X, sc = run_generic(SFS, w, WORLD, nit, lit, scalars=8 + 7 * (lit + 2))
    for r in range(WORLD):
        assert costs[r] == costs[0]           # every rank reports the global energy
    c = np.array(costs[0])
    assert len(c) == len(ref)                  # the same LM step count
    assert np.all(np.abs(c - ref) / ref <= _floor_bar(ref, pert)), (c, ref, pert)
    act = np.abs(Xref) < 1e3
    assert np.abs(X - Xref)[act].max() <= 1e-4 * np.abs(Xref[act]).max()
    # the fused step23's beta numerator (identity over the apply's fp64 sums, products in
    # fp64 on both sides) against the direct r.z of the same pass, every PCG
    # iteration of the last LM step on the 8 all-reduced slabs (stencil_plan.h slots:
    # rz(i) = 8 + 7 i, its identity value at rz(i) + 6; LM's residual-reset iteration 9
    # takes the classic sequence; a zeta exit leaves later slots unwritten)
    for i in range(1, lit):
        rz, rzx, rzp = sc[8 + 7 * i], sc[8 + 7 * i + 6], sc[8 + 7 * (i - 1)]
        if i == 9 or rz == 0:
            continue
        assert abs(rzx - rz) <= 1e-4 * rz + 1e-12 * rzp, (i, rz, rzx, rzp)


def test_sfs_4096_split_halo_overlap_is_bitwise_the_blocking_exchange(monkeypatch, sfs4096):
    monkeypatch.setenv("OPT_AMD_HALO_OVERLAP", "0")
    c0, X0 = run_generic(SFS, sfs4096, WORLD, 2, 10)
    monkeypatch.setenv("OPT_AMD_HALO_OVERLAP", "1")
    c1, X1 = run_generic(SFS, sfs4096, WORLD, 2, 10)
    assert c1[0] == c0[0]
    assert np.array_equal(X1, X0)


@pytest.fixture(scope="module")
def iw4096():
    return workloads.image_warping(N, N, seed=1234)


def test_image_warping_gn_4096_split_8_ways_matches_single_domain(iw4096):
    w = iw4096
    nit, lit = 2, 10

    def single(off):
        s = solver(N, N)
        s.set_solver_params({"nIterations": nit, "lIterations": lit})
        prm = device_params(dict(w, Offset=off))
        c = np.array(s.profiled_solve(prm))
        return c, prm[0].cpu().numpy().astype(np.float64), prm[1].cpu().numpy().astype(np.float64)

    ref, Oref, Aref = single(w["Offset"])
    pert, Op, Ap = single(_ulp(w["Offset"], 1))
    costs, O, A = run_decomposed(w, WORLD, nit, lit)
    for r in range(WORLD):
        assert costs[r] == costs[0]
    c = np.array(costs[0])
    assert len(c) == len(ref)
    assert np.all(np.abs(c - ref) / ref <= _floor_bar(ref, pert)), (c, ref, pert)
    # the unknowns too: within 4x the single-domain solve's own response to
    # a 1-ulp input change, or 1e-5 of the largest magnitude
    dO = np.abs(O.astype(np.float64) - Oref).max()
    dA = np.abs(A.astype(np.float64) - Aref).max()
    assert dO <= max(4 * np.abs(Op - Oref).max(), 1e-5 * np.abs(Oref).max()), (dO, np.abs(Op - Oref).max())
    assert dA <= max(4 * np.abs(Ap - Aref).max(), 1e-5 * max(1.0, np.abs(Aref).max())), (dA, np.abs(Ap - Aref).max())


def test_image_warping_4096_split_halo_overlap_is_bitwise_the_blocking_exchange(monkeypatch, iw4096):
    monkeypatch.setenv("OPT_AMD_HALO_OVERLAP", "0")
    c0, O0, A0 = run_decomposed(iw4096, WORLD, 2, 10)
    monkeypatch.setenv("OPT_AMD_HALO_OVERLAP", "1")
    c1, O1, A1 = run_decomposed(iw4096, WORLD, 2, 10)
    assert c1 == c0
    assert np.array_equal(O1, O0) and np.array_equal(A1, A0)
