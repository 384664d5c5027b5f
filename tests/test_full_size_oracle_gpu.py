"""GPU: BASELINE configs 3 and 4 pinned against the oracle AT FULL SIZE.

Config 3 (shape_from_shading 4096^2 fp32, LM + PCG; the config north_star tiles across the
node) and config 4 (arap_mesh_deformation, 1M-vertex grid mesh, fp32 GN) were checked at
full size only through properties (monotone LM energy, descent, determinism) and the
8-way split only against the single-domain GPU solve. Here the oracle runs the same
problems on the host (oracle/sfs_impl.h + solver_impl.h: the reference's LM loop,
solverGPUGaussNewton.t:1042-1120, 2035-2292; oracle/arap_impl.h) in fp32 and in fp64, and:
  * the fp32 GPU energies lie within max(2 x the measured fp32 floor, 1e-5) of the fp64
    oracle, where the floor is the fp32 oracle's own distance from the fp64 oracle (running
    max over the steps): how far an fp32 evaluation of the same algorithm lands;
  * the LM accept / reject sequence is the oracle's (a rejected step leaves the energy
    unchanged: the step is reverted, :2283-2290), and the step count is the same;
  * the unknowns of valid pixels / all vertices within the same floor-based bar;
  * the fp64 GPU path against the double oracle within 1e-8 (energies and unknowns);
  * the 8-way row split (LocalGroup: the 8 ranks as threads of this process running the
    RCCL transport's solver code) against the same oracle with the same bars.
The oracle runs on the host cores this process may use (at most 16: the box's share)."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver, workloads
from oracle import oracle
from tests.iw_helpers import ROOT

pytestmark = pytest.mark.gpu

SFS_ENERGY = os.path.join(ROOT, "energies", "shape_from_shading.t")
ARAP_ENERGY = os.path.join(ROOT, "energies", "arap_mesh_deformation.t")
NIT, LIT = 3, 10


def host_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def to_np(t):
    return t.detach().cpu().numpy()


def sfs_params(w, double=False):
    import torch

    scal = [float(v) for v in w["params"]]
    X = w["X"].astype(np.float64) if double else w["X"].copy()
    arrs = [X, w["D_i"], w["Im"], w["edgeMaskR"], w["edgeMaskC"]]
    return scal + [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def accepted(c):
    """LM step outcomes from an energy sequence: a rejected step is reverted and leaves
    the energy bitwise unchanged."""
    c = np.asarray(c)
    return c[1:] != c[:-1]


def floor_bar(c32, c64):
    return np.maximum(2 * np.maximum.accumulate(np.abs(c32 - c64) / c64), 1e-5)


def check_energies(c, c32, c64, what):
    c = np.asarray(c)
    assert len(c) == len(c64) == len(c32), (what, c, c64)
    assert np.array_equal(accepted(c), accepted(c64)), (what, c, c64)
    err = np.abs(c - c64) / c64
    bar = floor_bar(c32, c64)
    print(f"{what}: GPU vs fp64 oracle {err}, fp32 oracle vs fp64 oracle {np.abs(c32 - c64) / c64}")
    assert np.all(err <= bar), (what, err, bar)


@pytest.fixture(scope="module")
def config3():
    """4096^2, the bench's --workload shape_from_shading inputs (seed 3), with the
    oracle's fp32 and fp64 LM solves (3 steps x 10 PCG) on the host threads."""
    N = 4096
    w = workloads.shape_from_shading(N, N, seed=3)
    nt = host_threads()
    X32, c32 = oracle.sfs_solve(w, NIT, LIT, lm=True, nthreads=nt)
    X64, c64 = oracle.sfs_solve(w, NIT, LIT, lm=True, nthreads=nt, double=True)
    act = w["D_i"] > 0
    return w, c32, c64, X32, X64, act


def _x_bar(X32, X64, act):
    scale = np.abs(X64[act]).max()
    return max(2 * np.abs(X32 - X64)[act].max() / scale, 1e-5), scale


@pytest.mark.timeout(400)
def test_config3_single_domain_matches_oracle(config3):
    w, c32, c64, X32, X64, act = config3
    N = w["W"]
    s = OptSolver([N, N], SFS_ENERGY, "LMGPU")
    prm = sfs_params(w)
    s.set_solver_params({"nIterations": NIT, "lIterations": LIT})
    c = s.profiled_solve(prm)
    check_energies(c, c32, c64, "config3 4096^2 fp32")
    X = to_np(prm[len(w["params"])])
    bar, scale = _x_bar(X32, X64, act)
    assert np.abs(X - X64)[act].max() <= bar * scale


@pytest.mark.timeout(400)
def test_config3_split_8_ways_matches_oracle(config3):
    """The 8 x (4096 x 512) row slabs (the slabs' default fused PCGStep2+3, halo overlap)
    against the oracle: the decomposition changes the summation order and the PCG
    arrangement, not the algorithm."""
    from tests.test_decomposition_generic_gpu import SFS, run as run_generic

    w, c32, c64, X32, X64, act = config3
    costs, X = run_generic(SFS, w, 8, NIT, LIT)
    for r in range(8):
        assert costs[r] == costs[0]
    check_energies(costs[0], c32, c64, "config3 4096^2 fp32, 8 slabs")
    bar, scale = _x_bar(X32, X64, act)
    assert np.abs(X - X64)[act].max() <= bar * scale


@pytest.mark.timeout(400)
def test_shape_from_shading_fp64_2048_matches_double_oracle():
    """doublePrecision at 2048^2 (fp64 unknowns and solver, known arrays float) against
    the double oracle (80-bit sums, oracle/iw_impl.h): energies and unknowns within 1e-8."""
    N = 2048
    w = workloads.shape_from_shading(N, N, seed=3)
    s = OptSolver([N, N], SFS_ENERGY, "LMGPU", double_precision=True)
    prm = sfs_params(w, double=True)
    s.set_solver_params({"nIterations": NIT, "lIterations": LIT})
    c = np.array(s.profiled_solve(prm))
    X64, c64 = oracle.sfs_solve(w, NIT, LIT, lm=True, nthreads=host_threads(), double=True)
    print("sfs 2048^2 fp64 vs double oracle", np.abs(c - c64) / c64)
    assert len(c) == len(c64) and np.array_equal(accepted(c), accepted(c64))
    np.testing.assert_allclose(c, c64, rtol=1e-8)
    act = w["D_i"] > 0
    X = to_np(prm[len(w["params"])])
    assert np.abs(X - X64)[act].max() <= 1e-8 * np.abs(X64[act]).max()


def arap_params(w, double=False):
    import torch

    dt = np.float64 if double else np.float32
    arrs = [w["Offset"].astype(dt).copy(), w["Angle"].astype(dt).copy(), w["UrShape"], w["Constraints"]]
    arrs = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]
    graph = [torch.from_numpy(g).cuda() for g in (w["v0"], w["v1"])]
    return [w["w_fitSqrt"], w["w_regSqrt"]] + arrs + [None] + graph


@pytest.mark.timeout(400)
def test_config4_one_million_vertices_matches_oracle():
    """Config 4 (1000 x 1000 grid mesh, ~6M directed edges), GN 3 x 10 PCG: fp32 against
    the fp64 oracle within the floor-based bar (it was 1e-4), Offset / Angle too; fp64
    against the double oracle within 1e-8."""
    w = workloads.arap_grid(1000, 1000, seed=9)
    O32, A32, c32 = oracle.arap_solve(w, NIT, LIT)
    O64, A64, c64 = oracle.arap_solve(w, NIT, LIT, double=True)
    s = OptSolver([w["N"], w["E"]], ARAP_ENERGY, "gaussNewtonGPU")
    prm = arap_params(w)
    s.set_solver_params({"nIterations": NIT, "lIterations": LIT})
    c = s.profiled_solve(prm)
    s.close()
    check_energies(c, c32, c64, "config4 1M vertices fp32")
    for got, u32, u64 in ((to_np(prm[2]), O32, O64), (to_np(prm[3]), A32, A64)):
        scale = np.abs(u64).max()
        assert np.abs(got - u64).max() <= max(2 * np.abs(u32 - u64).max(), 1e-5 * scale)
    s = OptSolver([w["N"], w["E"]], ARAP_ENERGY, "gaussNewtonGPU", double_precision=True)
    prm = arap_params(w, double=True)
    s.set_solver_params({"nIterations": NIT, "lIterations": LIT})
    c = np.array(s.profiled_solve(prm))
    print("config4 fp64 vs double oracle", np.abs(c - c64) / c64)
    np.testing.assert_allclose(c, c64, rtol=1e-8)
    for got, u64 in ((to_np(prm[2]), O64), (to_np(prm[3]), A64)):
        assert np.abs(got - u64).max() <= 1e-8 * np.abs(u64).max()
