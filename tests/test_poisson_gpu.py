"""GPU parity of the poisson_image_editing path (generic GN/LM driver + pie_* kernels)
against the C oracle, through the C ABI. BASELINE config 1 (512^2, 1 GN / 10 PCG,
reference CPU backend) runs through the backend_cpu host-pointer mode."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver, workloads
from oracle import oracle
from tests.iw_helpers import ROOT, rel_err

pytestmark = pytest.mark.gpu
ENERGY = os.path.join(ROOT, "energies", "poisson_image_editing.t")


def dev(w):
    import torch
    return [torch.from_numpy(w[k].copy()).cuda() for k in ("X", "T", "M")]


def to_np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("W,H", [(64, 48), (97, 61), (130, 7), (1, 30)])
def test_kernels_match_oracle(W, H):
    import torch

    w = workloads.poisson_image_editing(W, H, seed=W + H)
    rng = np.random.default_rng(3)
    w["X"] = (w["X"] + rng.normal(0, 2, w["X"].shape)).astype(np.float32)
    s = OptSolver([W, H], ENERGY)
    assert s.family() == "poisson_image_editing"
    prm = dev(w)
    assert s.eval_cost(prm) == pytest.approx(oracle.pie_cost(w), rel=1e-5, abs=1e-9)
    n = 4 * W * H
    r = torch.zeros(n, device="cuda")
    pre = torch.zeros(n, device="cuda")
    s.eval_jtf(prm, r, pre)
    r_ref, _ = oracle.pie_jtf(w)
    assert rel_err(to_np(r), r_ref) < 2e-5
    act = np.repeat(w["M"] == 0, 4)
    assert np.all(to_np(pre)[act] == 0.25) and np.all(to_np(pre)[~act] == 0)   # guardedInvert(1)
    p = rng.normal(size=n).astype(np.float32)
    p[~act] = 0
    Ap = torch.zeros(n, device="cuda")
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.pie_apply(w, p)
    assert rel_err(to_np(Ap), Ap_ref) < 2e-5
    assert pAp == pytest.approx(pAp_ref, rel=1e-5)


@pytest.mark.parametrize("kind,nit,lit", [("gaussNewtonGPU", 1, 10), ("gaussNewtonGPU", 3, 10),
                                          ("LMGPU", 4, 10), ("LMGPU", 3, 25)])
def test_solve_matches_oracle(kind, nit, lit):
    W, H = 120, 90
    w = workloads.poisson_image_editing(W, H, seed=11)
    s = OptSolver([W, H], ENERGY, kind)
    prm = dev(w)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    X_ref, c_ref = oracle.pie_solve(w, nit, lit, lm=(kind == "LMGPU"))
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-5)
    assert rel_err(to_np(prm[0]), X_ref) < 1e-5


def test_config1_cpu_backend_512():
    """BASELINE config 1: 512x512, 1 GN outer / 10 PCG inner, host (CPU-backend) buffers."""
    W = H = 512
    w = workloads.poisson_image_editing(W, H, seed=1)
    s = OptSolver([W, H], ENERGY, "gaussNewtonGPU", backend="backend_cpu")
    X = w["X"].copy()
    s.set_solver_params({"nIterations": 1, "lIterations": 10})
    costs = s.profiled_solve([X, w["T"], w["M"]])
    X_ref, c_ref = oracle.pie_solve(w, 1, 10)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-5)
    assert costs[1] < costs[0]
    assert rel_err(X, X_ref) < 1e-5


@pytest.mark.parametrize("kind,nit,lit", [("gaussNewtonGPU", 3, 10), ("LMGPU", 4, 10)])
@pytest.mark.parametrize("W,H", [(64, 48), (97, 61), (130, 7)])
def test_double_precision_matches_double_oracle(kind, nit, lit, W, H):
    """doublePrecision (Opt.h:11-14): X and the solver in double, T / M float, against the
    double oracle (oracle/pie_impl.h): J^T F, J^T J p within 1e-10 of their largest
    magnitude, the cost within 1e-12, GN / LM trajectories and X within 1e-8."""
    import torch

    w = workloads.poisson_image_editing(W, H, seed=W + 2 * H)
    rng = np.random.default_rng(4)
    w["X"] = (w["X"] + rng.normal(0, 2, w["X"].shape)).astype(np.float32)
    s = OptSolver([W, H], ENERGY, kind, double_precision=True)
    prm = [torch.from_numpy(w["X"].astype(np.float64)).cuda()] + dev(w)[1:]
    assert s.eval_cost(prm) == pytest.approx(oracle.pie_cost(w, double=True), rel=1e-12, abs=1e-12)
    n = 4 * W * H
    r = torch.zeros(n, device="cuda", dtype=torch.float64)
    pre = torch.zeros(n, device="cuda", dtype=torch.float64)
    s.eval_jtf(prm, r, pre)
    r_ref, _ = oracle.pie_jtf(w, double=True)
    assert rel_err(to_np(r), r_ref) < 1e-10
    act = np.repeat(w["M"] == 0, 4)
    p = rng.normal(size=n)
    p[~act] = 0
    Ap = torch.zeros(n, device="cuda", dtype=torch.float64)
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.pie_apply(w, p, double=True)
    assert rel_err(to_np(Ap), Ap_ref) < 1e-10
    assert pAp == pytest.approx(pAp_ref, rel=1e-10)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    X_ref, c_ref = oracle.pie_solve(w, nit, lit, lm=(kind == "LMGPU"), double=True)
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-8)
    assert rel_err(to_np(prm[0]), X_ref) < 1e-8
