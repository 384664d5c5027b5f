"""GPU parity of the optical_flow path (generic GN/LM driver + of_* kernels: sampled
fit term, cached gradient, 5-point regularizer) against the C oracle, through the C ABI,
in opt_float = float and double. BASELINE config 5 (3840x2160, fp64, LM) at full size."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver, workloads
from oracle import oracle
from tests.iw_helpers import ROOT, rel_err

pytestmark = pytest.mark.gpu
ENERGY = os.path.join(ROOT, "energies", "optical_flow.t")


def params(w, double=False, host=False):
    dt = np.float64 if double else np.float32
    X = w["X"].astype(dt)
    arrs = [w["I"], w["I_hat"], w["I_hat_dx"], w["I_hat_dy"]]
    if host:
        return [w["w_fitSqrt"], w["w_regSqrt"], X.copy()] + arrs
    import torch
    return [w["w_fitSqrt"], w["w_regSqrt"], torch.from_numpy(X.copy()).cuda()] + \
        [torch.from_numpy(a).cuda() for a in arrs]


def to_np(t):
    return t.detach().cpu().numpy() if hasattr(t, "detach") else t


def perturbed(W, H, seed, sigma=3.0, max_flow=1.0):
    w = workloads.optical_flow(W, H, seed=seed, sigma=sigma, max_flow=max_flow)
    w["X"] = np.random.default_rng(seed).uniform(-1.5, 1.5, 2 * W * H).astype(np.float32)
    return w


@pytest.mark.parametrize("double", [False, True])
@pytest.mark.parametrize("W,H,rows", [(64, 48, "16"), (97, 61, "16"), (130, 7, "16"), (1, 30, "16"), (124, 33, "5"),
                                      (125, 2, "16"), (63, 70, "1")])
def test_strip_apply_equals_flat_apply(monkeypatch, W, H, rows, double):
    """of_apply_strip (round 6: 62-column register strips, side-by-side waves, OPT_AMD_OF_ROWS
    rows per wave) against the flat per-pixel of_apply (OPT_AMD_OF_STRIP=0): the same terms
    per pixel in the same order — Ap within 1e-15 (fp64) / 1e-6 (fp32) relative (fp
    contraction may fuse differently in the two kernels), p.Ap likewise; strip edges at
    widths 62 k +- 1 and row chunks that do not divide the height."""
    import torch

    w = perturbed(W, H, seed=W + 7 * H)
    dt = torch.float64 if double else torch.float32
    n = 2 * W * H
    p = torch.from_numpy(np.random.default_rng(3).normal(size=n)).to("cuda", dt)
    out = {}
    for strip in ("1", "0"):
        monkeypatch.setenv("OPT_AMD_OF_STRIP", strip)
        monkeypatch.setenv("OPT_AMD_OF_ROWS", rows)
        s = OptSolver([W, H], ENERGY, "LMGPU", double_precision=double)
        prm = params(w, double)
        r = torch.zeros(n, device="cuda", dtype=dt)
        s.eval_jtf(prm, r, torch.zeros_like(r))   # caches the sampled gradient
        Ap = torch.zeros(n, device="cuda", dtype=dt)
        out[strip] = (s.apply_jtj(prm, p, Ap), to_np(Ap))
        s.close()
    tol = 1e-14 if double else 1e-6
    assert rel_err(out["1"][1], out["0"][1]) < tol
    assert out["1"][0] == pytest.approx(out["0"][0], rel=tol)


@pytest.mark.parametrize("double", [False, True])
@pytest.mark.parametrize("W,H", [(64, 48), (97, 61), (130, 7), (1, 30)])
def test_kernels_match_oracle(W, H, double):
    import torch

    w = perturbed(W, H, seed=W * H)
    s = OptSolver([W, H], ENERGY, "LMGPU", double_precision=double)
    assert s.family() == "optical_flow"
    prm = params(w, double)
    tol = 1e-12 if double else 2e-5
    assert s.eval_cost(prm) == pytest.approx(oracle.of_cost(w, double=double), rel=max(tol, 1e-6))
    dt = torch.float64 if double else torch.float32
    n = 2 * W * H
    r = torch.zeros(n, device="cuda", dtype=dt)
    pre = torch.zeros(n, device="cuda", dtype=dt)
    s.eval_jtf(prm, r, pre)
    r_ref, _ = oracle.of_jtf(w, double=double)
    assert rel_err(to_np(r), r_ref) < tol * 10
    assert np.all(to_np(pre) == 0.25)   # UsePreconditioner(false): guardedInvert(1)
    p = np.random.default_rng(2).normal(size=n)
    Ap = torch.zeros(n, device="cuda", dtype=dt)
    pAp = s.apply_jtj(prm, torch.from_numpy(p).to("cuda", dt), Ap)
    Ap_ref, pAp_ref = oracle.of_apply(w, p, double=double)
    assert rel_err(to_np(Ap), Ap_ref) < tol * 10
    assert pAp == pytest.approx(pAp_ref, rel=tol * 10)


@pytest.mark.parametrize("double", [False, True])
@pytest.mark.parametrize("kind,nit,lit", [("gaussNewtonGPU", 3, 10), ("LMGPU", 8, 10), ("LMGPU", 4, 25)])
def test_solve_matches_oracle(kind, nit, lit, double):
    W, H = 96, 64
    w = workloads.optical_flow(W, H, seed=8, sigma=5.0, max_flow=0.5 if kind == "gaussNewtonGPU" else 1.5)
    s = OptSolver([W, H], ENERGY, kind, double_precision=double)
    prm = params(w, double)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    X_ref, c_ref = oracle.of_solve(w, nit, lit, lm=(kind == "LMGPU"), double=double)
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-8 if double else 2e-5)
    assert rel_err(to_np(prm[2]), X_ref) < (1e-7 if double else 1e-4)


def test_host_buffers_equal_device_path():
    W, H = 80, 50
    w = workloads.optical_flow(W, H, seed=3, sigma=4.0, max_flow=1.0)
    sd = OptSolver([W, H], ENERGY, "LMGPU", double_precision=True)
    pd = params(w, True)
    sd.set_solver_params({"nIterations": 4, "lIterations": 10})
    cd = sd.profiled_solve(pd)
    sh = OptSolver([W, H], ENERGY, "LMGPU", double_precision=True, backend="backend_cpu")
    ph = params(w, True, host=True)
    sh.set_solver_params({"nIterations": 4, "lIterations": 10})
    ch = sh.profiled_solve(ph)
    np.testing.assert_array_equal(cd, ch)
    np.testing.assert_array_equal(to_np(pd[2]), ph[2])


def test_config5_full_size_fp64_lm():
    """BASELINE config 5: 3840x2160, fp64 unknowns, LM; energy trajectory vs the oracle
    (north star: final energy within 1e-5 relative) and LM monotonicity."""
    W, H = 3840, 2160
    w = workloads.optical_flow(W, H, seed=5)
    s = OptSolver([W, H], ENERGY, "LMGPU", double_precision=True)
    prm = params(w, True)
    s.set_solver_params({"nIterations": 8, "lIterations": 10})
    costs = s.profiled_solve(prm)
    assert np.all(np.diff(costs) <= 0)
    _, c_ref = oracle.of_solve(w, 8, 10, lm=True, double=True)
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-5)
