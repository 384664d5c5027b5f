"""GPU parity of image_warping under LMGPU (generic GN/LM driver + the strip kernels in
their LM variants: J^T F with the raw diagonal, J^T J p + CtC p with the device-side
zeta exit, model cost) against the C oracle's generic LM loop, through the C ABI."""
import numpy as np
import pytest

from oracle import oracle
from tests.iw_helpers import device_params, host_params, perturbed, rel_err, solver

pytestmark = pytest.mark.gpu


def to_np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("W,H,nit,lit", [(37, 29, 4, 10), (130, 70, 5, 10), (64, 64, 4, 25), (200, 3, 3, 10)])
def test_lm_solve_matches_oracle(W, H, nit, lit):
    w = perturbed(W, H, seed=W + H)
    s = solver(W, H, kind="LMGPU")
    prm = device_params(w)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    O_ref, A_ref, c_ref = oracle.iw_solve_generic(w, nit, lit, lm=True)
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=2e-5)
    assert rel_err(to_np(prm[0]), O_ref) < 1e-5
    A = to_np(prm[1])
    assert np.abs(A - A_ref).max() < 1e-4 * max(1.0, np.abs(A_ref).max())


def test_lm_plan_kernels_match_oracle():
    W, H = 97, 61
    w = perturbed(W, H, seed=9)
    s = solver(W, H, kind="LMGPU")
    prm = device_params(w)
    import torch

    n = 3 * W * H
    r = torch.zeros(n, device="cuda")
    pre = torch.zeros(n, device="cuda")
    rz = s.eval_jtf(prm, r, pre)
    r_ref, pre_ref, rz_ref = oracle.iw_eval_jtf(w)
    assert rel_err(to_np(r), r_ref) < 2e-5
    assert rel_err(to_np(pre), pre_ref) < 2e-5
    assert rz == pytest.approx(rz_ref, rel=1e-5)
    rng = np.random.default_rng(1)
    p = rng.normal(size=n).astype(np.float32)
    act = np.concatenate([np.repeat(w["Mask"] == 0, 2), w["Mask"] == 0])
    p[~act] = 0
    Ap = torch.zeros(n, device="cuda")
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.iw_apply_jtj(w, p)
    assert rel_err(to_np(Ap), Ap_ref) < 2e-5
    assert pAp == pytest.approx(pAp_ref, rel=1e-5)
    assert s.eval_cost(prm) == pytest.approx(oracle.iw_cost(w), rel=1e-5)


def test_lm_host_buffers_equal_device_path():
    W, H = 90, 50
    w = perturbed(W, H, seed=3)
    sd = solver(W, H, kind="LMGPU")
    prm = device_params(w)
    sd.set_solver_params({"nIterations": 3, "lIterations": 10})
    cd = sd.profiled_solve(prm)
    sh = solver(W, H, kind="LMGPU", backend="backend_cpu")
    hp = host_params(w)
    sh.set_solver_params({"nIterations": 3, "lIterations": 10})
    ch = sh.profiled_solve(hp)
    np.testing.assert_array_equal(cd, ch)
    np.testing.assert_array_equal(to_np(prm[0]), hp[0])
    np.testing.assert_array_equal(to_np(prm[1]), hp[1])


def test_lm_double_precision_tracks_float():
    W, H = 80, 60
    w = perturbed(W, H, seed=4)
    s32 = solver(W, H, kind="LMGPU")
    p32 = device_params(w)
    s32.set_solver_params({"nIterations": 3, "lIterations": 10})
    c32 = s32.profiled_solve(p32)
    s64 = solver(W, H, double=True, kind="LMGPU")
    p64 = device_params(w, double=True)
    s64.set_solver_params({"nIterations": 3, "lIterations": 10})
    c64 = s64.profiled_solve(p64)
    assert c64[-1] < c64[0]
    np.testing.assert_allclose(c64, c32, rtol=1e-3)
