"""CPU: pin the arap_mesh_deformation oracle (parity unpinned otherwise: no reference
golden outputs) to an independent float64 numpy restatement of
examples/arap_mesh_deformation/arap_mesh_deformation.t (Rotate3D from API/src/lib.t:84-98)
with a finite-difference Jacobian."""
import numpy as np
import pytest

from opt_amd import workloads
from oracle import oracle


def rot3(a):
    al, be, ga = a
    ca, cb, cg, sa, sb, sg = np.cos(al), np.cos(be), np.cos(ga), np.sin(al), np.sin(be), np.sin(ga)
    return np.array([[cg * cb, -sg * ca + cg * sb * sa, sg * sa + cg * sb * ca],
                     [sg * cb, cg * ca + sg * sb * sa, -cg * sa + sg * sb * ca],
                     [-sb, cb * sa, cb * ca]])


def residuals64(w, x):
    N = w["N"]
    O = x[:3 * N].reshape(N, 3)
    A = x[3 * N:].reshape(N, 3)
    U = w["UrShape"].reshape(N, 3).astype(np.float64)
    C = w["Constraints"].reshape(N, 3).astype(np.float64)
    wf, wr = float(np.float32(w["w_fitSqrt"])), float(np.float32(w["w_regSqrt"]))
    fit = np.where((C[:, 0] >= -999999.9)[:, None], wf * (O - np.where(np.isfinite(C), C, 0)), 0.0)
    reg = [wr * ((O[a] - O[b]) - rot3(A[a]) @ (U[a] - U[b])) for a, b in zip(w["v0"], w["v1"])]
    return np.concatenate([fit.ravel(), np.array(reg).ravel()])


def small():
    w = workloads.arap_grid(7, 5, seed=2, n_handles=3)
    rng = np.random.default_rng(2)
    w["Offset"] = (w["Offset"] + 0.05 * rng.normal(size=w["Offset"].size)).astype(np.float32)
    w["Angle"] = (0.3 * rng.normal(size=w["Angle"].size)).astype(np.float32)
    return w


def jac(w):
    x0 = np.concatenate([w["Offset"], w["Angle"]]).astype(np.float64)
    F = residuals64(w, x0)
    J = np.zeros((F.size, x0.size))
    for j in range(x0.size):
        xp, xm = x0.copy(), x0.copy()
        xp[j] += 1e-6
        xm[j] -= 1e-6
        J[:, j] = (residuals64(w, xp) - residuals64(w, xm)) / 2e-6
    return F, J


@pytest.mark.parametrize("double", [False, True])
def test_cost_jtf_apply_model_match_numpy(double):
    """float: within fp32 error; double (the checker of the fp64 GPU path): within 1e-6
    (the oracle, like the kernels, forms UrShape differences in float)."""
    t = 1e-6 if double else 1.0
    dt = np.float64 if double else np.float32
    w = small()
    F, J = jac(w)
    assert oracle.arap_cost(w, double=double) == pytest.approx(0.5 * F @ F, rel=min(1e-5, t))
    r, dg = oracle.arap_jtf(w, double=double)
    g = J.T @ F
    np.testing.assert_allclose(r, -g, atol=min(2e-5, t) * np.abs(g).max())
    np.testing.assert_allclose(dg, np.sum(J * J, axis=0), rtol=min(1e-4, t), atol=min(1e-6, t))
    rng = np.random.default_rng(5)
    p = rng.normal(size=J.shape[1]).astype(dt)
    Ap, pAp = oracle.arap_apply(w, p, double=double)
    ref = J.T @ (J @ p.astype(np.float64))
    np.testing.assert_allclose(Ap, ref, atol=min(2e-5, t) * np.abs(ref).max())
    assert pAp == pytest.approx(float(p @ ref), rel=min(1e-5, t))
    d = (0.01 * rng.normal(size=J.shape[1])).astype(dt)
    m = F + J @ d
    assert oracle.arap_model_cost(w, d, double=double) == pytest.approx(0.5 * m @ m, rel=min(1e-5, t))


@pytest.mark.parametrize("lm", [False, True])
def test_solve_descends(lm):
    w = workloads.arap_grid(40, 30, seed=4)
    _, _, c = oracle.arap_solve(w, 5, 20, lm=lm)
    assert c[-1] < 0.5 * c[0]
    if lm:
        assert np.all(np.diff(c) <= 0)
