"""CPU: pin the poisson_image_editing oracle to an independent float64 restatement of
the energy file and a finite-difference Jacobian (parity otherwise unpinned)."""
import numpy as np
import pytest

from opt_amd import workloads
from oracle import oracle

DIRS = [(1, 0), (-1, 0), (0, 1), (0, -1)]


def residuals64(w, X):
    W, H = w["W"], w["H"]
    X = X.reshape(H, W, 4)
    T = w["T"].reshape(H, W, 4).astype(np.float64)
    res = np.zeros((H, W, 4, 4))
    for y in range(H):
        for x in range(W):
            for k, (sx, sy) in enumerate(DIRS):
                tx, ty = x + sx, y + sy
                if 0 <= tx < W and 0 <= ty < H:
                    res[y, x, k] = (X[y, x] - X[ty, tx]) - (T[y, x] - T[ty, tx])
    return res


def small(W=6, H=5, seed=2):
    rng = np.random.default_rng(seed)
    w = workloads.poisson_image_editing(W, H, seed=seed)
    w["M"][:] = 0.0
    w["M"][[0, 7, 13]] = 255.0          # a few fixed (excluded) pixels incl. a corner
    w["X"] = (w["X"] + rng.normal(0, 3, w["X"].shape)).astype(np.float32)
    return w


def test_cost_jtf_apply_against_fd():
    w = small()
    W, H = w["W"], w["H"]
    act_px = w["M"] == 0
    act = np.repeat(act_px, 4)
    x0 = w["X"].astype(np.float64)
    res = residuals64(w, x0)
    # cost: 1/2 sum over active centres
    c64 = 0.5 * float(np.sum(res.reshape(H * W, 16)[act_px] ** 2))
    assert oracle.pie_cost(w) == pytest.approx(c64, rel=1e-5)
    # Jacobian of ALL residuals (gathers include residuals centred at excluded pixels)
    n = x0.size
    J = np.zeros((res.size, n))
    for j in range(n):
        xp, xm = x0.copy(), x0.copy()
        xp[j] += 1e-4
        xm[j] -= 1e-4
        J[:, j] = (residuals64(w, xp) - residuals64(w, xm)).ravel() / 2e-4
    g = J.T @ res.ravel()
    r, dg = oracle.pie_jtf(w)
    np.testing.assert_allclose(r[act], -g[act], atol=1e-3 * np.abs(g).max())
    np.testing.assert_allclose(dg[act], np.sum(J * J, axis=0)[act], rtol=1e-6)
    assert np.all(r[~act] == 0)
    rng = np.random.default_rng(1)
    p = rng.normal(size=n).astype(np.float32)
    p[~act] = 0
    Ap, pAp = oracle.pie_apply(w, p)
    ref = J.T @ (J @ p.astype(np.float64))
    np.testing.assert_allclose(Ap[act], ref[act], atol=1e-4 * np.abs(ref).max())
    assert pAp == pytest.approx(float(p @ ref), rel=1e-5)


def test_gn_and_lm_decrease_cost():
    w = workloads.poisson_image_editing(48, 40, seed=4)
    _, c = oracle.pie_solve(w, 2, 10)
    assert len(c) == 3 and c[1] < c[0] and c[2] <= c[1]
    _, c = oracle.pie_solve(w, 3, 10, lm=True)
    assert c[-1] < c[0]


def test_double_oracle_against_fd():
    """opt_float = double: X and the solver in double, T / M float (oracle/pie_impl.h)."""
    w = small()
    W, H = w["W"], w["H"]
    act_px = w["M"] == 0
    act = np.repeat(act_px, 4)
    x0 = w["X"].astype(np.float64)
    res = residuals64(w, x0)
    assert oracle.pie_cost(w, double=True) == pytest.approx(0.5 * float(np.sum(res.reshape(H * W, 16)[act_px] ** 2)),
                                                           rel=1e-13)
    n = x0.size
    J = np.zeros((res.size, n))
    for j in range(n):   # the residuals are linear: central differences are exact up to rounding
        xp, xm = x0.copy(), x0.copy()
        xp[j] += 0.5
        xm[j] -= 0.5
        J[:, j] = (residuals64(w, xp) - residuals64(w, xm)).ravel()
    g = J.T @ res.ravel()
    r, dg = oracle.pie_jtf(w, double=True)
    assert r.dtype == np.float64
    np.testing.assert_allclose(r[act], -g[act], atol=1e-12 * np.abs(g).max())
    np.testing.assert_array_equal(dg[act], np.sum(J * J, axis=0)[act])
    p = np.random.default_rng(1).normal(size=n)
    p[~act] = 0
    Ap, pAp = oracle.pie_apply(w, p, double=True)
    ref = J.T @ (J @ p)
    np.testing.assert_allclose(Ap[act], ref[act], atol=1e-12 * np.abs(ref).max())
    assert pAp == pytest.approx(float(p @ ref), rel=1e-12)
    Xd, cd = oracle.pie_solve(w, 2, 10, double=True)
    _, cf = oracle.pie_solve(w, 2, 10)
    assert Xd.dtype == np.float64 and cd[-1] < cd[0]
    np.testing.assert_allclose(cf, cd, rtol=1e-5)
