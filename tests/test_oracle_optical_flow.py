"""CPU: pin the optical_flow oracle (parity unpinned otherwise: no reference golden
vectors) to an independent float64 numpy restatement of examples/optical_flow/optical_flow.t.

The fit term's Jacobian is defined by the SampledImage derivative images (o.t:3270-3280),
not by differentiating the bilinear sample, so J is assembled analytically here:
fit row d/dX_c = -wf S(I_hat_d{x,y}); regularizer rows by finite differences.
"""
import numpy as np
import pytest

from opt_amd import workloads
from oracle import oracle

DIRS = [(1, 0), (-1, 0), (0, 1), (0, -1)]


def sample64(im, x, y):
    H, W = im.shape
    x0, x1, y0, y1 = int(np.floor(x)), int(np.ceil(x)), int(np.floor(y)), int(np.ceil(y))

    def get(a, b):
        return float(im[b, a]) if 0 <= a < W and 0 <= b < H else 0.0
    xn, yn = x - x0, y - y0
    u = (1 - xn) * get(x0, y0) + xn * get(x1, y0)
    b = (1 - xn) * get(x0, y1) + xn * get(x1, y1)
    return (1 - yn) * u + yn * b


def problem(W=9, H=7, seed=2):
    w = workloads.optical_flow(W, H, seed=seed, sigma=1.0, max_flow=1.5)
    rng = np.random.default_rng(seed)
    w["X"] = rng.uniform(-1.3, 1.3, 2 * W * H).astype(np.float32)
    return w


def residuals_and_jacobian(w, X):
    W, H = w["W"], w["H"]
    I = w["I"].reshape(H, W)
    Ih, Ihx, Ihy = (w[k].reshape(H, W) for k in ("I_hat", "I_hat_dx", "I_hat_dy"))
    wf, wr = float(np.float32(w["w_fitSqrt"])), float(np.float32(w["w_regSqrt"]))
    X = X.astype(np.float64)
    F, rows = [], []
    n = 2 * W * H
    for y in range(H):
        for x in range(W):
            k = y * W + x
            sx, sy = x + X[2 * k], y + X[2 * k + 1]
            F.append(wf * (I[y, x] - sample64(Ih, sx, sy)))
            row = np.zeros(n)
            row[2 * k] = -wf * sample64(Ihx, sx, sy)
            row[2 * k + 1] = -wf * sample64(Ihy, sx, sy)
            rows.append(row)
            for dx, dy in DIRS:
                tx, ty = x + dx, y + dy
                for c in range(2):
                    row = np.zeros(n)
                    if 0 <= tx < W and 0 <= ty < H:
                        t = ty * W + tx
                        F.append(wr * (X[2 * k + c] - X[2 * t + c]))
                        row[2 * k + c] += wr
                        row[2 * t + c] -= wr
                    else:
                        F.append(0.0)
                    rows.append(row)
    return np.array(F), np.array(rows)


@pytest.mark.parametrize("double", [False, True])
def test_cost_jtf_apply_model_match_numpy(double):
    w = problem()
    F, J = residuals_and_jacobian(w, w["X"])
    tol = 1e-12 if double else 2e-5
    assert oracle.of_cost(w, double=double) == pytest.approx(0.5 * F @ F, rel=max(tol, 1e-6))
    r, dg = oracle.of_jtf(w, double=double)
    g = J.T @ F
    np.testing.assert_allclose(r, -g, atol=tol * 50 * np.abs(g).max())
    np.testing.assert_allclose(dg, np.sum(J * J, axis=0), rtol=tol * 10)
    rng = np.random.default_rng(4)
    p = rng.normal(size=J.shape[1])
    Ap, pAp = oracle.of_apply(w, p, double=double)
    ref = J.T @ (J @ p)
    np.testing.assert_allclose(Ap, ref, atol=tol * 50 * np.abs(ref).max())
    assert pAp == pytest.approx(float(p @ ref), rel=tol * 50)
    d = 0.1 * rng.normal(size=J.shape[1])
    m = F + J @ d
    assert oracle.of_model_cost(w, d, double=double) == pytest.approx(0.5 * m @ m, rel=max(tol * 10, 1e-6))


def test_integer_positions_and_outside_samples():
    """x0 == x1 at integer flow; taps outside the image read 0 (Image:get)."""
    w = problem(6, 5, seed=3)
    W, H = 6, 5
    X = np.zeros(2 * W * H, np.float32)
    X[0::2] = 2.0        # integral shift; right columns sample outside
    X[1] = -7.25         # pixel 0 samples far above the image
    F, _ = residuals_and_jacobian(w, X)
    assert oracle.of_cost(w, X=X, double=True) == pytest.approx(0.5 * F @ F, rel=1e-12)


def test_gn_first_steps_decrease_cost_and_precisions_agree():
    w = workloads.optical_flow(64, 48, seed=6, sigma=5.0, max_flow=0.5)
    _, c32 = oracle.of_solve(w, 3, 10)
    _, c64 = oracle.of_solve(w, 3, 10, double=True)
    assert c64[0] > c64[1] > c64[2] > c64[3]
    np.testing.assert_allclose(c32, c64, rtol=1e-4)


def test_lm_is_monotone_and_precisions_agree():
    """LM never accepts an increase (trust-region rejections keep the cost)."""
    w = workloads.optical_flow(64, 48, seed=6, sigma=5.0, max_flow=1.0)
    _, c32 = oracle.of_solve(w, 12, 10, lm=True)
    _, c64 = oracle.of_solve(w, 12, 10, lm=True, double=True)
    assert np.all(np.diff(c64) <= 0) and c64[-1] < 0.9 * c64[0]
    n = min(len(c32), len(c64))
    np.testing.assert_allclose(c32[:n], c64[:n], rtol=1e-3)
