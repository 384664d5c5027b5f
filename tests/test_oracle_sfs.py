"""CPU: pin the shape_from_shading oracle (parity unpinned otherwise: the reference
holds inputs but no expected outputs for this energy) to an independent float64 numpy
restatement of examples/shape_from_shading/shape_from_shading.t.

The numpy side evaluates every residual of every centre directly from the depth image
(B_I recomputed from X, no gradient images) and differentiates by central finite
differences, so the oracle's analytic ComputedArray gradient images, its gathers and its
exclusion / cost-domain rules are all checked against first principles. `valid` is held
at its value at X (its gradient is zero: comparisons only)."""
import os

import numpy as np
import pytest

from opt_amd import workloads
from oracle import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sfs_default.npz")


def small(W=11, H=9, seed=4):
    w = workloads.shape_from_shading(W, H, seed=seed, valid_frac=0.8)
    rng = np.random.default_rng(seed)
    w["edgeMaskR"] = (rng.uniform(size=W * H) < 0.8).astype(np.uint8)
    w["edgeMaskC"] = (rng.uniform(size=W * H) < 0.8).astype(np.uint8)
    return w


def residuals64(w, X, valid_fixed):
    """All residual components of all centres: (values[N, 6], excluded-centre mask)."""
    W, H = w["W"], w["H"]
    p = w["params"].astype(np.float64)
    wp, ws, wg = np.sqrt(p[0]), np.sqrt(p[1]), np.sqrt(p[2])
    fx, fy, ux, uy = p[3:7]
    L = p[7:16]
    D = w["D_i"].reshape(H, W).astype(np.float64)
    Im = w["Im"].reshape(H, W).astype(np.float64)
    mR = w["edgeMaskR"].reshape(H, W).astype(np.float64)
    mC = w["edgeMaskC"].reshape(H, W).astype(np.float64)
    X = X.reshape(H, W).astype(np.float64)

    def g(a, x, y):
        return a[y, x] if 0 <= x < W and 0 <= y < H else 0.0

    def dv(x, y):
        return g(D, x, y) > 0

    def inbe(x, y):
        return 1 <= x < W - 1 and 1 <= y < H - 1

    B = workloads.sfs_shading(X, fx, fy, ux, uy, L)

    def BI(x, y):
        if not (inbe(x, y) and dv(x - 1, y) and dv(x, y) and dv(x, y - 1)):
            return 0.0
        I = g(Im, x, y) * 0.5 + 0.25 * (g(Im, x - 1, y) + g(Im, x, y - 1))
        return B[y, x] - I

    out = np.zeros((H * W, 6))
    for y in range(H):
        for x in range(W):
            k = y * W + x
            if dv(x, y):
                out[k, 0] = wp * (X[y, x] - D[y, x])
            if inbe(x, y):
                out[k, 1] = wg * (BI(x, y) - BI(x + 1, y)) * mR[y, x]
                out[k, 2] = wg * (BI(x, y) - BI(x, y + 1)) * mC[y, x]
            if valid_fixed[k] == 1:
                def pv(ox, oy):
                    d = g(X, x + ox, y + oy)
                    return np.array([((x + ox) - ux) / fx * d, ((y + oy) - uy) / fy * d, d])
                out[k, 3:6] = ws * (4 * pv(0, 0) - (pv(-1, 0) + pv(0, -1) + pv(1, 0) + pv(0, 1)))
    return out, ~(D.reshape(-1) > 0)


def jacobian(w, valid_fixed, h=1e-6):
    X0 = w["X"].astype(np.float64)
    F, excl = residuals64(w, X0, valid_fixed)
    J = np.zeros((F.size, X0.size))
    for j in range(X0.size):
        if excl[j]:
            continue   # excluded unknowns are constants
        xp, xm = X0.copy(), X0.copy()
        xp[j] += h
        xm[j] -= h
        J[:, j] = (residuals64(w, xp, valid_fixed)[0] - residuals64(w, xm, valid_fixed)[0]).reshape(-1) / (2 * h)
    return F, excl, J


def test_precomputed_gradient_images_match_finite_differences():
    w = small()
    W, H = w["W"], w["H"]
    pc = oracle.sfs_precompute(w)
    p = w["params"].astype(np.float64)
    X0 = w["X"].reshape(H, W).astype(np.float64)
    B0 = workloads.sfs_shading(X0, *p[3:7], p[7:16])
    for (ox, oy), G in (((0, 0), pc[1]), ((-1, 0), pc[2]), ((0, -1), pc[3])):
        Xp, Xm = X0.copy(), X0.copy()
        h = 1e-6
        fd = np.zeros((H, W))
        for y in range(1, H - 1):
            for x in range(1, W - 1):
                Xp[:] = X0; Xm[:] = X0
                Xp[y + oy, x + ox] += h
                Xm[y + oy, x + ox] -= h
                fd[y, x] = (workloads.sfs_shading(Xp, *p[3:7], p[7:16])[y, x] -
                            workloads.sfs_shading(Xm, *p[3:7], p[7:16])[y, x]) / (2 * h)
        m = G.reshape(H, W) != 0
        assert m.sum() > 20
        np.testing.assert_allclose(G.reshape(H, W)[m], fd[m], rtol=2e-3, atol=1e-3 * np.abs(fd).max())
    assert np.all(np.isin(pc[4], [0.0, 1.0]))
    del B0


@pytest.mark.parametrize("double", [False, True])
def test_cost_jtf_apply_model_match_numpy(double):
    """float: the fp32 oracle within fp32 + finite-difference error; double: the fp64
    instantiation (the checker of the fp64 GPU path) within 1e-6."""
    t = 1e-6 if double else 1.0
    dt = np.float64 if double else np.float32
    w = small()
    valid = oracle.sfs_precompute(w)[4]
    F, excl, J = jacobian(w, valid)
    Fc = F.copy()
    Fc[excl] = 0          # cost / model cost skip excluded centres
    assert oracle.sfs_cost(w, double=double) == pytest.approx(0.5 * np.sum(Fc ** 2), rel=min(1e-4, t))
    Jf = J.reshape(F.shape[0], 6, -1)
    Jall = Jf.reshape(-1, J.shape[1])
    g = Jall.T @ F.reshape(-1)   # gathers include residuals of excluded centres
    r, dg = oracle.sfs_jtf(w, double=double)
    act = ~excl
    np.testing.assert_allclose(r[act], -g[act], atol=min(2e-3, t) * np.abs(g).max())
    assert np.all(r[excl] == 0)
    np.testing.assert_allclose(dg[act], np.sum(Jall ** 2, axis=0)[act], rtol=min(5e-3, t), atol=min(1e-3, t) * dg.max())
    rng = np.random.default_rng(1)
    pvec = rng.normal(size=J.shape[1]).astype(dt)
    pvec[excl] = 0
    Ap, pAp = oracle.sfs_apply(w, pvec, double=double)
    ref = Jall.T @ (Jall @ pvec.astype(np.float64))
    np.testing.assert_allclose(Ap[act], ref[act], atol=min(3e-3, t) * np.abs(ref).max())
    assert pAp == pytest.approx(float(pvec @ ref), rel=min(3e-3, t))
    d = (1e-3 * rng.normal(size=J.shape[1])).astype(dt)
    d[excl] = 0
    Jc = Jf.copy()
    Jc[excl] = 0
    m = Fc.reshape(-1) + Jc.reshape(-1, J.shape[1]) @ d
    assert oracle.sfs_model_cost(w, d, double=double) == pytest.approx(0.5 * m @ m, rel=min(1e-4, t))


@pytest.mark.parametrize("lm", [False, True])
def test_double_and_float_oracles_agree(lm):
    w = small(23, 17, seed=2)
    _, c32 = oracle.sfs_solve(w, 3, 10, lm=lm)
    X64, c64 = oracle.sfs_solve(w, 3, 10, lm=lm, double=True)
    assert X64.dtype == np.float64 and len(c32) == len(c64)
    np.testing.assert_allclose(c32, c64, rtol=1e-3)


def test_lm_and_gn_decrease_cost_on_reference_inputs():
    """The reference's own example inputs (examples/data/shape_from_shading/default*,
    640x480, tests/golden/sfs_default.npz): LM monotone and both solvers descend."""
    z = np.load(GOLDEN)
    H, W = z["D_i"].shape
    crop = (slice(100, 196), slice(200, 328))   # 96 x 128 window keeps the CPU test short
    w = {"params": z["params"], "W": 128, "H": 96}
    for k in ("D_i", "Im", "edgeMaskR", "edgeMaskC"):
        w[k] = np.ascontiguousarray(z[k][crop]).reshape(-1)
    w["X"] = np.ascontiguousarray(z["X0"][crop]).reshape(-1)
    assert (w["D_i"] > 0).mean() > 0.3
    _, c = oracle.sfs_solve(w, 8, 10, lm=True)
    assert np.all(np.diff(c) <= 0) and c[-1] < c[0]
    _, c = oracle.sfs_solve(w, 2, 10, lm=False)
    assert c[-1] < c[0]


@pytest.mark.parametrize("double", [False, True])
def test_threaded_solve_matches_one_thread(double):
    """The row-slab split over threads (bench.py's config-3 CPU comparator,
    backend_cpu_mt.t:716-737): same per-pixel values, only the sums' order changes."""
    w = workloads.shape_from_shading(96, 72, seed=3)
    X1, c1 = oracle.sfs_solve(w, 3, 10, lm=True, double=double)
    X4, c4 = oracle.sfs_solve(w, 3, 10, lm=True, double=double, nthreads=4)
    assert len(c1) == len(c4)
    np.testing.assert_allclose(c4, c1, rtol=1e-10 if double else 1e-5)
    np.testing.assert_allclose(X4, X1, rtol=0, atol=(1e-10 if double else 1e-5) * np.abs(X1).max())
