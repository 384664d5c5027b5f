"""CPU: pin the C oracle to the energy definition (the reference known answer is in test_reference_costs.py).

The reference has no executable path and no golden vectors for this energy
(oracle/README.md), so the oracle is checked against an independent float64 numpy
restatement of examples/image_warping/image_warping.t and a finite-difference
Jacobian of it: cost = 1/2|r|^2, r_oracle = -J^T F, pre = 1/(1+sqrt(diag J^T J))^2,
Ap = J^T J p, plus symmetry / positive semi-definiteness and GN descent.
"""
import numpy as np
import pytest

from opt_amd import workloads
from oracle import oracle

DIRS = [(1, 0), (-1, 0), (0, 1), (0, -1)]


def residuals64(w, O, A, u_float_diff=False):
    """image_warping.t, restated independently in float64 (10 residuals per pixel).
    u_float_diff: UrShape differences as float subtractions (the generated code's Terra
    operation on two float loads, o.t:2418-2470), as in the reference's doublePrecision."""
    W, H = w["W"], w["H"]
    U32 = w["UrShape"].reshape(H, W, 2)
    U = U32.astype(np.float64)
    C = w["Constraints"].reshape(H, W, 2).astype(np.float64)
    M = w["Mask"].reshape(H, W)
    O = O.reshape(H, W, 2)
    A = A.reshape(H, W)
    act = M == 0
    res = np.zeros((H, W, 10))
    wf, wr = float(np.float32(w["w_fitSqrt"])), float(np.float32(w["w_regSqrt"]))
    for y in range(H):
        for x in range(W):
            if not act[y, x]:
                continue
            c, s = np.cos(A[y, x]), np.sin(A[y, x])
            for k, (sx, sy) in enumerate(DIRS):
                tx, ty = x + sx, y + sy
                if not (0 <= tx < W and 0 <= ty < H) or not act[ty, tx]:
                    continue
                d = (U32[y, x] - U32[ty, tx]).astype(np.float64) if u_float_diff else U[y, x] - U[ty, tx]
                rot = np.array([c * d[0] - s * d[1], s * d[0] + c * d[1]])
                res[y, x, 2 * k:2 * k + 2] = wr * ((O[y, x] - O[ty, tx]) - rot)
            if C[y, x, 0] >= 0 and C[y, x, 1] >= 0:
                res[y, x, 8:10] = wf * (O[y, x] - C[y, x])
    return res.reshape(-1)


def small_problem(W=7, H=6, seed=3):
    rng = np.random.default_rng(seed)
    w = workloads.image_warping(W, H, seed=seed, n_handles=2, hole=False)
    M = w["Mask"].reshape(H, W)
    M[2, 3] = 255.0  # a hole
    M[4, 1] = 255.0
    w["Offset"] = (w["Offset"] + rng.normal(0, 0.3, w["Offset"].shape)).astype(np.float32)
    w["Angle"] = rng.normal(0, 0.4, w["Angle"].shape).astype(np.float32)
    w["UrShape"] = (w["UrShape"] + rng.normal(0, 0.1, w["UrShape"].shape)).astype(np.float32)
    C = w["Constraints"].reshape(H, W, 2)
    C[3, 3] = (3.5, 2.2)  # an interior handle
    return w


def unknown_vec(w):
    N = w["W"] * w["H"]
    return np.concatenate([w["Offset"].astype(np.float64), w["Angle"].astype(np.float64)]), N


def jacobian64(w, u_float_diff=False):
    x0, N = unknown_vec(w)
    n = x0.size
    res = lambda O, A: residuals64(w, O, A, u_float_diff)   # noqa: E731
    r0 = res(x0[:2 * N], x0[2 * N:])
    J = np.zeros((r0.size, n))
    h = 1e-6
    for j in range(n):
        xp, xm = x0.copy(), x0.copy()
        xp[j] += h
        xm[j] -= h
        J[:, j] = (res(xp[:2 * N], xp[2 * N:]) - res(xm[:2 * N], xm[2 * N:])) / (2 * h)
    return J, r0


def active_unknowns(w):
    N = w["W"] * w["H"]
    act = w["Mask"] == 0
    return np.concatenate([np.repeat(act, 2), act])


def test_residuals_and_cost():
    w = small_problem()
    x0, N = unknown_vec(w)
    r64 = residuals64(w, x0[:2 * N], x0[2 * N:])
    r32 = oracle.iw_residuals(w)
    np.testing.assert_allclose(r32, r64, rtol=1e-5, atol=2e-5)
    c = oracle.iw_cost(w)
    assert c == pytest.approx(0.5 * np.sum(r64 ** 2), rel=1e-5)


def test_jtf_and_preconditioner_match_fd_jacobian():
    w = small_problem()
    J, r0 = jacobian64(w)
    act = active_unknowns(w)
    g = J.T @ r0
    diag = np.sum(J * J, axis=0)
    r, pre, rz = oracle.iw_eval_jtf(w)
    scale = np.abs(g).max()
    np.testing.assert_allclose(r[act], -g[act], atol=2e-5 * scale)
    assert np.all(r[~act] == 0) and np.all(pre[~act] == 0)
    np.testing.assert_allclose(pre[act], 1.0 / (1.0 + np.sqrt(diag[act])) ** 2, rtol=2e-4)
    assert rz == pytest.approx(float(np.sum(r * pre * r)), rel=1e-5)


def test_apply_matches_fd_jacobian_and_is_spd():
    w = small_problem()
    J, _ = jacobian64(w)
    act = active_unknowns(w)
    rng = np.random.default_rng(7)
    p = rng.normal(size=J.shape[1]).astype(np.float32)
    q = rng.normal(size=J.shape[1]).astype(np.float32)
    p[~act] = 0
    q[~act] = 0
    Ap, pAp = oracle.iw_apply_jtj(w, p)
    Aq, _ = oracle.iw_apply_jtj(w, q)
    ref = J.T @ (J @ p.astype(np.float64))
    np.testing.assert_allclose(Ap[act], ref[act], atol=2e-4 * np.abs(ref).max())
    assert np.all(Ap[~act] == 0)
    assert pAp == pytest.approx(float(p.astype(np.float64) @ ref), rel=1e-4)
    assert pAp > 0
    assert float(q @ Ap) == pytest.approx(float(p @ Aq), rel=1e-4)


def test_gn_solve_decreases_cost_and_threads_agree():
    w = workloads.image_warping(40, 30, seed=11, n_handles=5)
    _, _, c1, _ = oracle.iw_solve(w, 3, 10, nthreads=1)
    O4, A4, c4, _ = oracle.iw_solve(w, 3, 10, nthreads=4)
    assert c1[0] > c1[1] > c1[2] > c1[3]
    np.testing.assert_allclose(c4, c1, rtol=1e-6)


def test_generic_gn_loop_equals_image_warping_loop():
    """The generic GN/LM loop (solver_impl.h) run as GN reproduces the image_warping
    specific PCG loop bit for bit (same float operations, same order)."""
    w = workloads.image_warping(40, 30, seed=5, n_handles=5)
    O1, A1, c1, _ = oracle.iw_solve(w, 3, 10)
    O2, A2, c2 = oracle.iw_solve_generic(w, 3, 10, lm=False)
    np.testing.assert_array_equal(c1, c2)
    np.testing.assert_array_equal(O1, O2)
    np.testing.assert_array_equal(A1, A2)


def test_model_cost_is_the_gauss_newton_quadratic():
    """m(d) = 1/2|F + J d|^2 = cost - r.d + 1/2 d.J^T J d (r = -J^T F), m(0) = cost."""
    w = small_problem()
    act = active_unknowns(w)
    rng = np.random.default_rng(5)
    d = (0.05 * rng.normal(size=act.size)).astype(np.float32)
    d[~act] = 0
    c = oracle.iw_cost(w)
    assert oracle.iw_model_cost(w, np.zeros_like(d)) == pytest.approx(c, rel=1e-6)
    r, dg = oracle.iw_jtf_diag(w)
    Ad, _ = oracle.iw_apply_jtj(w, d)
    quad = c - float(r.astype(np.float64) @ d) + 0.5 * float(d.astype(np.float64) @ Ad)
    assert oracle.iw_model_cost(w, d) == pytest.approx(quad, rel=1e-4)
    J, _ = jacobian64(w)
    np.testing.assert_allclose(dg[act], np.sum(J * J, axis=0)[act], rtol=2e-4)


def test_lm_solve_decreases_cost():
    w = workloads.image_warping(40, 30, seed=11, n_handles=5)
    _, _, c = oracle.iw_solve_generic(w, 5, 10, lm=True)
    assert len(c) >= 2 and np.all(np.diff(c) <= 0) and c[-1] < c[0]


def test_fp32_noise_floor_of_the_gn_trajectory():
    """The image_warping energy is evaluated as (O_k - O_t) - R(U_k - U_t) with O, U
    absolute pixel coordinates, so a 1-ulp change of Offset is a large relative change
    of the residuals; with lIterations = 10 the fp32 GN trajectory then moves at the
    1e-2 level. This is the floor below which no two fp32 implementations (nor the
    reference's own atomics-ordered runs) can agree; the GPU parity tests compare
    long-PCG trajectories against it (test_image_warping_gpu.py)."""
    w = workloads.image_warping(256, 192, seed=7, n_handles=6, max_move=0.1)
    _, _, c0, _ = oracle.iw_solve(w, 2, 10)
    rng = np.random.default_rng(0)
    w2 = dict(w)
    w2["Offset"] = (w["Offset"] * (1 + 2.0 ** -24 * rng.standard_normal(w["Offset"].size))).astype(np.float32)
    _, _, c1, _ = oracle.iw_solve(w2, 2, 10)
    drift = np.abs(c1 - c0) / c0
    assert drift[0] < 1e-6          # the energy itself barely moves
    assert drift[1] > 1e-3          # one GN step (10 PCG iterations) amplifies it
    _, _, s0, _ = oracle.iw_solve(w, 1, 2)
    _, _, s1, _ = oracle.iw_solve(w2, 1, 2)
    assert abs(s1[1] - s0[1]) / s0[1] < 1e-4   # one short-PCG step stays tight


# ---------------------------------------------------------------- opt_float = double
def test_double_oracle_matches_the_float64_restatement():
    """doublePrecision (Opt.h:11-14): the double instantiation of the same body
    (oracle/iw_impl.h) against the float64 restatement and its central-difference
    Jacobian at fp64 tolerances (the float form meets them only at 1e-5)."""
    w = small_problem()
    x0, N = unknown_vec(w)
    r64 = residuals64(w, x0[:2 * N], x0[2 * N:], u_float_diff=True)
    assert oracle.iw_cost(w, double=True) == pytest.approx(0.5 * np.sum(r64 ** 2), rel=1e-13)
    J, r0 = jacobian64(w, u_float_diff=True)
    act = active_unknowns(w)
    g = J.T @ r0
    r, pre, rz = oracle.iw_eval_jtf(w, double=True)
    assert r.dtype == np.float64
    np.testing.assert_allclose(r[act], -g[act], atol=1e-7 * np.abs(g).max())
    diag = np.sum(J * J, axis=0)
    np.testing.assert_allclose(pre[act], 1.0 / (1.0 + np.sqrt(diag[act])) ** 2, rtol=1e-7)
    assert rz == pytest.approx(float(np.sum(r * pre * r)), rel=1e-13)
    p = np.random.default_rng(7).normal(size=J.shape[1])
    p[~act] = 0
    Ap, pAp = oracle.iw_apply_jtj(w, p, double=True)
    ref = J.T @ (J @ p)
    np.testing.assert_allclose(Ap[act], ref[act], atol=1e-7 * np.abs(ref).max())
    assert np.all(Ap[~act] == 0)
    assert pAp == pytest.approx(float(p @ ref), rel=1e-8)
    # the double form of the GN-quadratic model cost and the raw diagonal
    d = 0.05 * np.random.default_rng(5).normal(size=act.size)
    d[~act] = 0
    rg, dg = oracle.iw_jtf_diag(w, double=True)
    Ad, _ = oracle.iw_apply_jtj(w, d, double=True)
    quad = oracle.iw_cost(w, double=True) - float(rg @ d) + 0.5 * float(d @ Ad)
    assert oracle.iw_model_cost(w, d, double=True) == pytest.approx(quad, rel=1e-12)
    np.testing.assert_allclose(dg[act], diag[act], rtol=1e-7)


def test_double_gn_loops_agree_and_track_the_float_loop():
    w = workloads.image_warping(40, 30, seed=5, n_handles=5)
    O1, A1, c1, _ = oracle.iw_solve(w, 3, 10, double=True)
    O2, A2, c2 = oracle.iw_solve_generic(w, 3, 10, lm=False, double=True)
    # the same double operations; only the dot products' summation order differs (pixel
    # order vs vector-layout order), which float's rounding of alpha / beta hides and
    # double's does not (a 1e-16 change moves this trajectory by ~1e-12)
    np.testing.assert_allclose(c2, c1, rtol=1e-10)
    np.testing.assert_allclose(O2, O1, rtol=0, atol=1e-10 * np.abs(O1).max())
    _, _, c4, _ = oracle.iw_solve(w, 3, 10, nthreads=4, double=True)
    np.testing.assert_allclose(c4, c1, rtol=1e-10)
    assert c1[0] > c1[1] > c1[2] > c1[3]
    # one short-PCG GN step: float and double agree to the float rounding of the inputs
    _, _, s32, _ = oracle.iw_solve(w, 1, 2)
    _, _, s64, _ = oracle.iw_solve(w, 1, 2, double=True)
    assert abs(s32[1] - s64[1]) / s64[1] < 1e-5
    _, _, cl = oracle.iw_solve_generic(w, 4, 10, lm=True, double=True)
    assert cl[-1] < cl[0]
