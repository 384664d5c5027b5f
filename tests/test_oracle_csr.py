"""CPU: the CSR restatement (oracle/csr.c) against the reference's own known-answer
test, and the materialized-Jacobian oracle against the matrix-free one.

Golden vectors: API/src/linalg_cpu_test.t:49-176 (a 3x4 matrix A, its transpose, A x
for x = (3, 5, 7, 9) and A^T A), the only numeric fixture the reference holds for
its sparse path."""
import numpy as np
import pytest

from opt_amd import workloads
from oracle import oracle
from tests.iw_helpers import perturbed, rel_err

# linalg_cpu_test.t:49-80
KAT_ROWPTR = np.array([0, 3, 5, 7], np.int32)
KAT_COLIND = np.array([0, 2, 3, 1, 3, 0, 2], np.int32)
KAT_VAL = np.array([1, 3, 4, 9, 2, 7, 8], np.float32)
KAT_X = np.array([3, 5, 7, 9], np.float32)
# linalg_cpu_test.t:95-118
KAT_AT_ROWPTR = [0, 2, 3, 5, 7]
KAT_AT_COLIND = [0, 2, 1, 0, 2, 0, 1]
KAT_AT_VAL = [1, 7, 9, 3, 8, 4, 2]
KAT_Y = [60, 63, 77]
# linalg_cpu_test.t:147-172
KAT_ATA_ROWPTR = [0, 3, 5, 8, 12]
KAT_ATA_COLIND = [0, 2, 3, 1, 3, 0, 2, 3, 0, 1, 2, 3]
KAT_ATA_VAL = [50, 59, 4, 81, 18, 59, 73, 12, 4, 18, 12, 20]


def test_transpose_known_answer():
    rp, ci, v = oracle.csr_transpose(3, 4, KAT_ROWPTR, KAT_COLIND, KAT_VAL)
    assert rp.tolist() == KAT_AT_ROWPTR
    assert ci.tolist() == KAT_AT_COLIND
    assert v.tolist() == KAT_AT_VAL


def test_spmv_known_answer():
    assert oracle.csr_spmv(3, 4, KAT_ROWPTR, KAT_COLIND, KAT_VAL, KAT_X).tolist() == KAT_Y


def test_ata_known_answer():
    rp, ci, v = oracle.csr_ata(3, 4, KAT_ROWPTR, KAT_COLIND, KAT_VAL)
    assert rp.tolist() == KAT_ATA_ROWPTR
    assert ci.tolist() == KAT_ATA_COLIND
    assert v.tolist() == KAT_ATA_VAL


def random_csr(rows, cols, per_row, seed):
    rng = np.random.default_rng(seed)
    rp = [0]
    ci = []
    for _ in range(rows):
        k = int(rng.integers(0, per_row + 1))
        ci += sorted(rng.choice(cols, size=min(k, cols), replace=False).tolist())
        rp.append(len(ci))
    return (np.array(rp, np.int32), np.array(ci, np.int32),
            rng.normal(size=len(ci)).astype(np.float32))


def dense(rows, cols, rp, ci, v):
    A = np.zeros((rows, cols))
    for r in range(rows):
        for k in range(rp[r], rp[r + 1]):
            A[r, ci[k]] += v[k]
    return A


@pytest.mark.parametrize("shape", [(1, 1, 1), (40, 17, 5), (300, 200, 9), (50, 400, 3)])
def test_random_matrices_match_dense_algebra(shape):
    rows, cols, per = shape
    rp, ci, v = random_csr(rows, cols, per, seed=rows)
    A = dense(rows, cols, rp, ci, v)
    rpT, ciT, vT = oracle.csr_transpose(rows, cols, rp, ci, v)
    np.testing.assert_array_equal(dense(cols, rows, rpT, ciT, vT), A.T)
    for r in range(cols):   # rows of A ascending inside every row of A^T
        assert np.all(np.diff(ciT[rpT[r]:rpT[r + 1]]) > 0)
    x = np.random.default_rng(1).normal(size=cols).astype(np.float32)
    np.testing.assert_allclose(oracle.csr_spmv(rows, cols, rp, ci, v, x), A @ x, rtol=1e-5, atol=1e-5)
    rpA, ciA, vA = oracle.csr_ata(rows, cols, rp, ci, v)
    np.testing.assert_allclose(dense(cols, cols, rpA, ciA, vA), A.T @ A, rtol=1e-5, atol=1e-5)
    # the pattern is the structural one: every stored entry, zeros included
    S = dense(rows, cols, rp, ci, np.ones_like(v)) != 0
    np.testing.assert_array_equal(dense(cols, cols, rpA, ciA, np.ones_like(vA)) != 0, (S.T.astype(int) @ S) > 0)


# ---------------------------------------------------------------- image_warping
@pytest.mark.parametrize("W,H", [(9, 7), (33, 20)])
def test_iw_jacobian_reproduces_matrix_free_operators(W, H):
    w = perturbed(W, H, seed=W)
    N = W * H
    rp, ci, v = oracle.iw_dump_j(w)
    assert rp[-1] == 26 * N and np.all(np.diff(rp) >= 0)
    for r in range(10 * N):
        assert np.all(np.diff(ci[rp[r]:rp[r + 1]]) > 0)   # sortCol
    assert ci.min() >= 0 and ci.max() < 3 * N              # wrap()
    J = dense(10 * N, 3 * N, rp, ci, v)
    act = np.repeat(w["Mask"] == 0, 1)
    act3 = np.concatenate([np.repeat(act, 2), act])
    # J^T F = -r on the active unknowns (evalJTF, o.t:2870-2913)
    F = oracle.iw_residuals(w).astype(np.float64)
    r, dg = oracle.iw_jtf_diag(w)
    np.testing.assert_allclose((J.T @ F)[act3], -r[act3], rtol=2e-4, atol=2e-4 * np.abs(r).max())
    np.testing.assert_allclose((J * J).sum(0)[act3], dg[act3], rtol=1e-4, atol=1e-6)
    # J^T J p = the matrix-free apply (applyJTJ, o.t:2770-2830), p zero off the solve
    p = np.random.default_rng(3).normal(size=3 * N).astype(np.float32) * act3
    Ap_free, _ = oracle.iw_apply_jtj(w, p)
    for fused in (True, False):
        Ap, pAp = oracle.iw_apply_materialized(w, p, fused=fused)
        assert np.all(Ap[~act3] == 0)
        assert rel_err(Ap[act3], Ap_free[act3]) < 1e-5
        assert abs(pAp - float(p @ Ap)) < 1e-6 * abs(pAp) + 1e-9


def test_iw_materialized_solve_tracks_matrix_free():
    w = perturbed(24, 18, seed=2)
    _, _, free = oracle.iw_solve_generic(w, 3, 4)
    for fused in (True, False):
        _, _, mat = oracle.iw_solve_materialized(w, 3, 4, fused=fused)
        np.testing.assert_allclose(mat, free, rtol=1e-4)
        assert mat[-1] < mat[0]


# ---------------------------------------------------------------- poisson
def test_pie_jacobian_reproduces_matrix_free_operators():
    w = workloads.poisson_image_editing(12, 9, seed=4)
    N = 12 * 9
    rp, ci, v = oracle.pie_dump_j(w)
    J = dense(16 * N, 4 * N, rp, ci, v)
    act4 = np.repeat(w["M"] == 0, 4)
    r, dg = oracle.pie_jtf(w)
    # J^T F = -r on the active unknowns; F = the 16 residuals of every pixel
    X = w["X"].reshape(9, 12, 4).astype(np.float64)
    T = w["T"].reshape(9, 12, 4).astype(np.float64)
    F = np.zeros((9, 12, 4, 4))
    for s, (dx, dy) in enumerate([(1, 0), (-1, 0), (0, 1), (0, -1)]):
        for y in range(9):
            for x in range(12):
                if 0 <= x + dx < 12 and 0 <= y + dy < 9:
                    F[y, x, s] = (X[y, x] - X[y + dy, x + dx]) - (T[y, x] - T[y + dy, x + dx])
    np.testing.assert_allclose((J.T @ F.reshape(-1))[act4], -r[act4], rtol=1e-4, atol=1e-4)
    p = np.random.default_rng(0).normal(size=4 * N).astype(np.float32) * act4
    Ap_free, _ = oracle.pie_apply(w, p)
    np.testing.assert_allclose((J.T @ (J @ p))[act4], Ap_free[act4], rtol=1e-5, atol=1e-5)


def test_pie_materialized_solve_tracks_matrix_free():
    w = workloads.poisson_image_editing(20, 16, seed=1)
    _, free = oracle.pie_solve(w, 1, 10)
    for fused in (True, False):
        _, mat = oracle.pie_solve_materialized(w, 1, 10, fused=fused)
        np.testing.assert_allclose(mat, free, rtol=1e-4)
