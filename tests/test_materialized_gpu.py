"""GPU: the materialized-Jacobian path (useMaterializedJTJ / useFusedJTJ) through the
C ABI — the device CSR kernels on the reference's known-answer vectors
(API/src/linalg_cpu_test.t:49-176) and against the CSR oracle, the families' J
assembly against the oracle's, and whole solves against the oracle's materialized
solver and the matrix-free path."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver, api, workloads
from oracle import oracle
from tests.iw_helpers import ENERGY, device_params, perturbed, rel_err
from tests.test_oracle_csr import (KAT_AT_COLIND, KAT_AT_ROWPTR, KAT_AT_VAL, KAT_ATA_COLIND, KAT_ATA_ROWPTR,
                                   KAT_ATA_VAL, KAT_COLIND, KAT_ROWPTR, KAT_VAL, KAT_X, KAT_Y, random_csr)

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PIE = os.path.join(ROOT, "energies", "poisson_image_editing.t")


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_known_answer_vectors():
    rp, ci, v = dev(KAT_ROWPTR), dev(KAT_COLIND), dev(KAT_VAL)
    rpT, ciT, vT = api.csr_transpose(3, 4, rp, ci, v)
    assert rpT.cpu().tolist() == KAT_AT_ROWPTR
    assert ciT.cpu().tolist() == KAT_AT_COLIND
    assert vT.cpu().tolist() == KAT_AT_VAL
    assert api.csr_spmv(3, 4, rp, ci, v, dev(KAT_X)).cpu().tolist() == KAT_Y
    rpA, ciA, vA = api.csr_ata(3, 4, rp, ci, v)
    assert rpA.cpu().tolist() == KAT_ATA_ROWPTR
    assert ciA.cpu().tolist() == KAT_ATA_COLIND
    assert vA.cpu().tolist() == KAT_ATA_VAL


@pytest.mark.parametrize("shape", [(1, 1, 1), (257, 100, 7), (5000, 3000, 12), (2000, 70000, 3)])
def test_csr_kernels_match_oracle(shape):
    rows, cols, per = shape
    rp, ci, v = random_csr(rows, cols, per, seed=cols)
    rpT, ciT, vT = oracle.csr_transpose(rows, cols, rp, ci, v)
    g = api.csr_transpose(rows, cols, dev(rp), dev(ci), dev(v))
    np.testing.assert_array_equal(g[0].cpu().numpy(), rpT)
    np.testing.assert_array_equal(g[1].cpu().numpy(), ciT)
    np.testing.assert_array_equal(g[2].cpu().numpy(), vT)
    rpA, ciA, vA = oracle.csr_ata(rows, cols, rp, ci, v)
    ga = api.csr_ata(rows, cols, dev(rp), dev(ci), dev(v))
    np.testing.assert_array_equal(ga[0].cpu().numpy(), rpA)
    np.testing.assert_array_equal(ga[1].cpu().numpy(), ciA)
    # same products and the same summation order (rows of A ascending), no contraction
    np.testing.assert_array_equal(ga[2].cpu().numpy(), vA)
    x = np.random.default_rng(2).normal(size=cols).astype(np.float32)
    y = api.csr_spmv(rows, cols, dev(rp), dev(ci), dev(v), dev(x)).cpu().numpy()
    # entries summed in order with rounded products: bitwise applyAtoVector
    np.testing.assert_array_equal(y, oracle.csr_spmv(rows, cols, rp, ci, v, x))


def test_csr_fp64():
    import torch

    rp, ci, v = random_csr(600, 400, 8, seed=9)
    vd = v.astype(np.float64)
    x = np.random.default_rng(4).normal(size=400)
    y = api.csr_spmv(600, 400, dev(rp), dev(ci), dev(vd), dev(x)).cpu().numpy()
    A = np.zeros((600, 400))
    for r in range(600):
        A[r, ci[rp[r]:rp[r + 1]]] = vd[rp[r]:rp[r + 1]]
    np.testing.assert_allclose(y, A @ x, rtol=1e-12, atol=1e-12)
    rpA, ciA, vA = api.csr_ata(600, 400, dev(rp), dev(ci), dev(vd))
    assert vA.dtype == torch.float64
    D = np.zeros((400, 400))
    rpA, ciA, vA = rpA.cpu().numpy(), ciA.cpu().numpy(), vA.cpu().numpy()
    for r in range(400):
        D[r, ciA[rpA[r]:rpA[r + 1]]] = vA[rpA[r]:rpA[r + 1]]
    np.testing.assert_allclose(D, A.T @ A, rtol=1e-12, atol=1e-12)


def iw_solver(W, H, fused, kind="gaussNewtonGPU", materialized=True):
    return OptSolver([W, H], ENERGY, kind, materialized=materialized, fused_jtj=fused)


@pytest.mark.parametrize("W,H", [(9, 7), (67, 45)])
def test_iw_jacobian_matches_oracle(W, H):
    import torch

    w = perturbed(W, H, seed=H)
    s = iw_solver(W, H, fused=True)
    rows, nnz = s.jacobian_shape()
    assert (rows, nnz) == (10 * W * H, 26 * W * H)
    rp = torch.empty(rows + 1, dtype=torch.int32, device="cuda")
    ci = torch.empty(nnz, dtype=torch.int32, device="cuda")
    v = torch.empty(nnz, dtype=torch.float32, device="cuda")
    s.eval_jacobian(device_params(w), rp, ci, v)
    orp, oci, ov = oracle.iw_dump_j(w)
    np.testing.assert_array_equal(rp.cpu().numpy(), orp)
    np.testing.assert_array_equal(ci.cpu().numpy(), oci)
    # angle partials go through sin/cos: a few ulp apart
    np.testing.assert_allclose(v.cpu().numpy(), ov, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fused", [True, False])
def test_iw_materialized_apply_equals_matrix_free(fused):
    import torch

    W, H = 80, 61
    w = perturbed(W, H, seed=11)
    prm = device_params(w)
    act = np.repeat(w["Mask"] == 0, 1)
    act3 = np.concatenate([np.repeat(act, 2), act])
    p = (np.random.default_rng(5).normal(size=3 * W * H) * act3).astype(np.float32)
    mat = iw_solver(W, H, fused)
    Ap = torch.zeros(3 * W * H, device="cuda")
    pAp = mat.apply_jtj(prm, dev(p), Ap)
    ref, ref_pAp = oracle.iw_apply_materialized(w, p, fused=fused)
    assert rel_err(Ap.cpu().numpy(), ref) < 1e-5
    assert abs(pAp - ref_pAp) < 1e-5 * abs(ref_pAp)
    free = OptSolver([W, H], ENERGY, "LMGPU")   # generic driver, matrix-free
    Ap2 = torch.zeros(3 * W * H, device="cuda")
    free.apply_jtj(prm, dev(p), Ap2)
    assert rel_err(Ap.cpu().numpy(), Ap2.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("kind", ["gaussNewtonGPU", "LMGPU"])
def test_iw_materialized_solve_matches_oracle(fused, kind):
    W, H = 48, 40
    w = perturbed(W, H, seed=3)
    s = iw_solver(W, H, fused, kind=kind)
    s.set_solver_params({"nIterations": 3, "lIterations": 4})
    costs = s.profiled_solve(device_params(w))
    lm = kind == "LMGPU"
    _, _, ref = oracle.iw_solve_materialized(w, 3, 4, lm=lm, fused=fused)
    np.testing.assert_allclose(costs, ref, rtol=1e-5)
    assert costs[-1] < costs[0]
    assert "J^TJp" in s.apply_kernel_name() or "J^T" in s.apply_kernel_name()


@pytest.mark.parametrize("fused", [True, False])
def test_pie_materialized_solve_matches_oracle(fused):
    import torch

    W, H = 64, 48
    w = workloads.poisson_image_editing(W, H, seed=2)
    s = OptSolver([W, H], PIE, "gaussNewtonGPU", materialized=True, fused_jtj=fused)
    rows, nnz = s.jacobian_shape()
    assert (rows, nnz) == (16 * W * H, 32 * W * H)
    X = torch.from_numpy(w["X"].copy()).cuda()
    prm = [X, dev(w["T"]), dev(w["M"])]
    s.set_solver_params({"nIterations": 1, "lIterations": 10})
    costs = s.profiled_solve(prm)
    Xr, ref = oracle.pie_solve_materialized(w, 1, 10, fused=fused)
    np.testing.assert_allclose(costs, ref, rtol=1e-5)
    assert rel_err(X.cpu().numpy(), Xr) < 1e-5


def test_families_without_assembly_use_the_generated_kernels():
    """shape_from_shading's hand-written family has no J assembly: a materialized plan of
    that energy runs on the generated kernels (generic.hip), which assemble any energy."""
    s = OptSolver([32, 32], os.path.join(ROOT, "energies", "shape_from_shading.t"), "LMGPU", materialized=True)
    assert s.family() == "generic"


@pytest.mark.parametrize("fused", [True, False])
def test_pie_materialized_apply_is_bitwise_the_oracle(fused):
    """J of this energy is exact (+-1 entries), so J^T, J^T J (reference summation order)
    and the SELL-64 SpMV (row order, rounded products) reproduce the CPU restatement of
    the reference's CSR path bit for bit."""
    import torch

    W, H = 70, 37
    w = workloads.poisson_image_editing(W, H, seed=8)
    act4 = np.repeat(w["M"] == 0, 4)
    p = (np.random.default_rng(1).normal(size=4 * W * H) * act4).astype(np.float32)
    s = OptSolver([W, H], PIE, "gaussNewtonGPU", materialized=True, fused_jtj=fused)
    Ap = torch.zeros(4 * W * H, device="cuda")
    s.apply_jtj([dev(w["X"]), dev(w["T"]), dev(w["M"])], dev(p), Ap)
    ref, _ = oracle.pie_apply_materialized(w, p, fused=fused)
    np.testing.assert_array_equal(Ap.cpu().numpy(), ref)
