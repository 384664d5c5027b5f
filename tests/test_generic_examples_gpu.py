"""GPU: the reference's four example energies that have no hand-written family
(cotangent_mesh_smoothing, embedded_mesh_deformation, robust_nonrigid_alignment,
volumetric_mesh_deformation — energies/*.t lower to exactly the reference files'
residual templates, tests/test_generic_frontend.py) on kernels generated for them, on
small synthetic meshes / lattices, fp64:
* -J^T F from the generated kernels equals the central-difference gradient of the
  generated cost (which is 1/2 |F|^2, the reference's createcost);
* J^T J p from the matrix-free apply equals J^T (J p) with J assembled by the generated
  saveJToCRS kernels (two independent emissions of the same partials);
* GN and LM solves decrease the energy."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver
from opt_amd.harness import problems

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def E(name):
    return os.path.join(ROOT, "energies", name + ".t")


def cuda(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def mesh():
    v = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    f = np.array([[0, 2, 4], [2, 1, 4], [1, 3, 4], [3, 0, 4], [2, 0, 5], [1, 2, 5], [3, 1, 5], [0, 3, 5]], np.int32)
    P, _, F = problems.sqrt3_subdivide(v, f)
    return P.astype(np.float64), F


def directed_edges(F):
    und = problems.mesh_edges(F)
    d = np.array(und + [(b, a) for a, b in und], np.int32)
    return d[:, 0].copy(), d[:, 1].copy()


def cot_edges(F):
    opp = {}
    for a, b, c in F:
        for u, w, o in ((a, b, c), (b, c, a), (c, a, b)):
            opp.setdefault((min(u, w), max(u, w)), []).append(o)
    v0, v1, v2, v3 = [], [], [], []
    for (a, b), (c, d) in opp.items():
        for s, t in ((a, b), (b, a)):
            v0.append(s); v1.append(t); v2.append(c); v3.append(d)
    return [np.array(x, np.int32) for x in (v0, v1, v2, v3)]


def problem(name, rng):
    """(dims, params in declared-index order, unknown tensors in index order)"""
    if name == "volumetric_mesh_deformation":
        W, H, D = 4, 3, 3
        n = W * H * D
        zz, yy, xx = np.mgrid[0:D, 0:H, 0:W]
        U = np.stack([xx, yy, zz], -1).reshape(-1, 3).astype(np.float32)
        C = np.full((n, 3), -np.inf, np.float32)
        C[0] = U[0] + 0.3
        C[-1] = U[-1] - 0.2
        O = cuda(U.astype(np.float64) + 0.05 * rng.normal(size=U.shape))
        A = cuda(0.1 * rng.normal(size=(n, 3)))
        return [W, H, D], [O, A, cuda(U), cuda(C), 2.0, 1.0], [O, A]
    P, F = mesh()
    N = len(P)
    if name == "cotangent_mesh_smoothing":
        v = cot_edges(F)
        X = cuda(P + 0.05 * rng.normal(size=P.shape))
        return [N, len(v[0])], [1.0, 0.5, X, cuda(P.astype(np.float32)), None] + [cuda(e) for e in v], [X]
    v0, v1 = directed_edges(F)
    U = P.astype(np.float32)
    C = np.full((N, 3), -np.inf, np.float32)
    C[[0, 3, 7]] = U[[0, 3, 7]] + 0.2
    if name == "embedded_mesh_deformation":
        O = cuda(P + 0.05 * rng.normal(size=P.shape))
        R = cuda(np.tile(np.eye(3).reshape(1, 9), (N, 1)) + 0.05 * rng.normal(size=(N, 9)))
        return [N, len(v0)], [2.0, 1.0, 0.5, O, R, cuda(U), cuda(C), None, cuda(v0), cuda(v1)], [O, R]
    # robust_nonrigid_alignment
    nrm = rng.normal(size=(N, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    O = cuda(P + 0.05 * rng.normal(size=P.shape))
    A = cuda(0.1 * rng.normal(size=(N, 3)))
    Wt = cuda(np.full(N, 0.9) + 0.05 * rng.normal(size=N))
    return [N, len(v0)], [2.0, 1.0, O, A, Wt, cuda(U), cuda(C), cuda(nrm.astype(np.float32)), None,
                          cuda(v0), cuda(v1)], [O, A, Wt]


NAMES = ["cotangent_mesh_smoothing", "embedded_mesh_deformation", "robust_nonrigid_alignment",
         "volumetric_mesh_deformation"]


@pytest.mark.parametrize("name", NAMES)
def test_generated_gradient_matches_finite_differences_of_the_cost(name):
    import torch

    dims, prm, unk = problem(name, np.random.default_rng(5))
    s = OptSolver(dims, E(name), "gaussNewtonGPU", double_precision=True)
    assert s.family() == "generic"
    n = s.unknown_count()
    assert n == sum(u.numel() for u in unk)
    r = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre = torch.zeros_like(r)
    s.eval_jtf(prm, r, pre)
    g = np.zeros(n)
    h = 1e-6
    k = 0
    for u in unk:
        flat = u.view(-1)
        for i in range(flat.numel()):
            x0 = flat[i].item()
            flat[i] = x0 + h
            cp = s.eval_cost(prm)
            flat[i] = x0 - h
            cm = s.eval_cost(prm)
            flat[i] = x0
            g[k] = (cp - cm) / (2 * h)
            k += 1
    rr = r.cpu().numpy()
    assert np.abs(rr + g).max() <= 1e-5 * max(np.abs(g).max(), 1.0)


@pytest.mark.parametrize("name", NAMES)
def test_generated_apply_equals_assembled_jacobian(name):
    import torch
    import scipy.sparse as sp

    dims, prm, _ = problem(name, np.random.default_rng(6))
    s = OptSolver(dims, E(name), "gaussNewtonGPU", double_precision=True)
    n = s.unknown_count()
    p = np.random.default_rng(1).normal(size=n)
    Ap = torch.zeros(n, dtype=torch.float64, device="cuda")
    s.apply_jtj(prm, cuda(p), Ap)
    m = OptSolver(dims, E(name), "gaussNewtonGPU", double_precision=True, materialized=True)
    rows, nnz = m.jacobian_shape()
    rp = torch.empty(rows + 1, dtype=torch.int32, device="cuda")
    ci = torch.empty(nnz, dtype=torch.int32, device="cuda")
    v = torch.empty(nnz, dtype=torch.float64, device="cuda")
    m.eval_jacobian(prm, rp, ci, v)
    J = sp.csr_matrix((v.cpu().numpy(), ci.cpu().numpy(), rp.cpu().numpy()), shape=(rows, n))
    ref = J.T @ (J @ p)
    assert np.abs(Ap.cpu().numpy() - ref).max() <= 1e-10 * max(np.abs(ref).max(), 1.0)


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("kind", ["gaussNewtonGPU", "LMGPU"])
def test_generated_solves_decrease_the_energy(name, kind):
    dims, prm, _ = problem(name, np.random.default_rng(7))
    s = OptSolver(dims, E(name), kind, double_precision=True)
    s.set_solver_params({"nIterations": 4, "lIterations": 20})
    costs = s.profiled_solve(prm)
    assert costs[-1] < costs[0] and all(np.isfinite(costs))
