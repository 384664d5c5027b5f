"""GPU parity of the arap_mesh_deformation graph path (CSR gathers built from the edge
list, generic GN/LM driver) against the C oracle's edge-scatter restatement, through the
C ABI. BASELINE config 4 (1M-vertex grid mesh, fp32, GN) at full size."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver, workloads
from oracle import oracle
from tests.iw_helpers import ROOT, rel_err

pytestmark = pytest.mark.gpu
ENERGY = os.path.join(ROOT, "energies", "arap_mesh_deformation.t")


def params(w, host=False, double=False):
    dt = np.float64 if double else np.float32
    arrs = [w["Offset"].astype(dt).copy(), w["Angle"].astype(dt).copy(), w["UrShape"], w["Constraints"]]
    graph = [w["v0"], w["v1"]]
    if not host:
        import torch
        arrs = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]
        graph = [torch.from_numpy(g).cuda() for g in graph]
    return [w["w_fitSqrt"], w["w_regSqrt"]] + arrs + [None] + graph


def to_np(t):
    return t.detach().cpu().numpy() if hasattr(t, "detach") else t


def solver(w, kind="gaussNewtonGPU", **kw):
    return OptSolver([w["N"], w["E"]], ENERGY, kind, **kw)


def perturbed(nx, ny, seed):
    w = workloads.arap_grid(nx, ny, seed=seed)
    rng = np.random.default_rng(seed)
    w["Offset"] = (w["Offset"] + 0.02 * rng.normal(size=w["Offset"].size)).astype(np.float32)
    w["Angle"] = (w["Angle"] + 0.2 * rng.normal(size=w["Angle"].size)).astype(np.float32)
    return w


@pytest.mark.parametrize("nx,ny", [(7, 5), (40, 30), (3, 200)])
def test_kernels_match_oracle(nx, ny):
    import torch

    w = perturbed(nx, ny, seed=nx + ny)
    s = solver(w)
    assert s.family() == "arap_mesh_deformation"
    prm = params(w)
    assert s.eval_cost(prm) == pytest.approx(oracle.arap_cost(w), rel=1e-5)
    n = 6 * w["N"]
    r = torch.zeros(n, device="cuda")
    pre = torch.zeros(n, device="cuda")
    s.eval_jtf(prm, r, pre)
    r_ref, dg = oracle.arap_jtf(w)
    assert rel_err(to_np(r), r_ref) < 2e-5
    assert rel_err(to_np(pre), 1.0 / (1.0 + np.sqrt(dg)) ** 2) < 1e-5
    p = np.random.default_rng(4).normal(size=n).astype(np.float32)
    Ap = torch.zeros(n, device="cuda")
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.arap_apply(w, p)
    assert rel_err(to_np(Ap), Ap_ref) < 2e-5
    assert pAp == pytest.approx(pAp_ref, rel=2e-5)


@pytest.mark.parametrize("kind,nit,lit", [("gaussNewtonGPU", 4, 20), ("LMGPU", 6, 20), ("LMGPU", 3, 25)])
def test_solve_matches_oracle(kind, nit, lit):
    w = perturbed(40, 30, seed=8)
    s = solver(w, kind)
    prm = params(w)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    O_ref, A_ref, c_ref = oracle.arap_solve(w, nit, lit, lm=(kind == "LMGPU"))
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-4)
    assert rel_err(to_np(prm[2]), O_ref) < 1e-4
    assert np.abs(to_np(prm[3]) - A_ref).max() < 1e-3


def test_edge_order_does_not_matter():
    """A shuffled edge list gives the same CSR up to per-vertex order (tolerance only)."""
    w = perturbed(30, 20, seed=3)
    s = solver(w)
    prm = params(w)
    s.set_solver_params({"nIterations": 3, "lIterations": 10})
    c1 = s.profiled_solve(prm)
    perm = np.random.default_rng(0).permutation(w["E"])
    w2 = dict(w, v0=np.ascontiguousarray(w["v0"][perm]), v1=np.ascontiguousarray(w["v1"][perm]))
    s2 = solver(w2)
    prm2 = params(w2)
    s2.set_solver_params({"nIterations": 3, "lIterations": 10})
    c2 = s2.profiled_solve(prm2)
    np.testing.assert_allclose(c2, c1, rtol=1e-5)


def test_host_buffers_equal_device_path():
    w = perturbed(25, 20, seed=6)
    sd = solver(w, "LMGPU")
    pd = params(w)
    sd.set_solver_params({"nIterations": 4, "lIterations": 10})
    cd = sd.profiled_solve(pd)
    sh = solver(w, "LMGPU", backend="backend_cpu")
    ph = params(w, host=True)
    sh.set_solver_params({"nIterations": 4, "lIterations": 10})
    ch = sh.profiled_solve(ph)
    np.testing.assert_array_equal(cd, ch)
    np.testing.assert_array_equal(to_np(pd[2]), ph[2])


def test_config4_one_million_vertices():
    """BASELINE config 4: 1000x1000 grid mesh (1M vertices, ~6M directed edges), GN:
    energy trajectory vs the oracle, descent, bitwise determinism."""
    w = workloads.arap_grid(1000, 1000, seed=9)
    assert w["N"] == 1000000 and 5.9e6 < w["E"] < 6.1e6
    runs = []
    for _ in range(2):
        s = solver(w)
        prm = params(w)
        s.set_solver_params({"nIterations": 3, "lIterations": 10})
        runs.append((s.profiled_solve(prm), to_np(prm[2])))
        s.close()
    c = runs[0][0]
    assert c[-1] < c[0]
    np.testing.assert_array_equal(runs[1][0], c)
    np.testing.assert_array_equal(runs[1][1], runs[0][1])
    _, _, c_ref = oracle.arap_solve(w, 3, 10)
    np.testing.assert_allclose(c, c_ref, rtol=1e-4)


# ---- fp64 (doublePrecision = 1) against the double instantiation of the oracle
@pytest.mark.parametrize("nx,ny", [(7, 5), (40, 30)])
def test_fp64_kernels_match_fp64_oracle(nx, ny):
    import torch

    w = perturbed(nx, ny, seed=nx + ny)
    s = solver(w, double_precision=True)
    prm = params(w, double=True)
    assert s.eval_cost(prm) == pytest.approx(oracle.arap_cost(w, double=True), rel=1e-10)
    n = 6 * w["N"]
    r = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre = torch.zeros_like(r)
    s.eval_jtf(prm, r, pre)
    r_ref, dg = oracle.arap_jtf(w, double=True)
    assert rel_err(to_np(r), r_ref) < 1e-10
    assert rel_err(to_np(pre), 1.0 / (1.0 + np.sqrt(dg)) ** 2) < 1e-10
    p = np.random.default_rng(4).normal(size=n)
    Ap = torch.zeros(n, dtype=torch.float64, device="cuda")
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.arap_apply(w, p, double=True)
    assert rel_err(to_np(Ap), Ap_ref) < 1e-10
    assert pAp == pytest.approx(pAp_ref, rel=1e-10)


@pytest.mark.parametrize("kind,nit,lit", [("gaussNewtonGPU", 4, 20), ("LMGPU", 6, 20)])
def test_fp64_solve_matches_fp64_oracle(kind, nit, lit):
    w = perturbed(40, 30, seed=8)
    s = solver(w, kind, double_precision=True)
    prm = params(w, double=True)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    O_ref, A_ref, c_ref = oracle.arap_solve(w, nit, lit, lm=(kind == "LMGPU"), double=True)
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-8)
    assert rel_err(to_np(prm[2]), O_ref) < 1e-8
    assert rel_err(to_np(prm[3]), A_ref) < 1e-8


@pytest.mark.parametrize("kind,nit,lit", [("gaussNewtonGPU", 4, 20), ("LMGPU", 6, 20)])
def test_fp32_trajectory_within_the_fp32_noise_floor(kind, nit, lit):
    """The fp32 bars above (1e-4) measured: the fp32 GPU trajectory is no further from the
    fp64 oracle's than fp32 oracle runs on 1-ulp perturbed inputs (x2 + 1e-7)."""
    from tests.test_sfs_gpu import fp32_noise_floor

    w = perturbed(40, 30, seed=8)
    s = solver(w, kind)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = np.array(s.profiled_solve(params(w)))
    lm = kind == "LMGPU"
    c64, floor = fp32_noise_floor(lambda ww, double=False: oracle.arap_solve(ww, nit, lit, lm=lm, double=double)[2],
                                  w, "Offset")
    drift = np.abs(costs - c64) / c64
    assert np.all(drift <= 2 * floor + 1e-7), (drift, floor)


# ---- irregular graphs: hubs of up to 1000 edges, isolated vertices, one-way edges
def irregular(seed=13):
    rng = np.random.default_rng(seed)
    w = workloads.arap_grid(60, 50, seed=seed)
    N = w["N"]
    e0, e1 = list(w["v0"]), list(w["v1"])
    for hub, deg in ((17, 700), (63, 300), (64, 129), (2500, 1000)):
        nb = rng.choice(N, size=deg, replace=False)
        nb = nb[nb != hub]
        e0 += [hub] * len(nb) + list(nb[: deg // 3])
        e1 += list(nb) + [hub] * len(nb[: deg // 3])
    keep = np.array([not (a in (5, 6, 7) or b in (5, 6, 7)) for a, b in zip(e0, e1)])
    e0, e1 = np.array(e0)[keep], np.array(e1)[keep]
    perm = rng.permutation(len(e0))
    w["v0"] = np.ascontiguousarray(e0[perm].astype(np.int32))
    w["v1"] = np.ascontiguousarray(e1[perm].astype(np.int32))
    w["E"] = len(e0)
    w["Offset"] = (w["Offset"] + 0.02 * rng.normal(size=w["Offset"].size)).astype(np.float32)
    w["Angle"] = (w["Angle"] + 0.3 * rng.normal(size=w["Angle"].size)).astype(np.float32)
    return w


@pytest.mark.parametrize("double", [False, True])
def test_apply_on_irregular_graphs(double):
    import torch

    w = irregular()
    dt = torch.float64 if double else torch.float32
    n = 6 * w["N"]
    p = torch.from_numpy(np.random.default_rng(3).normal(size=n)).to(dt).cuda()
    s = solver(w, double_precision=double)
    prm = params(w, double=double)
    Ap = torch.zeros(n, dtype=dt, device="cuda")
    pAp = s.apply_jtj(prm, p, Ap)
    Ap_ref, pAp_ref = oracle.arap_apply(w, to_np(p), double=double)
    tol = 1e-10 if double else 2e-5
    assert rel_err(to_np(Ap), Ap_ref) < tol
    assert pAp == pytest.approx(pAp_ref, rel=tol)
    r = torch.zeros(n, dtype=dt, device="cuda")
    pre = torch.zeros_like(r)
    s.eval_jtf(prm, r, pre)
    r_ref, _ = oracle.arap_jtf(w, double=double)
    assert rel_err(to_np(r), r_ref) < (1e-10 if double else 5e-5)


@pytest.mark.parametrize("kind", ["gaussNewtonGPU", "LMGPU"])
@pytest.mark.parametrize("double", [False, True])
def test_fused_step3_is_bitwise_the_separate_passes(monkeypatch, kind, double):
    """PCGStep3 folded into the K pass of the next apply (arap_kdir<T, true>, the generic
    driver's HasFusedStep3 hook): the same expressions per element, so whole solves
    are bitwise those of step3_kernel + the whole apply."""
    w = perturbed(23, 17, seed=4)
    out = {}
    for f in ("1", "0"):
        monkeypatch.setenv("OPT_AMD_FUSE_STEP3", f)
        s = solver(w, kind, double_precision=double)
        prm = params(w, double=double)
        s.set_solver_params({"nIterations": 4, "lIterations": 10})
        out[f] = (s.profiled_solve(prm), to_np(prm[2]), to_np(prm[3]))
        s.close()
    assert out["1"][0] == out["0"][0]
    assert np.array_equal(out["1"][1], out["0"][1]) and np.array_equal(out["1"][2], out["0"][2])


@pytest.mark.parametrize("double", [False, True])
def test_merged_neighbour_list_matches_the_two_lists(monkeypatch, double):
    """arap_apply_merged (one list: out-neighbours flagged when they also send an edge
    here, then the unmatched in-neighbours) against the separate out / in lists, on the
    grid mesh (every neighbour both ways) and on irregular hub graphs (one-way edges,
    duplicates): the same terms in another in-edge order, so J^T J p agrees to rounding
    and the solves to the fp32 noise floor (fp64: 1e-12)."""
    import torch

    for w in (perturbed(31, 19, seed=6), irregular(seed=21)):
        out = {}
        for m in ("1", "0"):
            monkeypatch.setenv("OPT_AMD_ARAP_MERGED", m)
            s = solver(w, double_precision=double)
            prm = params(w, double=double)
            n = s.unknown_count()
            dt = torch.float64 if double else torch.float32
            p = torch.from_numpy(np.random.default_rng(5).normal(size=n)).to(dt).cuda()
            Ap = torch.zeros_like(p)
            pAp = s.apply_jtj(prm, p, Ap)
            s.set_solver_params({"nIterations": 3, "lIterations": 10})
            out[m] = (to_np(Ap), pAp, s.profiled_solve(params(w, double=double)))
            s.close()
        assert rel_err(out["1"][0], out["0"][0]) < (1e-13 if double else 1e-5)
        assert out["1"][1] == pytest.approx(out["0"][1], rel=1e-12 if double else 1e-5)
        np.testing.assert_allclose(out["1"][2], out["0"][2], rtol=1e-12 if double else 1e-4)


def test_graph_without_edges_and_isolated_vertices():
    """Edge cases of the adjacency build (CSR, sliced ELL, merged list): a graph with no
    edges at all (only the fit term: J^T J p = w_fit^2 p on constrained vertices), and a
    vertex count that is not a multiple of the 64-vertex slice with isolated vertices;
    the apply against the oracle, whole solves against the oracle's trajectory."""
    import torch

    w = perturbed(9, 7, seed=3)          # 63 vertices
    N = w["N"]
    for keep in (0, len(w["v0"]) // 3):
        w2 = dict(w)
        w2["v0"] = np.ascontiguousarray(w["v0"][:keep])
        w2["v1"] = np.ascontiguousarray(w["v1"][:keep])
        w2["E"] = keep
        s = solver(w2)
        prm = params(w2)
        p = torch.from_numpy(np.random.default_rng(1).normal(size=6 * N).astype(np.float32)).cuda()
        Ap = torch.zeros_like(p)
        pAp = s.apply_jtj(prm, p, Ap)
        Ap_ref, pAp_ref = oracle.arap_apply(w2, to_np(p))
        assert rel_err(to_np(Ap), Ap_ref) < 2e-5
        assert pAp == pytest.approx(pAp_ref, rel=1e-5, abs=1e-12)
        if keep == 0:
            fit = np.repeat(w["Constraints"].reshape(-1, 3)[:, 0] >= -999999.9, 3)
            expect = np.concatenate([np.where(fit, w["w_fitSqrt"] ** 2 * to_np(p)[:3 * N], 0.0), np.zeros(3 * N)])
            np.testing.assert_allclose(to_np(Ap), expect, rtol=1e-6, atol=1e-7)
        # with no edges the system is diagonal: one PCG iteration solves it, after which the
        # reference's unguarded alpha = rz / pAp (solverGPUGaussNewton.t:696) is 0/0 or
        # rounding noise depending on whether r came out exactly 0 — so that case takes one
        # GN step of one PCG iteration
        nit, lit = (1, 1) if keep == 0 else (2, 5)
        s.set_solver_params({"nIterations": nit, "lIterations": lit})
        costs = s.profiled_solve(params(w2))
        ref = oracle.arap_solve(w2, nit, lit)[2]
        assert len(costs) == len(ref)
        np.testing.assert_allclose(costs, ref, rtol=1e-4, atol=1e-8 * ref[0])
        s.close()


@pytest.mark.parametrize("double", [False, True])
def test_merged_batch_size_is_bitwise(monkeypatch, double):
    """arap_apply_merged with 2 or 3 merged slots per load batch (OPT_AMD_ARAP_EB; the ELL
    widths padded to it): the slots are summed in the same order either way, padding slots
    add exact zeros, so whole GN solves are bitwise equal."""
    w = perturbed(23, 17, seed=6)
    out = {}
    for eb in ("2", "3"):
        monkeypatch.setenv("OPT_AMD_ARAP_EB", eb)
        s = solver(w, "gaussNewtonGPU", double_precision=double)
        prm = params(w, double=double)
        s.set_solver_params({"nIterations": 3, "lIterations": 10})
        out[eb] = (s.profiled_solve(prm), to_np(prm[2]), to_np(prm[3]))
        s.close()
    assert out["2"][0] == out["3"][0]
    assert np.array_equal(out["2"][1], out["3"][1]) and np.array_equal(out["2"][2], out["3"][2])


def test_adjacency_over_the_index_range_is_an_error_not_an_exit():
    """a mesh whose sliced-ELL adjacency needs >= 2^31 slots (here 34,000 64-vertex
    slices, each holding one vertex with 1,100 out-edges: 64 x 34,000 x 1,100 = 2.39e9 slots)
    is refused when the edges are bound — through the plan's error path (optamd::PlanError:
    Init stops, Step returns 0, OptAMD_PlanError holds the message, the wrapper raises) —
    and the process goes on: a normal solve runs afterwards in the same process."""
    from opt_amd.api import OptError

    ns, deg = 34000, 1100
    N, E = 64 * ns, ns * deg
    rng = np.random.default_rng(5)
    P = rng.uniform(0, 1, 3 * N).astype(np.float32)
    C = np.full(3 * N, -np.inf, np.float32)
    v0 = np.repeat(np.arange(ns, dtype=np.int32) * 64, deg)
    v1 = rng.integers(0, N, E, dtype=np.int32)
    w = {"Offset": P, "Angle": np.zeros(3 * N, np.float32), "UrShape": P, "Constraints": C, "v0": v0, "v1": v1,
         "N": N, "E": E, "w_fitSqrt": 2.0, "w_regSqrt": 1.0}
    s = solver(w)
    s.set_solver_params({"nIterations": 1, "lIterations": 1})
    with pytest.raises(OptError, match="adjacency too large"):
        s.init(params(w))
    assert np.isnan(s.cost())
    with pytest.raises(OptError, match="adjacency too large"):   # Step returns 0; the wrapper raises
        s.step()
    s.close()
    # the extension entry points bind too (StencilPlan::prepare -> build_csr);
    # the PlanError is caught at the C boundary there as well (no std::terminate through the
    # extern "C" frame), on a fresh plan whose first call is the extension
    import torch

    for call in ("eval_cost", "eval_jtf", "apply_jtj"):
        s = solver(w)
        prm = params(w)
        x = torch.zeros(6 * N, dtype=torch.float32, device="cuda")
        y = torch.zeros_like(x)
        with pytest.raises(OptError, match="adjacency too large"):
            if call == "eval_cost":
                s.eval_cost(prm)
            elif call == "eval_jtf":
                s.eval_jtf(prm, x, y)
            else:
                s.apply_jtj(prm, x, y)
        s.close()
    del w, v0, v1, P, C
    w2 = perturbed(7, 5, seed=3)
    s2 = solver(w2)
    s2.set_solver_params({"nIterations": 2, "lIterations": 10})
    c = s2.profiled_solve(params(w2))
    assert np.isfinite(c).all() and c[-1] < c[0]
