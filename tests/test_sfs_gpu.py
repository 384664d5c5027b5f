"""GPU parity of the shape_from_shading path (generic GN/LM driver + sfs_* kernels:
ComputedArray precompute with gradient images, radius-2 gathers) against the C oracle,
through the C ABI, on synthetic inputs and on the reference's own example inputs
(tests/golden/sfs_default.npz, 640x480). BASELINE config 3 (4096^2, LM) at full size
through size-independent properties (LM monotonicity, determinism)."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver, workloads
from oracle import oracle
from tests.iw_helpers import ROOT, rel_err

pytestmark = pytest.mark.gpu
ENERGY = os.path.join(ROOT, "energies", "shape_from_shading.t")
GOLDEN = os.path.join(ROOT, "tests", "golden", "sfs_default.npz")


def params(w, host=False):
    scal = [float(v) for v in w["params"]]
    arrs = [w["X"].copy(), w["D_i"], w["Im"], w["edgeMaskR"], w["edgeMaskC"]]
    if host:
        return scal + arrs
    import torch
    return scal + [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def to_np(t):
    return t.detach().cpu().numpy() if hasattr(t, "detach") else t


def synthetic(W, H, seed):
    w = workloads.shape_from_shading(W, H, seed=seed, valid_frac=0.7)
    rng = np.random.default_rng(seed)
    w["edgeMaskR"] = (rng.uniform(size=W * H) < 0.9).astype(np.uint8)
    w["edgeMaskC"] = (rng.uniform(size=W * H) < 0.9).astype(np.uint8)
    return w


def reference_inputs(crop=None):
    z = np.load(GOLDEN)
    H, W = z["D_i"].shape
    sl = crop or (slice(0, H), slice(0, W))
    w = {"params": z["params"]}
    for k in ("D_i", "Im", "edgeMaskR", "edgeMaskC"):
        w[k] = np.ascontiguousarray(z[k][sl]).reshape(-1)
    X = np.ascontiguousarray(z["X0"][sl])
    w["H"], w["W"] = X.shape
    w["X"] = X.reshape(-1)
    return w


@pytest.mark.parametrize("W,H", [(64, 48), (97, 61), (130, 9), (5, 40)])
def test_kernels_match_oracle(W, H):
    import torch

    w = synthetic(W, H, seed=W + H)
    s = OptSolver([W, H], ENERGY, "LMGPU")
    assert s.family() == "shape_from_shading"
    prm = params(w)
    assert s.eval_cost(prm) == pytest.approx(oracle.sfs_cost(w), rel=2e-5)
    n = W * H
    r = torch.zeros(n, device="cuda")
    pre = torch.zeros(n, device="cuda")
    s.eval_jtf(prm, r, pre)
    r_ref, _ = oracle.sfs_jtf(w)
    assert rel_err(to_np(r), r_ref) < 5e-5
    act = w["D_i"] > 0
    assert np.all(to_np(pre)[act] == 0.25) and np.all(to_np(pre)[~act] == 0)
    p = np.random.default_rng(3).normal(size=n).astype(np.float32)
    p[~act] = 0
    Ap = torch.zeros(n, device="cuda")
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.sfs_apply(w, p)
    assert rel_err(to_np(Ap), Ap_ref) < 5e-5
    assert pAp == pytest.approx(pAp_ref, rel=5e-5)


@pytest.mark.parametrize("kind,nit,lit", [("gaussNewtonGPU", 3, 10), ("LMGPU", 6, 10), ("LMGPU", 3, 25)])
def test_solve_matches_oracle_synthetic(kind, nit, lit):
    W, H = 96, 72
    w = synthetic(W, H, seed=12)
    s = OptSolver([W, H], ENERGY, kind)
    prm = params(w)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    X_ref, c_ref = oracle.sfs_solve(w, nit, lit, lm=(kind == "LMGPU"))
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-4)
    assert rel_err(to_np(prm[16]), X_ref) < 1e-4


def test_solve_matches_oracle_reference_inputs():
    """The reference's own example (examples/data/shape_from_shading/default*), 640x480,
    LM, the harness's X0 = initialUnknown."""
    w = reference_inputs()
    s = OptSolver([w["W"], w["H"]], ENERGY, "LMGPU")
    prm = params(w)
    s.set_solver_params({"nIterations": 5, "lIterations": 10})
    costs = s.profiled_solve(prm)
    X_ref, c_ref = oracle.sfs_solve(w, 5, 10, lm=True)
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-4)
    act = w["D_i"] > 0
    # the GPU gathers are re-associated (sfs.hip: J^T J p as a chain of 3-point stencils),
    # so fp32 rounding differs from the oracle's per-residual gather; five LM steps on
    # this ill-conditioned real-data problem amplify that to ~1e-4 in the depths
    assert rel_err(to_np(prm[16])[act], X_ref[act]) < 3e-4
    assert costs[-1] < costs[0]


def test_host_buffers_equal_device_path():
    w = reference_inputs((slice(120, 220), slice(250, 400)))
    W, H = w["W"], w["H"]
    sd = OptSolver([W, H], ENERGY, "LMGPU")
    pd = params(w)
    sd.set_solver_params({"nIterations": 4, "lIterations": 10})
    cd = sd.profiled_solve(pd)
    sh = OptSolver([W, H], ENERGY, "LMGPU", backend="backend_cpu")
    ph = params(w, host=True)
    sh.set_solver_params({"nIterations": 4, "lIterations": 10})
    ch = sh.profiled_solve(ph)
    np.testing.assert_array_equal(cd, ch)
    np.testing.assert_array_equal(to_np(pd[16]), ph[16])


def test_config3_full_size_properties():
    """BASELINE config 3 (4096^2, LM): monotone LM energy, descent, bitwise determinism."""
    W = H = 4096
    w = workloads.shape_from_shading(W, H, seed=3)
    runs = []
    for _ in range(2):
        s = OptSolver([W, H], ENERGY, "LMGPU")
        prm = params(w)
        s.set_solver_params({"nIterations": 4, "lIterations": 10})
        runs.append((s.profiled_solve(prm), to_np(prm[16])))
        s.close()
    c, X = runs[0]
    assert np.all(np.diff(c) <= 0) and c[-1] < c[0]
    np.testing.assert_array_equal(runs[1][0], c)
    np.testing.assert_array_equal(runs[1][1], X)


# ---- fp64 (doublePrecision = 1): unknowns and solver vectors in double, known arrays
# float, against the double instantiation of the same oracle (oracle/sfs_impl.h)
def params64(w):
    import torch
    scal = [float(v) for v in w["params"]]
    arrs = [w["X"].astype(np.float64), w["D_i"], w["Im"], w["edgeMaskR"], w["edgeMaskC"]]
    return scal + [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


@pytest.mark.parametrize("W,H", [(64, 48), (97, 61), (5, 40)])
def test_fp64_kernels_match_fp64_oracle(W, H):
    import torch

    w = synthetic(W, H, seed=W + H)
    s = OptSolver([W, H], ENERGY, "LMGPU", double_precision=True)
    prm = params64(w)
    assert s.eval_cost(prm) == pytest.approx(oracle.sfs_cost(w, double=True), rel=1e-10)
    n = W * H
    r = torch.zeros(n, dtype=torch.float64, device="cuda")
    pre = torch.zeros_like(r)
    s.eval_jtf(prm, r, pre)
    r_ref, _ = oracle.sfs_jtf(w, double=True)
    assert rel_err(to_np(r), r_ref) < 1e-10
    p = np.random.default_rng(3).normal(size=n)
    p[~(w["D_i"] > 0)] = 0
    Ap = torch.zeros(n, dtype=torch.float64, device="cuda")
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.sfs_apply(w, p, double=True)
    assert rel_err(to_np(Ap), Ap_ref) < 1e-10
    assert pAp == pytest.approx(pAp_ref, rel=1e-10)


@pytest.mark.parametrize("kind,nit,lit", [("gaussNewtonGPU", 3, 10), ("LMGPU", 6, 10), ("LMGPU", 3, 25)])
def test_fp64_solve_matches_fp64_oracle(kind, nit, lit):
    w = synthetic(96, 72, seed=12)
    s = OptSolver([96, 72], ENERGY, kind, double_precision=True)
    prm = params64(w)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    X_ref, c_ref = oracle.sfs_solve(w, nit, lit, lm=(kind == "LMGPU"), double=True)
    assert len(costs) == len(c_ref)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-8)
    assert rel_err(to_np(prm[16]), X_ref) < 1e-8


def test_fp64_reference_inputs_match_fp64_oracle():
    w = reference_inputs()
    s = OptSolver([w["W"], w["H"]], ENERGY, "LMGPU", double_precision=True)
    prm = params64(w)
    s.set_solver_params({"nIterations": 5, "lIterations": 10})
    costs = s.profiled_solve(prm)
    X_ref, c_ref = oracle.sfs_solve(w, 5, 10, lm=True, double=True)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-8)
    act = w["D_i"] > 0
    assert rel_err(to_np(prm[16])[act], X_ref[act]) < 1e-8


def fp32_noise_floor(solve, w, key, n_pert=4):
    """Relative distance of fp32 oracle trajectories from the fp64 one, over the input
    and n_pert copies with every unknown moved by one ulp (random sign), running max
    over the steps: how far apart two fp32 evaluations of the same algorithm land."""
    c64 = solve(w, double=True)
    rng = np.random.default_rng(0)
    worst = np.abs(solve(w) - c64) / c64
    for _ in range(n_pert):
        x = w[key]
        up = rng.uniform(size=x.size) < 0.5
        xp = np.where(up, np.nextafter(x, np.float32(np.inf)), np.nextafter(x, np.float32(-np.inf))).astype(np.float32)
        worst = np.maximum(worst, np.abs(solve(dict(w, **{key: xp})) - c64) / c64)
    return c64, np.maximum.accumulate(worst)


@pytest.mark.parametrize("case", ["synthetic", "reference"])
def test_fp32_trajectory_within_the_fp32_noise_floor(case):
    """The fp32 bars above (1e-4) measured: the fp32 GPU trajectory is no further from the
    fp64 oracle's than fp32 oracle runs on 1-ulp perturbed inputs are (x2 + 1e-7), i.e.
    the GPU-vs-oracle drift is fp32 rounding amplified by the problem, not a different
    algorithm."""
    w = synthetic(96, 72, seed=12) if case == "synthetic" else reference_inputs((slice(120, 280), slice(200, 440)))
    nit, lit = (6, 10) if case == "synthetic" else (5, 10)
    s = OptSolver([w["W"], w["H"]], ENERGY, "LMGPU")
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = np.array(s.profiled_solve(params(w)))
    c64, floor = fp32_noise_floor(lambda ww, double=False: oracle.sfs_solve(ww, nit, lit, lm=True, double=double)[1],
                                  w, "X", n_pert=3)
    drift = np.abs(costs - c64) / c64
    assert np.all(drift <= 2 * floor + 1e-7), (drift, floor)


@pytest.mark.parametrize("W,H", [(97, 61), (130, 9), (300, 257)])
def test_cost_strip_equals_per_pixel_cost(monkeypatch, W, H):
    """sfs_cost_strip (register strip, DPP neighbours) against the per-pixel sfs_cost:
    the cost, and the model cost through whole LM trajectories."""
    w = synthetic(W, H, seed=W)
    out = {}
    for strip in ("1", "0"):
        monkeypatch.setenv("OPT_AMD_SFS_COST_STRIP", strip)
        s = OptSolver([W, H], ENERGY, "LMGPU")
        prm = params(w)
        c0 = s.eval_cost(prm)
        s.set_solver_params({"nIterations": 5, "lIterations": 10})
        out[strip] = (c0, s.profiled_solve(prm))
        s.close()
    assert out["1"][0] == pytest.approx(out["0"][0], rel=1e-6)
    assert out["1"][0] == pytest.approx(oracle.sfs_cost(w), rel=2e-5)
    np.testing.assert_allclose(out["1"][1], out["0"][1], rtol=1e-5)


@pytest.mark.parametrize("W,H", [(97, 61), (130, 9), (300, 257)])
@pytest.mark.parametrize("double", [False, True])
def test_jtf_strip_equals_tile_jtf(monkeypatch, W, H, double):
    """J^T F + diag(J^T J) + flags by the register strip (sfs_strip<T, true>) against the
    LDS-tile kernel (sfs_tiles<T, true>): the same expressions in the same order; the two
    kernels may contract different multiply-adds into FMAs, so r and the preconditioner
    agree to a few ulps, and whole LM trajectories to the fp32 noise floor."""
    import torch

    w = synthetic(W, H, seed=W + 7)
    out = {}
    for strip in ("1", "0"):
        monkeypatch.setenv("OPT_AMD_SFS_JTF_STRIP", strip)
        s = OptSolver([W, H], ENERGY, "LMGPU", double_precision=double)
        mk = params64 if double else params
        prm = mk(w)
        n = s.unknown_count()
        dt = torch.float64 if double else torch.float32
        r = torch.zeros(n, dtype=dt, device="cuda")
        pre = torch.zeros_like(r)
        s.eval_jtf(prm, r, pre)
        s.set_solver_params({"nIterations": 4, "lIterations": 10})
        out[strip] = (to_np(r), to_np(pre), s.profiled_solve(mk(w)))
        s.close()
    tol = 1e-13 if double else 2e-6
    assert rel_err(out["1"][0], out["0"][0]) < tol
    assert rel_err(out["1"][1], out["0"][1]) < tol
    np.testing.assert_array_equal(out["1"][1] == 0, out["0"][1] == 0)   # flags (pre = 0 off them)
    # fp32: ulp-level J^T F differences grow along an LM trajectory like any 1-ulp input
    # change (test_fp32_trajectory_within_the_fp32_noise_floor measures that floor)
    np.testing.assert_allclose(out["1"][2], out["0"][2], rtol=1e-12 if double else 5e-5)


@pytest.mark.parametrize("W,H", [(97, 61), (130, 9), (300, 257)])
@pytest.mark.parametrize("double", [False, True])
def test_precompute_strip_equals_per_pixel(monkeypatch, W, H, double):
    """sfs_precompute_strip (register strips, DPP neighbours) against the per-pixel
    sfs_precompute: B_I, its gradient images and valid feed every later kernel, so the
    cost after init and whole LM trajectories agree."""
    w = synthetic(W, H, seed=W + 11)
    mk = params64 if double else params
    out = {}
    for strip in ("1", "0"):
        monkeypatch.setenv("OPT_AMD_SFS_PRE_STRIP", strip)
        s = OptSolver([W, H], ENERGY, "LMGPU", double_precision=double)
        c0 = s.eval_cost(mk(w))
        s.set_solver_params({"nIterations": 4, "lIterations": 10})
        out[strip] = (c0, s.profiled_solve(mk(w)))
        s.close()
    assert out["1"][0] == pytest.approx(out["0"][0], rel=1e-12 if double else 1e-6)
    np.testing.assert_allclose(out["1"][1], out["0"][1], rtol=1e-12 if double else 5e-5)


@pytest.mark.parametrize("kind", ["LMGPU", "gaussNewtonGPU"])
@pytest.mark.parametrize("double", [False, True])
@pytest.mark.parametrize("W,H,lit", [(97, 61, 10), (64, 48, 4), (130, 9, 1)])
def test_fused_pcg_step_matches_classic(monkeypatch, kind, double, W, H, lit):
    """PCGStep2 + PCGStep3 as one pass (step23_kernel, beta's numerator from the identity
    over the apply's fp64 sums r.W Ap, Ap.W Ap, r.W r) against the classic apply / step2 /
    step3 loop (OPT_AMD_FUSE23=0): energy trajectories within 1e-5 (fp32: the classic loop
    sums p.Ap and r.z per thread in fp32, the fused one in fp64 — 1.2e-6 measured after
    three GN steps of 10 PCG iterations) / 1e-11 (fp64);
    and in every fused iteration the identity agrees with the direct rz (fp64 sums of the
    same r) to 1e-7 relative (fp32 rounds r_{i+1} once more than the identity sees)."""
    import torch

    w = synthetic(W, H, seed=2 * W + H)
    out = {}
    for f in ("0", "1"):
        monkeypatch.setenv("OPT_AMD_FUSE23", f)
        s = OptSolver([W, H], ENERGY, kind, double_precision=double)
        s.set_solver_params({"nIterations": 3, "lIterations": lit})
        prm = params(w)
        if double:
            prm[16] = prm[16].double()
        out[f] = (np.array(s.profiled_solve(prm)), to_np(prm[16]).astype(np.float64), s.scalars(8 + 7 * (lit + 2)))
        s.close()
    tol = 1e-11 if double else 1e-5
    np.testing.assert_allclose(out["1"][0], out["0"][0], rtol=tol)
    assert rel_err(out["1"][1], out["0"][1]) < (1e-10 if double else 1e-4)
    sc = np.array(out["1"][2])
    for i in range(1, lit):
        rz, rz_id = sc[8 + 7 * i], sc[8 + 7 * i + 6]
        if rz == 0:
            continue
        assert abs(rz_id - rz) <= (1e-12 if double else 1e-7) * abs(rz) + 1e-300, (i, rz, rz_id)


@pytest.mark.parametrize("fuse", ["1", "0"])
def test_lm_far_past_convergence_with_residual_resets_stays_finite(monkeypatch, fuse):
    """the fused LM loop (step23_kernel: a zero step where p.Ap <= 0, beta = 0
    where the identity's rz <= 0) runs the classic halves on its residual-reset iterations
    (every residual_reset_period = 10, solverGPUGaussNewton.t:738-801); those now carry the
    same guards (half1_kernel / step3_kernel GUARD). A 7 x 5 image (35 unknowns) with
    lIterations = 120 and the zeta exit disabled (q_tolerance = 0) takes every PCG iteration
    far past convergence, through 12 resets per LM step: the energies and depths stay finite
    and the LM energy never increases (a rejected step is reverted). Both the fused loop
    (OPT_AMD_FUSE23=1) and the classic one (0) are run; the classic loop divides as the
    reference does, so only its finiteness where the reference's is finite is asserted."""
    monkeypatch.setenv("OPT_AMD_FUSE23", fuse)
    W, H = 7, 5
    w = synthetic(W, H, seed=4)
    s = OptSolver([W, H], ENERGY, "LMGPU")
    prm = params(w)
    s.set_solver_params({"nIterations": 4, "lIterations": 120, "q_tolerance": 0.0})
    costs = np.array(s.profiled_solve(prm))
    X = to_np(prm[16])
    print(f"FUSE23={fuse}: energies {costs}")
    if fuse == "1":
        assert np.all(np.isfinite(costs)) and np.all(np.isfinite(X[w["D_i"] > 0]))
        assert np.all(np.diff(costs) <= 0) and costs[-1] <= costs[0]


@pytest.mark.parametrize("double", [False, True])
def test_fused_lm_reset_iteration_with_zero_pap_keeps_delta_finite(monkeypatch, double):
    """the fused LM loop's residual-reset iterations launch the guarded
    half1_kernel (alpha = 0 unless p.Ap > 0, as step23_kernel). With no depth anywhere every
    unknown is excluded (Exclude(Not(has_depth)), shape_from_shading.t), so r_0 = p_0 = 0 and
    p.Ap = 0 exactly; residual_reset_period = 1 makes every PCG iteration a reset. The
    unguarded division (0 / 0) would put NaN into delta, and half2's q = 1/2 delta.(r + b)
    would carry it: every rz / q slot stays finite (zero) and the unknowns are unchanged."""
    monkeypatch.setenv("OPT_AMD_FUSE23", "1")
    W, H, lit = 16, 12, 4
    w = synthetic(W, H, seed=11)
    w["D_i"] = np.zeros_like(w["D_i"])
    s = OptSolver([W, H], ENERGY, "LMGPU", double_precision=double)
    s.set_solver_params({"nIterations": 2, "lIterations": lit, "residual_reset_period": 1, "q_tolerance": 0.0})
    prm = params64(w) if double else params(w)
    X0 = to_np(prm[16]).copy()
    costs = np.array(s.profiled_solve(prm))
    sc = np.array(s.scalars(8 + 7 * (lit + 2)))
    s.close()
    assert np.all(np.isfinite(costs)), costs
    for i in range(lit + 1):
        rz, q = sc[8 + 7 * i], sc[8 + 7 * i + 1]
        assert np.isfinite(rz) and np.isfinite(q), (i, rz, q)
    np.testing.assert_array_equal(to_np(prm[16]), X0)
