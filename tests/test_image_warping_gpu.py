"""GPU parity of the image_warping hot path (through the C ABI) against the C oracle.

Tolerances (float32 path; the reference computes in opt_float = float, config.t:3-5):
per-unknown kernel outputs (J^T F, pre, J^T J p) within 2e-5 of the largest
magnitude (different but equally valid summation orders, sincosf vs cosf/sinf ULPs);
scalar reductions within 1e-5 relative; GN energies within 1e-5 relative (the
north_star bar). Integer/flag work is exact by construction.
"""
import numpy as np
import pytest

from oracle import oracle
from opt_amd import OptSolver
from tests.iw_helpers import ENERGY, device_params, host_params, perturbed, rel_err, solver

pytestmark = pytest.mark.gpu

SIZES = [(37, 29), (62, 5), (63, 64), (130, 70), (250, 131), (5, 3), (1, 9), (200, 1)]
# |rz_i by the identity - rz_i direct| / rz_i allowed in any PCG iteration of the fused loop
IDENTITY_BOUND = 1e-6   # measured round 4: <= 7.5e-8 over 500 iterations


def to_np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("W,H", SIZES)
def test_cost_jtf_apply_match_oracle(W, H):
    import torch

    w = perturbed(W, H, seed=W * 7 + H)
    s = solver(W, H)
    prm = device_params(w)
    n = 3 * W * H
    assert s.unknown_count() == n
    assert s.family() == "image_warping"
    # cost
    c_gpu = s.eval_cost(prm)
    c_ref = oracle.iw_cost(w)
    assert c_gpu == pytest.approx(c_ref, rel=1e-5, abs=1e-12)
    # J^T F and preconditioner
    r = torch.zeros(n, device="cuda")
    pre = torch.zeros(n, device="cuda")
    rz = s.eval_jtf(prm, r, pre)
    r_ref, pre_ref, rz_ref = oracle.iw_eval_jtf(w)
    assert rel_err(to_np(r), r_ref) < 2e-5
    assert rel_err(to_np(pre), pre_ref) < 2e-5
    assert rz == pytest.approx(rz_ref, rel=1e-5, abs=1e-20)
    # J^T J p
    rng = np.random.default_rng(1)
    p = rng.normal(size=n).astype(np.float32)
    Ap = torch.zeros(n, device="cuda")
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.iw_apply_jtj(w, p)
    assert rel_err(to_np(Ap), Ap_ref) < 2e-5
    assert pAp == pytest.approx(pAp_ref, rel=1e-5, abs=1e-20)


@pytest.mark.parametrize("W,H,nit,lit", [(37, 29, 4, 10), (130, 70, 3, 10), (250, 131, 2, 20), (64, 64, 6, 5)])
def test_gn_solve_matches_oracle(W, H, nit, lit):
    w = perturbed(W, H, seed=17 + W)
    s = solver(W, H)
    prm = device_params(w)
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    costs = s.profiled_solve(prm)
    O_ref, A_ref, c_ref, _ = oracle.iw_solve(w, nit, lit)
    assert len(costs) == nit + 1
    np.testing.assert_allclose(costs, c_ref, rtol=1e-5)
    assert costs[-1] < costs[0]
    assert rel_err(to_np(prm[0]), O_ref) < 1e-5
    assert np.abs(to_np(prm[1]) - A_ref).max() < 1e-4 * max(1.0, np.abs(A_ref).max())
    assert s.iterations() == nit


def test_solve_is_bitwise_deterministic():
    W, H = 300, 200
    w = perturbed(W, H, seed=99)
    outs = []
    for _ in range(2):
        s = solver(W, H)
        prm = device_params(w)
        s.set_solver_params({"nIterations": 3, "lIterations": 10})
        c = s.solve(prm)
        outs.append((c, to_np(prm[0]).copy(), to_np(prm[1]).copy()))
    assert outs[0][0] == outs[1][0]
    assert np.array_equal(outs[0][1], outs[1][1]) and np.array_equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("backend", ["backend_cpu", "backend_cpu_mt"])
def test_host_buffer_backends_equal_device_path(backend):
    W, H = 97, 61
    w = perturbed(W, H, seed=4)
    sd = solver(W, H)
    pd = device_params(w)
    sd.set_solver_params({"nIterations": 2, "lIterations": 8})
    cd = sd.solve(pd)
    sh = solver(W, H, backend=backend)
    ph = host_params(w)
    sh.set_solver_params({"nIterations": 2, "lIterations": 8})
    ch = sh.solve(ph)
    assert ch == cd
    assert np.array_equal(ph[0], to_np(pd[0])) and np.array_equal(ph[1], to_np(pd[1]))


@pytest.mark.parametrize("W,H", [(90, 70), (37, 29), (130, 5), (64, 64)])
@pytest.mark.parametrize("fused", [1, 0])
def test_double_precision_path(monkeypatch, W, H, fused):
    """doublePrecision (Opt.h:11-14) against the double oracle (oracle/iw_impl.h, REAL =
    double: unknowns and solver in double, known arrays float): J^T F, pre and J^T J p
    within 1e-10 of their largest magnitude, the GN trajectory (3 GN x 10 PCG) within
    1e-8 relative, the unknowns within 1e-8. Both the fused loop (iw_jtf_apply +
    iw_apply_res) and the separate passes."""
    import torch

    monkeypatch.setenv("OPT_AMD_IW_FUSED_INIT", str(fused))
    monkeypatch.setenv("OPT_AMD_IW_FUSED_RES", str(fused))
    w = perturbed(W, H, seed=8 + W)
    s = solver(W, H, double=True)
    prm = device_params(w, double=True)
    n = 3 * W * H
    r = torch.zeros(n, device="cuda", dtype=torch.float64)
    pre = torch.zeros(n, device="cuda", dtype=torch.float64)
    rz = s.eval_jtf(prm, r, pre)
    r_ref, pre_ref, rz_ref = oracle.iw_eval_jtf(w, double=True)
    assert rel_err(to_np(r), r_ref) < 1e-10
    assert rel_err(to_np(pre), pre_ref) < 1e-10
    assert rz == pytest.approx(rz_ref, rel=1e-10)
    assert s.eval_cost(prm) == pytest.approx(oracle.iw_cost(w, double=True), rel=1e-12)
    p = torch.randn(n, device="cuda", dtype=torch.float64)
    Ap = torch.zeros_like(p)
    pAp = s.apply_jtj(prm, p, Ap)
    Ap_ref, pAp_ref = oracle.iw_apply_jtj(w, to_np(p), double=True)
    assert rel_err(to_np(Ap), Ap_ref) < 1e-10
    assert pAp == pytest.approx(pAp_ref, rel=1e-10)
    s.set_solver_params({"nIterations": 3, "lIterations": 10})
    costs = s.profiled_solve(prm)
    O_ref, A_ref, c_ref, _ = oracle.iw_solve(w, 3, 10, double=True)
    np.testing.assert_allclose(costs, c_ref, rtol=1e-8)
    assert rel_err(to_np(prm[0]), O_ref) < 1e-8
    assert np.abs(to_np(prm[1]) - A_ref).max() < 1e-8 * max(1.0, np.abs(A_ref).max())


def test_fully_masked_image_is_a_no_op():
    W, H = 70, 40
    w = perturbed(W, H, seed=2)
    w["Mask"][:] = 255.0
    s = solver(W, H)
    prm = device_params(w)
    O0, A0 = to_np(prm[0]).copy(), to_np(prm[1]).copy()
    s.set_solver_params({"nIterations": 2, "lIterations": 3})
    assert s.solve(prm) == 0.0
    assert np.array_equal(to_np(prm[0]), O0) and np.array_equal(to_np(prm[1]), A0)


@pytest.mark.parametrize("W,H", [(2048, 2048), (4096, 4096)])
def test_full_size_properties(W, H):
    """Size-independent properties at the BASELINE sizes: J^T J symmetric, PSD,
    linear; cost equals the oracle's; one GN step lowers the energy."""
    import torch

    w = perturbed(W, H, seed=1, angle_sigma=0.01, offset_sigma=0.1)
    s = solver(W, H)
    prm = device_params(w)
    n = 3 * W * H
    g = torch.Generator(device="cuda").manual_seed(0)
    p = torch.randn(n, device="cuda", generator=g)
    q = torch.randn(n, device="cuda", generator=g)
    Ap, Aq, Apq = (torch.zeros(n, device="cuda") for _ in range(3))
    pAp = s.apply_jtj(prm, p, Ap)
    s.apply_jtj(prm, q, Aq)
    s.apply_jtj(prm, p + q, Apq)
    act = torch.from_numpy(np.concatenate([np.repeat(w["Mask"] == 0, 2), w["Mask"] == 0])).cuda()
    pm, qm = p * act, q * act
    assert pAp > 0
    qAp = float(torch.dot(qm.double(), Ap.double()))
    pAq = float(torch.dot(pm.double(), Aq.double()))
    assert qAp == pytest.approx(pAq, rel=1e-5)
    lin = float((Apq - Ap - Aq).abs().max()) / float(Apq.abs().max())
    assert lin < 1e-5
    assert s.eval_cost(prm) == pytest.approx(oracle.iw_cost(w, nthreads=8), rel=1e-5)
    s.set_solver_params({"nIterations": 1, "lIterations": 10})
    costs = s.profiled_solve(prm)
    assert costs[1] < costs[0]


def _perturb_offset(w, seed):
    w2 = dict(w)
    rng = np.random.default_rng(seed)
    w2["Offset"] = (w["Offset"] * (1 + 2.0 ** -24 * rng.standard_normal(w["Offset"].size))).astype(np.float32)
    return w2


@pytest.mark.parametrize("N", [96, 1024])
def test_fp64_kernels_at_the_bench_workload(N):
    """No precision leak in the fp64 path at size: on the bench workload the
    fp64 cost, J^T F, pre, r.z, J^T J p and p.Ap agree with the double oracle within 1e-13
    (measured round 5: <= 4.6e-16 at 96^2, 1024^2 and 2048^2, tools/fp64_gap.py,
    profiles/r05_fp64_gap.txt)."""
    import torch
    from opt_amd import workloads

    w = workloads.image_warping(N, N, seed=1234)
    n = 3 * N * N
    s = solver(N, N, double=True)
    prm = device_params(w, double=True)
    assert s.eval_cost(prm) == pytest.approx(oracle.iw_cost(w, nthreads=16, double=True), rel=1e-13)
    r = torch.zeros(n, device="cuda", dtype=torch.float64)
    pre = torch.zeros_like(r)
    rz = s.eval_jtf(prm, r, pre)
    r_ref, pre_ref, rz_ref = oracle.iw_eval_jtf(w, nthreads=16, double=True)
    assert rel_err(to_np(r), r_ref) < 1e-13 and rel_err(to_np(pre), pre_ref) < 1e-13
    assert rz == pytest.approx(rz_ref, rel=1e-13)
    p = np.random.default_rng(3).standard_normal(n)
    Ap = torch.zeros_like(r)
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.iw_apply_jtj(w, p, nthreads=16, double=True)
    assert rel_err(to_np(Ap), Ap_ref) < 1e-13
    assert pAp == pytest.approx(pAp_ref, rel=1e-13)


@pytest.mark.parametrize("N", [96, 256])
@pytest.mark.parametrize("fused", [1, 0])
def test_fp64_bench_workload_matches_double_oracle(monkeypatch, N, fused):
    """The bench workload (handles moved by up to 5 % of the width: the energy falls
    2400-fold in the first GN step) in fp64, 2 GN x 10 PCG, against the double oracle
    within 1e-8 — the fused loop and the separate passes (measured round 5 at 96^2:
    4.4e-10 / 1.9e-10)."""
    from opt_amd import workloads

    monkeypatch.setenv("OPT_AMD_IW_FUSED_INIT", str(fused))
    monkeypatch.setenv("OPT_AMD_IW_FUSED_RES", str(fused))
    w = workloads.image_warping(N, N, seed=1234)
    _, _, truth, _ = oracle.iw_solve(w, 2, 10, nthreads=16, double=True)
    s = solver(N, N, double=True)
    prm = device_params(w, double=True)
    s.set_solver_params({"nIterations": 2, "lIterations": 10})
    c = np.array(s.profiled_solve(prm))
    print(f"N={N} fused={fused}: fp64 GPU vs double oracle {np.abs(c - truth) / truth}")
    np.testing.assert_allclose(c, truth, rtol=1e-8)


@pytest.mark.parametrize("N", [1024, 2048, 4096])
def test_fp64_trajectory_at_size_within_the_fp64_floor(N):
    """The fp64 headline trajectory at 1024^2 and 2048^2 (2 GN x 10 PCG) against the
    double oracle. Round 4 measured 2-5e-7 here and suspected a precision leak; round 5
     found none:
      * the kernels agree at 1e-16 (test_fp64_kernels_at_the_bench_workload);
      * fp-contract is not it: the oracle built with -ffp-contract=fast -mfma moves by
        6e-10, not 2e-7;
      * the gap was the oracle's own summation order: with double accumulators its energy
        after one GN step moved by up to 3.5e-7 between 1 and 16 slab threads. From PCG
        iteration 5 on this workload's PCG scalars lose about three digits per iteration
        (loss of orthogonality), so one rounding of a dot product anywhere moves the
        energy after 10 iterations by 1e-8 .. 1e-6.
    The oracle now sums in 80-bit (OACC, oracle/iw_impl.h), and its remaining spread over
    slab counts (16 vs 7 threads) is the fp64 floor of the trajectory. Assert: the fp64 GPU
    path within max(1e-8, 2 x that spread) (measured round 5: 1.4e-8 / 1.0e-8 at 1024^2
    against a spread of 1.2e-8 / 1.0e-8; 2.1e-8 / 7.9e-8 at 2048^2 against 8.6e-8 /
    2.2e-7), the initial energy within 1e-13. 4096^2 is the headline size (fp64
    parity pinned there too, with the same spread-derived bar)."""
    from opt_amd import workloads

    w = workloads.image_warping(N, N, seed=1234)
    _, _, truth, _ = oracle.iw_solve(w, 2, 10, nthreads=16, double=True)
    _, _, alt, _ = oracle.iw_solve(w, 2, 10, nthreads=7, double=True)
    spread = np.abs(alt - truth) / truth
    s = solver(N, N, double=True)
    prm = device_params(w, double=True)
    s.set_solver_params({"nIterations": 2, "lIterations": 10})
    c = np.array(s.profiled_solve(prm))
    e64 = np.abs(c - truth) / truth
    print(f"N={N}: fp64 GPU vs double oracle {e64}, oracle 7 vs 16 threads {spread}")
    assert e64[0] < 1e-13
    assert np.all(e64[1:] <= np.maximum(1e-8, 2 * spread[1:])), (e64, spread)


# fp32 GPU error against the fp64 truth after GN steps 1 / 2, measured with the round-5/6 loop
# (iw_pcg, every p_i kept: bitwise the same trajectory in both rounds; round 4's separate
# passes measured 3.3e-4 / 1.9e-4, 8.2e-4 / 3.4e-4, 1.2e-3 / 1.2e-4)
FP32_RECORDED = {1024: (6.8e-4, 5.4e-4), 2048: (1.13e-3, 4.0e-4), 4096: (9.7e-4, 7.8e-5)}


@pytest.mark.parametrize("N", [1024, 2048, 4096])
def test_bench_workload_trajectory_against_fp64_truth(N):
    """The bench generator's workload (seeded) at 1024^2, config 2's 2048^2
    and the headline's 4096^2, 2 GN steps x 10 PCG (solverGPUGaussNewton.t:1913-2349),
    measured against the TRUE trajectory: the double oracle (doublePrecision, Opt.h:11-14,
    80-bit sums), whose own fp64 floor is ~1e-8 .. 1e-6 at these sizes
    (test_fp64_trajectory_at_size_within_the_fp64_floor). VERDICT r5 #4: the bar is the fp32
    GPU path's OWN floor, not the fp32 oracle's (which sits 10-100x further from the truth):
      * the error at every step is at most twice the worst error of the same GPU path on two
        1-ulp perturbations of Offset (what fp32 rounding of the inputs alone moves), or 1e-5;
      * and at most twice the error recorded for this path (FP32_RECORDED: 9.7e-4 / 7.8e-5 at
        4096^2), so a systematic regression that moves all three runs together fails too;
      * the initial energy within 1e-6, and one short-PCG step (1 GN x 1 PCG) within 1e-5
        of the fp32 oracle.
    The errors are printed (1e-4 .. 1e-3 after one 10-iteration PCG solve: the energy is
    evaluated in absolute pixel coordinates)."""
    from opt_amd import workloads

    W = H = N
    w = workloads.image_warping(W, H, seed=1234)
    _, _, truth, _ = oracle.iw_solve(w, 2, 10, nthreads=16, double=True)

    def gpu(wi):
        s = solver(W, H)
        prm = device_params(wi)
        s.set_solver_params({"nIterations": 2, "lIterations": 10})
        c = np.array(s.profiled_solve(prm))
        s.close()
        return c

    c = gpu(w)
    e_gpu = np.abs(c - truth) / truth
    floor = np.zeros_like(truth)
    for seed in (1, 2):
        floor = np.maximum(floor, np.abs(gpu(_perturb_offset(w, seed)) - truth) / truth)
    rec = np.array((0.0,) + FP32_RECORDED[N])
    print(f"N={N} vs fp64 truth: fp32 GPU {e_gpu}, on 1-ulp perturbed inputs (max of 2) {floor}, recorded {rec}")
    assert len(c) == len(truth)
    assert e_gpu[0] < 1e-6
    assert np.all(e_gpu[1:] <= np.maximum(2 * floor[1:], 1e-5)), (e_gpu, floor)
    assert np.all(e_gpu[1:] <= 2 * rec[1:]), (e_gpu, rec)
    s1 = solver(W, H)
    p1 = device_params(w)
    s1.set_solver_params({"nIterations": 1, "lIterations": 1})
    c1 = s1.profiled_solve(p1)
    _, _, r1, _ = oracle.iw_solve(w, 1, 1, nthreads=16)
    np.testing.assert_allclose(c1, r1, rtol=1e-5)


def _step_scalars(s, prm, nit, lit):
    """GN energies and, per step, the PCG scalar slots of that step (rz_i direct and rz_i
    by the identity: slots 2 + 5 i and 2 + 5 i + 4, image_warping.hip kScBase / kSlots)."""
    s.set_solver_params({"nIterations": nit, "lIterations": lit})
    s.init(prm)
    costs, sc = [s.cost()], []
    for _ in range(nit):
        assert s.step(prm)
        costs.append(s.cost())
        sc.append(np.array(s.scalars(2 + 5 * (lit + 2))))
    return np.array(costs), sc


@pytest.mark.parametrize("case,lit", [("cat512", 200), ("cat512", 500), ("bench1024", 200), ("bench1024", 500)])
def test_fused_loop_at_the_examples_pcg_depth(monkeypatch, case, lit):
    """The fused GN loop (iw_apply_res: beta_i from the identity over the previous pass's
    fp64 sums, delta deferred in pairs over three p buffers) at the PCG depths the
    reference's examples run (CombinedSolverParameters.h:14 default 200;
    examples/image_warping/src/main.cpp:190,212: 400 / 500), 2 GN steps, on the
    reference's own cat512 input and on the bench workload at 1024^2:
      * in every PCG iteration of both steps the identity's rz_i agrees with the direct
        sum of the same pass: |rz_id - rz| <= IDENTITY_BOUND rz + 1e-12 rz_{i-1}. The second
        term is the identity's own conditioning: it subtracts fp64 sums of size rz_{i-1},
        so its absolute error is ~1e-14 rz_{i-1}, i.e. an absolute error of ~1e-14 in
        beta_i, whatever rz_i / rz_{i-1} is (a non-positive identity value
        gives beta_i = 0, iw_apply_res);
      * the true trajectory is the fp64 path's (doublePrecision, fused loop; pinned to the
        double oracle by test_double_precision_path); its own floor is the fp64
        separate-pass loop's distance from it. Hundreds of PCG iterations amplify fp64
        rounding too: measured round 4, cat512 at 200 iterations moves by 1.5e-3 / 1.4e-2
        after GN steps 1 / 2 between the two fp64 loops, and the double oracle lands
        7.5e-3 / 2.4e-2 from the GPU (its products and sums round differently), so this
        energy at that depth has no trajectory to pin below the percent level in ANY
        precision; the fp32 floor there is 0.14 / 0.09. So at this depth the TRAJECTORY
        parity is unpinned (bars of 2 x those floors, i.e. 20-30 % on cat512); the tight
        assertion is the identity against the direct sum above;
      * the fp32 fused loop and the fp32 separate-pass loop (OPT_AMD_IW_FUSED_RES=0) lie
        within twice the larger floor — fp32's (the worst error of the fp32 fused loop on
        two 1-ulp perturbations of Offset) or fp64's — of that truth, or 1e-5."""
    from opt_amd import workloads
    from tests.reference_inputs import image_warping_cat512

    w = image_warping_cat512() if case == "cat512" else workloads.image_warping(1024, 1024, seed=1234)
    W, H = w["W"], w["H"]

    def run(fused, double=False, wi=w):
        monkeypatch.setenv("OPT_AMD_IW_FUSED_RES", str(fused))
        s = solver(W, H, double=double)
        return _step_scalars(s, device_params(wi, double=double), 2, lit)

    fused32, sep32 = run(1), run(0)
    worst = worst_abs = 0.0
    for k, sc in enumerate(fused32[1]):
        for i in range(1, lit):
            rz, rzx, rzp = sc[2 + 5 * i], sc[2 + 5 * i + 4], sc[2 + 5 * (i - 1)]
            assert np.isfinite(rzx) and rz > 0
            assert abs(rzx - rz) <= IDENTITY_BOUND * rz + 1e-12 * rzp, (k, i, rz, rzx, rzp)
            worst = max(worst, abs(rzx - rz) / rz)
            worst_abs = max(worst_abs, abs(rzx - rz) / rzp)
    truth = run(1, double=True)[0]
    sep64 = run(0, double=True)[0]
    floor64 = np.abs(sep64 - truth) / truth
    floor = np.zeros_like(truth)
    for seed in (1, 2):
        c, _ = run(1, wi=_perturb_offset(w, seed))
        floor = np.maximum(floor, np.abs(c - truth) / truth)
    e_f = np.abs(fused32[0] - truth) / truth
    e_s = np.abs(sep32[0] - truth) / truth
    print(f"{case} lIterations={lit}: identity vs direct rz worst {worst:.3g} of rz_i, {worst_abs:.3g} of "
          f"rz_(i-1); vs fp64 truth: fused {e_f}, separate {e_s}, fp32 floor {floor}, fp64 floor {floor64}")
    bar = np.maximum(2 * np.maximum(floor, floor64), 1e-5)
    assert np.all(e_f <= bar) and np.all(e_s <= bar), (e_f, e_s, floor)


@pytest.mark.parametrize("W,H,lit", [(5, 4, 120), (9, 7, 400)])
def test_pcg_far_past_convergence_stays_finite(monkeypatch, W, H, lit):
    """lIterations far past convergence on tiny problems (60 and 189 unknowns, CG's
    exact-arithmetic bound): once rz reaches the rounding floor, the identity
    r_i.W r_i = rz_{i-1} - 2 alpha rAp + alpha^2 ApAp is a difference of fp64 sums of size
    rz_{i-1}; should it cancel to <= 0, iw_apply_res takes beta_i = 0 (a restart) instead
    of a negative or huge beta. The fused loop must stay finite and land where it lands
    with just enough iterations to converge (the 2 GN steps are then the same Newton
    steps up to fp32 rounding). The reference's own PCGStep2/3 divide without a guard
    (alpha = rz / pAp, beta = rz_new / rz_old, solverGPUGaussNewton.t:696,842), and so does
    our separate-pass loop (OPT_AMD_IW_FUSED_RES=0), which measured NaN energies on the
    5x4 case (round 4): past convergence those divisions meet 0 / 0. The count of
    non-positive identity values (kept raw in the scalar slot at +4) is printed."""
    from opt_amd import workloads

    w = workloads.image_warping(W, H, seed=7)
    n = 3 * W * H

    def run(lit_):
        monkeypatch.setenv("OPT_AMD_IW_FUSED_RES", "1")
        s = solver(W, H)
        prm = device_params(w)
        costs, sc = _step_scalars(s, prm, 2, lit_)
        return costs, sc, [t.cpu().numpy() for t in prm[0:2]]   # Offset, Angle after the steps

    cf, scf, xf = run(lit)
    cn, _, xn = run(n)
    restarts = sum(int(sc[2 + 5 * i + 4] <= 0.0) for sc in scf for i in range(1, lit))
    print(f"{W}x{H} lIterations={lit}: {restarts} iterations with a non-positive identity value; "
          f"energies {cf}, at lIterations={n}: {cn}")
    assert np.all(np.isfinite(cf)) and all(np.all(np.isfinite(x)) for x in xf)
    np.testing.assert_allclose(cf, cn, rtol=1e-4, atol=1e-6 * cn[0])
    for a, b in zip(xf, xn):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-3)


# ---- Step-time rebinding (Opt.h:64-65, solverGPUGaussNewton.t:2001,2028): every Step
# evaluates PCGInit1 from the arrays as they are at that Step, so a caller may update
# problem parameters IN PLACE (same pointers) between Steps. The oracle replays the
# same updates one GN step at a time.
CHANGES = ["none", "weight", "offset", "angle", "urshape", "constraints", "mask", "all"]


def _mutate(change, k, O, A, U, C, M, weights, W):
    """The in-place update made before step k (numpy arrays or torch tensors alike)."""
    rng = np.random.default_rng(100 + k)
    if change in ("weight", "all") and k == 2:
        weights[1] *= 1.7
    if change in ("offset", "all") and k in (1, 3):
        d = rng.normal(0, 0.5, O.shape).astype(np.float32)
        O += d if isinstance(O, np.ndarray) else _t(d, O)
    if change in ("angle", "all") and k == 2:
        d = rng.normal(0, 0.05, A.shape).astype(np.float32)
        A += d if isinstance(A, np.ndarray) else _t(d, A)
    if change in ("urshape", "all") and k == 1:
        d = rng.normal(0, 0.3, U.shape).astype(np.float32)
        U += d if isinstance(U, np.ndarray) else _t(d, U)
    if change in ("constraints", "all") and k == 2:
        C[C >= 0] += 1.0
    if change in ("mask", "all") and k == 3:
        M.reshape(-1, W)[20:40, 30:60] = 255.0


def _t(d, like):
    import torch

    return torch.from_numpy(d).to(like.device)


@pytest.mark.parametrize("fused", [1, 0])
@pytest.mark.parametrize("change", CHANGES)
def test_in_place_updates_between_steps_match_oracle(monkeypatch, change, fused):
    monkeypatch.setenv("OPT_AMD_IW_FUSED_INIT", str(fused))
    W, H, nsteps, lit = 150, 110, 5, 8
    w = perturbed(W, H, seed=21)
    s = solver(W, H)
    s.set_solver_params({"nIterations": nsteps, "lIterations": lit})
    prm = device_params(w)
    s.init(prm)
    weights = [prm[5], prm[6]]
    ptrs = [t.data_ptr() for t in prm[:5]]
    gpu = []
    for k in range(nsteps):
        _mutate(change, k, prm[0], prm[1], prm[2], prm[3], prm[4], weights, W)
        prm[5], prm[6] = weights
        assert s.step(prm)
        gpu.append(s.cost())
    assert [t.data_ptr() for t in prm[:5]] == ptrs   # every update was in place
    def replay(ulp):
        wo = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in w.items()}
        if ulp:   # 1-ulp input perturbation: the oracle's own fp32 sensitivity
            rng = np.random.default_rng(ulp)
            wo["Offset"] = (wo["Offset"] * (1 + 2.0 ** -24 * rng.standard_normal(wo["Offset"].size))).astype(np.float32)
        wts = [float(w["w_fitSqrt"]), float(w["w_regSqrt"])]
        ref = []
        for k in range(nsteps):
            _mutate(change, k, wo["Offset"], wo["Angle"], wo["UrShape"], wo["Constraints"], wo["Mask"], wts, W)
            wo["w_fitSqrt"], wo["w_regSqrt"] = wts
            O, A, c, _ = oracle.iw_solve(wo, 1, lit)
            wo["Offset"], wo["Angle"] = O, A
            ref.append(c[1])
        return np.array(ref), wo

    # energies within 1e-5 relative, or within twice the oracle's own spread under 1-ulp
    # input changes (two samples; the fp32 noise floor of this energy)
    # where that is larger; the first step must match at 1e-5 in every case
    ref, wo = replay(0)
    reps = [replay(1), replay(2)]
    floor = np.max([np.abs(r2 - ref) / ref for r2, _ in reps], axis=0)
    drift = np.abs(np.array(gpu) - ref) / ref
    assert drift[0] < 1e-5 and np.all(drift <= np.maximum(2 * floor, 1e-5)), (drift, floor)
    fO = max(np.abs(w2["Offset"] - wo["Offset"]).max() for _, w2 in reps) / np.abs(wo["Offset"]).max()
    assert rel_err(to_np(prm[0]), wo["Offset"]) <= max(2 * fO, 1e-5)
    fA = max(np.abs(w2["Angle"] - wo["Angle"]).max() for _, w2 in reps)
    assert np.abs(to_np(prm[1]) - wo["Angle"]).max() <= max(2 * fA, 1e-4 * max(1.0, np.abs(wo["Angle"]).max()))


def _oracle_trajectory_floor(w, nit, lit):
    """The oracle's GN energies and its fp32 noise floor: the largest relative change of
    each energy under three 1-ulp perturbations of Offset."""
    _, _, ref, _ = oracle.iw_solve(w, nit, lit)
    spread = np.zeros_like(ref)
    for seed in (1, 2, 3):
        w2 = dict(w)
        rng = np.random.default_rng(seed)
        w2["Offset"] = (w["Offset"] * (1 + 2.0 ** -24 * rng.standard_normal(w["Offset"].size))).astype(np.float32)
        _, _, r2, _ = oracle.iw_solve(w2, nit, lit)
        spread = np.maximum(spread, np.abs(r2 - ref) / ref)
    return ref, spread


def _fused_vs_separate(monkeypatch, env, W, H, lit, seed, energy=ENERGY, oracle_floor=True, both=False):
    """One GN step with `env` = 0 and = 1: energies within 1e-6, unknowns within 1e-6 of
    their largest magnitude (the per-pixel values are the same; only reductions group
    differently). Three steps: both settings within 4x the oracle's fp32 noise floor (or
    1e-5) of the oracle's energies — three 1-ulp samples underestimate the spread that
    other summation orders reach (the separate-pass path itself lands at 4.2x on the
    150 x 110 problem)."""
    def run(val, nit):
        monkeypatch.setenv(env, str(val))
        w = perturbed(W, H, seed=seed)
        s = OptSolver([W, H], energy, "gaussNewtonGPU")
        s.set_solver_params({"nIterations": nit, "lIterations": lit})
        prm = device_params(w)
        c = np.array(s.profiled_solve(prm))
        return c, to_np(prm[0]).astype(np.float64), to_np(prm[1]).astype(np.float64), s.scalars(2 + 5 * (lit + 2)), w

    a, b = run(0, 1), run(1, 1)
    np.testing.assert_allclose(b[0], a[0], rtol=1e-6, atol=1e-9 * a[0][0])
    for k in (1, 2):
        assert np.abs(b[k] - a[k]).max() <= 1e-6 * max(1.0, np.abs(a[k]).max())
    a3, b3 = run(0, 3), run(1, 3)
    if oracle_floor:
        ref, floor = _oracle_trajectory_floor(a3[4], 3, lit)
        bar = np.maximum(4 * floor, 1e-5)
        for c in (a3[0], b3[0]):
            assert np.all(np.abs(c - ref) / ref <= bar), (c, ref, floor)
    else:
        np.testing.assert_allclose(b3[0], a3[0], rtol=1e-4)
        assert b3[0][-1] < b3[0][0]
    return (a, b) if both else b


@pytest.mark.parametrize("W,H,lit", [(150, 110, 8), (37, 29, 1), (5, 3, 4), (200, 1, 3), (700, 300, 10)])
def test_fused_init_apply_equals_separate_passes(monkeypatch, W, H, lit):
    """iw_jtf_apply (PCGInit1 + the first apply in one pass) against iw_jtf followed by
    iw_apply<1,0> (and the separate loop that goes with them)."""
    _fused_vs_separate(monkeypatch, "OPT_AMD_IW_FUSED_INIT", W, H, lit, W + H)


@pytest.mark.parametrize("W,H,lit", [(150, 110, 8), (5, 3, 4), (200, 1, 3), (700, 300, 10), (64, 64, 2)])
@pytest.mark.parametrize("use_pre", [True, False])
def test_fused_residual_equals_separate_passes(monkeypatch, tmp_path, W, H, lit, use_pre):
    """iw_apply_res (iteration i's apply with iteration i-1's residual update folded in,
    beta_i's numerator from the exact identity over the previous pass's sums) against
    iw_apply<2> + iw_residual. Both UsePreconditioner settings (PCGInit1 weights r by 1/4
    without one, PCGStep2 by 1); the oracle implements the preconditioned energy."""
    energy = ENERGY
    if not use_pre:
        text = open(ENERGY).read().replace("UsePreconditioner(true)", "UsePreconditioner(false)")
        assert "UsePreconditioner(false)" in text
        energy = str(tmp_path / "iw_nopre.t")
        open(energy, "w").write(text)
    b = _fused_vs_separate(monkeypatch, "OPT_AMD_IW_FUSED_RES", W, H, lit, W + 2 * H, energy, use_pre)
    # beta's numerator by the identity against the direct sum of the same pass
    sc = np.array(b[3])
    for i in range(1, lit):
        rz, rzx = sc[2 + 5 * i], sc[2 + 5 * i + 4]
        assert abs(rzx - rz) <= 1e-6 * abs(rz) + 1e-30, (i, rz, rzx)



@pytest.mark.parametrize("W,H,lit", [(150, 110, 10), (37, 29, 1), (64, 64, 2), (5, 3, 3), (200, 1, 4), (700, 300, 7)])
def test_deferred_delta_is_bitwise_the_per_iteration_update(monkeypatch, W, H, lit):
    """iw_apply_res folding the delta terms of odd PCG iterations into the next even one
    (p in three rotating buffers, p_{i-2} read again) and iw_update taking whatever is
    still pending: every delta is the same chain of fmas, so the GN trajectory (energies,
    Offset, Angle, PCG scalars) is bitwise that of the per-iteration update."""
    out = []
    for val in (0, 1):
        monkeypatch.setenv("OPT_AMD_IW_DEFER", str(val))
        w = perturbed(W, H, seed=5 * W + H)
        s = OptSolver([W, H], ENERGY, "gaussNewtonGPU")
        s.set_solver_params({"nIterations": 3, "lIterations": lit})
        prm = device_params(w)
        c = np.array(s.profiled_solve(prm))
        out.append((c, to_np(prm[0]), to_np(prm[1]), np.array(s.scalars(2 + 5 * (lit + 2)))))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("W,H", [(37, 29), (130, 70), (250, 131), (520, 260)])
def test_side_by_side_waves_match_stacked(monkeypatch, W, H):
    """OPT_AMD_IW_SIDE=1: iw_apply_res with the block's four waves side by side over four
    adjacent strips (Args::side) — the same per-pixel arithmetic, only the reduction's
    tile partition differs: the GN trajectory within 1e-6 of the stacked geometry."""
    w = perturbed(W, H, seed=W + 3 * H)
    out = []
    for side in ("0", "1"):
        monkeypatch.setenv("OPT_AMD_IW_SIDE", side)
        s = solver(W, H)
        prm = device_params(w)
        s.set_solver_params({"nIterations": 3, "lIterations": 6})
        out.append((np.array(s.profiled_solve(prm)), to_np(prm[0]), to_np(prm[1])))
    np.testing.assert_allclose(out[1][0], out[0][0], rtol=1e-6)
    assert rel_err(out[1][1], out[0][1]) < 1e-6 and rel_err(out[1][2], out[0][2]) < 1e-5


@pytest.mark.parametrize("W,H,lit", [(150, 110, 8), (5, 3, 4), (200, 1, 3), (700, 300, 10), (64, 64, 2),
                                     (61, 2, 5), (1, 9, 4), (125, 66, 3)])
def test_pcg_pass_without_stored_ap_matches_apply_res(monkeypatch, W, H, lit):
    """iw_pcg (Ap_{i-1} recomputed from p_{i-1} on 60-column strips; Ap never stored)
    against iw_apply_res (Ap stored and read back, 64-column strips): the same per-pixel
    expressions, only the reduction's tile partition differs — one GN step within 1e-6,
    three within the oracle's fp32 floor; beta's identity against the direct sum."""
    a, b = _fused_vs_separate(monkeypatch, "OPT_AMD_IW_APFREE", W, H, lit, 3 * W + H, both=True)
    # the identity's distance from the direct sum is fp32 rounding of r_i amplified by
    # rz_{i-1} / rz_i (1e-5 on the 1 x 9 image, whose first iteration cuts rz 1e4-fold):
    # no further from it than iw_apply_res's, or 1e-6
    sa, sb = np.array(a[3]), np.array(b[3])
    for i in range(1, lit):
        rz, rzx = sb[2 + 5 * i], sb[2 + 5 * i + 4]
        old = abs(sa[2 + 5 * i + 4] - sa[2 + 5 * i])
        assert abs(rzx - rz) <= max(1e-6 * abs(rz), 2 * old) + 1e-30, (i, rz, rzx, old)


@pytest.mark.parametrize("W,H", [(90, 70), (130, 5), (256, 190)])
def test_pcg_pass_without_stored_ap_fp64(monkeypatch, W, H):
    """The same in fp64 (3 GN x 10 PCG): within 1e-9 of iw_apply_res and of the double
    oracle's energies."""
    w = perturbed(W, H, seed=8 + W)
    out = []
    for v in ("0", "1"):
        monkeypatch.setenv("OPT_AMD_IW_APFREE", v)
        s = solver(W, H, double=True)
        prm = device_params(w, double=True)
        s.set_solver_params({"nIterations": 3, "lIterations": 10})
        out.append((np.array(s.profiled_solve(prm)), to_np(prm[0]), to_np(prm[1])))
    np.testing.assert_allclose(out[1][0], out[0][0], rtol=1e-9)
    assert rel_err(out[1][1], out[0][1]) < 1e-9
    _, _, c_ref, _ = oracle.iw_solve(w, 3, 10, double=True)
    np.testing.assert_allclose(out[1][0], c_ref, rtol=1e-8)


@pytest.mark.parametrize("W,H,lit", [(150, 110, 10), (5, 3, 4), (200, 1, 3), (700, 300, 10), (61, 2, 5),
                                     (1, 9, 4), (240, 97, 7), (333, 131, 17)])
@pytest.mark.parametrize("double", [False, True])
def test_pcg_row_pairs_are_bitwise_one_row_per_trip(monkeypatch, W, H, lit, double):
    """OPT_AMD_IW_PCG_U2 (default 1): iw_pcg walking two rows per loop trip with the row
    records swapping roles (1), and with two raw rows in flight (2), against one row per
    trip (0): the same arithmetic in the same order — the trajectory is bitwise the same
    (odd and even row counts per wave, one-row images, the deferred-delta loop at 17)."""
    out = []
    for v in ("0", "1", "2"):
        monkeypatch.setenv("OPT_AMD_IW_PCG_U2", v)
        w = perturbed(W, H, seed=3 * W + H)
        s = solver(W, H, double=double)
        prm = device_params(w, double=double)
        s.set_solver_params({"nIterations": 3, "lIterations": lit})
        c = np.array(s.profiled_solve(prm))
        out.append((c, to_np(prm[0]), to_np(prm[1]), np.array(s.scalars(2 + 5 * (lit + 2)))))
    for o in out[1:]:
        for a, b in zip(out[0], o):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("W,H,lit", [(150, 110, 10), (5, 3, 4), (200, 1, 3), (700, 300, 10), (64, 64, 2),
                                     (61, 2, 5), (1, 9, 4), (121, 66, 1), (240, 97, 7), (90, 70, 16), (90, 70, 17)])
@pytest.mark.parametrize("double", [False, True])
def test_kept_p_update_is_bitwise_the_deferred_delta(monkeypatch, W, H, lit, double):
    """OPT_AMD_IW_ALLP (default 1, lIterations 2..16): every p_i kept and delta formed once
    by iw_update_all (alpha_0 p_0, then one fma per iteration) against the deferred delta
    (pairs folded by the even passes): the trajectory is bitwise the same, fp32 and fp64
    (lIterations 1 and 17 take the deferred path either way). ADVICE r5: when the kept
    vectors do not fit in HBM the Step falls back to the deferred delta — forced here with
    OPT_AMD_IW_ALLP_LIMIT_MB=0 — and is again bitwise the same; so is iw_update_all one pixel
    per thread against pixel pairs (OPT_AMD_IW_UPD_PAIRS, taken where N % 4 == 0)."""
    out = []
    for v in ("0", "1", "fallback", "nopairs"):
        monkeypatch.setenv("OPT_AMD_IW_ALLP", "0" if v == "0" else "1")
        monkeypatch.setenv("OPT_AMD_IW_ALLP_LIMIT_MB", "0" if v == "fallback" else "-1")
        monkeypatch.setenv("OPT_AMD_IW_UPD_PAIRS", "0" if v == "nopairs" else "1")
        w = perturbed(W, H, seed=5 * W + H)
        s = solver(W, H, double=double)
        prm = device_params(w, double=double)
        s.set_solver_params({"nIterations": 3, "lIterations": lit})
        c = np.array(s.profiled_solve(prm))
        out.append((c, to_np(prm[0]), to_np(prm[1]), np.array(s.scalars(2 + 5 * (lit + 2)))))
    for k in (1, 2, 3):
        for a, b in zip(out[0], out[k]):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("W,H,lit", [(150, 110, 10), (5, 3, 4), (200, 1, 3), (700, 300, 10), (61, 2, 5), (1, 9, 4),
                                     (240, 97, 7), (130, 257, 12)])
@pytest.mark.parametrize("double", [False, True])
def test_recomputed_angle_pre_is_bitwise_the_stored(monkeypatch, W, H, lit, double):
    """Round 6 (iw_pcg PRC, default on): the passes after the first recompute the angle
    channel's Jacobi preconditioner from the stencil geometry (diag_a2 over the four edges
    in iw_jtf's order, pre_angle) instead of reading the value iw_jtf_apply stored; every
    rounding of that formula is explicit, so the trajectory (energies, Offset, Angle, PCG
    scalars) is bitwise the stored-pre one (OPT_AMD_IW_PCG_PRC=0), fp32 and fp64."""
    out = []
    for v in ("0", "1"):
        monkeypatch.setenv("OPT_AMD_IW_PCG_PRC", v)
        w = perturbed(W, H, seed=11 * W + H)
        s = solver(W, H, double=double)
        prm = device_params(w, double=double)
        s.set_solver_params({"nIterations": 3, "lIterations": lit})
        c = np.array(s.profiled_solve(prm))
        out.append((c, to_np(prm[0]), to_np(prm[1]), np.array(s.scalars(2 + 5 * (lit + 2)))))
        s.close()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("W,H,lit", [(150, 110, 10), (5, 3, 4), (200, 1, 3), (700, 300, 10), (61, 2, 5), (1, 9, 4),
                                     (240, 97, 7)])
@pytest.mark.parametrize("double", [False, True])
def test_step_cost_from_flags_is_bitwise_the_mask_cost(monkeypatch, W, H, lit, double):
    """Round 6 (iw_cost60 FL, default on): the cost at the end of a Step takes the active and
    fit tests from the flag byte this Step's J^T F pass wrote and reads Constraints only at
    fit pixels, instead of Mask and every Constraint (OPT_AMD_IW_COST_FLAGS=0): the energies
    and the trajectory are bitwise the same, fp32 and fp64 (the masked pixels and the
    constraint pixels of perturbed() included)."""
    out = []
    for v in ("0", "1"):
        monkeypatch.setenv("OPT_AMD_IW_COST_FLAGS", v)
        w = perturbed(W, H, seed=13 * W + H)
        s = solver(W, H, double=double)
        prm = device_params(w, double=double)
        s.set_solver_params({"nIterations": 3, "lIterations": lit})
        c = np.array(s.profiled_solve(prm))
        out.append((c, to_np(prm[0]), to_np(prm[1]), np.array(s.scalars(2 + 5 * (lit + 2)))))
        s.close()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("W,H,lit", [(150, 110, 10), (5, 3, 4), (200, 1, 3), (700, 300, 10), (61, 2, 5), (1, 9, 4),
                                     (240, 97, 7), (121, 66, 1), (300, 200, 9)])
@pytest.mark.parametrize("double", [False, True])
def test_reversed_tile_order_is_bitwise_the_forward(monkeypatch, W, H, lit, double):
    """Round 6 (Args::rev, OPT_AMD_IW_MALL_REV): the odd PCG passes, and the update or the
    cost after them, take their tiles (pixels) in reverse order so that each kernel starts
    on what the previous one wrote last. Every tile keeps its reduction slot, so the
    trajectory is bitwise the forward one, fp32 and fp64."""
    out = []
    for v in ("0", "1"):
        monkeypatch.setenv("OPT_AMD_IW_MALL_REV", v)
        w = perturbed(W, H, seed=17 * W + H)
        s = solver(W, H, double=double)
        prm = device_params(w, double=double)
        s.set_solver_params({"nIterations": 3, "lIterations": lit})
        c = np.array(s.profiled_solve(prm))
        out.append((c, to_np(prm[0]), to_np(prm[1]), np.array(s.scalars(2 + 5 * (lit + 2)))))
        s.close()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("W,H,lit", [(150, 110, 10), (5, 3, 4), (200, 1, 3), (700, 300, 10), (64, 64, 2),
                                     (61, 2, 5), (1, 9, 4), (121, 66, 1), (240, 97, 7)])
@pytest.mark.parametrize("double", [False, True])
def test_rec_layout_is_bitwise_the_image_layout(monkeypatch, W, H, lit, double):
    """OPT_AMD_IW_REC=1 (default 0): the fused loop's PCG vectors as one record per pixel
    ([r.xy | p.xy | r.t p.t]) and the per-Step S record ([u.x u.y angle pre_t]) against the
    unknown layout: the same per-pixel arithmetic (one-expression contraction, so every
    instantiation rounds alike), the same tiles and sums — the trajectory (energies, Offset,
    Angle, PCG scalars) is bitwise the same, fp32 and fp64."""
    out = []
    for v in ("0", "1"):
        monkeypatch.setenv("OPT_AMD_IW_REC", v)
        w = perturbed(W, H, seed=7 * W + H)
        s = solver(W, H, double=double)
        prm = device_params(w, double=double)
        s.set_solver_params({"nIterations": 3, "lIterations": lit})
        c = np.array(s.profiled_solve(prm))
        out.append((c, to_np(prm[0]), to_np(prm[1]), np.array(s.scalars(2 + 5 * (lit + 2)))))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)
