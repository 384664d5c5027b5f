"""GPU: the reference's own end-to-end known answers (examples/test_final_cost.py:55-66)
through the C ABI on every solver path the reference test exercises (matrix-free GN,
materialized J^T (J p), materialized J^T J) plus our GN fast path / generic driver and
the host-buffer backends, within the reference test's 1e-5 relative tolerance."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver
from tests.iw_helpers import ENERGY, device_params, host_params
from tests.reference_inputs import (REFERENCE_FINAL_COST, REFERENCE_RTOL, arap_armadillo, image_warping_cat512,
                                   optical_flow_dogdance)

pytestmark = pytest.mark.gpu


def rel(a, b):
    return abs(a - b) / abs(b)


@pytest.mark.parametrize("mode", ["matrix_free", "materialized", "materialized_fused"])
@pytest.mark.parametrize("backend", ["backend_cuda", "backend_cpu", "backend_cpu_mt"])
def test_image_warping_cat512_final_cost(mode, backend):
    w = image_warping_cat512()
    s = OptSolver([w["W"], w["H"]], ENERGY, "gaussNewtonGPU", backend=backend,
                  materialized=mode != "matrix_free", fused_jtj=mode == "materialized_fused")
    s.set_solver_params({"nIterations": 1, "lIterations": 1})
    prm = device_params(w) if backend == "backend_cuda" else host_params(w)
    s.solve(prm)
    assert rel(s.cost(), REFERENCE_FINAL_COST["image_warping"]) < REFERENCE_RTOL
    s.close()


def test_image_warping_cat512_fp64():
    """doublePrecision = 1 (unknowns and solver vectors fp64, known arrays fp32)"""
    w = image_warping_cat512()
    s = OptSolver([w["W"], w["H"]], ENERGY, "gaussNewtonGPU", double_precision=True)
    s.set_solver_params({"nIterations": 1, "lIterations": 1})
    s.solve(device_params(w, double=True))
    assert rel(s.cost(), REFERENCE_FINAL_COST["image_warping"]) < REFERENCE_RTOL


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


MODES = {"matrix_free": {}, "materialized": {"materialized": True},
         "materialized_fused": {"materialized": True, "fused_jtj": True}}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("double", [False, True])
def test_optical_flow_dogdance_final_cost(double, mode):
    w = optical_flow_dogdance(1)
    s = OptSolver([w["W"], w["H"]], os.path.join(ROOT, "energies", "optical_flow.t"), "gaussNewtonGPU",
                  double_precision=double, **MODES[mode])
    s.set_solver_params({"nIterations": 1, "lIterations": 1})
    X = dev(w["X"].astype(np.float64 if double else np.float32))
    s.solve([w["w_fitSqrt"], w["w_regSqrt"], X] + [dev(w[k]) for k in ("I", "I_hat", "I_hat_dx", "I_hat_dy")])
    assert rel(s.cost(), REFERENCE_FINAL_COST["optical_flow"]) < REFERENCE_RTOL


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("backend", ["backend_cuda", "backend_cpu"])
def test_arap_armadillo_final_cost(backend, mode):
    w = arap_armadillo()
    s = OptSolver([w["N"], w["E"]], os.path.join(ROOT, "energies", "arap_mesh_deformation.t"), "gaussNewtonGPU",
                  backend=backend, **MODES[mode])
    s.set_solver_params({"nIterations": 1, "lIterations": 1})
    conv = dev if backend == "backend_cuda" else (lambda a: np.ascontiguousarray(a).copy())
    prm = [w["w_fitSqrt"], w["w_regSqrt"]] + [conv(w[k]) for k in ("Offset", "Angle", "UrShape", "Constraints")] + \
          [None, conv(w["v0"]), conv(w["v1"])]
    s.solve(prm)
    assert rel(s.cost(), REFERENCE_FINAL_COST["arap_mesh_deformation"]) < REFERENCE_RTOL


# ---- the reference's example energies with no hand-written family, on kernels the
# general front end generates for energies/<name>.t
from opt_amd.harness import problems  # noqa: E402
from tests.reference_inputs import GENERATED_EXAMPLES, REFERENCE_KIND  # noqa: E402


@pytest.mark.parametrize("name", sorted(GENERATED_EXAMPLES))
@pytest.mark.parametrize("double", [False, True])
def test_generated_example_known_answers(name, double):
    w = GENERATED_EXAMPLES[name]()
    s = OptSolver(problems.dims(name, w), os.path.join(ROOT, "energies", name + ".t"),
                  REFERENCE_KIND.get(name, "gaussNewtonGPU"), double_precision=double)
    assert s.family() == "generic"
    s.set_solver_params({"nIterations": 1, "lIterations": 1})
    s.solve(problems.problem_params(name, w, dev, double=double))
    assert rel(s.cost(), REFERENCE_FINAL_COST[name]) < REFERENCE_RTOL, (s.cost(), REFERENCE_FINAL_COST[name])


@pytest.mark.parametrize("name", ["cotangent_mesh_smoothing", "volumetric_mesh_deformation"])
@pytest.mark.parametrize("mode", ["materialized", "materialized_fused"])
def test_generated_example_known_answers_materialized(name, mode):
    """useMaterializedJTJ (test_final_cost.py:91-93 runs every example this way too)"""
    w = GENERATED_EXAMPLES[name]()
    s = OptSolver(problems.dims(name, w), os.path.join(ROOT, "energies", name + ".t"), "gaussNewtonGPU",
                  **MODES[mode])
    s.set_solver_params({"nIterations": 1, "lIterations": 1})
    s.solve(problems.problem_params(name, w, dev))
    assert rel(s.cost(), REFERENCE_FINAL_COST[name]) < REFERENCE_RTOL, (s.cost(), REFERENCE_FINAL_COST[name])


ROBUST_REFERENCE = 66.784683   # examples/test_final_cost.py:64 ("CUDA cost of first!!! solve"; broken, :41-43)


def _robust_first(arg_order):
    z = np.load(os.path.join(ROOT, "tests", "golden", "squat_first.npz"))
    w = problems.robust_nonrigid_alignment(z["src_verts"], z["src_faces"], z["tets"], z["tgt_verts"], z["tgt_faces"],
                                           arg_order=arg_order)
    prm = [w["w_fitSqrt"], w["w_regSqrt"]] + [dev(w[k]) for k in ("Offset", "Angle", "RobustWeights", "UrShape",
                                                                  "Constraints", "ConstraintNormals")] + \
          [None, dev(w["v0"]), dev(w["v1"])]
    s = OptSolver([w["N"], w["E"]], os.path.join(ROOT, "energies", "robust_nonrigid_alignment.t"), "LMGPU")
    assert s.family() == "generic"
    s.set_solver_params({"nIterations": 1, "lIterations": 1, "function_tolerance": 1e-7})
    s.solve(prm)
    return s.cost()


def test_robust_nonrigid_alignment_first_solve_brackets_the_reference():
    """robust_nonrigid_alignment, flagged broken by the reference's own test, is pinned only
    loosely: its first solve's cost depends on harness details C++ leaves to the platform
    — the order make_float3(normal(), normal(), normal()) evaluates its arguments in, and
    libstdc++'s distribution algorithms — through the 5 % spurious correspondences, which
    move it by several percent (tools/robust_first_solve.py on the first target in sorted
    directory order: 69.23 evaluating right to left, as GCC does on x86-64, 65.71 left to
    right; GCC 11's uniform_int 69.36 / 65.85; the other targets further off). The draws
    themselves match this image's libstdc++ bit for bit (test_harness_rng.py). The
    reference's 66.784683 lies between the two argument orders' costs, each within 4 %."""
    ltr, rtl = _robust_first("ltr"), _robust_first("rtl")
    assert ltr < ROBUST_REFERENCE < rtl, (ltr, rtl)
    assert rel(ltr, ROBUST_REFERENCE) < 0.04 and rel(rtl, ROBUST_REFERENCE) < 0.04, (ltr, rtl)
