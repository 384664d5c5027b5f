"""GPU: the reference's own end-to-end known answers (examples/test_final_cost.py:55-66)
through the C ABI on every solver path the reference test exercises (matrix-free GN,
materialized J^T (J p), materialized J^T J) plus our GN fast path / generic driver and
the host-buffer backends, within the reference test's 1e-5 relative tolerance."""
import numpy as np
import pytest

from opt_amd import OptSolver
from tests.iw_helpers import ENERGY, device_params, host_params
from tests.reference_inputs import REFERENCE_FINAL_COST, REFERENCE_RTOL, image_warping_cat512

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
