"""GPU: the solver log at verbosityLevel > 0 (the examples set verbosityLevel = 1 and
collectPerKernelTimingInfo = 1, examples/shared/OptSolver.h:46-49): "final cost=%.16f"
when Step returns 0 (cleanup, solverGPUGaussNewton.t:1902-1910) — the line the
reference's examples/test_final_cost.py parses — the LM trust-region lines
(:1505-1513, 2254-2283) and the per-kernel timing table; nothing at verbosityLevel 0."""
import re

import numpy as np
import pytest

from opt_amd import OptSolver
from tests.iw_helpers import ENERGY as IW_ENERGY, device_params, perturbed
from tests.reference_inputs import REFERENCE_FINAL_COST, image_warping_cat512

pytestmark = pytest.mark.gpu


def final_costs(out):
    return [float(m) for m in re.findall(r"final cost=([-+0-9.eE]+)", out)]


def test_final_cost_line_is_what_test_final_cost_parses(capfd):
    w = image_warping_cat512()
    s = OptSolver([w["W"], w["H"]], IW_ENERGY, "gaussNewtonGPU", verbosity=1, kernel_timing=True)
    s.set_solver_params({"nIterations": 1, "lIterations": 1})
    s.solve(device_params(w))
    out = capfd.readouterr().out
    fc = final_costs(out)
    assert len(fc) == 1 and fc[0] == pytest.approx(s.cost(), rel=1e-15)
    # examples/test_final_cost.py:100-121: re.search + 1e-5 relative
    m = re.search("final cost=(.*)", out)
    assert abs(float(m.group(1)) - REFERENCE_FINAL_COST["image_warping"]) / REFERENCE_FINAL_COST["image_warping"] < 1e-5
    # the timing table (collectPerKernelTimingInfo): with lIterations = 1 the step is
    # PCGInit1 fused with the only apply, the update and the cost
    for k in ("iw_jtf_apply", "iw_update", "iw_cost", "TIMING total"):
        assert k in out, (k, out)


def test_lm_log_and_silence_at_verbosity_zero(capfd):
    W, H = 48, 40
    w = perturbed(W, H, seed=2)
    s = OptSolver([W, H], IW_ENERGY, "LMGPU", verbosity=1)
    s.set_solver_params({"nIterations": 3, "lIterations": 5})
    s.solve(device_params(w))
    out = capfd.readouterr().out
    assert out.count(" model_cost=") >= 1 and out.count(" cost=") >= 1
    assert len(final_costs(out)) == 1 and final_costs(out)[0] == pytest.approx(s.cost(), rel=1e-15)
    s0 = OptSolver([W, H], IW_ENERGY, "LMGPU")
    s0.set_solver_params({"nIterations": 3, "lIterations": 5})
    s0.solve(device_params(w))
    assert "final cost" not in capfd.readouterr().out
