"""The reference's own end-to-end known answers (examples/test_final_cost.py): final
costs its CUDA backend produced on the example inputs at nIterations = lIterations = 1,
checked within the reference test's 1e-5 relative tolerance (test_final_cost.py:121).

CPU: the oracle (every restated solver path) against those values. This pins the
restatement to the reference's actual output, not only to finite differences.
The GPU paths are checked against the same values in test_reference_costs_gpu.py."""
import pytest

from oracle import oracle
from tests.reference_inputs import (REFERENCE_FINAL_COST, REFERENCE_RTOL, arap_armadillo, image_warping_cat512,
                                   optical_flow_dogdance)


def rel(a, b):
    return abs(a - b) / abs(b)


def test_image_warping_gn_fast_path_oracle():
    w = image_warping_cat512()
    _, _, costs, _ = oracle.iw_solve(w, 1, 1)
    assert rel(costs[-1], REFERENCE_FINAL_COST["image_warping"]) < REFERENCE_RTOL


def test_image_warping_generic_loop_oracle():
    w = image_warping_cat512()
    _, _, costs = oracle.iw_solve_generic(w, 1, 1)
    assert rel(costs[-1], REFERENCE_FINAL_COST["image_warping"]) < REFERENCE_RTOL


@pytest.mark.parametrize("fused", [True, False])
def test_image_warping_materialized_oracle(fused):
    """the reference test runs the same check with useMaterializedJTJ / useFusedJTJ
    (test_final_cost.py:91-93) against the same expected cost"""
    w = image_warping_cat512()
    _, _, costs = oracle.iw_solve_materialized(w, 1, 1, fused=fused)
    assert rel(costs[-1], REFERENCE_FINAL_COST["image_warping"]) < REFERENCE_RTOL


def test_optical_flow_oracle():
    """first solve of the two-level harness (the sigma-5 level), fp32 GN"""
    _, costs = oracle.of_solve(optical_flow_dogdance(1), 1, 1)
    assert rel(costs[-1], REFERENCE_FINAL_COST["optical_flow"]) < REFERENCE_RTOL


def test_arap_mesh_deformation_oracle():
    """small_armadillo after one sqrt(3) subdivision (386 vertices, 2304 directed edges)"""
    w = arap_armadillo()
    assert (w["N"], w["E"]) == (386, 2304)
    _, _, costs = oracle.arap_solve(w, 1, 1)
    assert rel(costs[-1], REFERENCE_FINAL_COST["arap_mesh_deformation"]) < REFERENCE_RTOL
