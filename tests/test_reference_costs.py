"""The reference's own end-to-end known answers (examples/test_final_cost.py): final
costs its CUDA backend produced on the example inputs at nIterations = lIterations = 1,
checked within the reference test's 1e-5 relative tolerance (test_final_cost.py:121).

CPU: the oracle (every restated solver path) against those values. This pins the
restatement to the reference's actual output, not only to finite differences.
The GPU paths are checked against the same values in test_reference_costs_gpu.py."""
import numpy as np
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


# ---- the example energies with no hand-written family: float64 AD restatements of the
# reference's energy files (oracle/examples_ad.py) driven by the oracle's generic loop
from tests.reference_inputs import GENERATED_EXAMPLES, REFERENCE_KIND  # noqa: E402

USE_PRE = {"intrinsic_image_decomposition": False}   # the energy file's UsePreconditioner


@pytest.mark.parametrize("name", sorted(GENERATED_EXAMPLES))
def test_generated_example_known_answers_oracle(name):
    from oracle import examples_ad

    w = GENERATED_EXAMPLES[name]()
    costs = examples_ad.solve(examples_ad.BUILDERS[name](w), 1, 1, lm=REFERENCE_KIND.get(name) == "LMGPU",
                              use_pre=USE_PRE.get(name, True))
    assert len(costs) == 2 and costs[-1] < costs[0]
    assert rel(costs[-1], REFERENCE_FINAL_COST[name]) < REFERENCE_RTOL


def test_cotangent_preconditioner_counts_each_vertex_access():
    """head.ply has two valence-2 boundary vertices whose edges list the same vertex as
    both prev and next (v2 == v3). The reference's diagonal adds one squared partial per
    graph slot; with the square of the summed partial instead, the one-step cost misses
    the known answer (1.3e-5 relative)."""
    from oracle import examples_ad

    w = GENERATED_EXAMPLES["cotangent_mesh_smoothing"]()
    assert int((w["v2"] == w["v3"]).sum()) == 2
    m = examples_ad.BUILDERS["cotangent_mesh_smoothing"](w)
    J = m.jacobian()
    summed = np.asarray(J.multiply(J).sum(0)).reshape(-1)
    assert np.abs(summed - m.diag_access).max() > 0
