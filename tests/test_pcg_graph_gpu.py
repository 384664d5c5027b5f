"""The generic driver's PCG loop replayed as a hipGraph (stencil_plan.h: pcg_graph_begin)
gives bitwise the same iterates as eager launches (OPT_AMD_NO_GRAPH=1), for GN and for LM
(device-side zeta exit inside the graph), and re-captures when a scalar parameter the
launches bake in changes between steps."""
import os

import numpy as np
import pytest

from opt_amd import OptSolver, workloads
from tests.iw_helpers import ROOT, device_params, perturbed, solver

pytestmark = pytest.mark.gpu
POISSON = os.path.join(ROOT, "energies", "poisson_image_editing.t")


def _poisson(monkeypatch, graph, kind):
    import torch

    monkeypatch.setenv("OPT_AMD_NO_GRAPH", "0" if graph else "1")
    w = workloads.poisson_image_editing(96, 80, seed=4)
    prm = [torch.from_numpy(w[k].copy()).cuda() for k in ("X", "T", "M")]
    s = OptSolver([96, 80], POISSON, kind)
    s.set_solver_params({"nIterations": 4, "lIterations": 10})
    costs = s.profiled_solve(prm)
    return costs, prm[0].cpu().numpy()


@pytest.mark.parametrize("kind", ["gaussNewtonGPU", "LMGPU"])
def test_graph_replay_is_bitwise_eager(monkeypatch, kind):
    c_eager, x_eager = _poisson(monkeypatch, False, kind)
    c_graph, x_graph = _poisson(monkeypatch, True, kind)
    assert c_graph == c_eager
    np.testing.assert_array_equal(x_graph, x_eager)


def _iw_lm_with_weight_change(monkeypatch, graph):
    monkeypatch.setenv("OPT_AMD_NO_GRAPH", "0" if graph else "1")
    w = perturbed(70, 50, seed=8)
    s = solver(70, 50, kind="LMGPU")
    s.set_solver_params({"nIterations": 6, "lIterations": 10})
    prm = device_params(w)
    s.init(prm)
    costs = []
    for k in range(6):
        prm[-1] = float(w["w_regSqrt"]) * (1.0 + 0.5 * (k >= 3))   # new value from step 3 on
        if not s.step(prm):
            break
        costs.append(s.cost())
    return costs, prm[0].cpu().numpy()


def test_graph_recaptures_on_parameter_change(monkeypatch):
    c_eager, o_eager = _iw_lm_with_weight_change(monkeypatch, False)
    c_graph, o_graph = _iw_lm_with_weight_change(monkeypatch, True)
    assert len(c_eager) >= 4
    assert c_graph == c_eager
    np.testing.assert_array_equal(o_graph, o_eager)


def _generated_iw_rebinding(monkeypatch, graph):
    """Generated kernels (OPT_AMD_GENERIC=1): new buffers for every array from step 3 on,
    so a replay keyed on stale pointers would read freed / old memory."""
    import torch

    monkeypatch.setenv("OPT_AMD_NO_GRAPH", "0" if graph else "1")
    monkeypatch.setenv("OPT_AMD_GENERIC", "1")
    w = perturbed(60, 40, seed=9)
    s = solver(60, 40, kind="LMGPU")
    assert s.family() == "generic"
    s.set_solver_params({"nIterations": 6, "lIterations": 10})
    prm = device_params(w)
    s.init(prm)
    costs = []
    for k in range(6):
        if k == 3:
            prm = [p.clone() if isinstance(p, torch.Tensor) else p for p in prm]
        if not s.step(prm):
            break
        costs.append(s.cost())
    return costs, prm[0].cpu().numpy()


def test_generated_graph_replay_follows_rebound_buffers(monkeypatch):
    c_eager, o_eager = _generated_iw_rebinding(monkeypatch, False)
    c_graph, o_graph = _generated_iw_rebinding(monkeypatch, True)
    assert len(c_eager) >= 4
    assert c_graph == c_eager
    np.testing.assert_array_equal(o_graph, o_eager)


def _embedded_rebinding(monkeypatch, graph):
    """A graph energy whose declarations the simple parser cannot read (RotMatrix): new
    edge arrays in a different order, on new buffers, between steps."""
    import torch
    from tests.test_generic_examples_gpu import E, problem

    monkeypatch.setenv("OPT_AMD_NO_GRAPH", "0" if graph else "1")
    dims, prm, _ = problem("embedded_mesh_deformation", np.random.default_rng(3))
    s = OptSolver(dims, E("embedded_mesh_deformation"), "gaussNewtonGPU", double_precision=True)
    s.set_solver_params({"nIterations": 5, "lIterations": 10})
    s.init(prm)
    costs = []
    perm = np.random.default_rng(4).permutation(prm[-1].numel())
    for k in range(5):
        if k == 2:
            prm = list(prm)
            prm[-2] = torch.from_numpy(prm[-2].cpu().numpy()[perm].copy()).cuda()
            prm[-1] = torch.from_numpy(prm[-1].cpu().numpy()[perm].copy()).cuda()
        if not s.step(prm):
            break
        costs.append(s.cost())
    return costs, prm[3].cpu().numpy()


def test_graph_energy_rebinding_edges_matches_eager(monkeypatch):
    c_eager, o_eager = _embedded_rebinding(monkeypatch, False)
    c_graph, o_graph = _embedded_rebinding(monkeypatch, True)
    assert len(c_eager) >= 3
    assert c_graph == c_eager
    np.testing.assert_array_equal(o_graph, o_eager)


def _gn_delta(monkeypatch, d3, generic):
    """A GN solve with PCGStep2's delta update in PCGStep3 (d3) or in PCGStep2."""
    monkeypatch.setenv("OPT_AMD_DELTA_IN_STEP3", "1" if d3 else "0")
    if generic:
        monkeypatch.setenv("OPT_AMD_GENERIC", "1")
        w = perturbed(61, 43, seed=12)
        s = solver(61, 43, kind="gaussNewtonGPU")
        assert s.family() == "generic"
        prm = device_params(w)
        s.set_solver_params({"nIterations": 4, "lIterations": 10})
        return s.profiled_solve(prm), prm[0].cpu().numpy()
    return _poisson(monkeypatch, True, "gaussNewtonGPU")


@pytest.mark.parametrize("generic", [False, True])
def test_delta_in_step3_is_bitwise_step2(monkeypatch, generic):
    """The generic GN driver forms delta += alpha p_old in PCGStep3 (stencil_driver.h
    step3_kernel DM) instead of PCGStep2: the same expression on the same operands, so
    whole solves are bitwise those with the reference's placement (:665-731)."""
    c1, x1 = _gn_delta(monkeypatch, True, generic)
    c0, x0 = _gn_delta(monkeypatch, False, generic)
    assert c1 == c0
    np.testing.assert_array_equal(x1, x0)
