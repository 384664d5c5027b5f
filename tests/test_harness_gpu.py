"""GPU: the example harness end to end (python -m opt_amd.harness) on small synthetic
data written in the reference's formats and file names: the logged "final cost=" equals
a direct OptSolver run of the same problem, results.csv and the result file are written."""
import io
import os
import struct
from contextlib import redirect_stdout

import numpy as np
import pytest

from opt_amd import OptSolver
from opt_amd.harness import formats, problems
from opt_amd.harness.__main__ import ROOT, run

pytestmark = pytest.mark.gpu


def write_data(d, rng):
    os.makedirs(os.path.join(d, "shape_from_shading"), exist_ok=True)
    H, W = 40, 56
    m = np.zeros((H, W, 4), np.uint8)
    m[10:30, 15:40, 0] = 255
    m[..., 3] = 255
    formats.write_png(os.path.join(d, "cat512_mask.png"), m)
    formats.write_constraints(os.path.join(d, "cat512.constraints"), np.array([[5, 5, 8, 6], [50, 35, 47, 30]]))
    img0 = rng.integers(0, 255, (H, W, 4)).astype(np.uint8)
    img1 = rng.integers(0, 255, (H, W, 4)).astype(np.uint8)
    formats.write_png(os.path.join(d, "poisson0.png"), img0)
    formats.write_png(os.path.join(d, "poisson1.png"), img1)
    formats.write_png(os.path.join(d, "poisson_mask.png"), m)
    yy, xx = np.mgrid[0:H, 0:W]
    base = (127 + 100 * np.sin(xx / 5.0) * np.cos(yy / 7.0)).astype(np.uint8)
    shifted = (127 + 100 * np.sin((xx - 1.3) / 5.0) * np.cos((yy + 0.7) / 7.0)).astype(np.uint8)
    formats.write_png(os.path.join(d, "dogdance0.png"), np.dstack([base] * 3 + [np.full_like(base, 255)]))
    formats.write_png(os.path.join(d, "dogdance1.png"), np.dstack([shifted] * 3 + [np.full_like(base, 255)]))
    v = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    f = np.array([[0, 2, 4], [2, 1, 4], [1, 3, 4], [3, 0, 4], [2, 0, 5], [1, 2, 5], [3, 1, 5], [0, 3, 5]], np.int32)
    formats.write_ply(os.path.join(d, "small_armadillo.ply"), v, f)
    formats.write_mrk(os.path.join(d, "small_armadillo.mrk"), np.array([[1.3, 0.1, 0], [0, 0, -1]], np.float32),
                      np.array([0.1, 0.1], np.float32), np.array([0, 5]))
    pre = os.path.join(d, "shape_from_shading", "default")
    p = np.zeros(39, np.float32)
    p[[0, 1, 3]] = [100.0, 100.0, 1.0]
    p[7:11] = [60.0, 60.0, W / 2, H / 2]
    p[27:36] = [0.3, 0.1, -0.2, 0.05, 0.01, 0.02, -0.03, 0.01, 0.02]
    p.tofile(pre + ".SFSSolverParameters")
    depth = (0.5 + 0.05 * np.sin(xx / 9.0)).astype(np.float32)
    depth[:3, :3] = -np.inf
    formats.write_imagedump(pre + "_targetDepth.imagedump", depth)
    formats.write_imagedump(pre + "_initialUnknown.imagedump", depth)
    formats.write_imagedump(pre + "_targetIntensity.imagedump", (0.4 + 0.1 * np.cos(yy / 4.0)).astype(np.float32))
    formats.write_imagedump(pre + "_maskEdgeMap.imagedump", np.ones((2 * H, W), np.uint8))


def direct_cost(name, data, kind, **kw):
    import torch

    w = problems.load_example(name, data, subdivisions=1 if name == "arap_mesh_deformation" else 0, **kw)
    prm = problems.problem_params(name, w, lambda x: torch.from_numpy(x).cuda())
    s = OptSolver(problems.dims(name, w), os.path.join(ROOT, "energies", name + ".t"), kind)
    s.set_solver_params({"nIterations": 2, "lIterations": 5})
    s.solve(prm)
    return s.cost()


@pytest.mark.parametrize("name,solver", [("image_warping", "--useOpt"), ("poisson_image_editing", "--useOpt"),
                                         ("optical_flow", "--useOptLM"), ("arap_mesh_deformation", "--useOpt"),
                                         ("shape_from_shading", "--useOptLM")])
def test_harness_runs_example(tmp_path, name, solver):
    data = str(tmp_path / "data")
    write_data(data, np.random.default_rng(1))
    out = str(tmp_path / "out")
    buf = io.StringIO()
    with redirect_stdout(buf):
        rc = run([name, "--data", data, "--out", out, "--backend", "backend_cuda", solver,
                  "--nIterations", "2", "--lIterations", "5", "--config", str(tmp_path / "none")])
    assert rc == 0
    txt = buf.getvalue()
    costs = [float(l.split("=")[1]) for l in txt.splitlines() if l.startswith("final cost=")]
    # optical_flow solves its two pyramid levels (coarse first, w_fit 30 then 50)
    assert len(costs) == (2 if name == "optical_flow" else 1)
    kind = "gaussNewtonGPU" if solver == "--useOpt" else "LMGPU"
    assert costs[0] == pytest.approx(direct_cost(name, data, kind), rel=1e-12)
    lines = open(os.path.join(out, "results.csv")).read().splitlines()
    assert lines[0].startswith("Iter, Ceres Error") and len(lines) >= 3
    assert "**Final Costs**" in txt
    assert len(os.listdir(out)) == 2   # results.csv + the example's result file


def test_optical_flow_schedule_matches_the_reference_harness(tmp_path):
    """CombinedSolver::solveAll of examples/optical_flow: level 1 (sigma 5) with w_fit 30,
    then level 0 (sigma 1) from a zero flow (preSingleSolve resets every level) with w_fit
    50, w_reg 0.1; the second logged cost equals that solve run directly."""
    import torch

    data = str(tmp_path / "data")
    write_data(data, np.random.default_rng(1))
    buf = io.StringIO()
    with redirect_stdout(buf):
        run(["optical_flow", "--data", data, "--out", str(tmp_path / "o"), "--backend", "backend_cuda", "--useOpt",
             "--nIterations", "2", "--lIterations", "5", "--config", str(tmp_path / "none")])
    costs = [float(l.split("=")[1]) for l in buf.getvalue().splitlines() if l.startswith("final cost=")]
    w = problems.load_example("optical_flow", data, level=0)
    w["w_fitSqrt"] = float(np.sqrt(np.float32(50.0)))
    prm = problems.problem_params("optical_flow", w, lambda x: torch.from_numpy(x).cuda())
    s = OptSolver(problems.dims("optical_flow", w), os.path.join(ROOT, "energies", "optical_flow.t"))
    s.set_solver_params({"nIterations": 2, "lIterations": 5})
    s.solve(prm)
    assert costs[1] == pytest.approx(s.cost(), rel=1e-12)
