"""CPU: the example-harness mirror (opt_amd/harness): data formats, problem builders
against the fixtures the pinned tests use, the results CSV and the option handling."""
import os

import numpy as np
import pytest

from opt_amd.harness import formats, problems, results
from opt_amd.harness.__main__ import parser, read_config, resolve

REF_DATA = "/root/reference/examples/data"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_imagedump_round_trip_and_infinity_clamp(tmp_path):
    a = np.arange(12, dtype=np.float32).reshape(3, 4)
    a[0, 1] = np.inf
    a[2, 3] = -np.inf
    formats.write_imagedump(tmp_path / "a.imagedump", a)
    b = formats.read_imagedump(tmp_path / "a.imagedump")
    assert b.shape == (3, 4) and b[0, 1] == np.finfo(np.float32).max and b[2, 3] == -10000.0
    assert np.isposinf(formats.read_imagedump(tmp_path / "a.imagedump", clamp_infinity=False)[0, 1])
    c = np.random.default_rng(0).integers(0, 255, (5, 2, 3)).astype(np.uint8)
    formats.write_imagedump(tmp_path / "c.imagedump", c)
    assert np.array_equal(formats.read_imagedump(tmp_path / "c.imagedump"), c)
    raw = open(tmp_path / "c.imagedump", "rb").read()
    assert np.frombuffer(raw[:16], np.int32).tolist() == [2, 5, 3, 1]   # width, height, channels, uchar


def test_markers_round_trip(tmp_path):
    c = np.array([[1, 2, 3, 4], [10, 20, 30, 40]], np.int32)
    formats.write_constraints(tmp_path / "x.constraints", c)
    assert np.array_equal(formats.read_constraints(tmp_path / "x.constraints"), c)
    pos = np.array([[0.5, -1.0, 2.0]], np.float32)
    formats.write_mrk(tmp_path / "x.mrk", pos, np.array([0.1], np.float32), np.array([7]))
    p, r, i = formats.read_mrk(tmp_path / "x.mrk")
    assert np.array_equal(p, pos) and i.tolist() == [7] and r[0] == np.float32(0.1)


def octahedron():
    v = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    f = np.array([[0, 2, 4], [2, 1, 4], [1, 3, 4], [3, 0, 4], [2, 0, 5], [1, 2, 5], [3, 1, 5], [0, 3, 5]], np.int32)
    return v, f


def test_meshes(tmp_path):
    v, f = octahedron()
    formats.write_ply(tmp_path / "o.ply", v, f)
    v2, f2 = formats.read_ply(tmp_path / "o.ply")
    assert np.array_equal(v, v2) and np.array_equal(f, f2)
    # binary little endian with an extra vertex property
    head = ("ply\nformat binary_little_endian 1.0\nelement vertex 6\nproperty float x\nproperty float y\n"
            "property float z\nproperty uchar red\nelement face 8\nproperty list uchar int vertex_indices\n"
            "end_header\n").encode()
    vr = np.zeros(6, np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1")]))
    vr["x"], vr["y"], vr["z"] = v[:, 0], v[:, 1], v[:, 2]
    fr = np.zeros(8, np.dtype([("n", "u1"), ("v", "<i4", (3,))]))
    fr["n"], fr["v"] = 3, f
    open(tmp_path / "b.ply", "wb").write(head + vr.tobytes() + fr.tobytes())
    v3, f3 = formats.read_ply(tmp_path / "b.ply")
    assert np.array_equal(v, v3) and np.array_equal(f, f3)
    with open(tmp_path / "o.off", "w") as fh:
        fh.write("OFF\n6 8 12\n" + "".join("%g %g %g\n" % tuple(p) for p in v) +
                 "".join("3 %d %d %d\n" % tuple(t) for t in f))
    v4, f4 = formats.read_off(tmp_path / "o.off")
    assert np.array_equal(v, v4) and np.array_equal(f, f4)


def test_sqrt3_subdivision_counts():
    v, f = octahedron()
    P, und, F = problems.sqrt3_subdivide(v, f)
    assert len(P) == 6 + 8 and len(F) == 3 * len(f) and len(und) == 3 * len(f) + 12
    w = problems.arap(v, f, v[:1], np.array([0]), subdivisions=2)
    assert w["N"] == 14 + 24 and w["E"] == 2 * 3 * w["N"] - 12   # closed triangle mesh: E = 3V - 6


def test_results_csv_matches_save_solver_results(tmp_path):
    gn = [results.SolverIteration(10.0, 1.5), results.SolverIteration(2.5, 0.5)]
    path = results.save_solver_results(str(tmp_path), "_x", [], gn, [], False)
    lines = open(path).read().splitlines()
    assert lines[0].startswith("Iter, Ceres Error, Opt(GN) Error (float),  Opt(LM) Error (float), ")
    assert lines[1] == ", ".join(["0", "%.20e" % 0, "%.20e" % 10.0, "%.20e" % 0, "%.20e" % 0, "%.20e" % 1.5,
                                  "%.20e" % 0, "%.20e" % 0, "%.20e" % 1.5, "%.20e" % 0])
    assert lines[2].split(", ")[2] == "%.20e" % 2.5 and lines[2].split(", ")[8] == "%.20e" % 2.0
    rep = results.report_final_costs("x", True, False, 2.5, 0)
    assert rep.splitlines()[-1] == "%.20e,," % 2.5


def test_options_follow_argparser_and_config(tmp_path):
    cfg = tmp_path / "args.config"
    cfg.write_text("nIterations = 7\nuseOpt=true # comment\nbackend = backend_cuda\n")
    assert read_config(str(cfg))["useOpt"] == "true"
    o = resolve(parser().parse_args(["image_warping", "--config", str(cfg), "--nIterations", "3"]))
    assert o["nIterations"] == 3 and o["useOpt"] and o["backend"] == "backend_cuda" and o["lIterations"] == 1
    o = resolve(parser().parse_args(["poisson_image_editing", "--config", str(tmp_path / "none")]))
    assert o["backend"] == "backend_cpu" and not o["useOpt"] and o["stride"] == 1   # ArgParser.h defaults


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference checkout not present")
def test_builders_from_reference_data_match_fixtures():
    from tests import reference_inputs as ri

    a = problems.load_example("image_warping", REF_DATA)
    b = ri.image_warping_cat512()
    for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask"):
        assert np.array_equal(a[k], b[k])
    a = problems.load_example("optical_flow", REF_DATA, stride=16)
    b = ri.optical_flow_dogdance()
    for k in ("I", "I_hat", "I_hat_dx", "I_hat_dy"):
        assert np.array_equal(a[k], b[k])
    a = problems.load_example("arap_mesh_deformation", REF_DATA)
    b = ri.arap_armadillo()
    for k in ("Offset", "Constraints", "v0", "v1"):
        assert np.array_equal(a[k], b[k])
    a = problems.load_example("shape_from_shading", REF_DATA)
    z = np.load(os.path.join(GOLDEN, "sfs_default.npz"))
    assert np.array_equal(a["params"], z["params"]) and np.array_equal(a["X"], z["X0"].reshape(-1))
    assert np.array_equal(a["edgeMaskC"], z["edgeMaskC"].reshape(-1))
    a = problems.load_example("poisson_image_editing", REF_DATA)
    assert a["X"].shape == (4 * a["W"] * a["H"],) and set(np.unique(a["M"])) <= {0.0, 255.0}
