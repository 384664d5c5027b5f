"""The drop-in boundary from C: a C99 program that includes only include/Opt.h (as the
reference's examples include it inside extern "C", examples/shared/OptSolver.h:5-7) and
the HIP runtime's C API for its own device arrays (as the examples use the CUDA runtime,
examples/shared/OptImage.h:49-51,95-105), compiled with gcc, linked with -lopt_amd,
following OptSolver.h:46-106's call sequence. It reproduces the reference's known
answers (examples/test_final_cost.py:61-63) for an image energy (image_warping cat512)
and a graph energy (arap_mesh_deformation small_armadillo: the Graph passed as an int*
edge count plus one int* per vertex slot, NamedParameters.h:35-49), with device arrays
(backend_cuda) and host arrays (backend_cpu, backend_cpu_mt)."""
import os
import re
import subprocess

import numpy as np
import pytest

from tests.reference_inputs import REFERENCE_FINAL_COST, REFERENCE_RTOL, arap_armadillo, image_warping_cat512

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c_caller", "caller.c")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
BACKENDS = ["backend_cuda", "backend_cpu", "backend_cpu_mt"]


@pytest.fixture(scope="module")
def caller(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("c_caller") / "caller")
    libdir = os.path.join(ROOT, "opt_amd")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-O2", "-D__HIP_PLATFORM_AMD__", "-o", out, SRC,
                    "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROCM, "include"),
                    "-L" + libdir, "-lopt_amd", "-Wl,-rpath," + libdir,
                    "-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-Wl,-rpath," + os.path.join(ROCM, "lib")],
                   check=True)
    return out


def test_c_program_compiles_against_opt_h_and_links(caller):
    assert os.path.exists(caller)


def _write_image(path, w):
    with open(path, "wb") as f:
        f.write(np.array([0, w["W"], w["H"]], np.int32).tobytes())
        for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask"):
            f.write(np.ascontiguousarray(w[k], np.float32).tobytes())
        f.write(np.array([w["w_fitSqrt"], w["w_regSqrt"]], np.float32).tobytes())


def _write_graph(path, w):
    with open(path, "wb") as f:
        f.write(np.array([1, w["N"], w["E"]], np.int32).tobytes())
        for k in ("Offset", "Angle", "UrShape", "Constraints"):
            f.write(np.ascontiguousarray(w[k], np.float32).tobytes())
        for k in ("v0", "v1"):
            f.write(np.ascontiguousarray(w[k], np.int32).tobytes())
        f.write(np.array([w["w_fitSqrt"], w["w_regSqrt"]], np.float32).tobytes())


def _run(caller, energy, path, backend):
    r = subprocess.run([caller, os.path.join(ROOT, "energies", energy), path, backend, "1", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    cost = float(re.search(r"final cost=(\S+)", r.stdout).group(1))
    sums = [float(v) for v in re.search(r"unknowns checksum=(\S+) (\S+)", r.stdout).groups()]
    return cost, sums


@pytest.mark.gpu
@pytest.mark.parametrize("backend", BACKENDS)
def test_c_program_reproduces_cat512(caller, tmp_path, backend):
    w = image_warping_cat512()
    path = str(tmp_path / "problem.bin")
    _write_image(path, w)
    cost, sums = _run(caller, "image_warping.t", path, backend)
    ref = REFERENCE_FINAL_COST["image_warping"]
    assert abs(cost - ref) / ref < REFERENCE_RTOL, (cost, ref)
    # the unknowns the program read back moved off their initial values
    assert sums[0] != pytest.approx(float(np.sum(w["Offset"], dtype=np.float64)), rel=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("backend", BACKENDS)
def test_c_program_reproduces_armadillo_graph(caller, tmp_path, backend):
    w = arap_armadillo()
    path = str(tmp_path / "problem.bin")
    _write_graph(path, w)
    cost, sums = _run(caller, "arap_mesh_deformation.t", path, backend)
    ref = REFERENCE_FINAL_COST["arap_mesh_deformation"]
    assert abs(cost - ref) / ref < REFERENCE_RTOL, (cost, ref)
    assert sums[0] != pytest.approx(float(np.sum(w["Offset"], dtype=np.float64)), rel=1e-9)


@pytest.mark.gpu
def test_c_program_backends_agree(caller, tmp_path):
    """Device arrays and host arrays give the same solve (bitwise: the arithmetic is the
    same GPU path)."""
    w = image_warping_cat512()
    path = str(tmp_path / "problem.bin")
    _write_image(path, w)
    outs = [_run(caller, "image_warping.t", path, b) for b in BACKENDS]
    assert outs[1] == outs[0] and outs[2] == outs[0]
