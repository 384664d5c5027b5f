"""The drop-in boundary from C: a C99 program that includes only include/Opt.h (as the
reference's examples include it inside extern "C", examples/shared/OptSolver.h:5-7),
compiled with gcc, linked with -lopt_amd, following OptSolver.h:46-106's call sequence,
reproduces the reference's cat512 known answer (examples/test_final_cost.py:61)."""
import os
import re
import subprocess

import numpy as np
import pytest

from tests.reference_inputs import REFERENCE_FINAL_COST, REFERENCE_RTOL, image_warping_cat512

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c_caller", "caller.c")


@pytest.fixture(scope="module")
def caller(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("c_caller") / "caller")
    libdir = os.path.join(ROOT, "opt_amd")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-O2", "-o", out, SRC, "-I" + os.path.join(ROOT, "include"),
                    "-L" + libdir, "-lopt_amd", "-Wl,-rpath," + libdir], check=True)
    return out


def test_c_program_compiles_against_opt_h_and_links(caller):
    assert os.path.exists(caller)


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["backend_cpu", "backend_cpu_mt"])
def test_c_program_reproduces_cat512(caller, tmp_path, backend):
    w = image_warping_cat512()
    path = str(tmp_path / "problem.bin")
    with open(path, "wb") as f:
        f.write(np.array([w["W"], w["H"]], np.int32).tobytes())
        for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask"):
            f.write(np.ascontiguousarray(w[k], np.float32).tobytes())
        f.write(np.array([w["w_fitSqrt"], w["w_regSqrt"]], np.float32).tobytes())
    r = subprocess.run([caller, os.path.join(ROOT, "energies", "image_warping.t"), path, backend, "1", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    cost = float(re.search(r"final cost=(\S+)", r.stdout).group(1))
    ref = REFERENCE_FINAL_COST["image_warping"]
    assert abs(cost - ref) / ref < REFERENCE_RTOL, (cost, ref)
