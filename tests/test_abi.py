"""CPU: the C-ABI library loads, exports every declared symbol, and its front end
reads the energy files (no device work: plans are only created on a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from opt_amd import api
from tests.conftest import gpu_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def header_symbols():
    names = []
    for h in ("Opt.h", "opt_amd.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names += re.findall(r"\b((?:Opt|OptAMD)_[A-Za-z]+)\s*\(", txt)
    return sorted(set(names))


def test_struct_layout():
    assert ctypes.sizeof(api.InitParams) == 44


def test_library_exports_every_header_symbol():
    lib = api.load_library()
    declared = header_symbols()
    assert "Opt_ProblemSolve" in declared and len(declared) >= 10 + 12
    out = subprocess.run(["nm", "-D", "--defined-only", api.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT\s+(\S+)", out))
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert sorted(api.EXPORTED_SYMBOLS) == declared
    for s in declared:
        assert hasattr(lib, s)


def _define(path, kind="gaussNewtonGPU"):
    lib = api.load_library()
    ip = api.InitParams()
    ip.backend = b"backend_cuda"
    st = lib.Opt_NewState(ip)
    assert st
    return lib, st, lib.Opt_ProblemDefine(st, path.encode(), kind.encode())


@pytest.mark.parametrize("name", ["image_warping", "poisson_image_editing", "optical_flow"])
def test_define_accepts_our_energy_files(energy, name):
    lib, st, pr = _define(energy(name))
    assert pr
    lib.Opt_ProblemDelete(st, pr)


def test_define_rejects_bad_input(tmp_path):
    lib, st, pr = _define(str(tmp_path / "missing.t"))
    assert not pr
    bad = tmp_path / "bad.t"
    bad.write_text('local W,H = Dim("W",0), Dim("H",1)\nlocal X = Unknown("X", opt_float,{W,H},0)\n'
                   'Energy(X(0,0)*X(0,0) +)\n')
    lib, st, pr = _define(str(bad))
    assert not pr  # neither a family nor a lowerable energy: nil, as problemPlan on error
    lib, st, pr = _define(str(tmp_path / "missing.t"), kind="notASolver")
    assert not pr


def test_new_state_rejects_unknown_backend():
    lib = api.load_library()
    ip = api.InitParams()
    ip.backend = b"backend_tpu"
    assert not lib.Opt_NewState(ip)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
@pytest.mark.parametrize("rel,kind", [
    ("examples/image_warping/image_warping.t", "gaussNewtonGPU"),
    ("examples/poisson_image_editing/poisson_image_editing.t", "gaussNewtonGPU"),
    ("examples/shape_from_shading/shape_from_shading.t", "LMGPU"),
    ("examples/arap_mesh_deformation/arap_mesh_deformation.t", "gaussNewtonGPU"),
    ("examples/optical_flow/optical_flow.t", "LMGPU"),
])
def test_define_reads_reference_energy_files(rel, kind):
    lib, st, pr = _define(os.path.join(REF, rel), kind)
    assert pr, rel


@pytest.mark.skipif(gpu_available(), reason="checks the no-device path")
def test_plan_without_device_returns_null(energy):
    lib, st, pr = _define(energy("image_warping"))
    dims = (ctypes.c_uint * 2)(64, 32)
    assert not lib.Opt_ProblemPlan(st, pr, dims)
