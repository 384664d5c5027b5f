"""CPU: the general energy front end (opt_amd/csrc/gen). It runs Opt energy files as Lua,
lowers them to residual templates (classifyexpression, API/src/o.t:2669-2715) and
generates HIP kernels for them (createjtfcentered / createjtjcentered / createcost ...,
o.t:2770-3129), which hiprtc compiles for gfx950 without a device.

Parity here is structural: two spellings of one energy must lower to identical templates
(the pool is hash-consed, so the printed expressions are canonical), the residual counts
match the reference's per-pixel residual layout (generateDumpJ rows), and every energy
the reference ships either lowers and compiles or is refused with the construct named.
Numeric parity of the generated kernels is in tests/test_generic_gpu.py."""
import ctypes
import os

import pytest

from opt_amd import api

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def E(name):
    return os.path.join(ROOT, "energies", name + ".t")


# residual templates per energy = J rows per pixel / vertex (+ per edge for graphs)
@pytest.mark.parametrize("name,count", [
    ("image_warping", 10),            # 4 edges x 2 channels + 2 fit rows (iw_dump_j)
    ("poisson_image_editing", 16),    # 4 edges x 4 channels (pie_dump_j)
    ("arap_mesh_deformation", 6),     # 3 fit rows per vertex + 3 rows per edge
    ("volume_denoise", 7),
    ("curve_smoothing", 7),
    ("intrinsic_image_decomposition", 19),   # 4 x 3 albedo + 4 shading + 3 fit
    ("shape_from_shading", 6),               # fit, 2 shading (through B_I), 3 smoothness
    ("optical_flow", 9),                     # 1 sampled fit + 4 x 2 regularizer rows
])
def test_residual_templates(name, count):
    d = api.generic_describe(E(name))
    assert len(d) == count
    if name == "arap_mesh_deformation":
        assert sum(l.startswith("graph0 ") for l in d) == 3
        # edge rows read Offset(v0), Offset(v1) and the angles of v0 the row's rotation
        # entries use (Rotate3D row z has no gamma)
        assert [l.split()[1] for l in d if l.startswith("graph0 ")] == ["5", "5", "4"]
    else:
        assert all(l.startswith("centred ") for l in d)


@pytest.mark.parametrize("name", ["image_warping", "poisson_image_editing", "arap_mesh_deformation",
                                  "volume_denoise", "curve_smoothing", "intrinsic_image_decomposition",
                                  "shape_from_shading", "optical_flow", "cotangent_mesh_smoothing",
                                  "embedded_mesh_deformation", "robust_nonrigid_alignment",
                                  "volumetric_mesh_deformation"])
def test_generated_source_compiles(name):
    src = api.generic_source(E(name))
    for k in ("gen_jtf", "gen_apply", "gen_cost", "gen_jtf_graph", "gen_apply_graph", "block_reduce_publish"):
        assert k in src
    assert "typedef float T;" in src
    assert "typedef double T;" in api.generic_source(E(name), double=True)
    # graph energies: the 32-bit gather form (plans with arrays below 2 GiB) differs only
    # in the slot reads; generic_compile_check compiles it too
    if "a.gnb[" in src:
        s32 = api.generic_source(E(name), off32=True)
        assert "opt_g32(p + a.uoff[" in s32 and "opt_g32(p + a.uoff[" not in src
    api.generic_compile_check(E(name))


def test_strip_wave_index_form_per_kernel():
    """The strip kernels take the wave index through readfirstlane only when they read no
    two-channel pair windows (codegen.cpp, OPT_AMD_GEN_WIDU=2, the default): image_warping's
    strips (Offset / UrShape pairs) ran 204-206 us with it against 165-166 without,
    shape_from_shading's 139-142 against 146-148."""
    if os.environ.get("OPT_AMD_GEN_WIDU") not in (None, "2"):
        pytest.skip("OPT_AMD_GEN_WIDU overrides the default")
    uni = "readfirstlane((int)opt_xcd_block()"
    iw = api.generic_source(E("image_warping"))
    assert "gen_apply_strip" in iw and "opt_ldm2" in iw and uni not in iw
    sfs = api.generic_source(E("shape_from_shading"))
    assert "gen_apply_strip" in sfs and uni in sfs


@pytest.mark.parametrize("name", ["image_warping", "poisson_image_editing", "arap_mesh_deformation",
                                  "volume_denoise", "curve_smoothing", "intrinsic_image_decomposition",
                                  "shape_from_shading", "optical_flow", "cotangent_mesh_smoothing",
                                  "embedded_mesh_deformation", "robust_nonrigid_alignment",
                                  "volumetric_mesh_deformation"])
def test_dump_j_columns_name_valid_channels(name):
    """saveJToCRS columns are uoff + channels * element + ch with ch < channels (a dangling
    pool reference in the generator once emitted garbage channels after diff() grew the pool)."""
    import re
    src = api.generic_source(E(name))
    cols = re.findall(r"cc\d+\[\d+\] = a\.uoff\[\d+\] \+ (\d+) \* .*? \+ (\d+);", src)
    assert cols
    for ch, c in cols:
        assert int(c) < int(ch), (ch, c)


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


HEAD = 'local W,H = Dim("W",0), Dim("H",1)\nlocal X = Unknown("X", opt_float2,{W,H},0)\n' \
       'local A = Array("A", opt_float2,{W,H},1)\nlocal w = Param("w", float, 2)\n'


def test_lua_constructs_lower_to_identical_templates(tmp_path):
    """Closures, varargs, while / repeat / numeric-for with a step, tables, string keys,
    method-style calls and math on numbers: the same energy as the plain spelling."""
    plain = HEAD + """
Energy(w * (X(0,0) - A(0,0)))
Energy(Select(InBounds(1,0), X(0,0) - X(1,0), 0))
Energy(Select(InBounds(0,1), X(0,0) - X(0,1), 0))
Energy(Select(InBounds(-1,0), X(0,0) - X(-1,0), 0))
"""
    fancy = HEAD + """
local function make_term(scale)
    return function(...)
        local args = {...}
        return scale * (X(0,0) - A(args[1], args[2]))
    end
end
local fit = make_term(w)
Energy(fit(0, 0))
local dirs = { east = {1, 0}, south = {0, 1} }
local order = {"east", "south"}
local i = 1
while i <= #order do
    local d = dirs[order[i]]
    Energy(Select(InBounds(d[1], d[2]), X(0,0) - X(d[1], d[2]), 0))
    i = i + 1
end
local n = 0
repeat n = n + 1 until n >= 3
for k = 3, 1, -2 do
    if k == 1 then
        local dx = math.floor(-1.5) + 1      -- -1
        Energy(Select(InBounds(dx, 0), X(0,0) - X(dx, 0), 0))
    end
end
assert(n == 3 and ("a" .. "b") == "ab", "lua semantics")
"""
    a = api.generic_describe(_write(tmp_path, "plain.t", plain))
    b = api.generic_describe(_write(tmp_path, "fancy.t", fancy))
    assert a == b and len(a) == 2 + 3 * 2


def test_vector_helpers_match_expanded_forms(tmp_path):
    """lib.t helpers (Rotate2D, Dot3 / length, vector indexing v[i] / v(i), All) against
    their expansions."""
    helpers = HEAD + """
local v = X(0,0) - X(1,0)
local r = Rotate2D(X(0,0)(0), A(0,0))
Energy(r[0] - v(1))
Energy(All(greater(A(0,0), 0)) * X(0,0)(0))
"""
    expanded = HEAD + """
local c, s = cos(X(0,0,0)), sin(X(0,0,0))
Energy(c * A(0,0,0) + (-s) * A(0,0,1) - (X(0,0,1) - X(1,0,1)))
Energy(greater(A(0,0,0), 0) * greater(A(0,0,1), 0) * X(0,0,0))
"""
    a = api.generic_describe(_write(tmp_path, "h.t", helpers))
    b = api.generic_describe(_write(tmp_path, "e.t", expanded))
    assert a == b


def test_front_end_errors_name_the_problem(tmp_path):
    with pytest.raises(api.OptError, match="line 3"):
        api.generic_describe(_write(tmp_path, "syntax.t", 'local W = Dim("W", 0)\n'
                                    'local X = Unknown("X", opt_float, {W}, 0)\nEnergy(X(0) + )\n'))
    with pytest.raises(api.OptError, match="derivatives are not defined"):
        api.generic_describe(_write(tmp_path, "s.t", HEAD + "local I = SampledImage(A)\n"
                                    "Energy(A(0,0,0) - I(X(0,0,0), X(0,0,1), 0))\n"))
    with pytest.raises(api.OptError, match="accessed with"):
        api.generic_describe(_write(tmp_path, "n.t", HEAD + "Energy(X(0,0,0,0))\n"))


def _define(path):
    lib = api.load_library()
    ip = api.InitParams()
    ip.backend = b"backend_cuda"
    st = lib.Opt_NewState(ip)
    return lib, st, lib.Opt_ProblemDefine(st, path.encode(), b"gaussNewtonGPU")


def test_define_routes_unrecognised_energies_to_the_front_end(tmp_path):
    for f in (E("volume_denoise"), E("curve_smoothing"),
              _write(tmp_path, "q.t", HEAD + "Energy(X(0,0) * X(0,0) - A(0,0))\n")):
        lib, st, pr = _define(f)
        assert pr, f
        lib.Opt_ProblemDelete(st, pr)
    lib, st, pr = _define(_write(tmp_path, "bad.t", 'local W,H = Dim("W",0), Dim("H",1)\n'
                                 'local X = Unknown("X", opt_float,{W,H},0)\nlocal A = Array("A", opt_float,{W,H},1)\n'
                                 'Energy(X(0,0) - SampledImage(A)(X(0,0), X(0,0)))\n'))
    assert not pr


LOWERED = ["arap_mesh_deformation", "cotangent_mesh_smoothing", "embedded_mesh_deformation", "image_warping",
           "intrinsic_image_decomposition", "poisson_image_editing", "robust_nonrigid_alignment",
           "shape_from_shading", "volumetric_mesh_deformation", "optical_flow"]
REFUSED = {}


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
@pytest.mark.parametrize("name", LOWERED + sorted(REFUSED))
def test_reference_example_energies(name):
    path = os.path.join(REF, "examples", name, name + ".t")
    if name in REFUSED:
        with pytest.raises(api.OptError, match=REFUSED[name]):
            api.generic_source(path)
        return
    d = api.generic_describe(path)
    assert d and all(l.split()[0] in ("centred", "graph0", "graph1", "graph2", "graph3") for l in d)
    api.generic_compile_check(path)


def test_computed_array_gradient_images(tmp_path):
    """ComputedArray (ProblemSpecAD:ComputedImage, o.t:1686-1718): a residual reading it is
    differentiated through its gradient images, its support includes the shifted unknown
    accesses behind them, and its bbox grows by the computed array's own bbox."""
    txt = HEAD + """
local C = ComputedArray("C", {W,H}, X(0,0,0) * X(-1,0,0))
Energy(C(1,0) - A(0,0,0))
"""
    d = api.generic_describe(_write(tmp_path, "c.t", txt))
    assert len(d) == 1
    dom, nsup, ex = d[0].split(" ", 2)
    assert (dom, nsup) == ("centred", "2")      # X(1,0) and X(0,0) through C(1,0)
    src = api.generic_source(_write(tmp_path, "c.t", txt))
    assert "gen_precompute_0" in src and "gen_precompute_1" not in src


@pytest.mark.parametrize("name", ["intrinsic_image_decomposition", "cotangent_mesh_smoothing", "shape_from_shading",
                                  "embedded_mesh_deformation", "robust_nonrigid_alignment",
                                  "volumetric_mesh_deformation", "image_warping", "optical_flow",
                                  "arap_mesh_deformation", "poisson_image_editing"])
def test_our_energy_files_lower_exactly_as_the_reference_files(name):
    """energies/<name>.t (our text) and the reference's examples/<name>/<name>.t produce
    identical residual templates (hash-consed expressions printed canonically)."""
    ref = os.path.join(REF, "examples", name, name + ".t")
    if not os.path.exists(ref):
        pytest.skip("reference checkout not present")
    assert api.generic_describe(E(name)) == api.generic_describe(ref)


@pytest.mark.parametrize("name,kernel", [("image_warping", "gen_apply_strip"), ("poisson_image_editing", "gen_apply_strip"),
                                         ("shape_from_shading", "gen_apply_strip"),
                                         ("intrinsic_image_decomposition", "gen_apply_strip"),
                                         ("optical_flow", "gen_apply_strip"), ("optical_flow:nocache", "gen_apply ")])
def test_apply_variant_rule(monkeypatch, name, kernel):
    """Static choice of the centred apply (codegen.cpp): the register strips for 2-D
    energies without sampled reads in their residuals, else tiles when the energy has many
    residual instances per centred residual. optical_flow's sample is cached per Step as a
    ComputedArray (lua.cpp cache_samples), so it takes the strip too; without the cache
    (OPT_AMD_GEN_SAMPLE_CACHE=0) the data-dependent sample keeps the gather."""
    if name.endswith(":nocache"):
        monkeypatch.setenv("OPT_AMD_GEN_SAMPLE_CACHE", "0")
        name = name.split(":")[0]
    head = api.generic_source(E(name)).splitlines()[0]
    assert head.startswith("// apply: " + kernel)
