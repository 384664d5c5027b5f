"""Pack the inputs of the reference's own end-to-end cost test into fixtures.

The reference's examples/test_final_cost.py runs every example at a small size with
nIterations = lIterations = 1 (examples/shared/ArgParser.h defaults, the example's
args.config) and checks the "final cost=" the solver logs (Opt_ProblemCurrentCost,
API/src/solverGPUGaussNewton.t:1903) against CUDA reference costs within 1e-5
relative (test_final_cost.py:55-66, 116-121). This script extracts the INPUT data
those runs read — data files only, nothing executable — exactly as the example
harness loads them:

  image_warping (examples/image_warping/src/main.cpp:92-183, file = 1, stride = 1):
    cat512_mask.png red channel (the Mask), cat512.constraints (marker list).
    The harness builds Offset = UrShape = (x, y), Angle = 1e-5, the border pins and
    the Constraints image from these (CombinedSolver.h:168-219); tests/reference_inputs.py
    restates that construction.

  optical_flow (examples/optical_flow/src/main.cpp:33-80, file = 1, stride = 16 as
    test_final_cost.py:78 sets): the RGB pixels of dogdance0.png / dogdance1.png at
    (16 i, 16 j). The grayscale conversion, the two Gaussian pyramid levels and the
    derivative images are restated in tests/reference_inputs.py.

  arap_mesh_deformation (examples/arap_mesh_deformation/src/main.cpp:17-70): the vertex
    positions and triangles of small_armadillo.ply (binary PLY) and its marker file
    small_armadillo.mrk (x y z radius vertex-index per marker). The harness's one
    sqrt(3) subdivision (OpenMesh Sqrt3T) and graph construction are restated in
    tests/reference_inputs.py.

  cotangent_mesh_smoothing / volumetric_mesh_deformation (their main.cpp read
    ../data/head.ply, numSubdivides 0): head.ply's vertex positions and triangles.

  embedded_mesh_deformation (main.cpp:17-45): raptor_simplify2k.off (positions,
    triangles) and raptor_simplify2k.mrk (markers).

  intrinsic_image_decomposition (main.cpp:19-40, stride 12 as test_final_cost.py:85
    sets): the RGB pixels of ye_high2.png at (12 x, 12 y).

  robust_nonrigid_alignment (main.cpp, CombinedSolver.h): squat_source.obj (positions,
    triangles), squat_tetmesh.ele (the tetrahedra the graph is built from) and the first
    target of squat_target/ in directory order (the first solve).

The problem construction of each (harness mirror, opt_amd/harness/problems.py) runs on
these at test time.

Data licence: public domain (cat512*), Middlebury flow data set (dogdance*), Stanford
3D Scanning Repository, research use with credit (small_armadillo*, head, raptor),
examples/data/copyright.txt.

    python tests/golden/make_reference_fixtures.py /root/reference
"""
import os
import sys

import numpy as np
from PIL import Image


def main(ref):
    data = os.path.join(ref, "examples", "data")
    here = os.path.dirname(os.path.abspath(__file__))
    mask = np.array(Image.open(os.path.join(data, "cat512_mask.png")))[..., 0].astype(np.uint8)   # .x of RGBA
    with open(os.path.join(data, "cat512.constraints")) as f:
        tok = f.read().split()
    n = int(tok[0])
    cons = np.array([int(t) for t in tok[1:1 + 4 * n]], np.int32).reshape(n, 4)
    out = os.path.join(here, "iw_cat512.npz")
    np.savez_compressed(out, mask=mask, constraints=cons)
    print(out, mask.shape, cons.shape)
    stride = 16
    rgb = []
    for name in ("dogdance0.png", "dogdance1.png"):
        a = np.array(Image.open(os.path.join(data, name)).convert("RGB"))
        H, W = a.shape[0] // stride, a.shape[1] // stride
        rgb.append(a[: H * stride: stride, : W * stride: stride].copy())
    out = os.path.join(here, "of_dogdance_s16.npz")
    np.savez_compressed(out, src=rgb[0], tar=rgb[1], stride=stride)
    print(out, rgb[0].shape)
    raw = open(os.path.join(data, "small_armadillo.ply"), "rb").read()
    head, body = raw.split(b"end_header\n", 1)
    nv = int(head.split(b"element vertex ")[1].split()[0])
    nf = int(head.split(b"element face ")[1].split()[0])
    verts = np.frombuffer(body[: 12 * nv], np.float32).reshape(nv, 3).copy()
    rec = np.dtype([("n", np.uint8), ("v", "<i4", (3,))])
    fr = np.frombuffer(body[12 * nv: 12 * nv + rec.itemsize * nf], rec)
    assert np.all(fr["n"] == 3)
    faces = fr["v"].astype(np.int32).copy()
    tok = open(os.path.join(data, "small_armadillo.mrk")).read().split()
    nm = int(tok[0])
    mk = np.array([float(t) for t in tok[1:1 + 5 * nm]], np.float64).reshape(nm, 5)
    out = os.path.join(here, "arap_armadillo.npz")
    np.savez_compressed(out, verts=verts, faces=faces, marker_pos=mk[:, :3].astype(np.float32),
                        marker_idx=mk[:, 4].astype(np.int32))
    print(out, verts.shape, faces.shape, mk.shape)
    sys.path.insert(0, os.path.dirname(os.path.dirname(here)))
    from opt_amd.harness import formats
    v, f = formats.read_ply(os.path.join(data, "head.ply"))
    out = os.path.join(here, "mesh_head.npz")
    np.savez_compressed(out, verts=v, faces=f)
    print(out, v.shape, f.shape)
    v, f = formats.read_off(os.path.join(data, "raptor_simplify2k.off"))
    pos, _, idx = formats.read_mrk(os.path.join(data, "raptor_simplify2k.mrk"))
    out = os.path.join(here, "mesh_raptor2k.npz")
    np.savez_compressed(out, verts=v, faces=f, marker_pos=pos, marker_idx=idx)
    print(out, v.shape, f.shape, pos.shape)
    stride = 12
    a = np.array(Image.open(os.path.join(data, "ye_high2.png")).convert("RGB"))
    H, W = a.shape[0] // stride, a.shape[1] // stride
    out = os.path.join(here, "iid_ye_s12.npz")
    np.savez_compressed(out, rgb=a[: H * stride: stride, : W * stride: stride].copy(), stride=stride)
    print(out, (H, W))
    # robust_nonrigid_alignment's first solve (the one test_final_cost.py's 66.784683 is
    # taken from): the source mesh, its tetrahedra and the first target in directory order
    sv, sf = formats.read_obj(os.path.join(data, "squat_source.obj"))
    first = sorted(os.listdir(os.path.join(data, "squat_target")))[0]
    tv, tf = formats.read_obj(os.path.join(data, "squat_target", first))
    te = formats.read_ele(os.path.join(data, "squat_tetmesh.ele"))
    out = os.path.join(here, "squat_first.npz")
    np.savez_compressed(out, src_verts=sv, src_faces=sf, tets=te, tgt_verts=tv, tgt_faces=tf, target=first)
    print(out, sv.shape, te.shape, first)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
