"""Problem construction of the reference's examples, from their data files.

Each builder restates what the example's main.cpp / CombinedSolver.h does with the files
(cited per function) and returns a dict of numpy arrays and scalars; `problem_params`
orders them by the declared indices of the matching energy in energies/ (the
reference's NamedParameters packing, examples/shared/NamedParameters.h:35-49).
"""
from __future__ import annotations

import os

import numpy as np

from . import formats

f32 = np.float32


# --------------------------------------------------------------- image_warping
def image_warping(mask: np.ndarray, constraints: np.ndarray, alpha: float = 1.0) -> dict:
    """examples/image_warping/src/main.cpp:92-183 and CombinedSolver.h:116-219: Offset =
    UrShape = (x, y), Angle = 1e-5, Mask = the mask image's red channel, Constraints =
    (-1, -1) except the marker targets (blended by alpha, setConstraintImage :199-219) and
    every border pixel pinned to itself, both only where Mask == 0; later markers overwrite
    earlier ones. w_fit = 100, w_reg = 0.01, square-rooted (:130-134)."""
    m = np.asarray(mask).astype(np.float32)
    H, W = m.shape
    cons = [list(map(int, c)) for c in constraints]
    for y in range(H):
        for x in range(W):
            if y == 0 or x == 0 or y == H - 1 or x == W - 1:
                cons.append([x, y, x, y])
    C = np.full((H, W, 2), -1.0, np.float32)
    a = f32(alpha)
    for x, y, nx, ny in cons:
        if m[y, x] == 0:
            C[y, x, 0] = (f32(1) - a) * f32(x) + a * f32(nx)
            C[y, x, 1] = (f32(1) - a) * f32(y) + a * f32(ny)
    ys, xs = np.mgrid[0:H, 0:W]
    U = np.stack([xs, ys], -1).astype(np.float32)
    return {
        "W": W, "H": H,
        "Offset": U.reshape(-1).copy(),
        "Angle": np.full(W * H, 1e-5, np.float32),
        "UrShape": U.reshape(-1).copy(),
        "Constraints": C.reshape(-1),
        "Mask": m.reshape(-1),
        "w_fitSqrt": float(np.sqrt(f32(100.0), dtype=f32)),
        "w_regSqrt": float(np.sqrt(f32(0.01), dtype=f32)),
    }


# ---------------------------------------------------------------- optical_flow
def filter_gaussian(img: np.ndarray, sigma: float) -> np.ndarray:
    """ImageHelper::filterGaussian (examples/optical_flow/src/ImageHelper.h:69-113): radius
    ceil(2 sigma), weights exp(-x^2 / (2 sigma^2)), renormalised at the borders, rows
    then columns, float arithmetic in the harness's order."""
    R = int(np.ceil(f32(2.0) * f32(sigma)))
    ker = [f32(np.exp(-(f32(i) * f32(i)) / (f32(2.0) * f32(sigma) * f32(sigma)))) for i in range(R + 1)]

    def one_dir(a, axis):
        out = np.zeros_like(a)
        n = a.shape[axis]
        for i in range(n):
            v = np.zeros(a.shape[1 - axis], f32)
            wsum = f32(0)
            for k in range(-R, R + 1):
                ik = i + k
                if 0 <= ik < n:
                    v = v + ker[abs(k)] * (a[:, ik] if axis == 1 else a[ik, :])
                    wsum = wsum + ker[abs(k)]
            if wsum > 0:
                v = v / wsum
            if axis == 1:
                out[:, i] = v
            else:
                out[i, :] = v
        return out

    return one_dir(one_dir(np.asarray(img).astype(f32), 1), 0)


def derivative(img: np.ndarray, axis: int) -> np.ndarray:
    """computeDU / computeDV (examples/optical_flow/src/CombinedSolver.h:143-170): 3x3
    difference / 8, zero border."""
    H, W = img.shape
    res = np.zeros_like(img)
    for j in range(1, H - 1):
        for i in range(1, W - 1):
            if axis == 0:
                d = (-img[j - 1, i - 1] - img[j, i - 1] - img[j + 1, i - 1]
                     + img[j - 1, i + 1] + img[j, i + 1] + img[j + 1, i + 1])
            else:
                d = (-img[j - 1, i - 1] - img[j - 1, i] - img[j - 1, i + 1]
                     + img[j + 1, i - 1] + img[j + 1, i] + img[j + 1, i + 1])
            res[j, i] = d / f32(8.0)
    return res


def grayscale(rgb: np.ndarray) -> np.ndarray:
    """mLib convertToGrayscale: (0.299 r + 0.587 g + 0.114 b) / 255 in float."""
    r, g, b = (rgb[..., c].astype(f32) for c in range(3))
    return (f32(0.299) * r + f32(0.587) * g + f32(0.114) * b) / f32(255.0)


def optical_flow(src_rgb: np.ndarray, tar_rgb: np.ndarray, level: int = 1) -> dict:
    """examples/optical_flow/src/main.cpp:33-80 and CombinedSolver.h:20-130: grayscale,
    pyramid level `level` filtered with sigma {1, 5}[level], I_hat_dx / dy by the 3x3
    formula, X = 0; the harness's weights for that level: w_fit = 10 + (50 - 10) / 2 for
    the first (coarse) solve (combinedSolveInit + preNonlinearSolve, :67-88), w_reg = 0.1,
    both square-rooted."""
    sigma = (1.0, 5.0)[level]
    src = filter_gaussian(grayscale(src_rgb), sigma)
    tar = filter_gaussian(grayscale(tar_rgb), sigma)
    H, W = src.shape
    w_fit = f32(10.0) + (f32(50.0) - f32(10.0)) / f32(2.0)
    return {
        "W": W, "H": H,
        "X": np.zeros(2 * W * H, f32),
        "I": src.reshape(-1).copy(),
        "I_hat": tar.reshape(-1).copy(),
        "I_hat_dx": derivative(tar, 0).reshape(-1).copy(),
        "I_hat_dy": derivative(tar, 1).reshape(-1).copy(),
        "w_fitSqrt": float(np.sqrt(w_fit, dtype=f32)),
        "w_regSqrt": float(np.sqrt(f32(0.1), dtype=f32)),
    }


# ------------------------------------------------------- arap_mesh_deformation
def sqrt3_subdivide(verts: np.ndarray, faces: np.ndarray):
    """One OpenMesh Sqrt3T step on a closed triangle mesh
    (examples/external/OpenMesh/.../Uniform/Sqrt3T.hh:165-273): old vertices relaxed to
    (1 - a_n) p + (a_n / n) sum(neighbours), a_n = (4 - 2 cos(2 pi / n)) / 9 (float
    weights from double, compute_weight :279-293); one new vertex per face at the
    centroid, indexed after the old ones in face order; every old edge flipped, i.e.
    replaced by the edge between the centroids of its two faces. Returns (positions,
    undirected edges, faces)."""
    nv, nf = len(verts), len(faces)
    nbrs = [set() for _ in range(nv)]
    edge_faces = {}
    for fi, (a, b, c) in enumerate(faces):
        for u, v in ((a, b), (b, c), (c, a)):
            nbrs[u].add(v)
            nbrs[v].add(u)
            edge_faces.setdefault((min(u, v), max(u, v)), []).append(fi)
    if not all(len(f) == 2 for f in edge_faces.values()):
        raise ValueError("sqrt(3) subdivision expects a closed triangle mesh")
    new = np.zeros((nv + nf, 3), f32)
    for v in range(nv):
        n = len(nbrs[v])
        alpha = f32((4.0 - 2.0 * np.cos(2.0 * np.pi / float(f32(n)))) / 9.0)
        w1, w2 = f32(1) - alpha, alpha / f32(n)
        pos = np.zeros(3, f32)
        for u in sorted(nbrs[v]):
            pos = pos + verts[u]
        new[v] = pos * w2 + w1 * verts[v]
    third = f32(1.0 / 3.0)
    for fi, (a, b, c) in enumerate(faces):
        new[nv + fi] = ((verts[a] + verts[b]) + verts[c]) * third
    edges = [(nv + fi, int(v)) for fi, f in enumerate(faces) for v in f]
    edges += [(nv + f[0], nv + f[1]) for f in edge_faces.values()]
    # the new triangles: each flipped edge (a, b) between faces f, g gives (a, c_f, c_g)
    # and (b, c_g, c_f) (orientation is irrelevant to the energy)
    new_faces = []
    for (a, b), (fa, fb) in edge_faces.items():
        new_faces.append((a, nv + fb, nv + fa))
        new_faces.append((b, nv + fa, nv + fb))
    return new, edges, np.array(new_faces, np.int32)


def mesh_edges(faces: np.ndarray):
    """Undirected edges of a polygon mesh."""
    e = set()
    for f in faces:
        for i in range(len(f)):
            u, v = int(f[i]), int(f[(i + 1) % len(f)])
            e.add((min(u, v), max(u, v)))
    return sorted(e)


def arap(verts, faces, marker_pos, marker_idx, subdivisions: int = 1) -> dict:
    """examples/arap_mesh_deformation/src/main.cpp:17-70 and CombinedSolver.h:16-170: the
    mesh subdivided `subdivisions` times by sqrt(3) (the harness raises numSubdivides to
    1), the graph = every mesh edge in both directions grouped by head vertex
    (initializeConnectivity + createGraphFromNeighborLists, OptGraph.h:78-90), Offset =
    UrShape = positions, Angle = 0.1, Constraints = marker targets on the marker vertices
    and -inf elsewhere, w_fit = 4, w_reg = 1 (square-rooted)."""
    P = np.asarray(verts, np.float32)
    F = np.asarray(faces, np.int32)
    und = None
    for _ in range(subdivisions):
        P, und, F = sqrt3_subdivide(P, F)
    if und is None:
        und = mesh_edges(F)
    N = len(P)
    und = np.array(und, np.int64)
    directed = np.concatenate([und, und[:, ::-1]])
    directed = directed[np.lexsort((directed[:, 1], directed[:, 0]))]
    C = np.full((N, 3), -np.inf, np.float32)
    for pos, idx in zip(marker_pos, marker_idx):
        C[idx] = pos
    return {
        "Offset": P.reshape(-1).copy(),
        "Angle": np.full(3 * N, 0.1, np.float32),
        "UrShape": P.reshape(-1).copy(),
        "Constraints": C.reshape(-1),
        "v0": np.ascontiguousarray(directed[:, 0].astype(np.int32)),
        "v1": np.ascontiguousarray(directed[:, 1].astype(np.int32)),
        "w_fitSqrt": float(np.sqrt(f32(4.0))),
        "w_regSqrt": float(np.sqrt(f32(1.0))),
        "N": N,
        "E": int(directed.shape[0]),
        "faces": F,
    }


# ------------------------------------------------------- poisson_image_editing
def poisson_image_editing(image0: np.ndarray, image1: np.ndarray, mask: np.ndarray, stride: int = 1) -> dict:
    """examples/poisson_image_editing/src/main.cpp:44-97 and CombinedSolver.h:66-91:
    X = image0 and T = image1 sampled at (stride x, stride y) with alpha 255, M = 0
    where the mask's red channel is 255 (solve) and 255 elsewhere. (The harness samples
    the already-strided mask at (stride x, stride y) again, out of bounds for stride > 1,
    main.cpp:95-101; the mask is sampled once here.)"""
    H, W = image0.shape[0] // stride, image0.shape[1] // stride
    X = image0[: H * stride: stride, : W * stride: stride].astype(np.float32).copy()
    T = image1[: H * stride: stride, : W * stride: stride].astype(np.float32).copy()
    X[..., 3] = 255.0
    T[..., 3] = 255.0
    m = mask[: H * stride: stride, : W * stride: stride, 0]
    M = np.where(m == 255, 0.0, 255.0).astype(np.float32)
    return {"W": W, "H": H, "X": X.reshape(-1), "T": T.reshape(-1), "M": M.reshape(-1)}


# ---------------------------------------------------------- shape_from_shading
def shape_from_shading(sfs_params: dict, X0, D, Im, mask_edge) -> dict:
    """examples/shape_from_shading/src/SFSSolverInput.h + CombinedSolver.h: parameters
    w_p = weightFitting, w_s = weightRegularizer, w_g = weightShading, f_x, f_y, u_x, u_y,
    L_1..L_9 (energy indices 0-15); X = initial unknown, D_i target depth, Im target
    intensity, the edge mask image = the row mask stacked over the column mask."""
    p = sfs_params["raw"]
    params = np.concatenate([p[[0, 1, 3, 7, 8, 9, 10]], p[27:36]]).astype(np.float32)
    D = np.asarray(D, np.float32)
    H, W = D.shape
    mask_edge = np.asarray(mask_edge)
    return {"W": W, "H": H, "params": params, "X": np.asarray(X0, np.float32).reshape(-1).copy(),
            "D_i": D.reshape(-1).copy(), "Im": np.asarray(Im, np.float32).reshape(-1).copy(),
            "edgeMaskR": np.ascontiguousarray(mask_edge[:H]).reshape(-1).astype(np.uint8),
            "edgeMaskC": np.ascontiguousarray(mask_edge[H:2 * H]).reshape(-1).astype(np.uint8)}


# --------------------------------------------------------- from the data folder
FILES = {  # file = 1 / 2 as the examples' main.cpp choose
    "image_warping": {1: ("cat512_mask.png", "cat512.constraints"), 2: ("cat4096_mask.png", "cat4096.constraints")},
    "poisson_image_editing": {1: ("poisson0.png", "poisson1.png", "poisson_mask.png")},
    "optical_flow": {1: ("dogdance0.png", "dogdance1.png")},
    "arap_mesh_deformation": {1: ("small_armadillo.ply", "small_armadillo.mrk"),
                              2: ("raptor_simplify2k.off", "raptor_simplify2k.mrk")},
    "shape_from_shading": {1: ("shape_from_shading/default",)},
}


def load_example(name: str, data: str, file: int = 1, stride: int = 1, level: int = 1,
                 subdivisions: int = 1, alpha: float = 1.0) -> dict:
    """Build example `name`'s problem from the reference's examples/data folder."""
    fs = [os.path.join(data, f) for f in FILES[name][file]]
    if name == "image_warping":
        return image_warping(formats.read_png(fs[0])[..., 0], formats.read_constraints(fs[1]), alpha)
    if name == "poisson_image_editing":
        return poisson_image_editing(*(formats.read_png(f) for f in fs), stride=stride)
    if name == "optical_flow":
        src, tar = (formats.read_png(f)[:, :, :3] for f in fs)
        H, W = src.shape[0] // stride, src.shape[1] // stride   # main.cpp:33-80: pixel (stride i, stride j)
        return optical_flow(src[: H * stride: stride, : W * stride: stride],
                            tar[: H * stride: stride, : W * stride: stride], level)
    if name == "arap_mesh_deformation":
        v, f = formats.read_ply(fs[0]) if fs[0].endswith(".ply") else formats.read_off(fs[0])
        pos, _, idx = formats.read_mrk(fs[1])
        return arap(v, f, pos, idx, subdivisions)
    if name == "shape_from_shading":
        pre = fs[0]
        return shape_from_shading(formats.read_sfs_parameters(pre + ".SFSSolverParameters"),
                                  formats.read_imagedump(pre + "_initialUnknown.imagedump"),
                                  formats.read_imagedump(pre + "_targetDepth.imagedump"),
                                  formats.read_imagedump(pre + "_targetIntensity.imagedump"),
                                  formats.read_imagedump(pre + "_maskEdgeMap.imagedump"))
    raise KeyError(name)


def dims(name: str, w: dict):
    return [w["N"], w["E"]] if name == "arap_mesh_deformation" else [w["W"], w["H"]]


def problem_params(name: str, w: dict, conv=lambda a: a, double: bool = False) -> list:
    """problemparams in the declared-index order of energies/<name>.t; `conv` maps each
    array (e.g. to a device tensor); unknowns in fp64 when `double`."""
    ut = np.float64 if double else np.float32
    U = lambda k: conv(np.ascontiguousarray(w[k].astype(ut)))  # noqa: E731
    A = lambda k: conv(np.ascontiguousarray(w[k]))  # noqa: E731
    if name == "image_warping":
        return [U("Offset"), U("Angle"), A("UrShape"), A("Constraints"), A("Mask"), w["w_fitSqrt"], w["w_regSqrt"]]
    if name == "poisson_image_editing":
        return [U("X"), A("T"), A("M")]
    if name == "optical_flow":
        return [w["w_fitSqrt"], w["w_regSqrt"], U("X"), A("I"), A("I_hat"), A("I_hat_dx"), A("I_hat_dy")]
    if name == "arap_mesh_deformation":
        return [w["w_fitSqrt"], w["w_regSqrt"], U("Offset"), U("Angle"), A("UrShape"), A("Constraints"), None,
                A("v0"), A("v1")]
    if name == "shape_from_shading":
        return [float(v) for v in w["params"]] + [U("X"), A("D_i"), A("Im"), A("edgeMaskR"), A("edgeMaskC")]
    raise KeyError(name)


# index of the (first) unknown in problem_params, for reading results back
UNKNOWN_INDEX = {"image_warping": 0, "poisson_image_editing": 0, "optical_flow": 2,
                 "arap_mesh_deformation": 2, "shape_from_shading": 16}
