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


# ------------------------------------------------------ meshes: neighbour fans
def vertex_fans(faces: np.ndarray, nv: int):
    """Each vertex's neighbours in the cyclic order of its triangle fan, as OpenMesh's
    vertex-vertex circulator visits them (the examples' initializeConnectivity loops).
    Only the cyclic order matters to the energies built from it (prev / next of each
    neighbour), not the start or the direction. A boundary vertex's fan is open: its
    neighbours run from one boundary neighbour to the other and close cyclically."""
    succ = [dict() for _ in range(nv)]
    for f in np.asarray(faces, np.int64):
        for i in range(len(f)):
            v, a, b = int(f[i]), int(f[(i + 1) % len(f)]), int(f[(i - 1) % len(f)])
            succ[v][a] = b      # around v: a then b (the face's orientation)
    fans = []
    for v in range(nv):
        nxt = succ[v]
        if not nxt:
            fans.append([])
            continue
        has_pred = set(nxt.values())
        starts = [a for a in nxt if a not in has_pred]
        if len(starts) > 1:
            raise ValueError("vertex %d is not manifold (%d fan pieces)" % (v, len(starts)))
        a = starts[0] if starts else min(nxt)
        ring = [a]
        while a in nxt and nxt[a] != ring[0]:
            a = nxt[a]
            ring.append(a)
        if len(set(ring)) != len(ring) or len(ring) != len(set(nxt) | has_pred):
            raise ValueError("vertex %d: inconsistent fan" % v)
        fans.append(ring)
    return fans


# ---------------------------------------------------- cotangent_mesh_smoothing
def cotangent_mesh_smoothing(verts, faces) -> dict:
    """examples/cotangent_mesh_smoothing/src/main.cpp:17-70 and CombinedSolver.h:16-160:
    X = A = the vertex positions (float3); the graph has one edge per (vertex, fan
    neighbour) as (head, curr, prev, next) with prev / next the cyclic fan neighbours of
    curr (initializeConnectivity :78-125, grouped by head); w_fit = 1, w_reg = 0.5,
    square-rooted (main.cpp:57-58)."""
    P = np.asarray(verts, np.float32)
    fans = vertex_fans(faces, len(P))
    e = [[], [], [], []]
    for h, ring in enumerate(fans):
        n = len(ring)
        for i, c in enumerate(ring):
            e[0].append(h)
            e[1].append(c)
            e[2].append(ring[(i + n - 1) % n])
            e[3].append(ring[(i + 1) % n])
    v = [np.array(x, np.int32) for x in e]
    return {"N": len(P), "E": len(v[0]), "X": P.reshape(-1).copy(), "A": P.reshape(-1).copy(),
            "v0": v[0], "v1": v[1], "v2": v[2], "v3": v[3],
            "w_fitSqrt": float(np.sqrt(f32(1.0))), "w_regSqrt": float(np.sqrt(f32(0.5)))}


# --------------------------------------------------- embedded_mesh_deformation
def _rot_axis(axis: str, deg) -> np.ndarray:
    """mLib Matrix3x3::setRotation{X,Y,Z} (float, angle in degrees,
    core-math/matrix3x3.h:126-170; degreesToRadians = x * (PIf / 180), utility.h:18)."""
    rad = f32(deg) * (f32(3.14159265358979323846) / f32(180.0))
    c, s = np.cos(rad, dtype=f32), np.sin(rad, dtype=f32)
    o, z = f32(1), f32(0)
    if axis == "x":
        m = [o, z, z, z, c, -s, z, s, c]
    elif axis == "y":
        m = [c, z, s, z, o, z, -s, z, c]
    else:
        m = [c, -s, z, s, c, z, z, z, o]
    return np.array(m, f32).reshape(3, 3)


def _matmul_f32(a, b):
    """mLib Matrix3x3 product in float, its summation order (matrix3x3.h:256-268)."""
    r = np.zeros((3, 3), f32)
    for i in range(3):
        for j in range(3):
            r[i, j] = (a[i, 0] * b[0, j] + a[i, 1] * b[1, j]) + a[i, 2] * b[2, j]
    return r


def embedded_mesh_deformation(verts, faces, marker_pos, marker_idx) -> dict:
    """examples/embedded_mesh_deformation/src/main.cpp:17-90 and CombinedSolver.h:16-170:
    Offset = UrShape = positions, RotMatrix = rotation(1e-3, 1e-3, 1e-3) degrees
    (yaw/pitch/roll: R_y R_x R_z, row-major) for every vertex, Constraints = marker
    targets (setConstraints(1): (1 - 1) p + 1 t) on the marker vertices and -inf
    elsewhere, the graph = every mesh edge in both directions grouped by head
    (createGraphFromNeighborLists), w_fit = 3, w_reg = 12, w_rot = 5 square-rooted."""
    P = np.asarray(verts, np.float32)
    N = len(P)
    R = _matmul_f32(_matmul_f32(_rot_axis("y", 1e-3), _rot_axis("x", 1e-3)), _rot_axis("z", 1e-3))
    und = np.array(mesh_edges(faces), np.int64)
    directed = np.concatenate([und, und[:, ::-1]])
    directed = directed[np.lexsort((directed[:, 1], directed[:, 0]))]
    C = np.full((N, 3), -np.inf, np.float32)
    for pos, i in zip(marker_pos, marker_idx):
        C[i] = (f32(1) - f32(1)) * P[i] + f32(1) * np.asarray(pos, f32)
    return {"N": N, "E": int(len(directed)), "Offset": P.reshape(-1).copy(),
            "RotMatrix": np.tile(R.reshape(1, 9), (N, 1)).reshape(-1).copy(), "UrShape": P.reshape(-1).copy(),
            "Constraints": C.reshape(-1), "v0": np.ascontiguousarray(directed[:, 0].astype(np.int32)),
            "v1": np.ascontiguousarray(directed[:, 1].astype(np.int32)),
            "w_fitSqrt": float(np.sqrt(f32(3.0))), "w_regSqrt": float(np.sqrt(f32(12.0))),
            "w_rotSqrt": float(np.sqrt(f32(5.0)))}


# ----------------------------------------------- intrinsic_image_decomposition
def intrinsic_image_decomposition(rgb: np.ndarray, stride: int = 1) -> dict:
    """examples/intrinsic_image_decomposition/src/main.cpp:19-40 (pixels (stride x,
    stride y) of the image) and CombinedSolver.h resetGPUMemory: v = rgb / 255,
    intensity = (r + g + b) / 3, i = log2(v + 0.01), r (albedo) = log2(v / intensity +
    0.01), s (shading) = log2(intensity + 0.01), in float; w_fit = 500, w_regAlbedo = 1000,
    w_regShading = 10000 square-rooted, pNorm = 0.8."""
    img = np.asarray(rgb)[..., :3]
    H, W = img.shape[0] // stride, img.shape[1] // stride
    v = img[: H * stride: stride, : W * stride: stride].astype(f32) / f32(255.0)
    inten = ((v[..., 0] + v[..., 1]) + v[..., 2]) / f32(3.0)
    eps = f32(0.01)
    chroma = v / inten[..., None]
    return {"W": W, "H": H,
            "r": np.log2(chroma + eps, dtype=f32).reshape(-1).copy(),
            "i": np.log2(v + eps, dtype=f32).reshape(-1).copy(),
            "s": np.log2(inten + eps, dtype=f32).reshape(-1).copy(),
            "w_fitSqrt": float(np.sqrt(f32(500.0))), "w_regSqrtAlbedo": float(np.sqrt(f32(1000.0))),
            "w_regSqrtShading": float(np.sqrt(f32(10000.0))), "pNorm": float(f32(0.8))}


# ------------------------------------------------- volumetric_mesh_deformation
def volumetric_mesh_deformation(verts, subdivisions: int = 0) -> dict:
    """examples/volumetric_mesh_deformation/src/main.cpp:17-45 and CombinedSolver.h: a
    lattice of (5 (s+1)) x (20 (s+1)) x (5 (s+1)) cells over the mesh's bounding box grown
    by 1e-6 (computeBoundingBox, resetGPUMemory), node (i, j, k) at min + (i, j, k) * delta,
    Angle = 0, Constraints = the node itself on the j = 0 layer, the top layer (j = dims.y)
    rotated by -90 degrees about z around its centre and moved by (2.5, -2.5, 0), -inf
    elsewhere (setConstraints(1)); w_fit = 1, w_reg = 0.05 square-rooted.

    The harness stores node (i, j, k) at i (Y+1)(Z+1) + j (Z+1) + k (getIndex1D), which
    the energy's x-fastest {X+1, Y+1, Z+1} image reads as coordinate (k, j, i): the
    lattice is laid out the same way here (the stencil energy is symmetric under that
    relabelling of axes; positions keep their own x, y, z)."""
    P = np.asarray(verts, np.float32)
    dx, dy, dz = 5 * (subdivisions + 1), 20 * (subdivisions + 1), 5 * (subdivisions + 1)
    mn = P.min(0).astype(f32) - f32(0.000001)
    mx = P.max(0).astype(f32) + f32(0.000001)
    delta = (mx - mn) / np.array([dx, dy, dz], f32)
    nx, ny, nz = dx + 1, dy + 1, dz + 1
    n = nx * ny * nz
    U = np.zeros((n, 3), f32)
    C = np.full((n, 3), -np.inf, f32)
    R = _rot_axis("z", -90.0)
    for i in range(nx):
        for j in range(ny):
            for k in range(nz):
                idx = i * (ny * nz) + j * nz + k
                v = mn + np.array([i, j, k], f32) * delta
                U[idx] = v
                # mat3f::diag(i, j, k) * delta: each row adds two zero products
                vc = mn + np.array([(f32(i) * delta[0] + f32(0) * delta[1]) + f32(0) * delta[2],
                                    (f32(0) * delta[0] + f32(j) * delta[1]) + f32(0) * delta[2],
                                    (f32(0) * delta[0] + f32(0) * delta[1]) + f32(k) * delta[2]], f32)
                if j == 0:
                    C[idx] = vc
                elif j == dy:
                    fd = np.array([f32(dx) / f32(2.0), f32(dy), f32(dz) / f32(2.0)], f32)
                    mid = mn + np.array([(fd[0] * delta[0] + f32(0) * delta[1]) + f32(0) * delta[2],
                                         (f32(0) * delta[0] + fd[1] * delta[1]) + f32(0) * delta[2],
                                         (f32(0) * delta[0] + f32(0) * delta[1]) + fd[2] * delta[2]], f32)
                    d = vc - mid
                    rv = np.array([(R[r, 0] * d[0] + R[r, 1] * d[1]) + R[r, 2] * d[2] for r in range(3)], f32)
                    C[idx] = (rv + mid) + np.array([2.5, -2.5, 0.0], f32)
    return {"W": nz, "H": ny, "D": nx, "Offset": U.reshape(-1).copy(), "Angle": np.zeros(3 * n, f32),
            "UrShape": U.reshape(-1).copy(), "Constraints": C.reshape(-1),
            "w_fitSqrt": float(np.sqrt(f32(1.0))), "w_regSqrt": float(np.sqrt(f32(0.05)))}


# --------------------------------------------------------- from the data folder
FILES = {  # file = 1 / 2 as the examples' main.cpp choose
    "image_warping": {1: ("cat512_mask.png", "cat512.constraints"), 2: ("cat4096_mask.png", "cat4096.constraints")},
    "poisson_image_editing": {1: ("poisson0.png", "poisson1.png", "poisson_mask.png")},
    "optical_flow": {1: ("dogdance0.png", "dogdance1.png")},
    "arap_mesh_deformation": {1: ("small_armadillo.ply", "small_armadillo.mrk"),
                              2: ("raptor_simplify2k.off", "raptor_simplify2k.mrk")},
    "shape_from_shading": {1: ("shape_from_shading/default",)},
    "cotangent_mesh_smoothing": {1: ("head.ply",)},
    "embedded_mesh_deformation": {1: ("raptor_simplify2k.off", "raptor_simplify2k.mrk")},
    "intrinsic_image_decomposition": {1: ("ye_high2.png",)},
    "volumetric_mesh_deformation": {1: ("head.ply",)},
}


def _read_mesh(path):
    return formats.read_ply(path) if path.endswith(".ply") else formats.read_off(path)


def load_example(name: str, data: str, file: int = 1, stride: int = 1, level: int = 1,
                 subdivisions=None, alpha: float = 1.0) -> dict:
    """Build example `name`'s problem from the reference's examples/data folder
    (subdivisions: numSubdivides; default 1 for arap, whose harness raises it to 1, else 0)."""
    if subdivisions is None:
        subdivisions = 1 if name == "arap_mesh_deformation" else 0
    if subdivisions and name in ("cotangent_mesh_smoothing", "embedded_mesh_deformation",
                                 "volumetric_mesh_deformation"):
        raise ValueError(name + ": numSubdivides > 0 is not mirrored (open meshes need OpenMesh's "
                         "boundary sqrt(3) rules)")
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
    if name == "cotangent_mesh_smoothing":
        return cotangent_mesh_smoothing(*_read_mesh(fs[0]))
    if name == "embedded_mesh_deformation":
        v, f = _read_mesh(fs[0])
        pos, _, idx = formats.read_mrk(fs[1])
        return embedded_mesh_deformation(v, f, pos, idx)
    if name == "intrinsic_image_decomposition":
        return intrinsic_image_decomposition(formats.read_png(fs[0]), stride=stride)
    if name == "volumetric_mesh_deformation":
        return volumetric_mesh_deformation(_read_mesh(fs[0])[0], subdivisions=max(0, subdivisions))
    raise KeyError(name)


GRAPH_EXAMPLES = ("arap_mesh_deformation", "cotangent_mesh_smoothing", "embedded_mesh_deformation")


def dims(name: str, w: dict):
    if name in GRAPH_EXAMPLES:
        return [w["N"], w["E"]]
    if name == "volumetric_mesh_deformation":
        return [w["W"], w["H"], w["D"]]
    return [w["W"], w["H"]]


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
    if name == "cotangent_mesh_smoothing":
        return [w["w_fitSqrt"], w["w_regSqrt"], U("X"), A("A"), None, A("v0"), A("v1"), A("v2"), A("v3")]
    if name == "embedded_mesh_deformation":
        return [w["w_fitSqrt"], w["w_regSqrt"], w["w_rotSqrt"], U("Offset"), U("RotMatrix"), A("UrShape"),
                A("Constraints"), None, A("v0"), A("v1")]
    if name == "intrinsic_image_decomposition":
        return [w["w_fitSqrt"], w["w_regSqrtAlbedo"], w["w_regSqrtShading"], w["pNorm"], U("r"), A("i"), U("s")]
    if name == "volumetric_mesh_deformation":
        return [U("Offset"), U("Angle"), A("UrShape"), A("Constraints"), w["w_fitSqrt"], w["w_regSqrt"]]
    raise KeyError(name)


# index of the (first) unknown in problem_params, for reading results back
UNKNOWN_INDEX = {"image_warping": 0, "poisson_image_editing": 0, "optical_flow": 2,
                 "arap_mesh_deformation": 2, "shape_from_shading": 16, "cotangent_mesh_smoothing": 2,
                 "embedded_mesh_deformation": 3, "intrinsic_image_decomposition": 4,
                 "volumetric_mesh_deformation": 0}


# ------------------------------------------------------- robust_nonrigid_alignment
class StdMt19937:
    """std::mt19937 (its init_genrand seeding = numpy's legacy MT19937 seeding)."""

    def __init__(self, seed: int):
        self.bg = np.random.MT19937(0)
        self.bg._legacy_seeding(seed)

    def __call__(self) -> int:
        return int(self.bg.random_raw())


def std_uniform_int(rng, a: int, b: int, lemire: bool = False) -> int:
    """libstdc++ std::uniform_int_distribution<int>(a, b) over a 32-bit engine: the
    downscaling loop of GCC < 11, or (lemire) GCC 11's nearly-divisionless method."""
    r = b - a + 1
    if lemire:
        prod = rng() * r
        low = prod & 0xFFFFFFFF
        if low < r:
            thr = ((1 << 32) - r) % r
            while low < thr:
                prod = rng() * r
                low = prod & 0xFFFFFFFF
        return (prod >> 32) + a
    scaling = 0xFFFFFFFF // r
    past = r * scaling
    while True:
        v = rng()
        if v < past:
            return v // scaling + a


class StdNormal:
    """libstdc++ std::normal_distribution<double>: Marsaglia's polar method (the second
    value saved for the next call) over generate_canonical<double, 53> (two 32-bit draws)."""

    def __init__(self, mean: float, stddev: float):
        self.mean, self.stddev, self.saved = mean, stddev, None

    def __call__(self, rng) -> float:
        if self.saved is not None:
            v, self.saved = self.saved, None
        else:
            def canon():
                s = (rng() + rng() * 4294967296.0) / 18446744073709551616.0
                return s if s < 1.0 else np.nextafter(1.0, 0.0)
            while True:
                x = 2.0 * canon() - 1.0
                y = 2.0 * canon() - 1.0
                r2 = x * x + y * y
                if 0.0 < r2 <= 1.0:
                    break
            mult = np.sqrt(-2.0 * np.log(r2) / r2)
            self.saved = x * mult
            v = y * mult
        return v * self.stddev + self.mean


def mesh_vertex_normals(v: np.ndarray, f: np.ndarray) -> np.ndarray:
    """OpenMesh update_normals(): per face the normalised (p2 - p1) x (p0 - p1), per vertex
    the normalised sum of its faces' normals (float32 as the SimpleMesh's Vec3f)."""
    p0, p1, p2 = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    n = np.cross(p2 - p1, p0 - p1).astype(np.float32)
    ln = np.sqrt((n * n).sum(1, dtype=np.float32))
    n = np.where(ln[:, None] != 0, n / np.where(ln == 0, 1, ln)[:, None], 0).astype(np.float32)
    vn = np.zeros_like(v, dtype=np.float32)
    for k in range(3):
        np.add.at(vn, f[:, k], n)
    lv = np.sqrt((vn * vn).sum(1, dtype=np.float32))
    return np.where(lv[:, None] != 0, vn / np.where(lv == 0, 1, lv)[:, None], 0).astype(np.float32)


def tet_graph(tets: np.ndarray, nv: int):
    """generateOptEdges with tetrahedra (CombinedSolver.h:381-404): every vertex's
    neighbours in its tets as a std::set (ascending), then the directed edges v -> n in
    that order (createGraphFromNeighborLists)."""
    nb = [set() for _ in range(nv)]
    for t in tets.tolist():
        for i in range(4):
            for j in range(1, 4):
                nb[t[i]].add(t[(i + j) % 4])
    v0 = np.array([i for i in range(nv) for _ in nb[i]], np.int32)
    v1 = np.array([n for i in range(nv) for n in sorted(nb[i])], np.int32)
    return v0, v1


def robust_nonrigid_alignment(src_v, src_f, tets, tgt_v, tgt_f, arg_order: str = "rtl",
                              lemire: bool = False, K: int = 20) -> dict:
    """The FIRST solve of the robust_nonrigid_alignment example (the one
    examples/test_final_cost.py's reference cost 66.784683 is taken from): CombinedSolver
    construction (CombinedSolver.h:72-137: average edge length, the mt19937(230948) draws
    of 5 % spurious target indices and their normal(0, 30 x edge length) offsets),
    combinedSolveInit (w_fit = sqrt 10, w_reg = sqrt 64), and preNonlinearSolve(0) on the
    first target (setConstraints, :266-352: per source vertex the K = 20 nearest target
    vertices (nanoflann, exact), the first within 5 edge lengths whose normal is within
    acos 0.7 of the source normal, else -inf; the spurious offsets added; every changed
    constraint's robust weight 1). arg_order: the order C++ evaluated
    make_float3(normal(), normal(), normal())'s arguments ("rtl" = GCC on x86-64)."""
    src_v = np.asarray(src_v, np.float32)
    tgt_v = np.asarray(tgt_v, np.float32)
    N = len(src_v)
    # average edge length (float edge lengths summed in double over the mesh's edges)
    e = np.concatenate([src_f[:, [0, 1]], src_f[:, [1, 2]], src_f[:, [2, 0]]])
    e = np.sort(e, axis=1)
    _, first = np.unique(e[:, 0].astype(np.int64) * N + e[:, 1], return_index=True)
    ue = e[np.sort(first)]
    d = src_v[ue[:, 1]] - src_v[ue[:, 0]]
    lens = np.sqrt((d * d).sum(1, dtype=np.float32)).astype(np.float32)
    avg = float(np.sum(lens.astype(np.float64))) / len(ue)
    # spurious correspondences
    rng = StdMt19937(230948)
    nd = StdNormal(0.0, avg * 30.0)
    spurious, noisy = [], []
    for _ in range(int(np.float32(N) * np.float32(0.05))):
        spurious.append(std_uniform_int(rng, 0, len(tgt_v) - 1, lemire))
        a, b, c = nd(rng), nd(rng), nd(rng)
        noisy.append((c, b, a) if arg_order == "rtl" else (a, b, c))
    noisy = np.array(noisy, np.float32)
    # correspondences of the initial mesh against the first target
    sn = mesh_vertex_normals(src_v, src_f)
    tn = mesh_vertex_normals(tgt_v, tgt_f)
    thr = np.float32(avg) * np.float32(5.0)
    C = np.full((N, 3), -np.inf, np.float32)
    CN = np.zeros((N, 3), np.float32)
    for s0 in range(0, N, 512):
        q = src_v[s0:s0 + 512]
        dd = q[:, None, :] - tgt_v[None, :, :]
        d2 = (dd[..., 0] * dd[..., 0] + dd[..., 1] * dd[..., 1]) + dd[..., 2] * dd[..., 2]
        nn = np.argpartition(d2, K, axis=1)[:, :K]
        for r in range(len(q)):
            cand = nn[r][np.lexsort((nn[r], d2[r, nn[r]]))]
            i = s0 + r
            for t in cand:
                dv = tgt_v[t] - src_v[i]
                dist = np.sqrt(np.float32(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]))
                if dist > thr:
                    break
                if np.float32(tn[t, 0] * sn[i, 0] + tn[t, 1] * sn[i, 1] + tn[t, 2] * sn[i, 2]) > np.float32(0.7):
                    C[i] = tgt_v[t]
                    CN[i] = tn[t]
                    break
    for k, idx in enumerate(spurious):
        if idx < N:
            C[idx] += noisy[k]
    v0, v1 = tet_graph(tets, N)
    return dict(N=N, E=len(v0), w_fitSqrt=float(np.sqrt(np.float32(10.0))), w_regSqrt=float(np.float32(8.0)),
                Offset=src_v.copy(), Angle=np.zeros((N, 3), np.float32), RobustWeights=np.ones(N, np.float32),
                UrShape=src_v.copy(), Constraints=C, ConstraintNormals=CN, v0=v0, v1=v1,
                average_edge_length=avg, spurious=np.array(spurious, np.int64))
