"""Problem inputs of the reference's own end-to-end cost test (examples/test_final_cost.py),
rebuilt from the data fixtures in tests/golden/ exactly as the example harness builds
them, plus the expected final costs that test holds (CUDA reference values,
test_final_cost.py:55-66; compared within 1e-5 relative, :116-121)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# examples/test_final_cost.py:58-66 (CUDA, small size, nIterations = lIterations = 1)
REFERENCE_FINAL_COST = {
    "image_warping": 1774.3405,
    "optical_flow": 0.52119255,     # cost of the first solve (the coarse level, sigma 5)
    "arap_mesh_deformation": 7183.464843,
}
# Not reproducible from the reference's files: poisson_image_editing (its harness reads
# the strided mask at (stride x, stride y) of the already-strided image,
# examples/poisson_image_editing/src/main.cpp:95-101, i.e. out of bounds for the
# test's stride 4), shape_from_shading (no reference value, test_final_cost.py:64).
REFERENCE_RTOL = 1e-5   # test_final_cost.py:121


def image_warping_cat512(alpha=1.0):
    """examples/image_warping/src/main.cpp:92-183 (file = 1, stride = 1) and
    CombinedSolver.h:116-219: Offset = UrShape = (x, y), Angle = 1e-5, Mask = red channel
    of cat512_mask.png, Constraints = (-1, -1) except the marker targets (blended by
    alpha) and every border pixel pinned to itself, both only where Mask == 0; later
    markers overwrite earlier ones. Weights w_fit = 100, w_reg = 0.01 (square-rooted)."""
    z = np.load(os.path.join(GOLDEN, "iw_cat512.npz"))
    m = z["mask"].astype(np.float32)
    H, W = m.shape
    cons = [list(map(int, c)) for c in z["constraints"]]
    for y in range(H):
        for x in range(W):
            if y == 0 or x == 0 or y == H - 1 or x == W - 1:
                cons.append([x, y, x, y])
    C = np.full((H, W, 2), -1.0, np.float32)
    a = np.float32(alpha)
    for x, y, nx, ny in cons:
        if m[y, x] == 0:
            C[y, x, 0] = (np.float32(1) - a) * np.float32(x) + a * np.float32(nx)
            C[y, x, 1] = (np.float32(1) - a) * np.float32(y) + a * np.float32(ny)
    ys, xs = np.mgrid[0:H, 0:W]
    U = np.stack([xs, ys], -1).astype(np.float32)
    return {
        "W": W, "H": H,
        "Offset": U.reshape(-1).copy(),
        "Angle": np.full(W * H, 1e-5, np.float32),
        "UrShape": U.reshape(-1).copy(),
        "Constraints": C.reshape(-1),
        "Mask": m.reshape(-1),
        "w_fitSqrt": float(np.sqrt(np.float32(100.0), dtype=np.float32)),
        "w_regSqrt": float(np.sqrt(np.float32(0.01), dtype=np.float32)),
    }


def _filter_gaussian(img, sigma):
    """ImageHelper::filterGaussian (examples/optical_flow/src/ImageHelper.h:69-113): radius
    ceil(2 sigma), weights exp(-x^2 / (2 sigma^2)), renormalised at the borders, rows
    then columns, float arithmetic in the harness's order."""
    f32 = np.float32
    R = int(np.ceil(f32(2.0) * f32(sigma)))
    ker = [f32(np.exp(-(f32(i) * f32(i)) / (f32(2.0) * f32(sigma) * f32(sigma)))) for i in range(R + 1)]
    H, W = img.shape

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

    return one_dir(one_dir(img.astype(f32), 1), 0)


def _derivative(img, axis):
    """computeDU / computeDV (CombinedSolver.h:143-170): 3x3 difference / 8, zero border"""
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
            res[j, i] = d / np.float32(8.0)
    return res


def optical_flow_dogdance(level=1):
    """examples/optical_flow/src/main.cpp:33-80 (stride 16) and CombinedSolver.h:20-130:
    grayscale (0.299 r + 0.587 g + 0.114 b) / 255 (mLib convertToGrayscale), pyramid
    level `level` filtered with sigma {1, 5}[level], I_hat_dx / dy by the 3x3 formula,
    X = 0. The first solve the harness runs is level 1 with w_fit = 10 + (50 - 10) / 2
    = 30 (combinedSolveInit + preNonlinearSolve, :67-88) and w_reg = 0.1, both square-rooted."""
    f32 = np.float32
    z = np.load(os.path.join(GOLDEN, "of_dogdance_s16.npz"))

    def gray(rgb):
        r, g, b = (rgb[..., c].astype(f32) for c in range(3))
        return (f32(0.299) * r + f32(0.587) * g + f32(0.114) * b) / f32(255.0)

    sigma = (1.0, 5.0)[level]
    src = _filter_gaussian(gray(z["src"]), sigma)
    tar = _filter_gaussian(gray(z["tar"]), sigma)
    H, W = src.shape
    w_fit = f32(10.0) + (f32(50.0) - f32(10.0)) / f32(2.0)
    return {
        "W": W, "H": H,
        "X": np.zeros(2 * W * H, f32),
        "I": src.reshape(-1).copy(),
        "I_hat": tar.reshape(-1).copy(),
        "I_hat_dx": _derivative(tar, 0).reshape(-1).copy(),
        "I_hat_dy": _derivative(tar, 1).reshape(-1).copy(),
        "w_fitSqrt": float(np.sqrt(w_fit, dtype=f32)),
        "w_regSqrt": float(np.sqrt(f32(0.1), dtype=f32)),
    }


def _sqrt3_subdivide(verts, faces):
    """One OpenMesh Sqrt3T step on a closed triangle mesh
    (examples/external/OpenMesh/.../Uniform/Sqrt3T.hh:165-273): old vertices relaxed to
    (1 - a_n) p + (a_n / n) sum(neighbours), a_n = (4 - 2 cos(2 pi / n)) / 9 (float
    weights from double, compute_weight :279-293); one new vertex per face at the
    centroid, indexed after the old ones in face order (add_vertex in faces_begin..end
    order); every old edge flipped, i.e. replaced by the edge between the centroids of
    its two faces. Returns (positions, undirected edges)."""
    f32 = np.float32
    nv, nf = len(verts), len(faces)
    nbrs = [set() for _ in range(nv)]
    edge_faces = {}
    for fi, (a, b, c) in enumerate(faces):
        for u, v in ((a, b), (b, c), (c, a)):
            nbrs[u].add(v)
            nbrs[v].add(u)
            edge_faces.setdefault((min(u, v), max(u, v)), []).append(fi)
    assert all(len(f) == 2 for f in edge_faces.values()), "expects a closed mesh"
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
    return new, edges


def arap_armadillo():
    """examples/arap_mesh_deformation/src/main.cpp:17-70 and CombinedSolver.h:16-170:
    small_armadillo.ply subdivided once by sqrt(3) (numSubdivides is raised to 1), the
    graph = every mesh edge in both directions grouped by head vertex
    (initializeConnectivity + createGraphFromNeighborLists, OptGraph.h:78-90), Offset =
    UrShape = positions, Angle = 0.1, Constraints = marker targets (alpha = 1) on the
    marker vertices and -inf elsewhere, w_fit = 4, w_reg = 1 (square-rooted)."""
    z = np.load(os.path.join(GOLDEN, "arap_armadillo.npz"))
    P, und = _sqrt3_subdivide(z["verts"].astype(np.float32), z["faces"])
    N = len(P)
    und = np.array(und, np.int64)
    directed = np.concatenate([und, und[:, ::-1]])
    directed = directed[np.lexsort((directed[:, 1], directed[:, 0]))]
    C = np.full((N, 3), -np.inf, np.float32)
    for pos, idx in zip(z["marker_pos"], z["marker_idx"]):
        C[idx] = pos
    return {
        "Offset": P.reshape(-1).copy(),
        "Angle": np.full(3 * N, 0.1, np.float32),
        "UrShape": P.reshape(-1).copy(),
        "Constraints": C.reshape(-1),
        "v0": np.ascontiguousarray(directed[:, 0].astype(np.int32)),
        "v1": np.ascontiguousarray(directed[:, 1].astype(np.int32)),
        "w_fitSqrt": float(np.sqrt(np.float32(4.0))),
        "w_regSqrt": float(np.sqrt(np.float32(1.0))),
        "N": N,
        "E": int(directed.shape[0]),
    }
