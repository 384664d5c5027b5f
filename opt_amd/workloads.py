"""Seeded synthetic inputs for the benchmark configurations.

No datasets can be fetched, so every configuration is generated with the shapes and
value distributions the reference's example harnesses build from their input files.
"""
from __future__ import annotations

import math

import numpy as np


def image_warping(W: int, H: int, seed: int = 1234, n_handles: int = 9, hole: bool = True,
                  max_move: float = 0.05):
    """image_warping inputs (examples/image_warping/src/CombinedSolver.h:166-223, main.cpp:163-177).

    UrShape(x,y) = (x,y); Offset = UrShape; Angle = 1e-5; Mask = 0 except a seeded
    elliptical hole (~5 % of the pixels, value 255); Constraints = (-1,-1) except the
    image border pinned to itself and `n_handles` seeded handles moved by up to
    max_move*W. Weights w_fit = 100, w_reg = 0.01 passed as square roots
    (CombinedSolver.h:130-134).

    Returns a dict of flat float32 arrays in the Opt layout (row-major, x fastest,
    channels interleaved) plus the two weights.
    """
    rng = np.random.default_rng(seed)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
    U = np.stack([xs, ys], axis=-1)
    M = np.zeros((H, W), np.float32)
    if hole:
        cx, cy = rng.uniform(0.35, 0.65) * W, rng.uniform(0.35, 0.65) * H
        ax, ay = 0.13 * W, 0.12 * H
        M[((xs - cx) / ax) ** 2 + ((ys - cy) / ay) ** 2 <= 1.0] = 255.0
    C = np.full((H, W, 2), -1.0, np.float32)
    border = np.zeros((H, W), bool)
    border[0, :] = border[-1, :] = border[:, 0] = border[:, -1] = True
    pin = border & (M == 0)
    C[pin] = U[pin]
    placed = 0
    tries = 0
    while placed < n_handles and tries < 100 * max(1, n_handles):
        tries += 1
        hx = int(rng.uniform(0.1, 0.9) * W)
        hy = int(rng.uniform(0.1, 0.9) * H)
        if M[hy, hx] != 0 or border[hy, hx]:
            continue
        tx = hx + rng.uniform(-max_move, max_move) * W
        ty = hy + rng.uniform(-max_move, max_move) * H
        C[hy, hx] = (max(tx, 0.0), max(ty, 0.0))
        placed += 1
    A = np.full((H, W), 1e-5, np.float32)
    return {
        "Offset": U.reshape(-1).copy(),
        "Angle": A.reshape(-1),
        "UrShape": U.reshape(-1).copy(),
        "Constraints": C.reshape(-1),
        "Mask": M.reshape(-1),
        "w_fitSqrt": float(math.sqrt(100.0)),
        "w_regSqrt": float(math.sqrt(0.01)),
        "W": W,
        "H": H,
    }


IMAGE_WARPING_ORDER = ["Offset", "Angle", "UrShape", "Constraints", "Mask", "w_fitSqrt", "w_regSqrt"]


def poisson_image_editing(W: int, H: int, seed: int = 7):
    """poisson_image_editing inputs (examples/poisson_image_editing/src/CombinedSolver.h:66-90).

    X = a smooth seeded RGBA base image (alpha 255), T = a second seeded image to be
    blended in, M = 0 (solve) inside a disk covering ~30 % of the image and 255 (fixed)
    outside; X starts as the base image everywhere.
    """
    rng = np.random.default_rng(seed)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)

    def smooth_image(k):
        img = np.zeros((H, W, 4), np.float32)
        for c in range(3):
            acc = np.zeros((H, W), np.float32)
            for _ in range(k):
                fx, fy, ph = rng.uniform(0.5, 4.0), rng.uniform(0.5, 4.0), rng.uniform(0, 2 * np.pi)
                acc += np.sin(2 * np.pi * (fx * xs / W + fy * ys / H) + ph).astype(np.float32)
            img[..., c] = 127.5 + 60.0 * acc / k
        img[..., 3] = 255.0
        return img

    X = smooth_image(4)
    T = smooth_image(3)
    cx, cy, rad = 0.5 * W, 0.5 * H, 0.31 * min(W, H)
    M = np.where((xs - cx) ** 2 + (ys - cy) ** 2 <= rad * rad, 0.0, 255.0).astype(np.float32)
    return {"X": X.reshape(-1).copy(), "T": T.reshape(-1).copy(), "M": M.reshape(-1).copy(), "W": W, "H": H}


POISSON_ORDER = ["X", "T", "M"]


def _sobel_like(img: np.ndarray, axis: int) -> np.ndarray:
    """examples/optical_flow/src/CombinedSolver.h computeDU / computeDV (float32, the
    same operation order; one-pixel border left at 0)."""
    d = np.zeros_like(img)
    c = img
    if axis == 0:   # DU: right column minus left column over the 3 rows
        v = (-c[:-2, :-2] - c[1:-1, :-2] - c[2:, :-2]) + c[:-2, 2:] + c[1:-1, 2:] + c[2:, 2:]
    else:           # DV: bottom row minus top row over the 3 columns
        v = (-c[:-2, :-2] - c[:-2, 1:-1] - c[:-2, 2:]) + c[2:, :-2] + c[2:, 1:-1] + c[2:, 2:]
    d[1:-1, 1:-1] = (v / np.float32(8.0)).astype(np.float32)
    return d


def optical_flow(W: int, H: int, seed: int = 5, sigma: float = 5.0, max_flow: float = 4.0):
    """optical_flow inputs (examples/optical_flow/src/CombinedSolver.h).

    I = Gaussian-filtered (sigma, the harness's coarse level) seeded noise scaled to
    [0, 255]; I_hat = I warped by a smooth seeded flow u with |u| <= max_flow px
    (I_hat(q) = I(q - u(q)), bilinear), so I(p) ~ I_hat(p + u); I_hat_dx / I_hat_dy by
    the harness's 3x3 difference formula; w_fit = 10, w_reg = 0.1 passed as square
    roots; X = 0.
    """
    from scipy import ndimage

    rng = np.random.default_rng(seed)
    noise = rng.normal(size=(H, W)).astype(np.float32)
    I = ndimage.gaussian_filter(noise, sigma, mode="nearest")
    I = (255.0 * (I - I.min()) / max(float(I.max() - I.min()), 1e-12)).astype(np.float32)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
    ph = rng.uniform(0, 2 * np.pi, 4)
    fx = rng.uniform(0.5, 2.0, 4)
    ux = 0.5 * max_flow * (np.sin(2 * np.pi * fx[0] * xs / W + ph[0]) + np.cos(2 * np.pi * fx[1] * ys / H + ph[1]))
    uy = 0.5 * max_flow * (np.cos(2 * np.pi * fx[2] * xs / W + ph[2]) + np.sin(2 * np.pi * fx[3] * ys / H + ph[3]))
    I_hat = ndimage.map_coordinates(I, [ys - uy, xs - ux], order=1, mode="nearest").astype(np.float32)
    return {
        "X": np.zeros(2 * W * H, np.float32),
        "I": I.reshape(-1).copy(),
        "I_hat": I_hat.reshape(-1).copy(),
        "I_hat_dx": _sobel_like(I_hat, 0).reshape(-1).copy(),
        "I_hat_dy": _sobel_like(I_hat, 1).reshape(-1).copy(),
        "w_fitSqrt": float(np.sqrt(np.float32(10.0))),
        "w_regSqrt": float(np.sqrt(np.float32(0.1))),
        "W": W,
        "H": H,
    }


# Param("w_fit",0), Param("w_reg",1), Unknown X 2, Arrays I 3, I_hat 4, I_hat_dx 5, I_hat_dy 6
OPTICAL_FLOW_ORDER = ["w_fitSqrt", "w_regSqrt", "X", "I", "I_hat", "I_hat_dx", "I_hat_dy"]


# lightingCoefficients of the reference's examples/data/shape_from_shading/default.SFSSolverParameters
SFS_LIGHTING = [0.6908318, 0.04459886, 0.0181296, -0.17731632, -0.04067883, 0.1446765, 0.02393525,
                -0.24658696, 0.005797]


def sfs_shading(X, fx, fy, ux, uy, L):
    """B(x,y) of shape_from_shading.t (normalAt / B, eq. 8-10) for a depth image X, float64."""
    X = X.astype(np.float64)
    H, W = X.shape
    j, i = np.mgrid[0:H, 0:W].astype(np.float64)
    d = X
    a = np.zeros_like(X); a[:, 1:] = X[:, :-1]    # X(-1,0)
    b = np.zeros_like(X); b[1:, :] = X[:-1, :]    # X(0,-1)
    nx = b * (d - a) / fy
    ny = a * (d - b) / fx
    nz = nx * (ux - i) / fx + ny * (uy - j) / fy - a * b / (fx * fy)
    sq = nx * nx + ny * ny + nz * nz
    inv = np.where(sq > 0, 1.0 / np.sqrt(np.where(sq > 0, sq, 1.0)), 1.0)
    Nx, Ny, Nz = inv * nx, inv * ny, inv * nz
    return (L[0] + L[1] * Ny + L[2] * Nz + L[3] * Nx + L[4] * Nx * Ny + L[5] * Ny * Nz +
            L[6] * (-Nx * Nx - Ny * Ny + 2 * Nz * Nz) + L[7] * Nz * Nx + L[8] * (Nx * Nx - Ny * Ny))


def shape_from_shading(W: int, H: int, seed: int = 3, valid_frac: float = 0.6, noise: float = 0.002):
    """shape_from_shading inputs (examples/shape_from_shading).

    D_i = a smooth seeded depth surface in [0.38, 0.56] (the range of the reference's
    default_targetDepth), invalid (-10000, as the harness clamps -inf) outside a seeded
    blob covering ~valid_frac of the image; Im = the surface's spherical-harmonics
    shading with the reference's lighting coefficients, plus seeded noise; camera
    f = 574.0528 * W / 640 (the reference intrinsics scaled to the width), u = (W/2, H/2);
    edge masks all 1; weights w_p = 100, w_s = 100, w_g = 1 (default.SFSSolverParameters);
    X0 = D_i plus seeded noise (so the fit and smoothness terms are active).
    """
    from scipy import ndimage

    rng = np.random.default_rng(seed)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    base = ndimage.gaussian_filter(rng.normal(size=(H, W)), max(W, H) / 24.0, mode="nearest")
    base = (base - base.min()) / max(base.max() - base.min(), 1e-12)
    depth = 0.38 + 0.18 * base
    blob = ndimage.gaussian_filter(rng.normal(size=(H, W)), max(W, H) / 16.0, mode="nearest")
    thr = np.quantile(blob, 1.0 - valid_frac)
    valid = blob >= thr
    fx = fy = 574.0528 * W / 640.0
    ux, uy = W / 2.0, H / 2.0
    Bimg = sfs_shading(depth, fx, fy, ux, uy, SFS_LIGHTING)
    Im = np.clip(Bimg + noise * rng.normal(size=(H, W)), 0.0, 1.0).astype(np.float32)
    D = np.where(valid, depth, -10000.0).astype(np.float32)
    X0 = np.where(valid, depth + 0.002 * rng.normal(size=(H, W)), -10000.0).astype(np.float32)
    params = [100.0, 100.0, 1.0, float(np.float32(fx)), float(np.float32(fy)), ux, uy] + list(SFS_LIGHTING)
    return {
        "params": np.array(params, np.float32),
        "X": X0.reshape(-1).copy(),
        "D_i": D.reshape(-1).copy(),
        "Im": Im.reshape(-1).copy(),
        "edgeMaskR": np.ones(W * H, np.uint8),
        "edgeMaskC": np.ones(W * H, np.uint8),
        "W": W,
        "H": H,
    }


def arap_grid(nx: int, ny: int, seed: int = 9, n_handles: int = 16, z_noise: float = 0.01,
              handle_move: float = 0.15):
    """arap_mesh_deformation inputs (examples/arap_mesh_deformation).

    A planar nx x ny grid mesh over [0,1]^2 (seeded z-noise), each quad split into two
    triangles; the graph holds every mesh edge in both directions, grouped by head vertex
    as createGraphFromNeighborLists builds it (examples/shared/OptGraph.h:78-90):
    ~6 directed edges per vertex. Constraints: the first and last grid rows pinned to
    themselves, n_handles seeded interior vertices moved by up to handle_move, all
    others -inf (CombinedSolver.h:84-101); Angle = 0.1 (CombinedSolver.h:166);
    w_fit = 4, w_reg = 1 passed as square roots (main.cpp).
    """
    rng = np.random.default_rng(seed)
    N = nx * ny
    ys, xs = np.mgrid[0:ny, 0:nx]
    P = np.stack([xs / max(nx - 1, 1), ys / max(ny - 1, 1), z_noise * rng.normal(size=(ny, nx))], -1)
    P = P.reshape(N, 3).astype(np.float32)
    idx = np.arange(N).reshape(ny, nx)
    und = [np.stack([idx[:, :-1].ravel(), idx[:, 1:].ravel()], 1),      # horizontal
           np.stack([idx[:-1, :].ravel(), idx[1:, :].ravel()], 1),      # vertical
           np.stack([idx[:-1, :-1].ravel(), idx[1:, 1:].ravel()], 1)]   # diagonal
    und = np.concatenate(und)
    directed = np.concatenate([und, und[:, ::-1]])
    order = np.lexsort((directed[:, 1], directed[:, 0]))   # by head, then tail
    directed = directed[order]
    C = np.full((N, 3), -np.inf, np.float32)
    pinned = np.concatenate([idx[0, :], idx[-1, :]])
    C[pinned] = P[pinned]
    interior = idx[1:-1, 1:-1].ravel()
    handles = rng.choice(interior, size=min(n_handles, interior.size), replace=False)
    C[handles] = P[handles] + rng.uniform(-handle_move, handle_move, (handles.size, 3)).astype(np.float32)
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
