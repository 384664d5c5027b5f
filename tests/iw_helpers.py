"""Shared helpers for the image_warping GPU tests."""
import os

import numpy as np

from opt_amd import OptSolver, workloads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENERGY = os.path.join(ROOT, "energies", "image_warping.t")


def device_params(w, double=False, device="cuda"):
    """problemparams in declared-index order (energies/image_warping.t)."""
    import torch

    ut = torch.float64 if double else torch.float32
    return [
        torch.from_numpy(w["Offset"]).to(device=device, dtype=ut).contiguous(),
        torch.from_numpy(w["Angle"]).to(device=device, dtype=ut).contiguous(),
        torch.from_numpy(w["UrShape"]).to(device),
        torch.from_numpy(w["Constraints"]).to(device),
        torch.from_numpy(w["Mask"]).to(device),
        float(w["w_fitSqrt"]),
        float(w["w_regSqrt"]),
    ]


def host_params(w, double=False):
    ut = np.float64 if double else np.float32
    return [
        w["Offset"].astype(ut).copy(),
        w["Angle"].astype(ut).copy(),
        w["UrShape"],
        w["Constraints"],
        w["Mask"],
        float(w["w_fitSqrt"]),
        float(w["w_regSqrt"]),
    ]


def solver(W, H, double=False, kind="gaussNewtonGPU", backend="backend_cuda", **kw):
    return OptSolver([W, H], ENERGY, kind, double_precision=double, backend=backend, **kw)


def perturbed(W, H, seed=5, n_handles=6, angle_sigma=0.05, offset_sigma=0.2, hole=True):
    """A problem away from its rest state so every term is non-trivial."""
    rng = np.random.default_rng(seed)
    w = workloads.image_warping(W, H, seed=seed, n_handles=n_handles, hole=hole, max_move=0.15)
    w["Offset"] = (w["Offset"] + rng.normal(0, offset_sigma, w["Offset"].shape)).astype(np.float32)
    w["Angle"] = rng.normal(0, angle_sigma, w["Angle"].shape).astype(np.float32)
    return w


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))
