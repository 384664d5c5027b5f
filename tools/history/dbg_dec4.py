"""Diagnose the 4-rank image_warping decomposition drift: run the single-domain and the
LocalGroup-decomposed solves with freed device memory poisoned (NaN) or zeroed before
each, and print the cost trajectories and the max angle difference."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from tests.iw_helpers import device_params, perturbed, solver
from tests.test_decomposition_gpu import run_decomposed


def poison(val):
    x = torch.full((1 << 28,), val, dtype=torch.float32, device="cuda")
    del x
    torch.cuda.synchronize()


W, H, world = 256, 200, 4
for fill in (0.0, float("nan"), 1.0):
    poison(fill)
    w = perturbed(W, H, seed=21 + world)
    s = solver(W, H)
    prm = device_params(w)
    s.set_solver_params({"nIterations": 3, "lIterations": 10})
    ref = s.profiled_solve(prm)
    s.close()
    poison(fill)
    costs, O, A = run_decomposed(w, world, 3, 10)
    ra = prm[1].cpu().numpy()
    print("fill", fill, "ref", ref, "dec", costs[0], "maxdA", float(np.abs(A - ra).max()), flush=True)
