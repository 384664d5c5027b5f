"""Debug: drift of the GPU image_warping GN trajectory from the oracle vs PCG length.
Run on the GPU box: python tools/dbg_iw.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opt_amd import workloads  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.iw_helpers import device_params, solver  # noqa: E402

CASES = [(256, 192, dict(seed=7, n_handles=6, max_move=0.1)), (256, 192, dict(seed=7, n_handles=6, max_move=0.02)),
         (2048, 2048, dict(seed=1234)), (4096, 4096, dict(seed=1234))]
for W, H, kw in CASES:
    w = workloads.image_warping(W, H, **kw)
    out = []
    for L in (1, 3, 10):
        s = solver(W, H)
        prm = device_params(w)
        s.set_solver_params({"nIterations": 2, "lIterations": L})
        c = s.profiled_solve(prm)
        _, _, ref, _ = oracle.iw_solve(w, 2, L, nthreads=16)
        out.append(f"L={L}: " + ",".join(f"{abs(a - b) / b:.1e}" for a, b in zip(c[1:], ref[1:])))
        s.close()
    print(W, H, kw, " | ".join(out), flush=True)
