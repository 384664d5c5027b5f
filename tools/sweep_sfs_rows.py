"""Rows per strip wave of the shape_from_shading kernels at one rank's slab shape:
LM step time for each OPT_AMD_SFS_ROWS in SWEEP_ROWS on a W x SWEEP_H image (one GPU).
    SWEEP_H=512 SWEEP_ROWS=20,12,8,6,4 python tools/sweep_sfs_rows.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from opt_amd import OptSolver, workloads  # noqa: E402


def main():
    W = int(os.environ.get("SWEEP_W", "4096"))
    H = int(os.environ.get("SWEEP_H", "512"))
    steps = int(os.environ.get("SWEEP_STEPS", "8"))
    w = workloads.shape_from_shading(W, H, seed=3)
    for rows in [int(r) for r in os.environ.get("SWEEP_ROWS", "20,12,8,6,4").split(",")]:
        os.environ["OPT_AMD_SFS_ROWS"] = str(rows)
        s = OptSolver([W, H], os.path.join(ROOT, "energies", "shape_from_shading.t"), "LMGPU")
        prm = [float(v) for v in w["params"]] + [torch.from_numpy(np.ascontiguousarray(w[k])).cuda()
                                                 for k in ("X", "D_i", "Im", "edgeMaskR", "edgeMaskC")]
        s.set_solver_params({"nIterations": 2 + 2 * steps, "lIterations": 10})
        s.init(prm)
        s.step()
        s.step()
        best = 1e9
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps // 2):
                s.step()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / (steps // 2))
        print(f"{W}x{H} rows {rows:3d}: LM step {1000 * best:.3f} ms", flush=True)
        s.close()


if __name__ == "__main__":
    main()
