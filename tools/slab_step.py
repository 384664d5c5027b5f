"""Row-slab GN step time on ONE GPU: `world` ranks of image_warping as
threads of this process (OptAMD_LocalGroup) splitting a W x H image into row slabs, each
rank running the same solver code as an RCCL rank. Prints the wall time per GN step of
the whole group (all ranks share the GPU, so this is the sum of the ranks' kernels plus
the host-side collectives) and each rank's energy.
Usage: python tools/slab_step.py WORLD W H [steps]   (env knobs as usual, e.g.
OPT_AMD_IW_FUSED_INIT=0 OPT_AMD_IW_APFREE=0 for round 4's slab loop)"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from opt_amd import api, workloads  # noqa: E402
from opt_amd import distributed as dd  # noqa: E402
from tests.iw_helpers import device_params, solver  # noqa: E402


def main():
    import torch

    world, W, H = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    w = workloads.image_warping(W, H, seed=1234)
    lib = api.load_library()
    group = lib.OptAMD_LocalGroupCreate(world)
    solvers, params = [], []
    for r in range(world):
        sv = solver(W, H)
        sl = dd.slab(H, r, world, sv.halo())
        sv.set_decomposition(lib.OptAMD_LocalGroupRank(group, r), sl.y_lo, sl.y_hi)
        sv.set_solver_params({"nIterations": steps + 3, "lIterations": 10})
        solvers.append(sv)
        params.append(device_params(dd.local_image_warping(w, sl)))
    costs = [None] * world

    def body(r, n, init):
        if init:
            solvers[r].init(params[r])
        for _ in range(n):
            solvers[r].step(params[r])
        costs[r] = solvers[r].cost()

    def run(n, init=False):
        th = [threading.Thread(target=body, args=(r, n, init)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()

    run(2, init=True)
    t0 = time.perf_counter()
    run(steps)
    dt = (time.perf_counter() - t0) / steps
    print(f"world={world} {W}x{H}: {1e3 * dt:.3f} ms per GN step (all ranks on one GPU); energy {costs[0]:.9g}",
          flush=True)
    for sv in solvers:
        sv.close()
    lib.OptAMD_LocalGroupDestroy(group)


if __name__ == "__main__":
    main()
