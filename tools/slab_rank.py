"""ONE rank's row slab on one GPU: rank `rank` of a `world`-way row split of
a W x H image, its owned rows plus the plan's halo rows bound as that rank's arrays, on a
1-rank communicator (OptAMD_LocalGroup of size 1: no halo exchange and no all-reduce run, so
the step is this rank's kernels alone — what each GPU of the split computes between its
collectives). Prints one JSON line: per-step wall time (ms, the Step call synchronises), the
kernel table of those steps (OptAMD_KernelReport), and the per-step collective volume the
same rank would move on the real split (halo planes and all-reduced doubles, counted from
the plan's exchange pattern), next to the whole image's step for comparison.
Usage: python tools/slab_rank.py {image_warping|shape_from_shading} WORLD RANK W H [steps]
(env knobs as usual: OPT_AMD_ROWS, OPT_AMD_FUSE23, OPT_AMD_IW_PCG_U2, ...).
Reference split restated: API/src/backend_cpu_mt.t:716-737 (row blocks per thread)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from opt_amd import OptSolver, api, workloads  # noqa: E402
from opt_amd import distributed as dd  # noqa: E402

ENERGY = {k: os.path.join(ROOT, "energies", k + ".t") for k in ("image_warping", "shape_from_shading")}
KIND = {"image_warping": "gaussNewtonGPU", "shape_from_shading": "LMGPU"}


def make(name, W, H):
    if name == "image_warping":
        return workloads.image_warping(W, H, seed=1234), dd.IW_CHANNELS
    return workloads.shape_from_shading(W, H, seed=3), dd.SFS_CHANNELS


def params(name, w, lw):
    import torch

    if name == "image_warping":
        return [torch.from_numpy(np.ascontiguousarray(lw[k])).cuda()
                for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask")] + [w["w_fitSqrt"], w["w_regSqrt"]]
    return [float(v) for v in w["params"]] + [torch.from_numpy(np.ascontiguousarray(lw[k])).cuda()
                                              for k in ("X", "D_i", "Im", "edgeMaskR", "edgeMaskC")]


def collectives(name, W, liter, halo, itemsize=4):
    """What the rank would exchange per step on the real split (interior rank: two
    neighbours). image_warping GN (image_warping.hip step()): the unknowns' halo after the
    update (3 channels), r_0 / pre / flags after the fused init, r_{i-1} and p_{i-1} before
    each of the L-1 iw_pcg passes; all-reduces: 4 doubles per PCG iteration + the cost.
    shape_from_shading LM with step23 on slabs (stencil_plan.h pcg_loop_fused): the unknown's
    halo, p before each apply; 6 doubles per iteration (rz, q with the apply's four sums)
    plus the init / cost / model-cost scalars."""
    plane = W * halo * itemsize          # one channel's halo rows on one side
    if name == "image_warping":
        planes = 3 + (3 + 1) + 0.25 + (liter - 1) * 6   # flags are 1 byte (0.25 of a 4-B plane)
        reduces = 4 * liter + 1
    else:
        planes = 1 + liter
        reduces = 6 * liter + 4
    return {"halo_bytes_per_step": int(2 * planes * plane), "allreduce_doubles_per_step": reduces,
            "allreduce_calls_per_step": liter + (1 if name == "image_warping" else 3)}


def main():
    import torch

    name, world, rank, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    steps = int(sys.argv[6]) if len(sys.argv) > 6 else 10
    liter = 10
    w, chans = make(name, W, H)
    lib = api.load_library()

    def run(split):
        s = OptSolver([W, H], ENERGY[name], KIND[name])
        group = None
        lw = w
        if split:
            group = lib.OptAMD_LocalGroupCreate(1)
            sl = dd.slab(H, rank, world, s.halo())
            s.set_decomposition(lib.OptAMD_LocalGroupRank(group, 0), sl.y_lo, sl.y_hi)
            lw = dd.local_image(w, sl, chans)
        prm = params(name, w, lw)
        s.set_solver_params({"nIterations": 2 * steps + 3, "lIterations": liter})
        s.init(prm)
        for _ in range(2):
            s.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            s.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        s.set_kernel_timing(1)
        for _ in range(steps):
            s.step()
        rep = s.kernel_report()
        cost = s.cost()
        s.close()
        if group:
            lib.OptAMD_LocalGroupDestroy(group)
        return dt, rep, cost

    dt, rep, cost = run(True)
    full, _, _ = run(False)
    sl = dd.slab(H, rank, world, 2)
    out = {"workload": name, "W": W, "H": H, "world": world, "rank": rank, "owned_rows": sl.rows,
           "mem_rows": sl.mem_rows, "ms_per_step_slab": round(1e3 * dt, 4),
           "ms_per_step_full_image": round(1e3 * full, 4),
           "slab_over_full_div_world": round(dt / (full / world), 3), "energy_after": cost,
           "env": {k: v for k, v in os.environ.items() if k.startswith("OPT_AMD_")},
           **collectives(name, W, liter, 2), "kernel_table": rep}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
