"""Why a J^T J p apply runs faster alone than inside the PCG loop: the
standalone timing (OptAMD_TimeApplyJTJ) replays ONE apply on the same p back to back, so
its inputs partly stay in the 256 MB Infinity Cache (MALL) between launches; in the PCG
loop every launch follows kernels that stream other vectors through it.

For the workload given, this prints (per-launch us from HIP events):
  warm   the same p, back to back (OptAMD_TimeApplyJTJ, the families table's figure)
  cold   p rotating over NBUF buffers, with a 1 GiB scrub written between launches
  loop   the bench's in-loop apply (kernel timing mode 2 over K LM / GN steps)
  python tools/apply_cache_study.py [shape_from_shading|image_warping] [NBUF]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from opt_amd import OptSolver, workloads  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "shape_from_shading"
    nbuf = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    N = 4096
    if wl == "shape_from_shading":
        w = workloads.shape_from_shading(N, N, seed=3)
        s = OptSolver([N, N], os.path.join(ROOT, "energies", "shape_from_shading.t"), "LMGPU")
        prm = [float(v) for v in w["params"]] + [torch.from_numpy(np.ascontiguousarray(w[k])).cuda()
                                                 for k in ("X", "D_i", "Im", "edgeMaskR", "edgeMaskC")]
        n = N * N
    else:
        w = workloads.image_warping(N, N, seed=1234)
        s = OptSolver([N, N], os.path.join(ROOT, "energies", "image_warping.t"), "gaussNewtonGPU")
        prm = [torch.from_numpy(w[k]).cuda() for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask")] + \
              [w["w_fitSqrt"], w["w_regSqrt"]]
        n = 3 * N * N
    s.set_solver_params({"nIterations": 1000, "lIterations": 10})
    s.init(prm)
    s.step()
    ps = [torch.randn(n, device="cuda") for _ in range(nbuf)]
    Ap = torch.empty(n, device="cuda")
    warm = s.time_apply(prm, ps[0], Ap, 20)
    scrub = torch.empty(1 << 28, device="cuda")   # 1 GiB
    name = s.apply_kernel_name()
    s.set_kernel_timing(2)
    for k in range(3 * nbuf):
        scrub.fill_(float(k))
        s.apply_jtj(prm, ps[k % nbuf], Ap)
    torch.cuda.synchronize()
    kc, msc = s.kernel_stat(name)
    s.set_kernel_timing(0)
    s.set_kernel_timing(2)
    for _ in range(5):
        s.step()
    torch.cuda.synchronize()
    kl, msl = s.kernel_stat(name)
    s.set_kernel_timing(0)
    print(f"{wl} {name}: warm {warm:.1f} us, cold {1000 * msc / max(kc, 1):.1f} us ({kc} launches), "
          f"loop {1000 * msl / max(kl, 1):.1f} us ({kl} launches)", flush=True)
    s.close()


if __name__ == "__main__":
    main()
