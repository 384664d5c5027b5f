"""where does the fp64 image_warping GPU path leave the double oracle at
size? Prints, for the bench workload at N^2 (fp64 unknowns, known arrays float):
  * per-kernel agreement (cost, J^T F, pre, J^T J p on a seeded p) as max|diff| / max|ref|;
  * the energy after 1 GN step of L PCG iterations for L in 1, 2, 3, 5, 10, relative to
    the double oracle, for the fused loop (default), the separate passes and the generated
    kernels (OPT_AMD_GENERIC=1);
  * 2 GN x 10 PCG against the oracle, and the oracle's own spread over its slab count
    (the summation order of its sums: the fp64 floor of this trajectory).
Usage: python tools/fp64_gap.py N [N ...]   (GPU; the oracle runs on 16 host threads)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from opt_amd import workloads  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.iw_helpers import device_params, rel_err, solver  # noqa: E402

NT = 16
VARIANTS = {
    "fused": {},
    "separate": {"OPT_AMD_IW_FUSED_INIT": "0", "OPT_AMD_IW_FUSED_RES": "0"},
    "generic": {"OPT_AMD_GENERIC": "1"},
}


def with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main(N):
    import torch

    W = H = N
    w = workloads.image_warping(W, H, seed=1234)
    n = 3 * W * H
    s = solver(W, H, double=True)
    prm = device_params(w, double=True)
    c = s.eval_cost(prm)
    cr = oracle.iw_cost(w, nthreads=NT, double=True)
    r = torch.zeros(n, device="cuda", dtype=torch.float64)
    pre = torch.zeros_like(r)
    rz = s.eval_jtf(prm, r, pre)
    r_ref, pre_ref, rz_ref = oracle.iw_eval_jtf(w, nthreads=NT, double=True)
    p = np.random.default_rng(3).standard_normal(n)
    Ap = torch.zeros_like(r)
    pAp = s.apply_jtj(prm, torch.from_numpy(p).cuda(), Ap)
    Ap_ref, pAp_ref = oracle.iw_apply_jtj(w, p, nthreads=NT, double=True)
    print(f"N={N} kernels: cost {abs(c - cr) / cr:.2e}  r {rel_err(r.cpu().numpy(), r_ref):.2e}  "
          f"pre {rel_err(pre.cpu().numpy(), pre_ref):.2e}  rz {abs(rz - rz_ref) / abs(rz_ref):.2e}  "
          f"Ap {rel_err(Ap.cpu().numpy(), Ap_ref):.2e}  pAp {abs(pAp - pAp_ref) / abs(pAp_ref):.2e}", flush=True)
    del s, prm
    for L in (1, 2, 3, 5, 10):
        _, _, ref, _ = oracle.iw_solve(w, 1, L, nthreads=NT, double=True)
        line = [f"N={N} 1 GN x {L:2d} PCG: oracle {ref[1]:.10e}"]
        for name, env in VARIANTS.items():
            def run():
                sv = solver(W, H, double=True)
                pv = device_params(w, double=True)
                sv.set_solver_params({"nIterations": 1, "lIterations": L})
                return np.array(sv.profiled_solve(pv))
            cg = with_env(env, run)
            line.append(f"{name} {abs(cg[1] - ref[1]) / ref[1]:.2e}")
        print("  ".join(line), flush=True)
    _, _, truth, _ = oracle.iw_solve(w, 2, 10, nthreads=NT, double=True)
    sv = solver(W, H, double=True)
    pv = device_params(w, double=True)
    sv.set_solver_params({"nIterations": 2, "lIterations": 10})
    cg = np.array(sv.profiled_solve(pv))
    print(f"N={N} 2 GN x 10 PCG: GPU fp64 vs the oracle {np.abs(cg - truth) / truth}", flush=True)
    for nt in (1, 7):
        _, _, cp, _ = oracle.iw_solve(w, 2, 10, nthreads=nt, double=True)
        print(f"N={N} 2 GN x 10 PCG: oracle on {nt} threads vs {NT}: {np.abs(cp - truth) / truth}", flush=True)

if __name__ == "__main__":
    for a in sys.argv[1:]:
        main(int(a))
