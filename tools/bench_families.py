"""Per-configuration measurements of every BASELINE.json config on one GPU.

For each config: the pure J^T J p apply (hipEvent loop over OptAMD_TimeApplyJTJ), its
algorithmic-byte roofline (SURVEY.md §8d per-unit bytes x units / apply time, against
8 TB/s), and the average solver step time (GN or LM iteration incl. all kernels) over
`--steps` timed steps after one warm-up step. Writes one JSON list (stdout or --out).
bench.py remains the driver's headline (image_warping 4096^2); this adds the other rows.

  python tools/bench_families.py [--out FILE] [--steps K] [--only name,...]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from opt_amd import OptSolver, workloads  # noqa: E402

PEAK = 8000.0
E = lambda n: os.path.join(ROOT, "energies", n + ".t")  # noqa: E731


def cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def iw(size):
    w = workloads.image_warping(size, size, seed=1234)
    prm = [cuda(w[k]) for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask")] + \
          [w["w_fitSqrt"], w["w_regSqrt"]]
    return dict(name=f"image_warping {size}x{size} fp32 GN", dims=[size, size], energy=E("image_warping"),
                kind="gaussNewtonGPU", double=False, prm=prm, units=size * size, unit="px", bytes_per_unit=48,
                dtype=torch.float32)


def poisson():
    w = workloads.poisson_image_editing(512, 512, seed=1)
    prm = [cuda(w[k]) for k in ("X", "T", "M")]
    return dict(name="poisson_image_editing 512x512 fp32 GN (1 GN / 10 PCG)", dims=[512, 512],
                energy=E("poisson_image_editing"), kind="gaussNewtonGPU", double=False, prm=prm, units=512 * 512,
                unit="px", bytes_per_unit=36, dtype=torch.float32, liter=10, nit=1)


def sfs():
    w = workloads.shape_from_shading(4096, 4096, seed=3)
    prm = [float(v) for v in w["params"]] + [cuda(w[k]) for k in ("X", "D_i", "Im", "edgeMaskR", "edgeMaskC")]
    return dict(name="shape_from_shading 4096x4096 fp32 LM", dims=[4096, 4096], energy=E("shape_from_shading"),
                # the timed apply alone (time_apply) gets no LM diagonal: 30 B/px; the PCG loop's
                # apply also reads CtC (34 B/px, bench.py --workload shape_from_shading)
                kind="LMGPU", double=False, prm=prm, units=4096 * 4096, unit="px", bytes_per_unit=30,
                dtype=torch.float32)


def arap():
    w = workloads.arap_grid(1000, 1000, seed=9)
    prm = [w["w_fitSqrt"], w["w_regSqrt"]] + [cuda(w[k]) for k in ("Offset", "Angle", "UrShape", "Constraints")] + \
          [None, cuda(w["v0"]), cuda(w["v1"])]
    return dict(name=f"arap_mesh_deformation 1M vertices ({w['E']} edges) fp32 GN", dims=[w["N"], w["E"]],
                energy=E("arap_mesh_deformation"), kind="gaussNewtonGPU", double=False, prm=prm, units=w["N"],
                unit="vertex", bytes_per_unit=132, dtype=torch.float32)


def oflow():
    w = workloads.optical_flow(3840, 2160, seed=5)
    prm = [w["w_fitSqrt"], w["w_regSqrt"], cuda(w["X"].astype(np.float64))] + \
          [cuda(w[k]) for k in ("I", "I_hat", "I_hat_dx", "I_hat_dy")]
    return dict(name="optical_flow 3840x2160 fp64 LM", dims=[3840, 2160], energy=E("optical_flow"), kind="LMGPU",
                double=True, prm=prm, units=3840 * 2160, unit="px", bytes_per_unit=72, dtype=torch.float64)


def materialized(cfg, fused):
    """The same config through the materialized-Jacobian path (useMaterializedJTJ)."""
    cfg = dict(cfg)
    cfg["name"] += " materialized " + ("J^T J (fused)" if fused else "J^T (J p)")
    cfg["materialized"] = True
    cfg["fused"] = fused
    return cfg


def generic(cfg):
    """The same config on the kernels the general front end generates (OPT_AMD_GENERIC=1)."""
    cfg = dict(cfg)
    cfg["name"] += " generated kernels"
    cfg["generic"] = True
    return cfg


CONFIGS = {"iw4096": lambda: iw(4096), "iw2048": lambda: iw(2048), "poisson": poisson, "sfs": sfs,
           "arap": arap, "optical_flow": oflow,
           "iw4096_mat_fused": lambda: materialized(iw(4096), True),
           "iw4096_mat_split": lambda: materialized(iw(4096), False),
           "poisson_mat_fused": lambda: materialized(poisson(), True),
           "iw4096_generic": lambda: generic(iw(4096)), "poisson_generic": lambda: generic(poisson()),
           "sfs_generic": lambda: generic(sfs()), "arap_generic": lambda: generic(arap()),
           "optical_flow_generic": lambda: generic(oflow())}


def spmv_bytes(rows, cols, nnz, x_len):
    """Compulsory bytes of one CSR SpMV: (value, column) per nonzero, row pointer and
    output per row, each input element once."""
    return 8 * nnz + 8 * rows + 4 + 4 * x_len


def measure(cfg, steps):
    mat = cfg.get("materialized", False)
    if cfg.get("generic"):
        os.environ["OPT_AMD_GENERIC"] = "1"
    try:
        s = OptSolver(cfg["dims"], cfg["energy"], cfg["kind"], double_precision=cfg["double"], materialized=mat,
                      fused_jtj=cfg.get("fused", False))
    finally:
        os.environ.pop("OPT_AMD_GENERIC", None)
    if cfg.get("generic"):
        assert s.family() == "generic"
    n = s.unknown_count()
    p = torch.randn(n, device="cuda", dtype=cfg["dtype"])
    Ap = torch.empty_like(p)
    apply_us = s.time_apply(cfg["prm"], p, Ap, 20)
    liter = cfg.get("liter", 10)
    nit = cfg.get("nit", steps + 1)
    s.set_solver_params({"nIterations": max(nit, steps + 1), "lIterations": liter})
    s.init(cfg["prm"])
    s.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    for _ in range(steps):
        if not s.step():
            break
        done += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    bytes_apply = cfg["bytes_per_unit"] * cfg["units"]
    bpu = cfg["bytes_per_unit"]
    if mat:
        nres, _ = s.jacobian_shape()
        nnzJ, nnzJTJ = s.materialized_nonzeros()
        if cfg["fused"]:   # one SpMV over J^T J (+ p read again for p.Ap: same vector, cached)
            bytes_apply = spmv_bytes(n, n, nnzJTJ, n)
        else:              # J p, then J^T (J p) with p read for p.Ap
            bytes_apply = spmv_bytes(nres, n, nnzJ, n) + spmv_bytes(n, nres, nnzJ, nres) + 4 * n
        bpu = bytes_apply / cfg["units"]
        apply_us = s.time_apply(cfg["prm"], p, Ap, 20)   # after the first step: steady-state J^T J
    gbs = bytes_apply / (apply_us * 1e-6) / 1e9
    out = {
        "config": cfg["name"], "unknowns": n, "apply_kernel": s.apply_kernel_name(), "apply_us": apply_us,
        "apply_unknowns_per_s": n / (apply_us * 1e-6),
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": PEAK, "unit": "GB/s", "frac": gbs / PEAK,
                     "bytes_per_unit": bpu, "unit_kind": cfg["unit"]},
        "lIterations": liter, "timed_steps": done,
        "step_ms": 1000.0 * dt / max(done, 1), "cost_after": s.cost(),
    }
    if mat:
        out["nnz_J"], out["nnz_JTJ"] = s.materialized_nonzeros()
        out["jacobian_rows"] = s.jacobian_shape()[0]
    s.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--only")
    a = ap.parse_args()
    names = a.only.split(",") if a.only else list(CONFIGS)
    res = []
    for nm in names:
        cfg = CONFIGS[nm]()
        r = measure(cfg, a.steps)
        print(json.dumps(r), flush=True)
        res.append(r)
        del cfg
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
