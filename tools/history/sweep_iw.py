"""Sweep the image_warping stencil-kernel geometry (rows per wavefront, prefetch depth)
on the GPU: pure apply time and per-kernel times inside GN steps at 4096^2."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from opt_amd import OptSolver, workloads  # noqa: E402


def main():
    W = H = int(os.environ.get("SWEEP_SIZE", "4096"))
    w = workloads.image_warping(W, H, seed=1234)
    base = [torch.from_numpy(w[k]).cuda() for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask")]
    rows_list = [int(x) for x in os.environ.get("SWEEP_ROWS", "8,16,32,64").split(",")]
    depths = [int(x) for x in os.environ.get("SWEEP_DEPTH", "1,2").split(",")]
    names = ["iw_apply", "iw_residual", "iw_jtf", "iw_update", "iw_cost"]
    print(f"{'rows':>5} {'depth':>5} {'pure_us':>9} {'step_ms':>8} " + " ".join(f"{n:>13}" for n in names))
    for rows in rows_list:
        for depth in depths:
            os.environ["OPT_AMD_ROWS"] = str(rows)
            os.environ["OPT_AMD_DEPTH"] = str(depth)
            prm = [t.clone() for t in base] + [w["w_fitSqrt"], w["w_regSqrt"]]
            s = OptSolver([W, H], os.path.join(ROOT, "energies", "image_warping.t"))
            p = torch.randn(s.unknown_count(), device="cuda")
            Ap = torch.empty_like(p)
            pure = s.time_apply(prm, p, Ap, 20)
            s.set_solver_params({"nIterations": 8, "lIterations": 10})
            s.init(prm)
            s.step()
            s.set_kernel_timing(1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                s.step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 5
            cols = []
            for n in names:
                k, ms = s.kernel_stat(n)
                cols.append(f"{1000 * ms / max(k, 1):13.1f}")
            print(f"{rows:5d} {depth:5d} {pure:9.1f} {1000 * dt:8.3f} " + " ".join(cols), flush=True)
            s.close()


if __name__ == "__main__":
    main()
