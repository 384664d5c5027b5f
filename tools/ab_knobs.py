"""A/B of per-Step knobs on ONE image_warping plan (same allocations: HBM placement moves
the step time by up to ~8% between plans). Rounds cycle through the configs.

AB_CONFIGS="OPT_AMD_IW_FUSED_RES=0;OPT_AMD_IW_FUSED_RES=1" AB_ROUNDS=4 AB_STEPS=10 AB_PLANS=2"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from opt_amd import OptSolver, workloads  # noqa: E402


def setenv(c):
    for kv in filter(None, c.split(",")):
        k, v = kv.split("=")
        os.environ[k] = v


def unsetenv(c):
    for kv in filter(None, c.split(",")):
        os.environ.pop(kv.split("=")[0], None)


def main():
    W = H = int(os.environ.get("AB_SIZE", "4096"))
    steps = int(os.environ.get("AB_STEPS", "10"))
    rounds = int(os.environ.get("AB_ROUNDS", "4"))
    nplans = int(os.environ.get("AB_PLANS", "2"))
    configs = os.environ.get("AB_CONFIGS", "").split(";")
    names = ["iw_apply", "iw_residual", "iw_jtf", "iw_jtf_apply", "iw_update", "iw_cost"]
    w = workloads.image_warping(W, H, seed=1234)
    base = [torch.from_numpy(w[k]).cuda() for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask")]
    for pl in range(nplans):
        prm = [t.clone() for t in base] + [w["w_fitSqrt"], w["w_regSqrt"]]
        s = OptSolver([W, H], os.path.join(ROOT, "energies", "image_warping.t"))
        s.set_solver_params({"nIterations": 10 ** 6, "lIterations": 10})
        s.init(prm)
        s.step()
        times = {c: [] for c in configs}
        for _ in range(rounds):
            for c in configs:
                setenv(c)
                s.step()   # the first step under the knobs: not timed
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    s.step()
                torch.cuda.synchronize()
                times[c].append(1000 * (time.perf_counter() - t0) / steps)
                unsetenv(c)
        for c in configs:
            setenv(c)
            s.set_kernel_timing(1)
            for _ in range(steps):
                s.step()
            torch.cuda.synchronize()
            cols = []
            for n in names:
                k, ms = s.kernel_stat(n)
                if k:
                    cols.append(f"{n}={1000 * ms / k:.1f}x{k // steps}")
            s.set_kernel_timing(0)
            unsetenv(c)
            print(f"plan{pl} {c or 'default':40s} step_ms " + " ".join(f"{t:.3f}" for t in times[c]) + "  " +
                  " ".join(cols), flush=True)
        s.close()
        del prm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
