"""A/B the image_warping GN step under plan environment knobs on the GPU.

SWEEP_CONFIGS="OPT_AMD_IW_SNAKE=0;OPT_AMD_IW_SNAKE=1,OPT_AMD_IW_NT=2" — each ';'-separated
config is applied to os.environ before a fresh plan is built (the plans read their knobs
at construction). Per config: wall time per GN step (no instrumentation) in ROUNDS
interleaved rounds, then the per-kernel averages from event timing."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from opt_amd import OptSolver, workloads  # noqa: E402


def main():
    W = H = int(os.environ.get("SWEEP_SIZE", "4096"))
    H = int(os.environ.get("SWEEP_H", H))   # e.g. 512: one rank's slab of the 8-GPU split
    steps = int(os.environ.get("SWEEP_STEPS", "10"))
    rounds = int(os.environ.get("SWEEP_ROUNDS", "3"))
    configs = [c for c in os.environ.get("SWEEP_CONFIGS", "").split(";")]
    w = workloads.image_warping(W, H, seed=1234)
    base = [torch.from_numpy(w[k]).cuda() for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask")]
    names = ["iw_apply", "iw_apply_res", "iw_residual", "iw_jtf", "iw_jtf_apply", "iw_update", "iw_cost"]
    solvers = []
    for c in configs:
        for kv in filter(None, c.split(",")):
            k, v = kv.split("=")
            os.environ[k] = v
        prm = [t.clone() for t in base] + [w["w_fitSqrt"], w["w_regSqrt"]]
        s = OptSolver([W, H], os.path.join(ROOT, "energies", "image_warping.t"))
        s.set_solver_params({"nIterations": 2 + rounds * steps + steps + 2, "lIterations": 10})
        s.init(prm)
        s.step()
        solvers.append((f"{len(solvers)}:{c or 'default'}", s))
        for kv in filter(None, c.split(",")):
            os.environ.pop(kv.split("=")[0])
    times = {c: [] for c, _ in solvers}
    for _ in range(rounds):
        for c, s in solvers:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                s.step()
            torch.cuda.synchronize()
            times[c].append(1000 * (time.perf_counter() - t0) / steps)
    for c, s in solvers:
        s.set_kernel_timing(1)
        for _ in range(steps):
            s.step()
        torch.cuda.synchronize()
        cols = []
        for n in names:
            k, ms = s.kernel_stat(n)
            cols.append(f"{n}={1000 * ms / max(k, 1):.1f}")
        print(f"{c:40s} step_ms " + " ".join(f"{t:.3f}" for t in times[c]) + "  " + " ".join(cols), flush=True)
        s.close()


if __name__ == "__main__":
    main()
