"""Per-kernel device-time table of one configuration (the reference's per-kernel timing
report, collectPerKernelTimingInfo, API/src/backend_cuda.t:231-297): hipEvent pairs
around every kernel of `--steps` solver steps after one warm-up step.

  python tools/kernel_table.py iw4096_mat_fused [--steps 2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from bench_families import CONFIGS  # noqa: E402
from opt_amd import OptSolver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]()
    s = OptSolver(cfg["dims"], cfg["energy"], cfg["kind"], double_precision=cfg["double"],
                  materialized=cfg.get("materialized", False), fused_jtj=cfg.get("fused", False))
    s.set_solver_params({"nIterations": a.steps + 2, "lIterations": cfg.get("liter", 10)})
    s.init(cfg["prm"])
    s.step()
    torch.cuda.synchronize()
    s.set_kernel_timing(1)
    for _ in range(a.steps):
        s.step()
    torch.cuda.synchronize()
    print(cfg["name"])
    print(s.kernel_report())


if __name__ == "__main__":
    main()
