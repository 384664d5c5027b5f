"""Where do OPT_AMD_IW_REC=0 and =1 first part? Runs W x H (fp32) for 1..n GN steps with
lIterations `lit` in both layouts and prints the first step whose energies, Offset, Angle
or PCG scalars differ, with the differing pixels.
Usage: python tools/layout_diag.py W H lit [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.iw_helpers import device_params, perturbed, solver  # noqa: E402


def run(W, H, lit, n, dup):
    os.environ["OPT_AMD_IW_REC"] = dup
    w = perturbed(W, H, seed=7 * W + H)
    s = solver(W, H)
    prm = device_params(w)
    s.set_solver_params({"nIterations": n, "lIterations": lit})
    c = np.array(s.profiled_solve(prm))
    sc = np.array(s.scalars(2 + 5 * (lit + 2)))
    out = (c, prm[0].cpu().numpy(), prm[1].cpu().numpy(), sc)
    s.close()
    return out


def main():
    W, H, lit = (int(v) for v in sys.argv[1:4])
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    for n in range(1, steps + 1):
        a, b = run(W, H, lit, n, "0"), run(W, H, lit, n, "1")
        names = ("energies", "Offset", "Angle", "scalars")
        bad = [nm for nm, x, y in zip(names, a, b) if not np.array_equal(x, y)]
        print(f"steps={n}: differ: {bad or 'none'}", flush=True)
        for nm, x, y in zip(names, a, b):
            if nm in bad:
                d = np.argwhere(x != y)
                print(f"  {nm}: {len(d)} differ; first {d[:8].tolist()}", flush=True)
                for idx in d[:4]:
                    t = tuple(idx)
                    print(f"    {t}: {x[t]!r} vs {y[t]!r}", flush=True)
        if bad:
            break


if __name__ == "__main__":
    main()
