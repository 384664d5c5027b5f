"""Per-iteration PCG scalars of the image_warping GN loop far past convergence (round-4
debugging of test_pcg_far_past_convergence_stays_finite):
  python tools/dbg_deep_pcg.py W H lIterations [fused(1|0)]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from opt_amd import workloads  # noqa: E402
from tests.iw_helpers import device_params, solver  # noqa: E402

W, H, L = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
fused = sys.argv[4] if len(sys.argv) > 4 else "1"
os.environ["OPT_AMD_IW_FUSED_RES"] = fused
w = workloads.image_warping(W, H, seed=7)
s = solver(W, H)
prm = device_params(w)
s.set_solver_params({"nIterations": 2, "lIterations": L})
s.init(prm)
print("cost0", s.cost())
for k in range(2):
    s.step(prm)
    sc = np.array(s.scalars(2 + 5 * (L + 2)))
    print("step", k + 1, "cost", s.cost())
    for i in range(L):
        rz, pap, rap, apap, rzx = sc[2 + 5 * i: 2 + 5 * i + 5]
        if i < 5 or i % 10 == 0 or not np.isfinite(rz) or i > L - 4:
            print(f"  i={i:3d} rz={rz:.4e} rz_id={rzx:.4e} pAp={pap:.4e} rAp={rap:.4e} ApAp={apap:.4e}")
