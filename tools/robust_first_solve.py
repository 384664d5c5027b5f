"""robust_nonrigid_alignment's first solve (examples/test_final_cost.py: 66.784683, "CUDA
cost of first!!! solve", the example flagged broken there) on generated kernels, for the
variants of the harness details C++ leaves open: make_float3's argument evaluation order
and libstdc++'s uniform_int_distribution algorithm (GCC < 11 downscaling / GCC 11 Lemire).
    python tools/robust_first_solve.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from opt_amd import OptSolver  # noqa: E402
from opt_amd.harness import problems  # noqa: E402

REF = 66.784683


def first_solve(w, double=False, lit=1):
    ut = torch.float64 if double else torch.float32
    c = lambda a, t=None: torch.from_numpy(np.ascontiguousarray(a)).cuda() if t is None else \
        torch.from_numpy(np.ascontiguousarray(a)).to("cuda", t)  # noqa: E731
    prm = [w["w_fitSqrt"], w["w_regSqrt"], c(w["Offset"], ut), c(w["Angle"], ut), c(w["RobustWeights"], ut),
           c(w["UrShape"]), c(w["Constraints"]), c(w["ConstraintNormals"]), None, c(w["v0"]), c(w["v1"])]
    s = OptSolver([w["N"], w["E"]], os.path.join(ROOT, "energies", "robust_nonrigid_alignment.t"), "LMGPU",
                  double_precision=double)
    s.set_solver_params({"nIterations": 1, "lIterations": lit, "function_tolerance": 1e-7})
    costs = s.profiled_solve(prm)
    s.close()
    return costs


if __name__ == "__main__":
    z = np.load(os.path.join(ROOT, "tests", "golden", "squat_first.npz"))
    for order in ("rtl", "ltr"):
        for lemire in (False, True):
            w = problems.robust_nonrigid_alignment(z["src_verts"], z["src_faces"], z["tets"], z["tgt_verts"],
                                                   z["tgt_faces"], arg_order=order, lemire=lemire)
            for double in (False, True):
                c = first_solve(w, double)
                print(order, "lemire" if lemire else "downscale", "fp64" if double else "fp32", c,
                      "rel", (c[-1] - REF) / REF, flush=True)


def all_targets(data):
    """Every squat target as the first solve's target (ml::Directory::enumerateFiles order
    is the file system's), fp32, the four harness variants."""
    from opt_amd.harness import formats
    sv, sf = formats.read_obj(os.path.join(data, "squat_source.obj"))
    te = formats.read_ele(os.path.join(data, "squat_tetmesh.ele"))
    for t in sorted(os.listdir(os.path.join(data, "squat_target"))):
        tv, tf = formats.read_obj(os.path.join(data, "squat_target", t))
        for order in ("rtl", "ltr"):
            for lemire in (False, True):
                w = problems.robust_nonrigid_alignment(sv, sf, te, tv, tf, arg_order=order, lemire=lemire)
                c = first_solve(w)
                print(t, order, "lemire" if lemire else "downscale", c, "rel", (c[-1] - REF) / REF, flush=True)
