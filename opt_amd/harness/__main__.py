"""Run one of the reference's examples on libopt_amd.so, as the example's main program
does: read its data files, build the problem, run the Opt GN and/or LM solvers with the
profiled Init/Step loop, log "final cost=" per solve (the line the reference's
solverGPUGaussNewton.t:1903 cleanup logs and examples/test_final_cost.py parses), write
results.csv (saveSolverResults) and print the final-cost report (reportFinalCosts).

Options mirror examples/shared/ArgParser.h (same names and defaults; `args.config` in the
working directory, or --config, supplies defaults below the command line as
boost::program_options does):

    python -m opt_amd.harness image_warping --data /path/to/examples/data --useOpt \\
        --backend backend_cuda --nIterations 10 --lIterations 10
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

from . import formats, problems, results

EXAMPLES = ["image_warping", "poisson_image_editing", "optical_flow", "arap_mesh_deformation", "shape_from_shading"]
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _bool(v):
    return str(v).lower() in ("1", "true", "yes", "on")


def parser():
    ap = argparse.ArgumentParser(prog="python -m opt_amd.harness", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("example", choices=EXAMPLES)
    ap.add_argument("--data", default=os.path.join("..", "data"), help="the reference's examples/data folder")
    ap.add_argument("--config", default="args.config")
    ap.add_argument("--energy", help="energy file (default: energies/<example>.t of this repository)")
    ap.add_argument("--out", default=".", help="directory for results.csv and result files")
    ap.add_argument("--double", action="store_true", help="doublePrecision = 1")
    ap.add_argument("--level", type=int, default=1, help="optical_flow: pyramid level of the solve (1 = coarse)")
    # examples/shared/ArgParser.h
    ap.add_argument("--backend", default=None)
    ap.add_argument("--numthreads", type=int, default=None)
    ap.add_argument("--oIterations", type=int, default=None)
    ap.add_argument("--nIterations", type=int, default=None)
    ap.add_argument("--lIterations", type=int, default=None)
    for b in ("useOpt", "useOptLM", "useCeres", "useMaterializedJTJ", "useFusedJTJ", "noOutput"):
        ap.add_argument("--" + b, nargs="?", const="true", default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--stride", type=int, default=None)
    ap.add_argument("--numSubdivides", type=int, default=None)
    ap.add_argument("--file", type=int, default=None)
    return ap


DEFAULTS = {"backend": "backend_cpu", "numthreads": 1, "oIterations": 1, "nIterations": 1, "lIterations": 1,
            "useOpt": "false", "useOptLM": "false", "useCeres": "false", "useMaterializedJTJ": "false",
            "useFusedJTJ": "false", "noOutput": "false", "width": 640, "height": 360, "stride": 1,
            "numSubdivides": 0, "file": 1}


def read_config(path):
    """boost::program_options config file: `key = value` lines, '#' comments."""
    out = {}
    if not os.path.exists(path):
        return out
    for line in open(path):
        line = line.split("#")[0].strip()
        if "=" in line:
            k, v = (t.strip() for t in line.split("=", 1))
            out[k] = v
    return out


def resolve(a):
    cfg = read_config(a.config)
    opts = {}
    for k, d in DEFAULTS.items():
        v = getattr(a, k)
        if v is None:
            v = cfg.get(k, d)
        opts[k] = type(d)(v) if not isinstance(d, str) or k == "backend" else v
    for b in ("useOpt", "useOptLM", "useCeres", "useMaterializedJTJ", "useFusedJTJ", "noOutput"):
        opts[b] = _bool(opts[b])
    return opts


def run(argv=None) -> int:
    a = parser().parse_args(argv)
    o = resolve(a)
    import torch  # noqa: F401  (one HIP runtime with torch, opt_amd/api.py)

    from ..api import OptSolver

    name = a.example
    energy = a.energy or os.path.join(ROOT, "energies", name + ".t")
    if o["useCeres"]:
        print("Ceres is not part of this runtime (the reference's comparison solver); skipped")
    # the arap harness raises numSubdivides to at least 1 (examples/arap_mesh_deformation/src/main.cpp)
    subdiv = max(1, o["numSubdivides"]) if name == "arap_mesh_deformation" else o["numSubdivides"]
    device = o["backend"] == "backend_cuda"
    conv = (lambda x: torch.from_numpy(x).cuda()) if device else (lambda x: x.copy())
    iters = {"gn": [], "lm": []}
    final = {"gn": 0.0, "lm": 0.0}
    last = None
    state = {"w_fit": 10.0}   # optical_flow: CombinedSolver::m_weightFit persists across solves
    for key, use, kind in (("gn", o["useOpt"], "gaussNewtonGPU"), ("lm", o["useOptLM"], "LMGPU")):
        if not use:
            continue
        w = problems.load_example(name, a.data, file=o["file"], stride=o["stride"], level=a.level,
                                  subdivisions=subdiv)
        prm = problems.problem_params(name, w, conv, double=a.double)
        s = OptSolver(problems.dims(name, w), energy, kind, backend=o["backend"], double_precision=a.double,
                      materialized=o["useMaterializedJTJ"], fused_jtj=o["useFusedJTJ"], numthreads=o["numthreads"])
        s.set_solver_params({"nIterations": o["nIterations"], "lIterations": o["lIterations"]})
        for prm in schedule(name, a, o, w, prm, conv, state):
            its = results.profiled_solve(s, prm)
            iters[key] += its
            print("final cost=%.16f" % s.cost(), flush=True)
        final[key] = s.cost()
        last = (w, prm)
        s.close()
    if not o["noOutput"]:
        os.makedirs(a.out, exist_ok=True)
        path = results.save_solver_results(a.out, "", [], iters["gn"], iters["lm"], a.double)
        print("wrote", path)
        if last is not None:
            write_result(name, last[0], last[1], a.out)
    print(results.report_final_costs(name, o["useOpt"], o["useOptLM"], final["gn"], final["lm"]))
    return 0


def schedule(name, a, o, w, prm, conv, state):
    """The example's sequence of single solves (CombinedSolverBase::singleSolve and the
    examples' solveAll overrides), yielding the problem parameters of each."""
    numIter = max(1, o["oIterations"])
    if name == "image_warping":
        # numIter solves with the constraints blended by alpha = (i + 1) / numIter
        # (examples/image_warping/src/CombinedSolver.h:150-160, setConstraintImage :199-219)
        cons = formats.read_constraints(os.path.join(a.data, problems.FILES[name][o["file"]][1]))
        for i in range(numIter):
            if numIter > 1:
                w2 = problems.image_warping(w["Mask"].reshape(w["H"], w["W"]), cons, (i + 1) / numIter)
                prm[3] = conv(np.ascontiguousarray(w2["Constraints"]))
            yield prm
    elif name == "optical_flow":
        # two pyramid levels (sigma 5, then 1), coarse first; before each level every flow
        # field is reset to zero (preSingleSolve -> resetGPU), and w_fit grows by
        # (50 - 10) / (numIter * levels) before every solve (preNonlinearSolve), the weight
        # carried over between solvers (examples/optical_flow/src/CombinedSolver.h:40-95)
        levels = {lv: problems.load_example(name, a.data, file=o["file"], stride=o["stride"], level=lv)
                  for lv in (1, 0)}
        step = np.float32(np.float32(50.0) - np.float32(10.0)) / np.float32(numIter * 2)
        ut = np.float64 if a.double else np.float32
        for lv in (1, 0):
            L = levels[lv]
            for k in ("I", "I_hat", "I_hat_dx", "I_hat_dy"):
                prm[3 + ("I", "I_hat", "I_hat_dx", "I_hat_dy").index(k)] = conv(np.ascontiguousarray(L[k]))
            for _ in range(numIter):
                prm[2] = conv(np.zeros(2 * L["W"] * L["H"], ut))
                state["w_fit"] = float(np.float32(state["w_fit"]) + step)
                prm[0] = float(np.sqrt(np.float32(state["w_fit"]), dtype=np.float32))
                yield prm
    else:
        for _ in range(numIter):
            yield prm


def write_result(name, w, prm, out):
    """The solved unknowns in the example's output format."""
    k = problems.UNKNOWN_INDEX[name]
    X = prm[k].detach().cpu().numpy() if hasattr(prm[k], "detach") else np.asarray(prm[k])
    if name == "image_warping":
        np.save(os.path.join(out, "offset.npy"), X.reshape(w["H"], w["W"], 2))
    elif name == "poisson_image_editing":
        formats.write_png(os.path.join(out, "output.png"),
                          np.clip(np.round(X.reshape(w["H"], w["W"], 4)), 0, 255).astype(np.uint8))
    elif name == "optical_flow":
        np.save(os.path.join(out, "flow.npy"), X.reshape(w["H"], w["W"], 2))
    elif name == "arap_mesh_deformation":
        formats.write_ply(os.path.join(out, "out.ply"), X.reshape(-1, 3), w.get("faces"))
    elif name == "shape_from_shading":
        formats.write_imagedump(os.path.join(out, "sfsOutput.imagedump"), X.reshape(w["H"], w["W"]).astype(np.float32))


if __name__ == "__main__":
    sys.exit(run())
