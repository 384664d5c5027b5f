"""SolverIteration bookkeeping, the results CSV and the final-cost report
(examples/shared/SolverIteration.h:12-86) and the profiled solve loop
(launchProfiledSolve, examples/shared/OptUtils.h:47-64)."""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import List


@dataclass
class SolverIteration:
    cost: float = -math.inf
    timeInMS: float = -math.inf


def profiled_solve(solver, problem_params, sync=None) -> List[SolverIteration]:
    """Init, then Step until it returns 0; one SolverIteration per call with the cost after
    it and its wall time (the reference times each call with a CUDA timer,
    OptUtils.h:47-64). `sync` waits for the device (the C ABI calls already return
    synchronised; kept for callers that queue their own work)."""
    its = []
    t0 = time.perf_counter()
    solver.init(problem_params)
    if sync:
        sync()
    its.append(SolverIteration(solver.cost(), 1000.0 * (time.perf_counter() - t0)))
    while True:
        t0 = time.perf_counter()
        more = solver.step()
        if sync:
            sync()
        its.append(SolverIteration(solver.cost(), 1000.0 * (time.perf_counter() - t0)))
        if not more:
            break
    return its


def _clamped(v: List[SolverIteration], i: int) -> SolverIteration:
    return v[0] if i < 0 else v[-1] if i >= len(v) else v[i]


def _sci(x: float) -> str:
    """std::scientific with setprecision(20)."""
    return "%.20e" % x


def save_solver_results(directory: str, suffix: str, ceres: List[SolverIteration], gn: List[SolverIteration],
                        lm: List[SolverIteration], double_precision: bool) -> str:
    """results<suffix>.csv exactly as saveSolverResults writes it (SolverIteration.h:28-66)."""
    import os

    col = " (double)" if double_precision else " (float)"
    lines = ["Iter, Ceres Error, Opt(GN) Error%s,  Opt(LM) Error%s, Ceres Iter Time(ms), "
             "Opt(GN) Iter Time(ms)%s, Opt(LM) Iter Time(ms)%s, Total Ceres Time(ms), "
             "Total Opt(GN) Time(ms)%s, Total Opt(LM) Time(ms)%s" % ((col,) * 6)]
    c = list(ceres) or [SolverIteration(0, 0)]
    g = list(gn) or [SolverIteration(0, 0)]
    m = list(lm) or [SolverIteration(0, 0)]
    sc = sg = sm = 0.0
    for i in range(max(len(c), len(g), len(m))):
        tc = c[i].timeInMS if len(c) > i else 0.0
        tg = g[i].timeInMS if len(g) > i else 0.0
        tm = m[i].timeInMS if len(m) > i else 0.0
        sc += tc
        sg += tg
        sm += tm
        lines.append(", ".join([str(i), _sci(_clamped(c, i).cost), _sci(_clamped(g, i).cost),
                                _sci(_clamped(m, i).cost), _sci(tc), _sci(tg), _sci(tm), _sci(sc), _sci(sg),
                                _sci(sm)]))
    path = os.path.join(directory, "results" + suffix + ".csv")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def report_final_costs(name: str, use_gn: bool, use_lm: bool, gn_cost: float, lm_cost: float,
                       use_ceres: bool = False, ceres_cost: float = 0.0) -> str:
    """reportFinalCosts (SolverIteration.h:69-86)."""
    out = ["===%s===" % name, "**Final Costs**", "Opt GN,Opt LM,CERES",
           (_sci(gn_cost) if use_gn else "") + "," + (_sci(lm_cost) if use_lm else "") + "," +
           (_sci(ceres_cost) if use_ceres else "")]
    return "\n".join(out)
