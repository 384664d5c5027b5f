"""ctypes binding of oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
(the checker and the timed CPU baseline). Parity status: pinned to the reference's own
known answers for image_warping, optical_flow, arap_mesh_deformation and the CSR
algebra (oracle/README.md).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_F = ctypes.POINTER(ctypes.c_float)
_D = ctypes.POINTER(ctypes.c_double)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
    lib = ctypes.CDLL(LIB)
    i, f, d = ctypes.c_int, ctypes.c_float, ctypes.c_double
    lib.oracle_iw_cost.restype = d
    lib.oracle_iw_cost.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, i]
    lib.oracle_iw_eval_jtf.restype = d
    lib.oracle_iw_eval_jtf.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, _F, _F, i]
    lib.oracle_iw_apply_jtj.restype = d
    lib.oracle_iw_apply_jtj.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, _F, _F, i]
    lib.oracle_iw_solve.restype = None
    lib.oracle_iw_solve.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, i, i, i, _D, _D]
    lib.oracle_iw_residuals.restype = None
    lib.oracle_iw_residuals.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, _F]
    _lib = lib
    return lib


def _f(a):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_F)


def _args(w):
    return (w["W"], w["H"], _f(w["Offset"]), _f(w["Angle"]), _f(w["UrShape"]), _f(w["Constraints"]),
            _f(w["Mask"]), w["w_fitSqrt"], w["w_regSqrt"])


def _iw_double_lib():
    lib = load()
    if not getattr(lib, "_iwd", False):
        i, f, d = ctypes.c_int, ctypes.c_float, ctypes.c_double
        base = [i, i, _D, _D, _F, _F, _F, f, f]
        lib.oracle_iw_cost_double.restype, lib.oracle_iw_cost_double.argtypes = d, base + [i]
        lib.oracle_iw_eval_jtf_double.restype, lib.oracle_iw_eval_jtf_double.argtypes = d, base + [_D, _D, i]
        lib.oracle_iw_apply_jtj_double.restype, lib.oracle_iw_apply_jtj_double.argtypes = d, base + [_D, _D, i]
        lib.oracle_iw_solve_double.restype, lib.oracle_iw_solve_double.argtypes = None, base + [i, i, i, _D, _D]
        lib.oracle_iw_solve_generic_double.restype = i
        lib.oracle_iw_solve_generic_double.argtypes = base + [i, i, i, i, _D]
        lib.oracle_iw_model_cost_double.restype, lib.oracle_iw_model_cost_double.argtypes = d, base + [_D]
        lib.oracle_iw_jtf_diag_double.restype, lib.oracle_iw_jtf_diag_double.argtypes = None, base + [_D, _D]
        lib._iwd = True
    return lib


def _dd(a):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_D)


def _args_double(w, O=None, A=None):
    """opt_float = double: the unknowns widened to double (or given), known arrays float."""
    O = np.ascontiguousarray(w["Offset"] if O is None else O, np.float64)
    A = np.ascontiguousarray(w["Angle"] if A is None else A, np.float64)
    return (O, A), (w["W"], w["H"], _dd(O), _dd(A), _f(w["UrShape"]), _f(w["Constraints"]), _f(w["Mask"]),
                    w["w_fitSqrt"], w["w_regSqrt"])


def iw_cost(w, nthreads=1, double=False):
    if double:
        keep, a = _args_double(w)
        return _iw_double_lib().oracle_iw_cost_double(*a, nthreads)
    return load().oracle_iw_cost(*_args(w), nthreads)


def iw_eval_jtf(w, nthreads=1, double=False):
    n = 3 * w["W"] * w["H"]
    if double:
        keep, a = _args_double(w)
        r, pre = np.zeros(n, np.float64), np.zeros(n, np.float64)
        rz = _iw_double_lib().oracle_iw_eval_jtf_double(*a, _dd(r), _dd(pre), nthreads)
        return r, pre, rz
    r = np.zeros(n, np.float32)
    pre = np.zeros(n, np.float32)
    rz = load().oracle_iw_eval_jtf(*_args(w), _f(r), _f(pre), nthreads)
    return r, pre, rz


def iw_apply_jtj(w, p, nthreads=1, double=False):
    if double:
        keep, a = _args_double(w)
        p = np.ascontiguousarray(p, np.float64)
        Ap = np.zeros_like(p)
        pAp = _iw_double_lib().oracle_iw_apply_jtj_double(*a, _dd(p), _dd(Ap), nthreads)
        return Ap, pAp
    p = np.ascontiguousarray(p, np.float32)
    Ap = np.zeros_like(p)
    pAp = load().oracle_iw_apply_jtj(*_args(w), _f(p), _f(Ap), nthreads)
    return Ap, pAp


def iw_residuals(w):
    """All residuals, 10 per pixel: for s in (+x,-x,+y,-y): (c=0,c=1), then fit (c=0,c=1)."""
    res = np.zeros(10 * w["W"] * w["H"], np.float32)
    load().oracle_iw_residuals(*_args(w), _f(res))
    return res


def iw_solve(w, n_iter, l_iter, nthreads=1, want_scalars=False, double=False):
    """Full GN solve; returns (Offset, Angle, costs[n_iter+1], scalars|None). double: the
    reference's doublePrecision mode (unknowns and solver in double, known arrays float)."""
    dt = np.float64 if double else np.float32
    O = w["Offset"].astype(dt)
    A = w["Angle"].astype(dt)
    costs = np.zeros(n_iter + 1, np.float64)
    sc = np.zeros(max(1, 3 * n_iter * l_iter), np.float64) if want_scalars else None
    scp = sc.ctypes.data_as(_D) if sc is not None else None
    if double:
        _iw_double_lib().oracle_iw_solve_double(w["W"], w["H"], _dd(O), _dd(A), _f(w["UrShape"]),
                                                _f(w["Constraints"]), _f(w["Mask"]), w["w_fitSqrt"],
                                                w["w_regSqrt"], n_iter, l_iter, nthreads, costs.ctypes.data_as(_D),
                                                scp)
    else:
        load().oracle_iw_solve(w["W"], w["H"], _f(O), _f(A), _f(w["UrShape"]), _f(w["Constraints"]),
                               _f(w["Mask"]), w["w_fitSqrt"], w["w_regSqrt"], n_iter, l_iter, nthreads,
                               costs.ctypes.data_as(_D), scp)
    return O, A, costs, (sc.reshape(n_iter, l_iter, 3) if sc is not None else None)


def _iwg_lib():
    lib = load()
    if not getattr(lib, "_iwg", False):
        i, f, d = ctypes.c_int, ctypes.c_float, ctypes.c_double
        lib.oracle_iw_solve_generic.restype = i
        lib.oracle_iw_solve_generic.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, i, i, i, i, _D]
        lib.oracle_iw_jtf_diag.restype = None
        lib.oracle_iw_jtf_diag.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, _F, _F]
        lib.oracle_iw_model_cost.restype = d
        lib.oracle_iw_model_cost.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, _F]
        lib._iwg = True
    return lib


def iw_jtf_diag(w, double=False):
    """r = -J^T F and the raw diagonal of J^T J (generic driver layout)."""
    n = 3 * w["W"] * w["H"]
    if double:
        keep, a = _args_double(w)
        r, dg = np.zeros(n, np.float64), np.zeros(n, np.float64)
        _iw_double_lib().oracle_iw_jtf_diag_double(*a, _dd(r), _dd(dg))
        return r, dg
    r = np.zeros(n, np.float32)
    dg = np.zeros(n, np.float32)
    _iwg_lib().oracle_iw_jtf_diag(*_args(w), _f(r), _f(dg))
    return r, dg


def iw_model_cost(w, delta, double=False):
    if double:
        keep, a = _args_double(w)
        return _iw_double_lib().oracle_iw_model_cost_double(*a, _dd(np.ascontiguousarray(delta, np.float64)))
    delta = np.ascontiguousarray(delta, np.float32)
    return _iwg_lib().oracle_iw_model_cost(*_args(w), _f(delta))


def iw_solve_generic(w, n_iter, l_iter, lm=False, nthreads=1, double=False):
    """GN or LM solve through the generic loop (solver_impl.h); returns (O, A, costs)."""
    if double:
        (O, A), a = _args_double(w, w["Offset"].astype(np.float64), w["Angle"].astype(np.float64))
        costs = np.zeros(n_iter + 1, np.float64)
        k = _iw_double_lib().oracle_iw_solve_generic_double(*a, int(lm), n_iter, l_iter, nthreads,
                                                            costs.ctypes.data_as(_D))
        return O, A, costs[: k + 1]
    O = w["Offset"].copy()
    A = w["Angle"].copy()
    costs = np.zeros(n_iter + 1, np.float64)
    k = _iwg_lib().oracle_iw_solve_generic(w["W"], w["H"], _f(O), _f(A), _f(w["UrShape"]), _f(w["Constraints"]),
                                           _f(w["Mask"]), w["w_fitSqrt"], w["w_regSqrt"], int(lm), n_iter, l_iter,
                                           nthreads, costs.ctypes.data_as(_D))
    return O, A, costs[: k + 1]


# ------------------------------------------------------------ poisson_image_editing
def _pie_lib():
    lib = load()
    if not getattr(lib, "_pie", False):
        i, d = ctypes.c_int, ctypes.c_double
        lib.oracle_pie_cost.restype = d
        lib.oracle_pie_cost.argtypes = [i, i, _F, _F, _F]
        lib.oracle_pie_jtf.restype = None
        lib.oracle_pie_jtf.argtypes = [i, i, _F, _F, _F, _F, _F]
        lib.oracle_pie_apply.restype = d
        lib.oracle_pie_apply.argtypes = [i, i, _F, _F, _F, _F, _F]
        lib.oracle_pie_solve.restype = i
        lib.oracle_pie_solve.argtypes = [i, i, _F, _F, _F, i, i, i, _D]
        lib.oracle_pie_cost_double.restype = d
        lib.oracle_pie_cost_double.argtypes = [i, i, _D, _F, _F]
        lib.oracle_pie_jtf_double.restype = None
        lib.oracle_pie_jtf_double.argtypes = [i, i, _D, _F, _F, _D, _D]
        lib.oracle_pie_apply_double.restype = d
        lib.oracle_pie_apply_double.argtypes = [i, i, _D, _F, _F, _D, _D]
        lib.oracle_pie_solve_double.restype = i
        lib.oracle_pie_solve_double.argtypes = [i, i, _D, _F, _F, i, i, i, _D]
        lib._pie = True
    return lib


def _pie_x(w, double, X=None):
    X = np.ascontiguousarray(w["X"] if X is None else X, np.float64 if double else np.float32)
    return X, (X.ctypes.data_as(_D if double else _F))


def pie_cost(w, double=False):
    X, xp = _pie_x(w, double)
    fn = _pie_lib().oracle_pie_cost_double if double else _pie_lib().oracle_pie_cost
    return fn(w["W"], w["H"], xp, _f(w["T"]), _f(w["M"]))


def pie_jtf(w, double=False):
    dt = np.float64 if double else np.float32
    n = 4 * w["W"] * w["H"]
    r = np.zeros(n, dt)
    dg = np.zeros(n, dt)
    X, xp = _pie_x(w, double)
    P = _D if double else _F
    fn = _pie_lib().oracle_pie_jtf_double if double else _pie_lib().oracle_pie_jtf
    fn(w["W"], w["H"], xp, _f(w["T"]), _f(w["M"]), r.ctypes.data_as(P), dg.ctypes.data_as(P))
    return r, dg


def pie_apply(w, p, double=False):
    dt = np.float64 if double else np.float32
    P = _D if double else _F
    p = np.ascontiguousarray(p, dt)
    Ap = np.zeros_like(p)
    X, xp = _pie_x(w, double)
    fn = _pie_lib().oracle_pie_apply_double if double else _pie_lib().oracle_pie_apply
    pAp = fn(w["W"], w["H"], xp, _f(w["T"]), _f(w["M"]), p.ctypes.data_as(P), Ap.ctypes.data_as(P))
    return Ap, pAp


def pie_solve(w, n_iter, l_iter, lm=False, double=False):
    X, xp = _pie_x(w, double, w["X"].astype(np.float64 if double else np.float32))
    costs = np.zeros(n_iter + 1, np.float64)
    fn = _pie_lib().oracle_pie_solve_double if double else _pie_lib().oracle_pie_solve
    k = fn(w["W"], w["H"], xp, _f(w["T"]), _f(w["M"]), int(lm), n_iter, l_iter, costs.ctypes.data_as(_D))
    return X, costs[: k + 1]


# ------------------------------------------------------------ optical_flow
def _of_lib():
    lib = load()
    if not getattr(lib, "_of", False):
        i, f, d = ctypes.c_int, ctypes.c_float, ctypes.c_double
        for R, P in (("float", _F), ("double", _D)):
            g = getattr(lib, "oracle_of_cost_" + R)
            g.restype, g.argtypes = d, [i, i, P, _F, _F, _F, _F, f, f]
            g = getattr(lib, "oracle_of_jtf_" + R)
            g.restype, g.argtypes = None, [i, i, P, _F, _F, _F, _F, f, f, P, P]
            g = getattr(lib, "oracle_of_apply_" + R)
            g.restype, g.argtypes = d, [i, i, P, _F, _F, _F, _F, f, f, P, P]
            g = getattr(lib, "oracle_of_model_cost_" + R)
            g.restype, g.argtypes = d, [i, i, P, _F, _F, _F, _F, f, f, P]
            g = getattr(lib, "oracle_of_solve_" + R)
            g.restype, g.argtypes = i, [i, i, P, _F, _F, _F, _F, f, f, i, i, i, _D]
        lib._of = True
    return lib


def _of_real(double):
    return (np.float64, _D, "double") if double else (np.float32, _F, "float")


def _of_args(w, X, double):
    dt, P, _ = _of_real(double)
    X = np.ascontiguousarray(X, dt)
    return X, (w["W"], w["H"], X.ctypes.data_as(P), _f(w["I"]), _f(w["I_hat"]), _f(w["I_hat_dx"]),
               _f(w["I_hat_dy"]), w["w_fitSqrt"], w["w_regSqrt"])


def of_cost(w, X=None, double=False):
    X, a = _of_args(w, w["X"] if X is None else X, double)
    return getattr(_of_lib(), "oracle_of_cost_" + _of_real(double)[2])(*a)


def of_jtf(w, X=None, double=False):
    dt, P, R = _of_real(double)
    X, a = _of_args(w, w["X"] if X is None else X, double)
    n = 2 * w["W"] * w["H"]
    r, dg = np.zeros(n, dt), np.zeros(n, dt)
    getattr(_of_lib(), "oracle_of_jtf_" + R)(*a, r.ctypes.data_as(P), dg.ctypes.data_as(P))
    return r, dg


def of_apply(w, p, X=None, double=False):
    dt, P, R = _of_real(double)
    X, a = _of_args(w, w["X"] if X is None else X, double)
    p = np.ascontiguousarray(p, dt)
    Ap = np.zeros_like(p)
    v = getattr(_of_lib(), "oracle_of_apply_" + R)(*a, p.ctypes.data_as(P), Ap.ctypes.data_as(P))
    return Ap, v


def of_model_cost(w, d, X=None, double=False):
    dt, P, R = _of_real(double)
    X, a = _of_args(w, w["X"] if X is None else X, double)
    d = np.ascontiguousarray(d, dt)
    return getattr(_of_lib(), "oracle_of_model_cost_" + R)(*a, d.ctypes.data_as(P))


def of_solve(w, n_iter, l_iter, lm=False, double=False, X=None):
    """GN / LM solve; returns (X, costs)."""
    X, a = _of_args(w, (w["X"] if X is None else X).copy(), double)
    costs = np.zeros(n_iter + 1, np.float64)
    k = getattr(_of_lib(), "oracle_of_solve_" + _of_real(double)[2])(*a, int(lm), n_iter, l_iter,
                                                                     costs.ctypes.data_as(_D))
    return X, costs[: k + 1]


# ------------------------------------------------------------ shape_from_shading
_U8 = ctypes.POINTER(ctypes.c_ubyte)


def _sfs_lib():
    lib = load()
    if not getattr(lib, "_sfs", False):
        i, d = ctypes.c_int, ctypes.c_double
        for suf, R in (("", _F), ("_double", _D)):
            base = [i, i, R, _F, _F, _U8, _U8, _F]
            for name, res, extra in (("precompute", None, [R]), ("cost", d, []), ("jtf", None, [R, R]),
                                     ("apply", d, [R, R]), ("model_cost", d, [R]), ("solve", i, [i, i, i, _D, i])):
                fn = getattr(lib, "oracle_sfs_" + name + suf)
                fn.restype, fn.argtypes = res, base + extra
        lib._sfs = True
    return lib


def _real(double):
    """(numpy dtype, ctypes pointer type, entry-point suffix) of opt_float"""
    return (np.float64, _D, "_double") if double else (np.float32, _F, "")


def _sfs_args(w, X, double=False):
    dt, R, _ = _real(double)
    X = np.ascontiguousarray(X, dt)
    keep = [np.ascontiguousarray(w["edgeMaskR"], np.uint8), np.ascontiguousarray(w["edgeMaskC"], np.uint8),
            np.ascontiguousarray(w["params"], np.float32)]
    return X, keep, (w["W"], w["H"], X.ctypes.data_as(R), _f(w["D_i"]), _f(w["Im"]), keep[0].ctypes.data_as(_U8),
                     keep[1].ctypes.data_as(_U8), _f(keep[2]))


def _sfs_fn(name, double):
    return getattr(_sfs_lib(), "oracle_sfs_" + name + _real(double)[2])


def sfs_precompute(w, X=None, double=False):
    """[B_I, dB_I/dX(0,0), dB_I/dX(-1,0), dB_I/dX(0,-1), valid], each W*H."""
    dt, R, _ = _real(double)
    X, keep, a = _sfs_args(w, w["X"] if X is None else X, double)
    out = np.zeros(5 * w["W"] * w["H"], dt)
    _sfs_fn("precompute", double)(*a, out.ctypes.data_as(R))
    return out.reshape(5, -1)


def sfs_cost(w, X=None, double=False):
    X, keep, a = _sfs_args(w, w["X"] if X is None else X, double)
    return _sfs_fn("cost", double)(*a)


def sfs_jtf(w, X=None, double=False):
    dt, R, _ = _real(double)
    X, keep, a = _sfs_args(w, w["X"] if X is None else X, double)
    n = w["W"] * w["H"]
    r, dg = np.zeros(n, dt), np.zeros(n, dt)
    _sfs_fn("jtf", double)(*a, r.ctypes.data_as(R), dg.ctypes.data_as(R))
    return r, dg


def sfs_apply(w, p, X=None, double=False):
    dt, R, _ = _real(double)
    X, keep, a = _sfs_args(w, w["X"] if X is None else X, double)
    p = np.ascontiguousarray(p, dt)
    Ap = np.zeros_like(p)
    v = _sfs_fn("apply", double)(*a, p.ctypes.data_as(R), Ap.ctypes.data_as(R))
    return Ap, v


def sfs_model_cost(w, d, X=None, double=False):
    dt, R, _ = _real(double)
    X, keep, a = _sfs_args(w, w["X"] if X is None else X, double)
    d = np.ascontiguousarray(d, dt)
    return _sfs_fn("model_cost", double)(*a, d.ctypes.data_as(R))


def sfs_solve(w, n_iter, l_iter, lm=True, double=False, nthreads=1):
    """LM (or GN) solve; nthreads: the stencil passes split over row slabs on that many
    threads (backend_cpu_mt.t:716-737), per-thread sums added in thread order."""
    X, keep, a = _sfs_args(w, w["X"].copy(), double)
    costs = np.zeros(n_iter + 1, np.float64)
    k = _sfs_fn("solve", double)(*a, int(lm), n_iter, l_iter, costs.ctypes.data_as(_D), nthreads)
    return X, costs[: k + 1]


# ------------------------------------------------------------ arap_mesh_deformation
_I = ctypes.POINTER(ctypes.c_int)


def _arap_lib():
    lib = load()
    if not getattr(lib, "_arap", False):
        i, f, d = ctypes.c_int, ctypes.c_float, ctypes.c_double
        for suf, R in (("", _F), ("_double", _D)):
            base = [i, i, R, R, _F, _F, _I, _I, f, f]
            for name, res, extra in (("cost", d, []), ("jtf", None, [R, R]), ("apply", d, [R, R]),
                                     ("model_cost", d, [R]), ("solve", i, [i, i, i, _D])):
                fn = getattr(lib, "oracle_arap_" + name + suf)
                fn.restype, fn.argtypes = res, base + extra
        lib._arap = True
    return lib


def _arap_fn(name, double):
    return getattr(_arap_lib(), "oracle_arap_" + name + _real(double)[2])


def _arap_args(w, O=None, A=None, double=False):
    dt, R, _ = _real(double)
    O = np.ascontiguousarray(w["Offset"] if O is None else O, dt)
    A = np.ascontiguousarray(w["Angle"] if A is None else A, dt)
    v0 = np.ascontiguousarray(w["v0"], np.int32)
    v1 = np.ascontiguousarray(w["v1"], np.int32)
    keep = (O, A, v0, v1)
    return keep, (w["N"], w["E"], O.ctypes.data_as(R), A.ctypes.data_as(R), _f(w["UrShape"]), _f(w["Constraints"]),
                  v0.ctypes.data_as(_I), v1.ctypes.data_as(_I), w["w_fitSqrt"], w["w_regSqrt"])


def arap_cost(w, double=False):
    keep, a = _arap_args(w, double=double)
    return _arap_fn("cost", double)(*a)


def arap_jtf(w, double=False):
    dt, R, _ = _real(double)
    keep, a = _arap_args(w, double=double)
    n = 6 * w["N"]
    r, dg = np.zeros(n, dt), np.zeros(n, dt)
    _arap_fn("jtf", double)(*a, r.ctypes.data_as(R), dg.ctypes.data_as(R))
    return r, dg


def arap_apply(w, p, double=False):
    dt, R, _ = _real(double)
    keep, a = _arap_args(w, double=double)
    p = np.ascontiguousarray(p, dt)
    Ap = np.zeros_like(p)
    v = _arap_fn("apply", double)(*a, p.ctypes.data_as(R), Ap.ctypes.data_as(R))
    return Ap, v


def arap_model_cost(w, d, double=False):
    dt, R, _ = _real(double)
    keep, a = _arap_args(w, double=double)
    d = np.ascontiguousarray(d, dt)
    return _arap_fn("model_cost", double)(*a, d.ctypes.data_as(R))


def arap_solve(w, n_iter, l_iter, lm=False, double=False):
    dt = _real(double)[0]
    O, A = w["Offset"].astype(dt), w["Angle"].astype(dt)
    keep, a = _arap_args(w, O, A, double)
    costs = np.zeros(n_iter + 1, np.float64)
    k = _arap_fn("solve", double)(*a, int(lm), n_iter, l_iter, costs.ctypes.data_as(_D))
    return O, A, costs[: k + 1]


# ------------------------------------------------------------ CSR / materialized J
_I = ctypes.POINTER(ctypes.c_int)


def _csr_lib():
    lib = load()
    if not getattr(lib, "_csr", False):
        i, f, d = ctypes.c_int, ctypes.c_float, ctypes.c_double
        lib.oracle_csr_pattern_at.restype = None
        lib.oracle_csr_pattern_at.argtypes = [i, i, i, _I, _I, _I, _I]
        lib.oracle_csr_at.restype = None
        lib.oracle_csr_at.argtypes = [i, i, i, _F, _I, _I, _F, _I, _I]
        lib.oracle_csr_pattern_ata.restype = i
        lib.oracle_csr_pattern_ata.argtypes = [i, i, i, _I, _I, _I, _I]
        lib.oracle_csr_ata.restype = None
        lib.oracle_csr_ata.argtypes = [i, i, i, i, _F, _I, _I, _F, _I, _I, _F, _I, _I]
        lib.oracle_csr_spmv.restype = None
        lib.oracle_csr_spmv.argtypes = [i, i, i, _F, _I, _I, _F, _F]
        lib.oracle_iw_dump_j.restype = None
        lib.oracle_iw_dump_j.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, _I, _I, _F]
        lib.oracle_iw_solve_materialized.restype = i
        lib.oracle_iw_solve_materialized.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, i, i, i, i, _D]
        lib.oracle_iw_apply_materialized.restype = d
        lib.oracle_iw_apply_materialized.argtypes = [i, i, _F, _F, _F, _F, _F, f, f, i, _F, _F]
        lib.oracle_pie_dump_j.restype = None
        lib.oracle_pie_dump_j.argtypes = [i, i, _F, _F, _F, _I, _I, _F]
        lib.oracle_pie_apply_materialized.restype = d
        lib.oracle_pie_apply_materialized.argtypes = [i, i, _F, _F, _F, i, _F, _F]
        lib.oracle_pie_solve_materialized.restype = i
        lib.oracle_pie_solve_materialized.argtypes = [i, i, _F, _F, _F, i, i, i, i, _D]
        lib._csr = True
    return lib


def _i(a):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_I)


def csr_transpose(n_rows, n_cols, rowPtr, colInd, val):
    """computeNnzPatternAT + computeAT (linalg_cpu.t:203-297, 512-551)."""
    lib = _csr_lib()
    nnz = len(colInd)
    rpT = np.zeros(n_cols + 1, np.int32)
    ciT = np.zeros(max(nnz, 1), np.int32)
    vT = np.zeros(max(nnz, 1), np.float32)
    lib.oracle_csr_pattern_at(n_cols, n_rows, nnz, _i(rowPtr), _i(colInd), _i(rpT), _i(ciT))
    lib.oracle_csr_at(n_cols, n_rows, nnz, _f(val), _i(rowPtr), _i(colInd), _f(vT), _i(rpT), _i(ciT))
    return rpT, ciT[:nnz], vT[:nnz]


def csr_ata(n_rows, n_cols, rowPtr, colInd, val):
    """computeNnzPatternATA + computeATA (linalg_cpu.t:300-508)."""
    lib = _csr_lib()
    nnz = len(colInd)
    rp = np.zeros(n_cols + 1, np.int32)
    m = lib.oracle_csr_pattern_ata(n_cols, n_rows, nnz, _i(rowPtr), _i(colInd), _i(rp), None)
    ci = np.zeros(max(m, 1), np.int32)
    lib.oracle_csr_pattern_ata(n_cols, n_rows, nnz, _i(rowPtr), _i(colInd), _i(rp), _i(ci))
    rpT, ciT, vT = csr_transpose(n_rows, n_cols, rowPtr, colInd, val)
    rpT = np.ascontiguousarray(rpT)
    ciT = np.ascontiguousarray(ciT)
    vT = np.ascontiguousarray(vT)
    v = np.zeros(max(m, 1), np.float32)
    lib.oracle_csr_ata(n_cols, n_rows, nnz, m, _f(val), _i(rowPtr), _i(colInd), _f(vT), _i(rpT), _i(ciT), _f(v),
                       _i(rp), _i(ci))
    return rp, ci[:m], v[:m]


def csr_spmv(n_rows, n_cols, rowPtr, colInd, val, x):
    """applyAtoVector (linalg_cpu.t:560-600)."""
    y = np.zeros(n_rows, np.float32)
    _csr_lib().oracle_csr_spmv(n_cols, n_rows, len(colInd), _f(val), _i(rowPtr), _i(colInd),
                               _f(np.ascontiguousarray(x, np.float32)), _f(y))
    return y


def iw_dump_j(w):
    """J of image_warping in the runtime's CSR layout: 10 rows / 26 nonzeros per pixel."""
    N = w["W"] * w["H"]
    rp = np.zeros(10 * N + 1, np.int32)
    ci = np.zeros(26 * N, np.int32)
    v = np.zeros(26 * N, np.float32)
    _csr_lib().oracle_iw_dump_j(*_args(w), _i(rp), _i(ci), _f(v))
    return rp, ci, v


def iw_apply_materialized(w, p, fused=True):
    p = np.ascontiguousarray(p, np.float32)
    Ap = np.zeros_like(p)
    pAp = _csr_lib().oracle_iw_apply_materialized(*_args(w), int(fused), _f(p), _f(Ap))
    return Ap, pAp


def iw_solve_materialized(w, n_iter, l_iter, lm=False, fused=True):
    O = w["Offset"].copy()
    A = w["Angle"].copy()
    costs = np.zeros(n_iter + 1, np.float64)
    k = _csr_lib().oracle_iw_solve_materialized(w["W"], w["H"], _f(O), _f(A), _f(w["UrShape"]),
                                                _f(w["Constraints"]), _f(w["Mask"]), w["w_fitSqrt"],
                                                w["w_regSqrt"], int(lm), int(fused), n_iter, l_iter,
                                                costs.ctypes.data_as(_D))
    return O, A, costs[: k + 1]


def pie_dump_j(w):
    N = w["W"] * w["H"]
    rp = np.zeros(16 * N + 1, np.int32)
    ci = np.zeros(32 * N, np.int32)
    v = np.zeros(32 * N, np.float32)
    _csr_lib().oracle_pie_dump_j(w["W"], w["H"], _f(w["X"]), _f(w["T"]), _f(w["M"]), _i(rp), _i(ci), _f(v))
    return rp, ci, v


def pie_solve_materialized(w, n_iter, l_iter, lm=False, fused=True):
    X = w["X"].copy()
    costs = np.zeros(n_iter + 1, np.float64)
    k = _csr_lib().oracle_pie_solve_materialized(w["W"], w["H"], _f(X), _f(w["T"]), _f(w["M"]), int(lm), int(fused),
                                                 n_iter, l_iter, costs.ctypes.data_as(_D))
    return X, costs[: k + 1]


def pie_apply_materialized(w, p, fused=True):
    p = np.ascontiguousarray(p, np.float32)
    Ap = np.zeros_like(p)
    pAp = _csr_lib().oracle_pie_apply_materialized(w["W"], w["H"], _f(w["X"]), _f(w["T"]), _f(w["M"]), int(fused),
                                                   _f(p), _f(Ap))
    return Ap, pAp
