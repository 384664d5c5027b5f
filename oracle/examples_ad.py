"""Float64 automatic-differentiation restatements of the reference example energies that
have no hand-written kernel family — TEST INFRASTRUCTURE ONLY (oracle/README.md).

Importable only from tests/ (the checker); libopt_amd.so never calls it. Each energy is
restated from the reference's example file and lib.t helpers (cited per function), not
from this repository's energies/*.t lowering, so it is an independent check of the
general front end + generated kernels:

* residuals are written term by term with torch (CPU, float64); Select is torch.where;
* each term's local Jacobian comes from forward-mode AD (torch.func.jacfwd, vmapped over
  the term's instances) and is scattered into one sparse J (scipy CSR);
* the GN / LM loop is the C oracle's generic restatement of solverGPUGaussNewton.t
  (oracle/solver_impl.h, REAL = double), driven through ctypes callbacks:
  cost = 1/2 |F|^2, r = -J^T F with diag(J^T J), J^T J p, model cost 1/2 |F + J d|^2.

Pinned to the reference's known answers (examples/test_final_cost.py:58-66, CUDA,
nIterations = lIterations = 1) by tests/test_reference_costs.py.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import oracle as _c

_D = ctypes.POINTER(ctypes.c_double)


def _torch():
    import torch
    return torch


# ------------------------------------------------------------ sparse LSQ model
class Model:
    """Unknown blocks (name -> (n, ch) float64), constant arrays, and residual terms.

    A term is (fn, args, k): args = list of ("u" | "c", name, index array (M,)); fn
    maps one instance's gathered rows (1-D tensors of each arg's channel count) to k
    residuals. Unknown layout: blocks in declaration order, channels interleaved."""

    def __init__(self, blocks, consts):
        self.names = [b[0] for b in blocks]
        self.x = {n: np.ascontiguousarray(v, np.float64).reshape(len(v), -1) for n, v in blocks}
        self.c = {n: np.ascontiguousarray(v, np.float64).reshape(len(v), -1) for n, v in consts.items()}
        self.off = {}
        o = 0
        for n in self.names:
            self.off[n] = o
            o += self.x[n].size
        self.n = o
        self.terms = []

    def term(self, fn, args, k):
        self.terms.append((fn, [(a, nm, np.asarray(ix, np.int64)) for a, nm, ix in args], k))

    # flat vector <-> blocks
    def get(self):
        return np.concatenate([self.x[n].reshape(-1) for n in self.names])

    def set(self, v):
        for n in self.names:
            o, s = self.off[n], self.x[n].shape
            self.x[n] = np.asarray(v[o: o + self.x[n].size], np.float64).reshape(s).copy()

    def _gather(self, args):
        torch = _torch()
        out = []
        for a, nm, ix in args:
            src = self.x[nm] if a == "u" else self.c[nm]
            out.append(torch.from_numpy(src[ix]))
        return out

    def residuals(self):
        torch = _torch()
        F = []
        for fn, args, k in self.terms:
            g = self._gather(args)
            F.append(torch.vmap(fn)(*g).reshape(-1).numpy())
        return np.concatenate(F)

    def jacobian(self):
        import scipy.sparse as sp
        torch = _torch()
        rows, cols, vals = [], [], []
        r0 = 0
        for fn, args, k in self.terms:
            g = self._gather(args)
            upos = [i for i, (a, _, _) in enumerate(args) if a == "u"]
            M = len(args[0][2])
            if upos:
                jac = torch.vmap(torch.func.jacfwd(fn, argnums=tuple(upos)))(*g)
                for j, i in enumerate(upos):
                    _, nm, ix = args[i]
                    Jb = jac[j].numpy()                       # (M, k, ch)
                    ch = Jb.shape[2]
                    rr = r0 + np.arange(M)[:, None, None] * k + np.arange(k)[None, :, None]
                    cc = self.off[nm] + ix[:, None, None] * ch + np.arange(ch)[None, None, :]
                    rows.append(np.broadcast_to(rr, Jb.shape).reshape(-1))
                    cols.append(np.broadcast_to(cc, Jb.shape).reshape(-1))
                    vals.append(Jb.reshape(-1))
            r0 += M * k
        vals, cols = np.concatenate(vals), np.concatenate(cols)
        # diag(J^T J) as the reference forms it: one squared partial per unknown ACCESS
        # (graph slot), so a vertex in two slots of one residual adds two squares, not the
        # square of their sum (PCGInit1_Graph scatters per slot, solverGPUGaussNewton.t
        # :570-602; o.t:2969-2994)
        self.diag_access = np.bincount(cols, weights=vals * vals, minlength=self.n)
        J = sp.csr_matrix((vals, (np.concatenate(rows), cols)), shape=(r0, self.n))
        J.sum_duplicates()
        return J

    def cost(self):
        F = self.residuals()
        return 0.5 * float(F @ F)


# ------------------------------------------------------------ solver (C loop)
class _Problem(ctypes.Structure):
    pass


_COST = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_void_p)
_JTF = ctypes.CFUNCTYPE(None, ctypes.c_void_p, _D, _D)
_APPLY = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_void_p, _D, _D)
_MODEL = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_void_p, _D)
_UPD = ctypes.CFUNCTYPE(None, ctypes.c_void_p, _D)
_VOID = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
_Problem._fields_ = [("n", ctypes.c_longlong), ("act", ctypes.c_void_p), ("use_pre", ctypes.c_int),
                     ("ctx", ctypes.c_void_p), ("cost", _COST), ("jtf", _JTF), ("apply", _APPLY),
                     ("model_cost", _MODEL), ("update", _UPD), ("save", _VOID), ("revert", _VOID),
                     ("materialize", ctypes.c_void_p), ("apply_mat", ctypes.c_void_p)]


class _Params(ctypes.Structure):
    _fields_ = [("nIterations", ctypes.c_int), ("lIterations", ctypes.c_int), ("residual_reset_period", ctypes.c_int)] + \
               [(k, ctypes.c_float) for k in ("min_relative_decrease", "min_trust_region_radius",
                                              "max_trust_region_radius", "q_tolerance", "function_tolerance",
                                              "trust_region_radius", "radius_decrease_factor", "min_lm_diagonal",
                                              "max_lm_diagonal")]


def default_params(n_iter, l_iter, **kw):
    """solverGPUGaussNewton.t:41-55 (oracle/solver.h: oracle_default_params)."""
    p = _Params(n_iter, l_iter, 10, 1e-3, 1e-32, 1e16, 0.0001, 0.000001, 1e4, 2.0, 1e-6, 1e32)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def solve(model: Model, n_iter: int, l_iter: int, lm: bool = False, use_pre: bool = True, active=None, **kw):
    """GN / LM solve of `model` by the C oracle's generic loop; returns the costs after
    init and after each step (Opt_ProblemCurrentCost)."""
    lib = _c.load()
    lib.oracle_solve_f64.restype = ctypes.c_int
    lib.oracle_solve_f64.argtypes = [ctypes.POINTER(_Problem), ctypes.c_int, ctypes.POINTER(_Params), _D]
    n = model.n
    st = {"J": None, "prev": None}

    def arr(ptr):
        return np.ctypeslib.as_array(ptr, shape=(n,))

    def J():
        if st["J"] is None:
            st["J"] = model.jacobian()
        return st["J"]

    def cost(_):
        return model.cost()

    def jtf(_, r, diag):
        st["J"] = None
        Jm = J()
        arr(r)[:] = -(Jm.T @ model.residuals())
        arr(diag)[:] = model.diag_access

    def apply(_, p, Ap):
        pv = arr(p).copy()
        out = J().T @ (J() @ pv)
        arr(Ap)[:] = out
        return float(pv @ out)

    def model_cost(_, d):
        m = model.residuals() + J() @ arr(d)
        return 0.5 * float(m @ m)

    def update(_, d):
        model.set(model.get() + arr(d))
        st["J"] = None

    def save(_):
        st["prev"] = model.get()

    def revert(_):
        model.set(st["prev"])
        st["J"] = None

    act = np.ones(n, np.uint8) if active is None else np.ascontiguousarray(active, np.uint8)
    cbs = [_COST(cost), _JTF(jtf), _APPLY(apply), _MODEL(model_cost), _UPD(update), _VOID(save), _VOID(revert)]
    P = _Problem(n, act.ctypes.data, int(use_pre), None, *cbs, None, None)
    sp = default_params(n_iter, l_iter, **kw)
    costs = np.zeros(n_iter + 1)
    k = lib.oracle_solve_f64(ctypes.byref(P), int(lm), ctypes.byref(sp), costs.ctypes.data_as(_D))
    return costs[: k + 1]


# -------------------------------------------------------------- lib.t helpers
def _dot3(a, b):
    """L.Dot3 (API/src/lib.t:53-55)."""
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _rotate3d(ang, v):
    """L.Rotate3D (lib.t:84-97): row-major matrix of (alpha, beta, gamma) times v."""
    torch = _torch()
    a, b, g = ang[0], ang[1], ang[2]
    ca, cb, cg, sa, sb, sg = torch.cos(a), torch.cos(b), torch.cos(g), torch.sin(a), torch.sin(b), torch.sin(g)
    m = [cg * cb, -sg * ca + cg * sb * sa, sg * sa + cg * sb * ca,
         sg * cb, cg * ca + sg * sb * sa, -cg * sa + sg * sb * ca,
         -sb, cb * sa, cb * ca]
    return torch.stack([m[0] * v[0] + m[1] * v[1] + m[2] * v[2], m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
                        m[6] * v[0] + m[7] * v[1] + m[8] * v[2]])


def _pinned(c):
    """greatereq(Constraints(0)(0), -999999.9): the example's 'has a target' test."""
    return c[0] >= -999999.9


# ------------------------------------------------------- the example energies
def cotangent_mesh_smoothing(w) -> Model:
    """examples/cotangent_mesh_smoothing/cotangent_mesh_smoothing.t: fit w_fit (X - A) per
    vertex; per graph edge (v0 head, v1 tail, v2 / v3 the opposite vertices) the weight
    sqrt(max(0.5 (cot(v2) + cot(v3)), 1e-4)) with cot(u, v) = u.v / sqrt(max(|u|^2 |v|^2
    - (u.v)^2, 1e-4)) of the normalized spokes, times w_reg (X(v1) - X(v0))."""
    torch = _torch()
    N = w["N"]
    m = Model([("X", w["X"].reshape(N, 3))], {"A": w["A"].reshape(N, 3)})
    wf, wr = w["w_fitSqrt"], w["w_regSqrt"]
    m.term(lambda x, a: wf * (x - a), [("u", "X", np.arange(N)), ("c", "A", np.arange(N))], 3)

    def nrm(v):
        return v / torch.sqrt(_dot3(v, v))

    def cot(u, v):
        d = _dot3(u, v)
        s2 = _dot3(u, u) * _dot3(v, v) - d * d
        s2 = torch.where(s2 > 0.0, s2, torch.full_like(s2, 0.0001))
        return _dot3(u, v) / torch.sqrt(s2)

    def edge(p0, p1, p2, p3):
        wt = 0.5 * (cot(nrm(p0 - p2), nrm(p1 - p2)) + cot(nrm(p0 - p3), nrm(p1 - p3)))
        wt = torch.sqrt(torch.where(wt > 0.0, wt, torch.full_like(wt, 0.0001)))
        return wr * wt * (p1 - p0)

    m.term(edge, [("u", "X", w["v0"]), ("u", "X", w["v1"]), ("u", "X", w["v2"]), ("u", "X", w["v3"])], 3)
    return m


def embedded_mesh_deformation(w) -> Model:
    """examples/embedded_mesh_deformation/embedded_mesh_deformation.t: fit w_fit (t -
    target) where a target exists; rotation regulariser w_rot (a_i . a_j for the three
    column pairs, |a_k|^2 - 1 per column) of the row-major RotMatrix; per edge w_reg
    ((t(v1) - t(v0)) - R(v0) (g(v1) - g(v0))) (lib.t Matrix3x3Mul, :46-51)."""
    torch = _torch()
    N = w["N"]
    m = Model([("Offset", w["Offset"].reshape(N, 3)), ("RotMatrix", w["RotMatrix"].reshape(N, 9))],
              {"UrShape": w["UrShape"].reshape(N, 3), "Constraints": w["Constraints"].reshape(N, 3)})
    wf, wr, wo = w["w_fitSqrt"], w["w_regSqrt"], w["w_rotSqrt"]
    ids = np.arange(N)

    def fit(t, q):
        return torch.where(_pinned(q), wf * (t - q), torch.zeros_like(t))

    m.term(fit, [("u", "Offset", ids), ("c", "Constraints", ids)], 3)

    def rot(A):
        c = [torch.stack([A[k], A[k + 3], A[k + 6]]) for k in range(3)]
        return torch.stack([wo * _dot3(c[0], c[1]), wo * _dot3(c[0], c[2]), wo * _dot3(c[1], c[2]),
                            wo * (_dot3(c[0], c[0]) - 1), wo * (_dot3(c[1], c[1]) - 1), wo * (_dot3(c[2], c[2]) - 1)])

    m.term(rot, [("u", "RotMatrix", ids)], 6)

    def edge(t0, t1, R0, g0, g1):
        d = g1 - g0
        Rd = torch.stack([R0[0] * d[0] + R0[1] * d[1] + R0[2] * d[2], R0[3] * d[0] + R0[4] * d[1] + R0[5] * d[2],
                          R0[6] * d[0] + R0[7] * d[1] + R0[8] * d[2]])
        return wr * ((t1 - t0) - Rd)

    m.term(edge, [("u", "Offset", w["v0"]), ("u", "Offset", w["v1"]), ("u", "RotMatrix", w["v0"]),
                  ("c", "UrShape", w["v0"]), ("c", "UrShape", w["v1"])], 3)
    return m


def volumetric_mesh_deformation(w) -> Model:
    """examples/volumetric_mesh_deformation/volumetric_mesh_deformation.t: fit w_fit
    (Offset - target) where a target exists; for each of the 6 face neighbours inside the
    lattice w_reg ((O(0) - O(n)) - Rotate3D(Angle(0), U(0) - U(n)))."""
    W, H, D = w["W"], w["H"], w["D"]
    n = W * H * D
    m = Model([("Offset", w["Offset"].reshape(n, 3)), ("Angle", w["Angle"].reshape(n, 3))],
              {"UrShape": w["UrShape"].reshape(n, 3), "Constraints": w["Constraints"].reshape(n, 3)})
    wf, wr = w["w_fitSqrt"], w["w_regSqrt"]
    torch = _torch()
    ids = np.arange(n)
    m.term(lambda o, q: torch.where(_pinned(q), wf * (o - q), torch.zeros_like(o)),
           [("u", "Offset", ids), ("c", "Constraints", ids)], 3)
    z, y, x = np.meshgrid(np.arange(D), np.arange(H), np.arange(W), indexing="ij")
    for a, b, c in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)):
        ok = (x + a >= 0) & (x + a < W) & (y + b >= 0) & (y + b < H) & (z + c >= 0) & (z + c < D)
        i0 = (x + W * (y + H * z))[ok]
        i1 = ((x + a) + W * ((y + b) + H * (z + c)))[ok]
        m.term(lambda o0, o1, A0, u0, u1: wr * ((o0 - o1) - _rotate3d(A0, u0 - u1)),
               [("u", "Offset", i0), ("u", "Offset", i1), ("u", "Angle", i0), ("c", "UrShape", i0),
                ("c", "UrShape", i1)], 3)
    return m


def intrinsic_image_decomposition(w) -> Model:
    """examples/intrinsic_image_decomposition/intrinsic_image_decomposition.t: for each of
    the 4 neighbours inside the image, w_albedo * L_p(r(0) - r(n), r_const(0) - r_const(n),
    p) with L_p (lib.t:113-121) = sqrt(pow(|v_const| + 1e-7, p - 2)) * v, the weight a
    ComputedArray of the current albedo treated as a constant; w_shading (s(0) - s(n));
    fit w_fit (r + s - i). The weights are re-evaluated from the current r on every
    residual evaluation (the reference's precompute after init / each update)."""
    torch = _torch()
    W, H = w["W"], w["H"]
    n = W * H
    m = Model([("r", w["r"].reshape(n, 3)), ("s", w["s"].reshape(n, 1))], {"i": w["i"].reshape(n, 3)})
    wf, wa, ws, p = w["w_fitSqrt"], w["w_regSqrtAlbedo"], w["w_regSqrtShading"], w["pNorm"]
    y, x = np.mgrid[0:H, 0:W]
    for dx, dy in ((1, 0), (-1, 0), (0, 1), (0, -1)):
        ok = (x + dx >= 0) & (x + dx < W) & (y + dy >= 0) & (y + dy < H)
        i0 = (x + W * y)[ok]
        i1 = ((x + dx) + W * (y + dy))[ok]

        def alb(r0, r1):
            vc = (r0 - r1).detach()
            sq = torch.sqrt(torch.pow(torch.sqrt(_dot3(vc, vc)) + 0.0000001, p - 2))
            return wa * (sq * (r0 - r1))

        m.term(alb, [("u", "r", i0), ("u", "r", i1)], 3)
        m.term(lambda s0, s1: ws * (s0 - s1), [("u", "s", i0), ("u", "s", i1)], 1)
    ids = np.arange(n)
    m.term(lambda r, s, i: wf * (r + s[0] - i), [("u", "r", ids), ("u", "s", ids), ("c", "i", ids)], 3)
    return m


BUILDERS = {"cotangent_mesh_smoothing": cotangent_mesh_smoothing,
            "embedded_mesh_deformation": embedded_mesh_deformation,
            "volumetric_mesh_deformation": volumetric_mesh_deformation,
            "intrinsic_image_decomposition": intrinsic_image_decomposition}
