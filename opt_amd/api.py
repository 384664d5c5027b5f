"""ctypes binding of libopt_amd.so and a Python mirror of the reference's OptSolver.

Mirrors examples/shared/OptSolver.h:46-106 (state/problem/plan lifetime, solve) and
examples/shared/OptUtils.h:47-64 (profiled Init/Step loop) and 108-112 (solver
parameters by name). Problem parameters are passed exactly as the reference's
NamedParameters::data() packs them (examples/shared/NamedParameters.h:35-49): one
``void*`` per declared index — a device (or, for the CPU backends, host) array
pointer for Array/Unknown, a pointer to the value for Param.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libopt_amd.so")


class OptError(RuntimeError):
    pass


class InitParams(ctypes.Structure):
    """Opt_InitializationParameters (include/Opt.h; reference Opt.h:10-35)."""

    _fields_ = [
        ("doublePrecision", ctypes.c_int),
        ("verbosityLevel", ctypes.c_int),
        ("collectPerKernelTimingInfo", ctypes.c_int),
        ("backend", ctypes.c_char * 20),
        ("numthreads", ctypes.c_int),
        ("useMaterializedJTJ", ctypes.c_int),
        ("useFusedJTJ", ctypes.c_int),
    ]


assert ctypes.sizeof(InitParams) == 44

_lib = None

# (name, restype, argtypes) for every symbol of include/Opt.h and include/opt_amd.h
_VP = ctypes.c_void_p
_SIGNATURES = [
    ("Opt_NewState", _VP, [InitParams]),
    ("Opt_ProblemDefine", _VP, [_VP, ctypes.c_char_p, ctypes.c_char_p]),
    ("Opt_ProblemDelete", None, [_VP, _VP]),
    ("Opt_ProblemPlan", _VP, [_VP, _VP, ctypes.POINTER(ctypes.c_uint)]),
    ("Opt_PlanFree", None, [_VP, _VP]),
    ("Opt_SetSolverParameter", None, [_VP, _VP, ctypes.c_char_p, _VP]),
    ("Opt_ProblemSolve", None, [_VP, _VP, ctypes.POINTER(_VP)]),
    ("Opt_ProblemInit", None, [_VP, _VP, ctypes.POINTER(_VP)]),
    ("Opt_ProblemStep", ctypes.c_int, [_VP, _VP, ctypes.POINTER(_VP)]),
    ("Opt_ProblemCurrentCost", ctypes.c_double, [_VP, _VP]),
    ("OptAMD_PlanUnknownCount", ctypes.c_longlong, [_VP]),
    ("OptAMD_PlanFamily", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_ProblemFamily", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_GenericSignature", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_EvalJTF", ctypes.c_int, [_VP, _VP, ctypes.POINTER(_VP), _VP, _VP, ctypes.POINTER(ctypes.c_double)]),
    ("OptAMD_ApplyJTJ", ctypes.c_int, [_VP, _VP, ctypes.POINTER(_VP), _VP, _VP, ctypes.POINTER(ctypes.c_double)]),
    ("OptAMD_EvalCost", ctypes.c_double, [_VP, _VP, ctypes.POINTER(_VP)]),
    ("OptAMD_TimeApplyJTJ", ctypes.c_double, [_VP, _VP, ctypes.POINTER(_VP), _VP, _VP, ctypes.c_int]),
    ("OptAMD_SetKernelTiming", None, [_VP, ctypes.c_int]),
    ("OptAMD_KernelStat", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]),
    ("OptAMD_ApplyKernelName", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_KernelReport", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_PlanStream", _VP, [_VP]),
    ("OptAMD_PlanIterations", ctypes.c_int, [_VP]),
    ("OptAMD_PlanScalars", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    ("OptAMD_RcclUniqueId", ctypes.c_int, [_VP]),
    ("OptAMD_CommCreateRccl", _VP, [_VP, ctypes.c_int, ctypes.c_int]),
    ("OptAMD_CommDestroy", None, [_VP]),
    ("OptAMD_CommSize", ctypes.c_int, [_VP]),
    ("OptAMD_CommRank", ctypes.c_int, [_VP]),
    ("OptAMD_CommKind", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_PlanError", ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_LocalGroupCreate", _VP, [ctypes.c_int]),
    ("OptAMD_LocalGroupRank", _VP, [_VP, ctypes.c_int]),
    ("OptAMD_LocalGroupDestroy", None, [_VP]),
    ("OptAMD_PlanHalo", ctypes.c_int, [_VP]),
    ("OptAMD_PlanSetDecomposition", ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.c_int]),
    ("OptAMD_PlanJacobianShape", ctypes.c_longlong, [_VP, ctypes.POINTER(ctypes.c_longlong)]),
    ("OptAMD_PlanMaterializedNonzeros", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_longlong),
                                                       ctypes.POINTER(ctypes.c_longlong)]),
    ("OptAMD_EvalJacobian", ctypes.c_int, [_VP, _VP, ctypes.POINTER(_VP), _VP, _VP, _VP]),
    ("OptAMD_CsrTranspose", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, _VP, _VP, _VP, _VP, _VP,
                                           _VP, ctypes.c_int]),
    ("OptAMD_CsrATA", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, _VP, _VP, _VP, _VP, _VP, _VP,
                                     ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]),
    ("OptAMD_CsrSpMV", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_longlong, _VP, _VP, _VP, _VP, _VP,
                                      ctypes.c_int]),
    ("OptAMD_GenericSource", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_GenericDescribe", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]),
    ("OptAMD_GenericCompileCheck", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
]
EXPORTED_SYMBOLS = [s[0] for s in _SIGNATURES]


def load_library(path: str = None):
    """Load libopt_amd.so (OPT_AMD_LIB overrides the in-tree path, for A/B builds);
    raise if it is missing (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("OPT_AMD_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise OptError(
            f"{path} not found: build the HIP runtime first "
            "(python -c 'import __graft_entry__ as g; g.build()' or `make`)"
        )
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7, and whichever
    # copy is loaded first serves both (same soname). Load torch's first when it is
    # installed, so tensors allocated by torch and our kernels share one runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, res, args in _SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is None:
            if os.path.abspath(path) != os.path.abspath(LIB_PATH):
                continue   # an older A/B build (OPT_AMD_LIB) may predate an extension entry point
            raise OptError(f"{path} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _ptr(obj) -> int:
    """Address of a problem parameter: torch tensor, numpy array, ctypes object or int."""
    if obj is None:
        return 0
    if isinstance(obj, int):
        return obj
    if hasattr(obj, "data_ptr"):  # torch.Tensor
        return obj.data_ptr()
    if hasattr(obj, "ctypes"):  # numpy.ndarray
        return obj.ctypes.data
    return ctypes.addressof(obj)


class ParamPack:
    """The void** problemparams array; keeps scalar boxes alive."""

    def __init__(self, values: Sequence):
        self._keep = []
        self.arr = (ctypes.c_void_p * max(1, len(values)))()
        for i, v in enumerate(values):
            if isinstance(v, float):
                box = ctypes.c_float(v)
                self._keep.append(box)
                self.arr[i] = ctypes.addressof(box)
            elif isinstance(v, tuple) and len(v) == 2 and v[0] in ("int", "float", "double"):
                box = {"int": ctypes.c_int, "float": ctypes.c_float, "double": ctypes.c_double}[v[0]](v[1])
                self._keep.append(box)
                self.arr[i] = ctypes.addressof(box)
            else:
                self._keep.append(v)
                self.arr[i] = _ptr(v)

    @property
    def ptr(self):
        return ctypes.cast(self.arr, ctypes.POINTER(ctypes.c_void_p))


class OptSolver:
    """One Opt_State + Opt_Problem + Opt_Plan (reference OptSolver, OptSolver.h:46-84)."""

    def __init__(
        self,
        dims: Sequence[int],
        energy_file: str,
        solver_kind: str = "gaussNewtonGPU",
        double_precision: bool = False,
        backend: str = "backend_cuda",
        verbosity: int = 0,
        kernel_timing: bool = False,
        numthreads: int = 1,
        materialized: bool = False,
        fused_jtj: bool = False,
    ):
        self.lib = load_library()
        ip = InitParams()
        ip.doublePrecision = int(double_precision)
        ip.verbosityLevel = verbosity
        ip.collectPerKernelTimingInfo = int(kernel_timing)
        ip.backend = backend.encode()
        ip.numthreads = numthreads
        ip.useMaterializedJTJ = int(materialized)
        ip.useFusedJTJ = int(fused_jtj)
        self.state = self.lib.Opt_NewState(ip)
        if not self.state:
            raise OptError("Opt_NewState failed")
        self.problem = self.lib.Opt_ProblemDefine(self.state, energy_file.encode(), solver_kind.encode())
        if not self.problem:
            raise OptError(f"Opt_ProblemDefine failed for {energy_file}")
        self._dims = (ctypes.c_uint * len(dims))(*dims)
        self.plan = self.lib.Opt_ProblemPlan(self.state, self.problem, self._dims)
        if not self.plan:
            raise OptError("Opt_ProblemPlan failed")
        self.double_precision = double_precision

    # ---- reference API ---------------------------------------------------------
    def set_solver_params(self, params: Dict[str, object]):
        """setAllSolverParameters (OptUtils.h:108-112): ints for the iteration counts."""
        keep = []
        for name, v in params.items():
            box = ctypes.c_int(v) if isinstance(v, int) else ctypes.c_float(v)
            keep.append(box)
            self.lib.Opt_SetSolverParameter(self.state, self.plan, name.encode(), ctypes.addressof(box))

    def solve(self, problem_params: Sequence, solver_params: Optional[Dict[str, object]] = None) -> float:
        if solver_params:
            self.set_solver_params(solver_params)
        pk = ParamPack(problem_params)
        self.lib.Opt_ProblemSolve(self.state, self.plan, pk.ptr)
        return self.cost()

    def init(self, problem_params: Sequence):
        self._pk = ParamPack(problem_params)
        self.lib.Opt_ProblemInit(self.state, self.plan, self._pk.ptr)
        self._raise_plan_error()

    def step(self, problem_params: Optional[Sequence] = None) -> int:
        if problem_params is not None:
            self._pk = ParamPack(problem_params)
        r = self.lib.Opt_ProblemStep(self.state, self.plan, self._pk.ptr)
        self._raise_plan_error()
        return r

    def _raise_plan_error(self):
        """OptAMD_PlanError: a problem the plan met when the arrays were bound."""
        buf = ctypes.create_string_buffer(512)
        if self.lib.OptAMD_PlanError(self.plan, buf, 512) > 0:
            raise OptError(buf.value.decode())

    def profiled_solve(self, problem_params: Sequence) -> List[float]:
        """launchProfiledSolve (OptUtils.h:47-64): cost after Init and after each Step."""
        self.init(problem_params)
        costs = [self.cost()]
        while self.step():
            costs.append(self.cost())
        return costs

    def cost(self) -> float:
        return self.lib.Opt_ProblemCurrentCost(self.state, self.plan)

    # ---- extensions (include/opt_amd.h) ----------------------------------------
    def unknown_count(self) -> int:
        return self.lib.OptAMD_PlanUnknownCount(self.plan)

    def family(self) -> str:
        buf = ctypes.create_string_buffer(64)
        self.lib.OptAMD_PlanFamily(self.plan, buf, 64)
        return buf.value.decode()

    def eval_jtf(self, problem_params, r, pre) -> float:
        pk = ParamPack(problem_params)
        out = ctypes.c_double()
        if self.lib.OptAMD_EvalJTF(self.state, self.plan, pk.ptr, _ptr(r), _ptr(pre), ctypes.byref(out)):
            self._raise_plan_error()
            raise OptError("OptAMD_EvalJTF failed")
        return out.value

    def apply_jtj(self, problem_params, p, Ap) -> float:
        pk = ParamPack(problem_params)
        out = ctypes.c_double()
        if self.lib.OptAMD_ApplyJTJ(self.state, self.plan, pk.ptr, _ptr(p), _ptr(Ap), ctypes.byref(out)):
            self._raise_plan_error()
            raise OptError("OptAMD_ApplyJTJ failed")
        return out.value

    def eval_cost(self, problem_params) -> float:
        pk = ParamPack(problem_params)
        c = self.lib.OptAMD_EvalCost(self.state, self.plan, pk.ptr)
        if c == -1.0:   # a cost is >= 0: the call failed (OptAMD_PlanError holds why)
            self._raise_plan_error()
            raise OptError("OptAMD_EvalCost failed")
        return c

    def time_apply(self, problem_params, p, Ap, reps: int) -> float:
        pk = ParamPack(problem_params)
        return self.lib.OptAMD_TimeApplyJTJ(self.state, self.plan, pk.ptr, _ptr(p), _ptr(Ap), reps)

    def set_kernel_timing(self, mode: int):
        self.lib.OptAMD_SetKernelTiming(self.plan, mode)

    def kernel_stat(self, name: str):
        n = ctypes.c_longlong()
        ms = ctypes.c_double()
        ok = self.lib.OptAMD_KernelStat(self.plan, name.encode(), ctypes.byref(n), ctypes.byref(ms)) == 0
        return (n.value, ms.value) if ok else (0, 0.0)

    def apply_kernel_name(self) -> str:
        buf = ctypes.create_string_buffer(64)
        self.lib.OptAMD_ApplyKernelName(self.plan, buf, 64)
        return buf.value.decode()

    def kernel_report(self) -> str:
        buf = ctypes.create_string_buffer(1 << 16)
        self.lib.OptAMD_KernelReport(self.plan, buf, 1 << 16)
        return buf.value.decode()

    def stream(self) -> int:
        return self.lib.OptAMD_PlanStream(self.plan) or 0

    def iterations(self) -> int:
        return self.lib.OptAMD_PlanIterations(self.plan)

    def scalars(self, n: int = 256):
        """The plan's device scalar slots after the last call (OptAMD_PlanScalars)."""
        buf = (ctypes.c_double * n)()
        k = self.lib.OptAMD_PlanScalars(self.plan, buf, n)
        return list(buf)[: max(k, 0)]

    def halo(self) -> int:
        return self.lib.OptAMD_PlanHalo(self.plan)

    def set_decomposition(self, comm, y_lo: int, y_hi: int):
        """Own global rows [y_lo, y_hi) of a row-slab decomposition (include/opt_amd.h)."""
        if self.lib.OptAMD_PlanSetDecomposition(self.plan, comm, y_lo, y_hi):
            raise OptError("OptAMD_PlanSetDecomposition failed")

    def jacobian_shape(self):
        """(residual rows, nonzeros) of the materialized J; nnz = -1 if the family has none."""
        rows = ctypes.c_longlong()
        nnz = self.lib.OptAMD_PlanJacobianShape(self.plan, ctypes.byref(rows))
        return rows.value, nnz

    def materialized_nonzeros(self):
        """(nnz J, nnz J^T J) of a materialized plan, None for a matrix-free one."""
        a, b = ctypes.c_longlong(), ctypes.c_longlong()
        if self.lib.OptAMD_PlanMaterializedNonzeros(self.plan, ctypes.byref(a), ctypes.byref(b)):
            return None
        return a.value, b.value

    def eval_jacobian(self, problem_params, rowPtr, colInd, val):
        """J at the current unknowns into device arrays (rowPtr rows+1, colInd/val nnz)."""
        pk = ParamPack(problem_params)
        if self.lib.OptAMD_EvalJacobian(self.state, self.plan, pk.ptr, _ptr(rowPtr), _ptr(colInd), _ptr(val)):
            raise OptError("OptAMD_EvalJacobian failed")

    def close(self):
        if getattr(self, "plan", None):
            self.lib.Opt_PlanFree(self.state, self.plan)
            self.plan = None
        if getattr(self, "problem", None):
            self.lib.Opt_ProblemDelete(self.state, self.problem)
            self.problem = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- device CSR building blocks (include/opt_amd.h) ---------------------------------
def csr_transpose(rows, cols, rowPtr, colInd, val=None):
    """(rowPtrT, colIndT, valT) of a device CSR matrix given as torch tensors."""
    import torch

    lib = load_library()
    nnz = colInd.numel()
    rpT = torch.empty(cols + 1, dtype=torch.int32, device=rowPtr.device)
    ciT = torch.empty(max(nnz, 1), dtype=torch.int32, device=rowPtr.device)
    vT = torch.empty(max(nnz, 1), dtype=val.dtype, device=rowPtr.device) if val is not None else None
    dp = int(val is not None and val.dtype == torch.float64)
    if lib.OptAMD_CsrTranspose(rows, cols, nnz, _ptr(rowPtr), _ptr(colInd), _ptr(val), _ptr(rpT), _ptr(ciT),
                               _ptr(vT), dp):
        raise OptError("OptAMD_CsrTranspose failed")
    return rpT, ciT[:nnz], (vT[:nnz] if vT is not None else None)


def csr_ata(rows, cols, rowPtr, colInd, val):
    """(rowPtrATA, colIndATA, valATA) of A^T A for a device CSR matrix A."""
    import torch

    lib = load_library()
    nnz = colInd.numel()
    dp = int(val.dtype == torch.float64)
    rp = torch.empty(cols + 1, dtype=torch.int32, device=rowPtr.device)
    n = ctypes.c_longlong()
    args = (rows, cols, nnz, _ptr(rowPtr), _ptr(colInd), _ptr(val), _ptr(rp))
    if lib.OptAMD_CsrATA(*args, None, None, ctypes.byref(n), dp):
        raise OptError("OptAMD_CsrATA (pattern) failed")
    ci = torch.empty(max(n.value, 1), dtype=torch.int32, device=rowPtr.device)
    v = torch.empty(max(n.value, 1), dtype=val.dtype, device=rowPtr.device)
    if lib.OptAMD_CsrATA(*args, _ptr(ci), _ptr(v), ctypes.byref(n), dp):
        raise OptError("OptAMD_CsrATA failed")
    return rp, ci[: n.value], v[: n.value]


def csr_spmv(rows, cols, rowPtr, colInd, val, x):
    import torch

    lib = load_library()
    y = torch.empty(rows, dtype=val.dtype, device=x.device)
    dp = int(val.dtype == torch.float64)
    if lib.OptAMD_CsrSpMV(rows, cols, colInd.numel(), _ptr(rowPtr), _ptr(colInd), _ptr(val), _ptr(x), _ptr(y), dp):
        raise OptError("OptAMD_CsrSpMV failed")
    return y


# ---- general energy front end (no device needed) ----------------------------------
def _text_call(fn, *args, cap: int = 1 << 23):
    buf = ctypes.create_string_buffer(cap)
    r = fn(*args, buf, cap)
    return r, buf.value.decode(errors="replace")


def generic_source(energy_file: str, double: bool = False, off32: bool = False) -> str:
    """HIP source the front end generates for `energy_file` (OptAMD_GenericSource); off32:
    the 32-bit gather addressing plans take for arrays below 2 GiB."""
    r, txt = _text_call(load_library().OptAMD_GenericSource, energy_file.encode(), int(double) | (2 if off32 else 0))
    if r < 0:
        raise OptError(txt)
    return txt


def generic_describe(energy_file: str) -> List[str]:
    """Residual templates of `energy_file`: '<centred|graphK> <n unknowns> <expression>'."""
    r, txt = _text_call(load_library().OptAMD_GenericDescribe, energy_file.encode())
    if r < 0:
        raise OptError(txt)
    return txt.splitlines()


def generic_signature(energy_file: str) -> str:
    """Structural signature of the lowered energy (OptAMD_GenericSignature)."""
    r, txt = _text_call(load_library().OptAMD_GenericSignature, energy_file.encode())
    if r < 0:
        raise OptError(txt)
    return txt


def problem_family(energy_file: str, solver_kind: str = "gaussNewtonGPU") -> str:
    """Kernel family Opt_ProblemDefine picks for `energy_file` (OptAMD_ProblemFamily):
    a hand-written family only if the file lowers to exactly its residual templates."""
    lib = load_library()
    ip = InitParams()
    ip.backend = b"backend_cuda"
    st = lib.Opt_NewState(ip)
    pr = lib.Opt_ProblemDefine(st, energy_file.encode(), solver_kind.encode())
    if not pr:
        raise OptError(f"Opt_ProblemDefine refused {energy_file}")
    buf = ctypes.create_string_buffer(64)
    lib.OptAMD_ProblemFamily(pr, buf, 64)
    lib.Opt_ProblemDelete(st, pr)
    return buf.value.decode()


def generic_compile_check(energy_file: str, double: bool = False) -> None:
    """Compile the generated source for gfx950 with hiprtc; raise with the log on error."""
    r, txt = _text_call(load_library().OptAMD_GenericCompileCheck, energy_file.encode(), int(double))
    if r != 0:
        raise OptError(txt)
