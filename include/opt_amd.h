/*
 * opt_amd.h — extension entry points of libopt_amd.so beyond the reference ABI.
 *
 * The reference exposes its solver only through Opt.h; its kernels are reachable
 * only from inside the generated step() (solverGPUGaussNewton.t:1913-2349). These
 * entry points expose the same kernels one at a time so the parity tests and the
 * benchmark can drive and time them without a full solve. Each cites the reference
 * kernel whose per-unknown result it returns. All pointers are device pointers into
 * the plan's unknown-vector layout: one contiguous block per unknown image in
 * declaration order, channels interleaved inside an image (reference UnknownType,
 * API/src/o.t:998-1100; e.g. image_warping = [Offset.xy * N | Angle * N]).
 * Element type is float, or double when the state was created with doublePrecision.
 * All calls are synchronous (they return after the device work completed).
 * Return value 0 = success, nonzero = invalid arguments (message on stderr).
 */
#pragma once
#include "Opt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Total number of scalar unknowns of the plan (e.g. 3*W*H for image_warping). */
long long OptAMD_PlanUnknownCount(Opt_Plan* plan);

/* Energy family the problem was lowered to ("image_warping", "poisson_image_editing",
 * ...); writes a NUL-terminated name into buf. Returns the name length. */
int OptAMD_PlanFamily(Opt_Plan* plan, char* buf, int buflen);

/* Kernel family Opt_ProblemDefine chose for the energy file: a hand-written family
 * only when the file lowers to exactly that family's residual templates, else
 * "generic" (kernels generated from the file at plan time). No device needed. */
int OptAMD_ProblemFamily(Opt_Problem* problem, char* buf, int buflen);

/* Structural signature of an energy file as the front end lowers it (declaration
 * kinds/types/indices, ComputedArray, Exclude and residual templates; names dropped):
 * two files with equal signatures define the same problem. Returns the length, or -1
 * with the error message in buf. No device needed. */
int OptAMD_GenericSignature(const char* filename, char* buf, int buflen);

/* r = -J^T F and the CERES-guarded Jacobi preconditioner pre = 1/(1+sqrt(diag J^TJ))^2
 * (or the reference's forced value when UsePreconditioner(false)) at the current
 * unknowns; *r_dot_pre_r = sum r.(pre*r) (reference kernels.PCGInit1,
 * solverGPUGaussNewton.t:521-563, with fmap.evalJTF o.t:2870-2913). Excluded
 * elements get r = 0, pre = 0. */
int OptAMD_EvalJTF(Opt_State* state, Opt_Plan* plan, void** problemparams,
                   void* r, void* pre, double* r_dot_pre_r);

/* Ap = J^T J p at the current unknowns (+ CtC*p for LM plans, with the CtC of the
 * last LM step) and *p_dot_Ap = p.Ap (reference kernels.PCGStep1,
 * solverGPUGaussNewton.t:607-632, with fmap.applyJTJ o.t:2770-2830). Excluded
 * elements get Ap = 0. */
int OptAMD_ApplyJTJ(Opt_State* state, Opt_Plan* plan, void** problemparams,
                    const void* p, void* Ap, double* p_dot_Ap);

/* Energy 1/2 sum r^2 at the current unknowns (reference kernels.computeCost,
 * solverGPUGaussNewton.t:971-997, fmap.cost o.t:3119-3129). */
double OptAMD_EvalCost(Opt_State* state, Opt_Plan* plan, void** problemparams);

/* Launch the apply `reps` times back to back on the plan's stream, bracketed by
 * hipEvents; returns the mean device time per launch in microseconds. */
double OptAMD_TimeApplyJTJ(Opt_State* state, Opt_Plan* plan, void** problemparams,
                           const void* p, void* Ap, int reps);

/* Per-kernel device-time accounting (hipEvent pairs on the plan's stream).
 * mode 0: off; 1: every kernel (the reference's collectPerKernelTimingInfo);
 * 2: only the PCG J^T J p apply kernel. Resets the accumulated statistics. */
void OptAMD_SetKernelTiming(Opt_Plan* plan, int mode);

/* Accumulated statistics for kernel `name` since the last reset: number of launches
 * and total device milliseconds. Returns 0 if the kernel was seen, 1 otherwise. */
int OptAMD_KernelStat(Opt_Plan* plan, const char* name, long long* launches, double* total_ms);

/* Name of the plan's dominant (PCG apply) kernel as it appears in KernelStat and in
 * rocprofv3 kernel traces. */
int OptAMD_ApplyKernelName(Opt_Plan* plan, char* buf, int buflen);

/* Human-readable table of every timed kernel (reference timer report,
 * backend_cuda.t:231-297). Returns the length written. */
int OptAMD_KernelReport(Opt_Plan* plan, char* buf, int buflen);

/* The HIP stream (hipStream_t) all of the plan's device work is issued on. */
void* OptAMD_PlanStream(Opt_Plan* plan);

/* Outer iterations completed since the last Init. */
int OptAMD_PlanIterations(Opt_Plan* plan);

/* Copy up to n of the plan's device scalar slots (fp64: costs, the PCG rz / pAp sums of
 * the last Step, ...) to `out` after synchronising; returns the number copied. The slot
 * layout is the family's (image_warping: opt_amd/csrc/image_warping.hip, kScBase /
 * kSlots); a parity/diagnostic hook with no reference counterpart. */
int OptAMD_PlanScalars(Opt_Plan* plan, double* out, int n);

/* ---- multi-GPU row-slab decomposition (no reference counterpart:
 * the reference is single-device, §2.3) ------------------------------------------ */
typedef struct OptAMD_Comm OptAMD_Comm;
typedef struct OptAMD_LocalGroup OptAMD_LocalGroup;

/* 128-byte RCCL unique id, created on one rank and shared with the others by the
 * caller (e.g. torch.distributed broadcast). Returns 0 on success. */
int OptAMD_RcclUniqueId(void* out128);
/* RCCL communicator over `nranks` processes, one GPU each (the current HIP device). */
OptAMD_Comm* OptAMD_CommCreateRccl(const void* id128, int rank, int nranks);
void OptAMD_CommDestroy(OptAMD_Comm* comm);
/* Number of ranks / this rank of a communicator (-1 for NULL): bench.py reports the
 * world size the solver actually runs on from here, not from the launcher's env. */
int OptAMD_CommSize(OptAMD_Comm* comm);
int OptAMD_CommRank(OptAMD_Comm* comm);
/* The transport behind a communicator, "rccl" or "local", copied into buf (at most
 * buflen bytes incl. the terminator); returns its length, -1 for NULL. */
int OptAMD_CommKind(OptAMD_Comm* comm, char* buf, int buflen);
/* The error that stopped the last Init / Step of this plan (a problem found only when
 * the arrays were bound, e.g. an arap graph whose adjacency exceeds 2^31 slots), copied
 * into buf; returns its length, 0 when there was none (-1 for NULL). After such an
 * error Opt_ProblemStep returns 0 and Opt_ProblemCurrentCost NaN; the process goes on. */
int OptAMD_PlanError(Opt_Plan* plan, char* buf, int buflen);
/* All ranks as threads of one process (shared device or peer devices): for testing
 * the decomposition on one GPU. The rank handles belong to the group. */
OptAMD_LocalGroup* OptAMD_LocalGroupCreate(int nranks);
OptAMD_Comm* OptAMD_LocalGroupRank(OptAMD_LocalGroup* group, int rank);
void OptAMD_LocalGroupDestroy(OptAMD_LocalGroup* group);

/* Stencil radius of the plan's energy (rows of neighbour data a slab needs). */
int OptAMD_PlanHalo(Opt_Plan* plan);
/* Make this plan one rank of a row-slab decomposition of the dims given to
 * Opt_ProblemPlan: it owns global rows [y_lo, y_hi). From then on every array in
 * problemparams (and every vector passed to the OptAMD_ kernels) holds rows
 * [y_lo - hl, y_hi + hh) with hl = min(halo, y_lo), hh = min(halo, H - y_hi); the
 * caller fills the known arrays' halo rows, the plan refreshes the unknowns' halo rows
 * itself. Energies, costs and dot products are global (summed over ranks).
 * Returns 0 on success. */
int OptAMD_PlanSetDecomposition(Opt_Plan* plan, OptAMD_Comm* comm, int y_lo, int y_hi);

/* ---- materialized Jacobian path (useMaterializedJTJ / useFusedJTJ, Opt.h) --------
 * Every array is a device pointer; CSR is zero-based with int32 indices (nnz < 2^31);
 * values are float, or double when doublePrecision is nonzero. Synchronous. */

/* Shape of the plan's assembled Jacobian: returns its nonzero count and stores the
 * residual (row) count in *nResiduals; -1 when the energy family has no J assembly. */
long long OptAMD_PlanJacobianShape(Opt_Plan* plan, long long* nResiduals);

/* Nonzeros of the J and (fused) J^T J a materialized plan holds (the J^T J count is
 * known after the first Step, 0 before and for useFusedJTJ = 0). Returns 1 for a
 * matrix-free plan. */
int OptAMD_PlanMaterializedNonzeros(Opt_Plan* plan, long long* nnzJ, long long* nnzJTJ);

/* J at the current unknowns (reference kernels.saveJToCRS, solverGPUGaussNewton.t:
 * 1004-1022, rows/columns as generateDumpJ :385-442: one block of rows per pixel,
 * columns = unknown indices wrapped into [0, nUnknowns) and sorted inside each row).
 * rowPtr: nResiduals+1, colInd / val: nnz. Returns 0 on success. */
int OptAMD_EvalJacobian(Opt_State* state, Opt_Plan* plan, void** problemparams,
                        int* rowPtr, int* colInd, void* val);

/* A^T of an nRowsA x nColsA matrix: rowPtrAT (nColsA+1), colIndAT and valAT (nnz), the
 * rows of A ascending inside each row of A^T (reference computeNnzPatternAT + computeAT,
 * API/src/linalg_cpu.t:203-297,512-551; cusparseScsr2csc, API/src/backend_cuda.t:600-612).
 * valA / valAT may be NULL (pattern only). */
int OptAMD_CsrTranspose(int nRowsA, int nColsA, long long nnz, const int* rowPtrA,
                        const int* colIndA, const void* valA, int* rowPtrAT, int* colIndAT,
                        void* valAT, int doublePrecision);

/* A^T A (nColsA x nColsA) of A with sorted columns in every row. First call with
 * colIndATA = valATA = NULL: fills rowPtrATA (nColsA+1) and *nnzATA; second call with
 * those arrays allocated: sorted column indices and the values, each summed over the
 * rows of A in ascending order (reference computeNnzPatternATA + computeATA,
 * API/src/linalg_cpu.t:300-508; cusparseXcsrgemmNnz / cusparseScsrgemm,
 * API/src/backend_cuda.t:556-596). Nonzero return: more than 2^31 nonzeros. */
int OptAMD_CsrATA(int nRowsA, int nColsA, long long nnz, const int* rowPtrA, const int* colIndA,
                  const void* valA, int* rowPtrATA, int* colIndATA, void* valATA,
                  long long* nnzATA, int doublePrecision);

/* y = A x (reference applyAtoVector, API/src/linalg_cpu.t:560-600; cusparseScsrmv,
 * API/src/backend_cuda.t:616-636). */
int OptAMD_CsrSpMV(int nRowsA, int nColsA, long long nnz, const int* rowPtrA, const int* colIndA,
                   const void* valA, const void* x, void* y, int doublePrecision);

/* General energy front end (the reference's energy compiler, API/src/o.t:1295-1348 and
 * 2669-3235): the HIP source generated for the energy file `filename` (float kernels, or
 * double with bit 0 of doublePrecision set; bit 1 selects the 32-bit gather addressing a
 * plan takes when its arrays are below 2 GiB), copied into buf (NUL-terminated, truncated
 * to n). Returns the full length, or -1 with the front end's message in buf. No device
 * needed. */
int OptAMD_GenericSource(const char* filename, int doublePrecision, char* buf, int n);

/* The residual templates the front end lowered `filename` to, one line each:
 * "<centred|graphK> <number of unknowns it reads> <expression>" (the reference's
 * toenergyspecs / classifyexpression result, API/src/o.t:2669-2715). Returns the residual
 * count, or -1 with the front end's message in buf. */
int OptAMD_GenericDescribe(const char* filename, char* buf, int n);

/* Compile that source for gfx950 with hiprtc (no device needed). 0 on success, -1 with
 * the compiler log (or the front end's message) in buf. */
int OptAMD_GenericCompileCheck(const char* filename, int doublePrecision, char* buf, int n);

#ifdef __cplusplus
}
#endif
