/*
 * oracle/arap.c — CPU restatement of the reference's arap_mesh_deformation solver, for
 * opt_float = float and double (the body is oracle/arap_impl.h).
 * TEST INFRASTRUCTURE ONLY (oracle/README.md). PINNED to the reference's own output:
 * its end-to-end test's CUDA final cost for the small_armadillo example
 * (examples/test_final_cost.py:55-66, 7183.464843) is reproduced within 1.2e-7
 * (tests/test_reference_costs.py); also checked against an independent float64 numpy
 * restatement with finite differences (tests/test_oracle_arap.py).
 *
 * Energy examples/arap_mesh_deformation/arap_mesh_deformation.t:
 *   unknowns Offset, Angle (float3 per vertex); knowns UrShape, Constraints (float3);
 *   graph G (edges v0 -> v1, int32); UsePreconditioner(true)
 *   e_fit(v) = Constraints(v).x >= -999999.9 ? w_fit (Offset(v) - Constraints(v)) : 0
 *   e_reg(e) = w_reg ((Offset(v0) - Offset(v1)) - Rotate3D(Angle(v0), UrShape(v0) - UrShape(v1)))
 * Rotate3D / Matrix3x3Mul: API/src/lib.t:46-98.
 * The fit term is a centred function over vertices (PCGInit1 / PCGStep1 / computeCost,
 * solverGPUGaussNewton.t:521-632, 971-997); the regulariser a graph function whose
 * J^T F, diag, J^T J p and cost are scattered per edge (createjtfgraph o.t:2969-2994,
 * createjtjgraph o.t:2833-2867, PCGInit1_Graph / PCGInit1_Finish / PCGStep1_Graph
 * solverGPUGaussNewton.t:570-602, 1188-1233). Here the edge scatters run sequentially
 * in edge order (the reference's float atomics have no fixed order).
 * Vector layout [Offset.xyz * N | Angle.xyz * N].
 */
#include <tgmath.h>
#include <stdlib.h>
#include <string.h>
#include "solver.h"

#define REAL float
#define OACC double
#include "arap_impl.h"
#undef REAL
#undef OACC
#define OACC long double
#define REAL double
#include "arap_impl.h"
#undef REAL

/* ------------------------------------------------------------- public API ---- */
/* float entry points: oracle_arap_*; double (unknowns and solver vectors in double,
 * known arrays float): oracle_arap_*_double */
#define ARAP_API(R, SUF, SOLVE)                                                                                \
    double oracle_arap_cost##SUF(int N, int E, R* O, R* A, const float* U, const float* C, const int* v0,       \
                                 const int* v1, float wf, float wr) {                                           \
        arap_ctx_##R c = {N, E, O, A, U, C, v0, v1, wf, wr, NULL, NULL};                                        \
        return arap_cost_fn_##R(&c);                                                                            \
    }                                                                                                           \
    void oracle_arap_jtf##SUF(int N, int E, R* O, R* A, const float* U, const float* C, const int* v0,          \
                              const int* v1, float wf, float wr, R* r, R* diag) {                               \
        arap_ctx_##R c = {N, E, O, A, U, C, v0, v1, wf, wr, NULL, NULL};                                        \
        arap_jtf_fn_##R(&c, r, diag);                                                                           \
    }                                                                                                           \
    double oracle_arap_apply##SUF(int N, int E, R* O, R* A, const float* U, const float* C, const int* v0,      \
                                  const int* v1, float wf, float wr, const R* p, R* Ap) {                       \
        arap_ctx_##R c = {N, E, O, A, U, C, v0, v1, wf, wr, NULL, NULL};                                        \
        return arap_apply_fn_##R(&c, p, Ap);                                                                    \
    }                                                                                                           \
    double oracle_arap_model_cost##SUF(int N, int E, R* O, R* A, const float* U, const float* C,               \
                                       const int* v0, const int* v1, float wf, float wr, const R* d) {          \
        arap_ctx_##R c = {N, E, O, A, U, C, v0, v1, wf, wr, NULL, NULL};                                        \
        return arap_model_fn_##R(&c, d);                                                                        \
    }                                                                                                           \
    int oracle_arap_solve##SUF(int N, int E, R* O, R* A, const float* U, const float* C, const int* v0,         \
                               const int* v1, float wf, float wr, int lm, int nIter, int lIter, double* costs) { \
        arap_ctx_##R c = {N, E, O, A, U, C, v0, v1, wf, wr, NULL, NULL};                                        \
        c.prevO = malloc(sizeof(R) * 3 * N);                                                                    \
        c.prevA = malloc(sizeof(R) * 3 * N);                                                                    \
        unsigned char* act = malloc(6 * (size_t)N);                                                             \
        memset(act, 1, 6 * (size_t)N);                                                                          \
        oracle_problem_##R P = {6LL * N, act, 1, &c, arap_cost_fn_##R, arap_jtf_fn_##R, arap_apply_fn_##R,      \
                                arap_model_fn_##R, arap_update_fn_##R, arap_save_fn_##R, arap_revert_fn_##R};   \
        oracle_params sp = oracle_default_params();                                                             \
        sp.nIterations = nIter;                                                                                 \
        sp.lIterations = lIter;                                                                                 \
        const int k = SOLVE(&P, lm, &sp, costs);                                                                \
        free(act); free(c.prevO); free(c.prevA);                                                                \
        return k;                                                                                               \
    }

ARAP_API(float, , oracle_solve_f32)
ARAP_API(double, _double, oracle_solve_f64)
