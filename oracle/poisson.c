/*
 * oracle/poisson.c — CPU restatement of the reference's poisson_image_editing solver.
 * TEST INFRASTRUCTURE ONLY (oracle/README.md). PARITY UNPINNED for this energy: the
 * reference's end-to-end test value (test_final_cost.py:63) comes from a harness run
 * that reads its mask out of bounds (examples/poisson_image_editing/src/main.cpp:95-101
 * at the test's stride 4), so it cannot be reproduced; checked against an independent
 * float64 restatement + finite differences (tests/test_oracle_poisson.py) and, through
 * the shared generic loop (solver_impl.h), by the pinned image_warping / optical_flow
 * solves.
 *
 * Energy: examples/poisson_image_editing/poisson_image_editing.t — X float4 unknown,
 * T float4, M mask; Exclude(M != 0); UsePreconditioner(false);
 *   e(k,s) = Select(InBounds(s), (X_k - X_{k+s}) - (T_k - T_{k+s}), 0), s in 4-neighbours.
 * Gathers follow o.t:2770-2830 (J^T J p) and 2870-2913 (J^T F, diag) literally:
 * per unknown X_c(k), residual instances centred at k (dr/dX = +1) and at k - s
 * (dr/dX = -1); excluded neighbours keep their X (Dirichlet) and have p = 0.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "solver.h"

static const int PX[4] = {1, -1, 0, 0};
static const int PY[4] = {0, 0, 1, -1};

#define REAL float
#define OACC double
#include "pie_impl.h"
#undef REAL
#undef OACC
#define OACC long double
#define REAL double
#include "pie_impl.h"
#undef REAL

/* the float instantiation under the names the rest of this file uses */
typedef pie_ctx_float pie_ctx;
#define pin pin_float
#define pact pact_float
#define pie_cost_fn pie_cost_fn_float
#define pie_jtf_fn pie_jtf_fn_float
#define pie_apply_fn pie_apply_fn_float
#define pie_model_fn pie_model_fn_float
#define pie_update_fn pie_update_fn_float
#define pie_save_fn pie_save_fn_float
#define pie_revert_fn pie_revert_fn_float

/* ------------------------------------------------------------- public API ---- */
double oracle_pie_cost(int W, int H, float* X, const float* T, const float* M) {
    pie_ctx c = {W, H, X, T, M, NULL};
    return pie_cost_fn(&c);
}
void oracle_pie_jtf(int W, int H, float* X, const float* T, const float* M, float* r, float* diag) {
    pie_ctx c = {W, H, X, T, M, NULL};
    pie_jtf_fn(&c, r, diag);
}
double oracle_pie_apply(int W, int H, float* X, const float* T, const float* M, const float* p, float* Ap) {
    pie_ctx c = {W, H, X, T, M, NULL};
    return pie_apply_fn(&c, p, Ap);
}
/* GN (lm = 0) or LM solve, X updated in place; returns completed steps. */
int oracle_pie_solve(int W, int H, float* X, const float* T, const float* M, int lm, int nIter, int lIter,
                     double* costs) {
    pie_ctx c = {W, H, X, T, M, NULL};
    const long long n = 4LL * W * H;
    unsigned char* act = malloc(n);
    for (long long e = 0; e < n; ++e) act[e] = M[e / 4] == 0.f;
    c.prev = malloc(sizeof(float) * n);
    oracle_problem_float P = {n, act, 0, &c, pie_cost_fn, pie_jtf_fn, pie_apply_fn, pie_model_fn,
                              pie_update_fn, pie_save_fn, pie_revert_fn};
    oracle_params sp = oracle_default_params();
    sp.nIterations = nIter;
    sp.lIterations = lIter;
    const int k = oracle_solve_f32(&P, lm, &sp, costs);
    free(act);
    free(c.prev);
    return k;
}

/* opt_float = double: X and the solver in double, T / M float */
double oracle_pie_cost_double(int W, int H, double* X, const float* T, const float* M) {
    pie_ctx_double c = {W, H, X, T, M, NULL};
    return pie_cost_fn_double(&c);
}
void oracle_pie_jtf_double(int W, int H, double* X, const float* T, const float* M, double* r, double* diag) {
    pie_ctx_double c = {W, H, X, T, M, NULL};
    pie_jtf_fn_double(&c, r, diag);
}
double oracle_pie_apply_double(int W, int H, double* X, const float* T, const float* M, const double* p,
                               double* Ap) {
    pie_ctx_double c = {W, H, X, T, M, NULL};
    return pie_apply_fn_double(&c, p, Ap);
}
int oracle_pie_solve_double(int W, int H, double* X, const float* T, const float* M, int lm, int nIter, int lIter,
                            double* costs) {
    pie_ctx_double c = {W, H, X, T, M, NULL};
    const long long n = 4LL * W * H;
    unsigned char* act = malloc(n);
    for (long long e = 0; e < n; ++e) act[e] = M[e / 4] == 0.f;
    c.prev = malloc(sizeof(double) * n);
    oracle_problem_double P = {n, act, 0, &c, pie_cost_fn_double, pie_jtf_fn_double, pie_apply_fn_double,
                               pie_model_fn_double, pie_update_fn_double, pie_save_fn_double, pie_revert_fn_double};
    oracle_params sp = oracle_default_params();
    sp.nIterations = nIter;
    sp.lIterations = lIter;
    const int k = oracle_solve_f64(&P, lm, &sp, costs);
    free(act);
    free(c.prev);
    return k;
}

/* ------------------------------------------- materialized Jacobian (oracle/csr.c) ---- */
/* saveJToCRS / generateDumpJ (solverGPUGaussNewton.t:385-442, 1004-1022): pixel k owns
 * rows 16k + 4s + ch, each {X_ch(k): b, X_ch(k+s): -b}, b = InBounds(k+s), columns
 * wrapped into [0, 4N) (:365-381) and sorted (sortCol). */
#include "csr.h"
static void pie_dump(void* v, int* rowPtr, int* colInd, float* val) {
    const pie_ctx* c = (const pie_ctx*)v;
    const long long N = (long long)c->W * c->H, n = 4 * N;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            for (int s = 0; s < 4; ++s) {
                const int in = pin(c, x + PX[s], y + PY[s]);
                const long long tn = k + PX[s] + (long long)PY[s] * c->W;
                for (int ch = 0; ch < 4; ++ch) {
                    const long long row = 16 * k + 4 * s + ch, nz = 2 * row;
                    long long c0 = 4 * k + ch, c1 = 4 * tn + ch;
                    c1 = c1 < 0 ? c1 + n : (c1 >= n ? c1 - n : c1);
                    float v0 = in ? 1.f : 0.f, v1 = in ? -1.f : 0.f;
                    if (c1 < c0) { long long t = c0; c0 = c1; c1 = t; float tv = v0; v0 = v1; v1 = tv; }
                    rowPtr[row] = (int)nz;
                    colInd[nz] = (int)c0; val[nz] = v0;
                    colInd[nz + 1] = (int)c1; val[nz + 1] = v1;
                }
            }
        }
    rowPtr[16 * N] = (int)(32 * N);
}
void oracle_pie_dump_j(int W, int H, float* X, const float* T, const float* M, int* rowPtr, int* colInd, float* val) {
    pie_ctx c = {W, H, X, T, M, NULL};
    pie_dump(&c, rowPtr, colInd, val);
}
typedef struct { pie_ctx c; oracle_mat m; } piem_ctx;
static void piem_materialize(void* v) { oracle_mat_build(&((piem_ctx*)v)->m); }
static double piem_apply(void* v, const float* p, float* Ap) { return oracle_mat_apply(&((piem_ctx*)v)->m, p, Ap); }
int oracle_pie_solve_materialized(int W, int H, float* X, const float* T, const float* M, int lm, int fused, int nIter,
                                  int lIter, double* costs) {
    piem_ctx c = {{W, H, X, T, M, NULL}};
    const long long n = 4LL * W * H;
    unsigned char* act = malloc(n);
    for (long long e = 0; e < n; ++e) act[e] = M[e / 4] == 0.f;
    c.c.prev = malloc(sizeof(float) * n);
    oracle_mat_init(&c.m, 16LL * W * H, 32LL * W * H, (int)n, fused, act, pie_dump, &c.c);
    oracle_problem_float P = {n, act, 0, &c, pie_cost_fn, pie_jtf_fn, pie_apply_fn, pie_model_fn,
                              pie_update_fn, pie_save_fn, pie_revert_fn, piem_materialize, piem_apply};
    oracle_params sp = oracle_default_params();
    sp.nIterations = nIter;
    sp.lIterations = lIter;
    const int k = oracle_solve_f32(&P, lm, &sp, costs);
    oracle_mat_free(&c.m);
    free(act);
    free(c.c.prev);
    return k;
}
double oracle_pie_apply_materialized(int W, int H, float* X, const float* T, const float* M, int fused,
                                     const float* p, float* Ap) {
    piem_ctx c = {{W, H, X, T, M, NULL}};
    const long long n = 4LL * W * H;
    unsigned char* act = malloc(n);
    for (long long e = 0; e < n; ++e) act[e] = M[e / 4] == 0.f;
    oracle_mat_init(&c.m, 16LL * W * H, 32LL * W * H, (int)n, fused, act, pie_dump, &c.c);
    oracle_mat_build(&c.m);
    const double d = oracle_mat_apply(&c.m, p, Ap);
    oracle_mat_free(&c.m);
    free(act);
    return d;
}
