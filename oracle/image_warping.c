/*
 * oracle/image_warping.c — CPU restatement of the reference's image_warping solver.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline; libopt_amd never calls it.
 *
 * PINNED to the reference's own output: the reference's end-to-end test
 * (examples/test_final_cost.py:55-66) holds the CUDA final cost of the cat512 example at
 * nIterations = lIterations = 1, 1774.3405; this restatement reproduces it within 5e-8
 * (tests/test_reference_costs.py), and so do the generic loop and the materialized
 * J^T J / J^T (J p) paths. Also checked by finite differences of the cost against
 * J^T F, of J^T F against J^T J, and the symmetry of J^T J (tests/test_oracle.py).
 *
 * What is restated (all float arithmetic, as opt_float = float: API/src/config.t:3-5):
 *   energy      examples/image_warping/image_warping.t:12-108
 *   residual    classification + automatic bbox select  API/src/o.t:2669-2710
 *   J^T J p     gather over residual instances touching x00  o.t:2770-2830
 *   J^T F, diag                                         o.t:2870-2913
 *   cost        1/2 sum r^2                              o.t:3119-3129
 *   PCG/GN      PCGInit1 :521-563, PCGStep1 :607-632, PCGStep2 :665-731,
 *               PCGStep3 :814-845, PCGLinearUpdate :854-859, step() :1913-2349
 *               (file solverGPUGaussNewton.t), guardedInvert CERES :478-507
 *   CPU-MT      outer-dimension slab split + per-thread partial sums
 *               (API/src/backend_cpu_mt.t:716-737, 350-414)
 * Dot products are accumulated in double (the reference uses float atomics whose
 * order is nondeterministic; double is the tighter restatement of the exact sum).
 *
 * opt_float = double (doublePrecision, API/release/include/Opt.h:11-14): the same body
 * (oracle/iw_impl.h) instantiated for REAL = double — unknowns, solver vectors and
 * parameters in double, known arrays float — behind the oracle_iw_*_double entry points.
 * PARITY of the double form is pinned by the float form's pins only through the shared
 * body; tests/test_oracle.py checks it against central differences of its own cost and
 * against the float form on well-conditioned problems.
 *
 * Vector layout (reference UnknownType, o.t:998-1100): [Offset.xy * N | Angle * N].
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "solver.h"

static const int SX[4] = {1, -1, 0, 0};
static const int SY[4] = {0, 0, 1, -1};

#define REAL float
#define OACC double
#define RCOS cosf
#define RSIN sinf
#define RSQRT sqrtf
#define SOLVE_FN oracle_solve_f32
#include "iw_impl.h"
#undef REAL
#undef RCOS
#undef RSIN
#undef RSQRT
#undef SOLVE_FN
#undef OACC
#define OACC long double
#define REAL double
#define RCOS cos
#define RSIN sin
#define RSQRT sqrt
#define SOLVE_FN oracle_solve_f64
#include "iw_impl.h"
#undef REAL
#undef RCOS
#undef RSIN
#undef RSQRT
#undef SOLVE_FN

/* the float instantiation under the names the rest of this file uses */
typedef iw_problem_float iw_problem;
typedef reg_res_float reg_res;
typedef iw_ctx_float iw_ctx;
#define excluded excluded_float
#define reg_residual reg_residual_float
#define fit_valid fit_valid_float
#define run_slabs run_slabs_float
#define w_cost w_cost_float
#define w_jtf w_jtf_float
#define w_apply w_apply_float
#define iwg_cost iwg_cost_float
#define iwg_jtf iwg_jtf_float
#define iwg_apply iwg_apply_float
#define iwg_model iwg_model_float
#define iwg_update iwg_update_float
#define iwg_save iwg_save_float
#define iwg_revert iwg_revert_float

/* ------------------------------------------------------------- public API ---- */
#define PROB iw_problem P = {W, H, O, A, U, C, M, wf, wr}

double oracle_iw_cost(int W, int H, const float* O, const float* A, const float* U, const float* C,
                      const float* M, float wf, float wr, int nthreads) {
    PROB;
    return run_slabs(&P, nthreads, w_cost, NULL, NULL, NULL);
}

double oracle_iw_eval_jtf(int W, int H, const float* O, const float* A, const float* U, const float* C,
                          const float* M, float wf, float wr, float* r, float* pre, int nthreads) {
    PROB;
    return run_slabs(&P, nthreads, w_jtf, NULL, r, pre);
}

double oracle_iw_apply_jtj(int W, int H, const float* O, const float* A, const float* U, const float* C,
                           const float* M, float wf, float wr, const float* p, float* Ap, int nthreads) {
    PROB;
    return run_slabs(&P, nthreads, w_apply, p, Ap, NULL);
}

/* Full GN solve in the reference's kernel order. O and A are updated in place;
 * costs[0] = initial cost, costs[i] = cost after GN iteration i (nIter+1 entries).
 * If scalars != NULL it receives, per GN iteration, 3*lIter values
 * (alpha_num, alpha_den, beta_num) of each PCG iteration. */
void oracle_iw_solve(int W, int H, float* O, float* A, const float* U, const float* C, const float* M,
                     float wf, float wr, int nIter, int lIter, int nthreads, double* costs,
                     double* scalars) {
    iw_solve_float(W, H, O, A, U, C, M, wf, wr, nIter, lIter, nthreads, costs, scalars);
}

/* ---- opt_float = double: unknowns O, A and the solver in double, known arrays float,
 * the weights widened from the float parameters the runtime passes ---- */
#define PROBD iw_problem_double P = {W, H, O, A, U, C, M, (double)wf, (double)wr}
double oracle_iw_cost_double(int W, int H, const double* O, const double* A, const float* U, const float* C,
                             const float* M, float wf, float wr, int nthreads) {
    PROBD;
    return run_slabs_double(&P, nthreads, w_cost_double, NULL, NULL, NULL);
}
double oracle_iw_eval_jtf_double(int W, int H, const double* O, const double* A, const float* U, const float* C,
                                 const float* M, float wf, float wr, double* r, double* pre, int nthreads) {
    PROBD;
    return run_slabs_double(&P, nthreads, w_jtf_double, NULL, r, pre);
}
double oracle_iw_apply_jtj_double(int W, int H, const double* O, const double* A, const float* U, const float* C,
                                  const float* M, float wf, float wr, const double* p, double* Ap, int nthreads) {
    PROBD;
    return run_slabs_double(&P, nthreads, w_apply_double, p, Ap, NULL);
}
void oracle_iw_solve_double(int W, int H, double* O, double* A, const float* U, const float* C, const float* M,
                            float wf, float wr, int nIter, int lIter, int nthreads, double* costs,
                            double* scalars) {
    iw_solve_double(W, H, O, A, U, C, M, (double)wf, (double)wr, nIter, lIter, nthreads, costs, scalars);
}
int oracle_iw_solve_generic_double(int W, int H, double* O, double* A, const float* U, const float* C,
                                   const float* M, float wf, float wr, int lm, int nIter, int lIter, int nthreads,
                                   double* costs) {
    return iw_solve_generic_double(W, H, O, A, U, C, M, (double)wf, (double)wr, lm, nIter, lIter, nthreads, costs);
}
double oracle_iw_model_cost_double(int W, int H, const double* O, const double* A, const float* U, const float* C,
                                   const float* M, float wf, float wr, const double* d) {
    iw_ctx_double c = {{W, H, O, A, U, C, M, (double)wf, (double)wr}, (double*)O, (double*)A, NULL, NULL, 1};
    return iwg_model_double(&c, d);
}
void oracle_iw_jtf_diag_double(int W, int H, const double* O, const double* A, const float* U, const float* C,
                               const float* M, float wf, float wr, double* r, double* diag) {
    iw_ctx_double c = {{W, H, O, A, U, C, M, (double)wf, (double)wr}, (double*)O, (double*)A, NULL, NULL, 1};
    iwg_jtf_double(&c, r, diag);
}

/* All residual values, 10 per pixel in template order: for s in (+x,-x,+y,-y) the two
 * components of e_reg, then the two components of e_fit. Residuals of excluded
 * pixels are 0 (their kernels never run; computeCost skips them, :971-997). */
void oracle_iw_residuals(int W, int H, const float* O, const float* A, const float* U, const float* C,
                         const float* M, float wf, float wr, float* res) {
    PROB;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int k = y * W + x;
            float* o = res + (size_t)10 * k;
            for (int j = 0; j < 10; ++j) o[j] = 0.f;
            if (excluded(&P, x, y)) continue;
            for (int s = 0; s < 4; ++s)
                for (int c = 0; c < 2; ++c) {
                    reg_res r = reg_residual(&P, x, y, s, c);
                    o[2 * s + c] = r.valid ? r.value : 0.f;
                }
            if (fit_valid(&P, k))
                for (int c = 0; c < 2; ++c) o[8 + c] = wf * (O[2 * k + c] - C[2 * k + c]);
        }
}

/* GN (lm = 0) or LM solve through the generic loop; returns completed steps. */
int oracle_iw_solve_generic(int W, int H, float* O, float* A, const float* U, const float* C, const float* M,
                            float wf, float wr, int lm, int nIter, int lIter, int nthreads, double* costs) {
    return iw_solve_generic_float(W, H, O, A, U, C, M, wf, wr, lm, nIter, lIter, nthreads, costs);
}
/* J^T F and the raw diagonal (generic layout), for the LM kernel tests */
void oracle_iw_jtf_diag(int W, int H, const float* O, const float* A, const float* U, const float* C,
                        const float* M, float wf, float wr, float* r, float* diag) {
    iw_ctx c = {{W, H, O, A, U, C, M, wf, wr}, (float*)O, (float*)A, NULL, NULL, 1};
    iwg_jtf(&c, r, diag);
}
double oracle_iw_model_cost(int W, int H, const float* O, const float* A, const float* U, const float* C,
                            const float* M, float wf, float wr, const float* d) {
    iw_ctx c = {{W, H, O, A, U, C, M, wf, wr}, (float*)O, (float*)A, NULL, NULL, 1};
    return iwg_model(&c, d);
}

/* ------------------------------------------- materialized Jacobian (oracle/csr.c) ---- */
/* saveJToCRS / generateDumpJ (solverGPUGaussNewton.t:385-442, 1004-1022): every pixel
 * k (excluded ones included) owns rows 10k..10k+9 — for s in (+x,-x,+y,-y): channel 0,
 * channel 1 (3 nonzeros each: O_c(k), O_c(k+s), A(k)); then fit channel 0, 1 (1 each)
 * — at nonzero offset 26k. Columns: image offset + channels * tooffset + channel,
 * wrapped into [0, 3N) (wrap :365-381), sorted inside the row (sortCol). Values are the
 * partials of the residual (0 where it is not valid). */
#include "csr.h"
static void iw_dump(void* v, int* rowPtr, int* colInd, float* val) {
    const iw_problem* P = (const iw_problem*)v;
    const long long N = (long long)P->W * P->H, n = 3 * N;
    for (int y = 0; y < P->H; ++y)
        for (int x = 0; x < P->W; ++x) {
            const long long k = (long long)y * P->W + x, rb = 10 * k, nb = 26 * k;
            for (int s = 0; s < 4; ++s) {
                const long long tn = k + SX[s] + (long long)SY[s] * P->W;
                for (int c = 0; c < 2; ++c) {
                    reg_res r = reg_residual(P, x, y, s, c);
                    const int row = 2 * s + c;
                    long long cc[3] = {2 * k + c, 2 * tn + c, 2 * N + k};
                    float vv[3] = {r.valid ? r.dOc : 0.f, r.valid ? r.dOsc : 0.f, r.valid ? r.dA : 0.f};
                    for (int q = 0; q < 3; ++q) cc[q] = cc[q] < 0 ? cc[q] + n : (cc[q] >= n ? cc[q] - n : cc[q]);
                    for (int a = 1; a < 3; ++a)   /* sortCol */
                        for (int b = a; b > 0 && cc[b] < cc[b - 1]; --b) {
                            long long tc = cc[b]; cc[b] = cc[b - 1]; cc[b - 1] = tc;
                            float tv = vv[b]; vv[b] = vv[b - 1]; vv[b - 1] = tv;
                        }
                    rowPtr[rb + row] = (int)(nb + 3 * row);
                    for (int q = 0; q < 3; ++q) { colInd[nb + 3 * row + q] = (int)cc[q]; val[nb + 3 * row + q] = vv[q]; }
                }
            }
            const int has = fit_valid(P, (int)k);
            for (int c = 0; c < 2; ++c) {
                rowPtr[rb + 8 + c] = (int)(nb + 24 + c);
                colInd[nb + 24 + c] = (int)(2 * k + c);
                val[nb + 24 + c] = has ? P->wf : 0.f;
            }
        }
    rowPtr[10 * N] = (int)(26 * N);
}
void oracle_iw_dump_j(int W, int H, const float* O, const float* A, const float* U, const float* C, const float* M,
                      float wf, float wr, int* rowPtr, int* colInd, float* val) {
    iw_problem P = {W, H, O, A, U, C, M, wf, wr};
    iw_dump(&P, rowPtr, colInd, val);
}

typedef struct { iw_ctx c; oracle_mat m; } iwm_ctx;
static void iwm_materialize(void* v) { oracle_mat_build(&((iwm_ctx*)v)->m); }
static double iwm_apply(void* v, const float* p, float* Ap) { return oracle_mat_apply(&((iwm_ctx*)v)->m, p, Ap); }
static void iwm_dump(void* v, int* rowPtr, int* colInd, float* val) { iw_dump(&((iw_ctx*)v)->P, rowPtr, colInd, val); }

/* GN / LM solve with the materialized J^T J (fused) or J^T (J p) apply */
int oracle_iw_solve_materialized(int W, int H, float* O, float* A, const float* U, const float* C, const float* M,
                                 float wf, float wr, int lm, int fused, int nIter, int lIter, double* costs) {
    const int N = W * H;
    iwm_ctx c = {{{W, H, O, A, U, C, M, wf, wr}, O, A, NULL, NULL, 1}};
    c.c.prevO = (float*)malloc(sizeof(float) * 2 * N);
    c.c.prevA = (float*)malloc(sizeof(float) * N);
    unsigned char* act = (unsigned char*)malloc((size_t)3 * N);
    for (int k = 0; k < N; ++k) act[2 * k] = act[2 * k + 1] = act[2 * N + k] = M[k] == 0.f;
    oracle_mat_init(&c.m, 10LL * N, 26LL * N, 3 * N, fused, act, iwm_dump, &c.c);
    oracle_problem_float P = {3LL * N, act, 1, &c, iwg_cost, iwg_jtf, iwg_apply, iwg_model,
                              iwg_update, iwg_save, iwg_revert, iwm_materialize, iwm_apply};
    oracle_params sp = oracle_default_params();
    sp.nIterations = nIter;
    sp.lIterations = lIter;
    const int k = oracle_solve_f32(&P, lm, &sp, costs);
    oracle_mat_free(&c.m);
    free(act); free(c.c.prevO); free(c.c.prevA);
    return k;
}
/* one materialized apply at the given unknowns (Ap = 0 on excluded unknowns) */
double oracle_iw_apply_materialized(int W, int H, const float* O, const float* A, const float* U, const float* C,
                                    const float* M, float wf, float wr, int fused, const float* p, float* Ap) {
    const int N = W * H;
    iwm_ctx c = {{{W, H, O, A, U, C, M, wf, wr}, (float*)O, (float*)A, NULL, NULL, 1}};
    unsigned char* act = (unsigned char*)malloc((size_t)3 * N);
    for (int k = 0; k < N; ++k) act[2 * k] = act[2 * k + 1] = act[2 * N + k] = M[k] == 0.f;
    oracle_mat_init(&c.m, 10LL * N, 26LL * N, 3 * N, fused, act, iwm_dump, &c.c);
    oracle_mat_build(&c.m);
    const double d = oracle_mat_apply(&c.m, p, Ap);
    oracle_mat_free(&c.m);
    free(act);
    return d;
}
