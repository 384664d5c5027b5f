/* oracle/optical_flow.c — TEST INFRASTRUCTURE ONLY: the optical_flow restatement
 * (optical_flow_impl.h) for opt_float = float and double, and its public entry points. */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "solver.h"

#define REAL float
#define OACC double
#include "optical_flow_impl.h"
#undef REAL
#undef OACC
#define OACC long double
#define REAL double
#include "optical_flow_impl.h"
#undef REAL

#define OF_API(R, P)                                                                                         \
    double oracle_of_cost_##R(int W, int H, R* X, const float* I, const float* Ih, const float* Ihx,         \
                              const float* Ihy, float wf, float wr) {                                       \
        of_ctx_##R c = of_make_##R(W, H, X, I, Ih, Ihx, Ihy, wf, wr);                                       \
        const double v = of_cost_##R(&c);                                                                   \
        free(c.G);                                                                                          \
        return v;                                                                                           \
    }                                                                                                       \
    void oracle_of_jtf_##R(int W, int H, R* X, const float* I, const float* Ih, const float* Ihx,           \
                           const float* Ihy, float wf, float wr, R* r, R* diag) {                           \
        of_ctx_##R c = of_make_##R(W, H, X, I, Ih, Ihx, Ihy, wf, wr);                                       \
        of_jtf_##R(&c, r, diag);                                                                            \
        free(c.G);                                                                                          \
    }                                                                                                       \
    double oracle_of_apply_##R(int W, int H, R* X, const float* I, const float* Ih, const float* Ihx,       \
                               const float* Ihy, float wf, float wr, const R* p, R* Ap) {                   \
        of_ctx_##R c = of_make_##R(W, H, X, I, Ih, Ihx, Ihy, wf, wr);                                       \
        const size_t n = 2 * (size_t)W * H;                                                                 \
        R* r = (R*)calloc(n, sizeof(R));                                                                    \
        R* dg = (R*)calloc(n, sizeof(R));                                                                   \
        of_jtf_##R(&c, r, dg);                                                                              \
        const double v = of_apply_##R(&c, p, Ap);                                                           \
        free(r); free(dg); free(c.G);                                                                       \
        return v;                                                                                           \
    }                                                                                                       \
    double oracle_of_model_cost_##R(int W, int H, R* X, const float* I, const float* Ih, const float* Ihx,  \
                                    const float* Ihy, float wf, float wr, const R* d) {                     \
        of_ctx_##R c = of_make_##R(W, H, X, I, Ih, Ihx, Ihy, wf, wr);                                       \
        const double v = of_model_##R(&c, d);                                                              \
        free(c.G);                                                                                          \
        return v;                                                                                           \
    }                                                                                                       \
    int oracle_of_solve_##R(int W, int H, R* X, const float* I, const float* Ih, const float* Ihx,          \
                            const float* Ihy, float wf, float wr, int lm, int nIter, int lIter,             \
                            double* costs) {                                                                \
        of_ctx_##R c = of_make_##R(W, H, X, I, Ih, Ihx, Ihy, wf, wr);                                       \
        const long long n = 2LL * W * H;                                                                    \
        unsigned char* act = (unsigned char*)malloc(n);                                                     \
        memset(act, 1, n);                                                                                  \
        c.prev = (R*)malloc(sizeof(R) * n);                                                                 \
        P P_ = {n, act, 0, &c, of_cost_##R, of_jtf_##R, of_apply_##R, of_model_##R,                         \
                of_update_##R, of_save_##R, of_revert_##R};                                                 \
        oracle_params sp = oracle_default_params();                                                         \
        sp.nIterations = nIter;                                                                             \
        sp.lIterations = lIter;                                                                             \
        const int k = oracle_solve_##R(&P_, lm, &sp, costs);                                                \
        free(act); free(c.prev); free(c.G);                                                                 \
        return k;                                                                                           \
    }

static int oracle_solve_float(oracle_problem_float* P, int lm, const oracle_params* sp, double* costs) {
    return oracle_solve_f32(P, lm, sp, costs);
}
static int oracle_solve_double(oracle_problem_double* P, int lm, const oracle_params* sp, double* costs) {
    return oracle_solve_f64(P, lm, sp, costs);
}
OF_API(float, oracle_problem_float)
OF_API(double, oracle_problem_double)
