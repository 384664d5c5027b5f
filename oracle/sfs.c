/*
 * oracle/sfs.c — CPU restatement of the reference's shape_from_shading solver, for
 * opt_float = float and double (the body is oracle/sfs_impl.h).
 * TEST INFRASTRUCTURE ONLY (oracle/README.md). PARITY UNPINNED for this energy: the
 * reference's end-to-end test holds no value for it (test_final_cost.py:64, -1); its own input files
 * (examples/data/shape_from_shading/default*) are used as inputs, and this restatement
 * is pinned by an independent float64 numpy restatement with finite differences
 * (tests/test_oracle_sfs.py).
 *
 * Energy examples/shape_from_shading/shape_from_shading.t. Unknown X (depth), knowns
 * D_i, Im (float), edgeMaskR/C (uint8); params w_p, w_s, w_g (square-rooted inside the
 * energy), f_x, f_y, u_x, u_y, L_1..L_9. Exclude(D_i <= 0).
 * ComputedArrays (ProblemSpecAD:ComputedImage, API/src/o.t:1686-1716): B_I and its
 * gradient images w.r.t. the three unknowns it reads, X(0,0), X(-1,0), X(0,-1), and
 * `valid` (comparisons only: constant gradient, not materialised); all recomputed by
 * `precompute` at init, after each update and after a revert
 * (solverGPUGaussNewton.t:1876, 2242, 2284).
 * Residual templates (value and partials w.r.t. X at offsets of the centre c):
 *   E_p   = DV(c) ? w_p (X - D_i) : 0
 *   E_g_h = InBoundsExpanded(c,1) ? w_g (B_I(c) - B_I(c+(1,0))) edgeMaskR(c) : 0
 *   E_g_v = InBoundsExpanded(c,1) ? w_g (B_I(c) - B_I(c+(0,1))) edgeMaskC(c) : 0
 *   E_s   = valid(c) == 1 ? w_s (4 p(0,0) - sum_4 p(o)) : 0     (3 components)
 * where a residual that reads B_I(c+o) depends on X(c+o+(0,0)), X(c+o+(-1,0)),
 * X(c+o+(0,-1)) through the gradient images read at c+o (ImageAccess:gradient,
 * o.t:1664-1676). Gathers: J^T F / diag o.t:2870-2913, J^T J p o.t:2770-2830 (every
 * residual instance containing X_k, centred anywhere, excluded centres included),
 * cost o.t:3119-3129 and model cost o.t:2915-2943 over non-excluded centres only
 * (computeCost / computeModelCost, solverGPUGaussNewton.t:971-997).
 * Image reads outside the image are 0 (Image:get, o.t:856-862).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "solver.h"


#define REAL float
#define OACC double
#include "sfs_impl.h"
#undef REAL
#undef OACC
#define OACC long double
#define REAL double
#include "sfs_impl.h"
#undef REAL

/* ------------------------------------------------------------- public API ---- */
/* prm: w_p, w_s, w_g, f_x, f_y, u_x, u_y, L_1..L_9 (16 floats, declaration order).
 * float entry points: oracle_sfs_*; double (unknowns and solver vectors in double,
 * known arrays float): oracle_sfs_*_double. */
#define SFS_API(R, SUF, SOLVE)                                                                                  \
    static sfs_ctx_##R make_ctx_##R(int W, int H, R* X, const float* D, const float* Im, const unsigned char* mR, \
                                    const unsigned char* mC, const float* prm) {                                  \
        sfs_ctx_##R c;                                                                                            \
        memset(&c, 0, sizeof(c));                                                                                 \
        c.W = W; c.H = H; c.X = X; c.D = D; c.Im = Im; c.mR = mR; c.mC = mC;                                      \
        c.wp = prm[0]; c.ws = prm[1]; c.wg = prm[2]; c.fx = prm[3]; c.fy = prm[4]; c.ux = prm[5]; c.uy = prm[6]; \
        for (int i = 0; i < 9; ++i) c.L[i] = prm[7 + i];                                                          \
        const size_t N = (size_t)W * H;                                                                           \
        c.BI = calloc(N, sizeof(R)); c.G00 = calloc(N, sizeof(R)); c.Gm0 = calloc(N, sizeof(R));                  \
        c.G0m = calloc(N, sizeof(R)); c.VAL = calloc(N, sizeof(R)); c.prev = calloc(N, sizeof(R));                \
        sfs_precompute_##R(&c);                                                                                   \
        return c;                                                                                                 \
    }                                                                                                             \
    static void free_ctx_##R(sfs_ctx_##R* c) {                                                                   \
        free(c->BI); free(c->G00); free(c->Gm0); free(c->G0m); free(c->VAL); free(c->prev);                       \
    }                                                                                                             \
    /* out = [B_I | dB_I/dX(0,0) | dB_I/dX(-1,0) | dB_I/dX(0,-1) | valid], 5 N values */                       \
    void oracle_sfs_precompute##SUF(int W, int H, R* X, const float* D, const float* Im, const unsigned char* mR, \
                                    const unsigned char* mC, const float* prm, R* out) {                          \
        sfs_ctx_##R c = make_ctx_##R(W, H, X, D, Im, mR, mC, prm);                                                \
        const size_t N = (size_t)W * H;                                                                           \
        memcpy(out, c.BI, N * sizeof(R)); memcpy(out + N, c.G00, N * sizeof(R));                                  \
        memcpy(out + 2 * N, c.Gm0, N * sizeof(R)); memcpy(out + 3 * N, c.G0m, N * sizeof(R));                     \
        memcpy(out + 4 * N, c.VAL, N * sizeof(R));                                                                \
        free_ctx_##R(&c);                                                                                         \
    }                                                                                                             \
    double oracle_sfs_cost##SUF(int W, int H, R* X, const float* D, const float* Im, const unsigned char* mR,    \
                                const unsigned char* mC, const float* prm) {                                      \
        sfs_ctx_##R c = make_ctx_##R(W, H, X, D, Im, mR, mC, prm);                                                \
        const double v = sfs_cost_fn_##R(&c);                                                                     \
        free_ctx_##R(&c);                                                                                         \
        return v;                                                                                                 \
    }                                                                                                             \
    void oracle_sfs_jtf##SUF(int W, int H, R* X, const float* D, const float* Im, const unsigned char* mR,       \
                             const unsigned char* mC, const float* prm, R* r, R* diag) {                          \
        sfs_ctx_##R c = make_ctx_##R(W, H, X, D, Im, mR, mC, prm);                                                \
        sfs_jtf_fn_##R(&c, r, diag);                                                                              \
        free_ctx_##R(&c);                                                                                         \
    }                                                                                                             \
    double oracle_sfs_apply##SUF(int W, int H, R* X, const float* D, const float* Im, const unsigned char* mR,   \
                                 const unsigned char* mC, const float* prm, const R* p, R* Ap) {                  \
        sfs_ctx_##R c = make_ctx_##R(W, H, X, D, Im, mR, mC, prm);                                                \
        const double v = sfs_apply_fn_##R(&c, p, Ap);                                                             \
        free_ctx_##R(&c);                                                                                         \
        return v;                                                                                                 \
    }                                                                                                             \
    double oracle_sfs_model_cost##SUF(int W, int H, R* X, const float* D, const float* Im,                      \
                                      const unsigned char* mR, const unsigned char* mC, const float* prm,         \
                                      const R* d) {                                                               \
        sfs_ctx_##R c = make_ctx_##R(W, H, X, D, Im, mR, mC, prm);                                                \
        const double v = sfs_model_fn_##R(&c, d);                                                                 \
        free_ctx_##R(&c);                                                                                         \
        return v;                                                                                                 \
    }                                                                                                             \
    /* nthreads: row slabs of every stencil pass over that many threads (backend_cpu_mt) */                    \
    int oracle_sfs_solve##SUF(int W, int H, R* X, const float* D, const float* Im, const unsigned char* mR,      \
                              const unsigned char* mC, const float* prm, int lm, int nIter, int lIter,            \
                              double* costs, int nthreads) {                                                      \
        sfs_ctx_##R c = make_ctx_##R(W, H, X, D, Im, mR, mC, prm);                                                \
        c.nthreads = nthreads;                                                                                    \
        const long long n = (long long)W * H;                                                                     \
        unsigned char* act = malloc(n);                                                                           \
        for (long long k = 0; k < n; ++k) act[k] = !excl_##R(&c, k);                                              \
        oracle_problem_##R P = {n, act, 0, &c, sfs_cost_fn_##R, sfs_jtf_fn_##R, sfs_apply_fn_##R,                 \
                                sfs_model_fn_##R, sfs_update_fn_##R, sfs_save_fn_##R, sfs_revert_fn_##R};         \
        oracle_params sp = oracle_default_params();                                                               \
        sp.nIterations = nIter;                                                                                   \
        sp.lIterations = lIter;                                                                                   \
        const int k = SOLVE(&P, lm, &sp, costs);                                                                  \
        free(act);                                                                                                \
        free_ctx_##R(&c);                                                                                         \
        return k;                                                                                                 \
    }

SFS_API(float, , oracle_solve_f32)
SFS_API(double, _double, oracle_solve_f64)
