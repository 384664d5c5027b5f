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
 * Vector layout (reference UnknownType, o.t:998-1100): [Offset.xy * N | Angle * N].
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int W, H;
    const float* O;   /* Offset, 2 per pixel (current unknowns) */
    const float* A;   /* Angle */
    const float* U;   /* UrShape, 2 per pixel */
    const float* C;   /* Constraints, 2 per pixel */
    const float* M;   /* Mask */
    float wf, wr;     /* w_fitSqrt, w_regSqrt */
} iw_problem;

static const int SX[4] = {1, -1, 0, 0};
static const int SY[4] = {0, 0, 1, -1};

static int inb(const iw_problem* P, int x, int y) { return x >= 0 && x < P->W && y >= 0 && y < P->H; }
/* Image:get zero-fills out-of-bounds reads (o.t:856-862) */
static float getM(const iw_problem* P, int x, int y) { return inb(P, x, y) ? P->M[y * P->W + x] : 0.f; }
/* fmap.exclude: Exclude(Not(eq(Mask(0,0),0))) */
static int excluded(const iw_problem* P, int x, int y) { return getM(P, x, y) != 0.f; }

/* Residual template s (0..3: stencil dir, component c) centered at (x,y):
 *   valid = InBounds(x,y) [bbox of the center, usesbounds]  &  InBounds(x+sx,y+sy)
 *           & Mask(x+sx,y+sy)==0 & Mask(x,y)==0
 *   value = wr*((O - O_s) - Rotate2D(A, U - U_s))_c
 * Partials w.r.t. its support {O_c(x,y), O_c(x+s), A(x,y)}. */
typedef struct { int valid; float value, dOc, dOsc, dA; } reg_res;

static reg_res reg_residual(const iw_problem* P, int x, int y, int s, int c) {
    reg_res r = {0, 0.f, 0.f, 0.f, 0.f};
    const int tx = x + SX[s], ty = y + SY[s];
    if (!inb(P, x, y) || !inb(P, tx, ty)) return r;
    if (getM(P, tx, ty) != 0.f || getM(P, x, y) != 0.f) return r;
    const int i = y * P->W + x, t = ty * P->W + tx;
    const float a = P->A[i];
    const float ca = cosf(a), sa = sinf(a);
    const float dx = P->U[2 * i] - P->U[2 * t], dy = P->U[2 * i + 1] - P->U[2 * t + 1];
    /* Rotate2D (lib.t): (cos*v0 - sin*v1, sin*v0 + cos*v1); its angle derivative */
    const float rot = c == 0 ? ca * dx - sa * dy : sa * dx + ca * dy;
    const float drot = c == 0 ? -sa * dx - ca * dy : ca * dx - sa * dy;
    r.valid = 1;
    r.value = P->wr * ((P->O[2 * i + c] - P->O[2 * t + c]) - rot);
    r.dOc = P->wr;
    r.dOsc = -P->wr;
    r.dA = -P->wr * drot;
    return r;
}
/* fit residual c at (x,y): wf*Select(All(Constraints>=0), O - C, 0) */
static int fit_valid(const iw_problem* P, int i) { return P->C[2 * i] >= 0.f && P->C[2 * i + 1] >= 0.f; }

typedef struct {
    const iw_problem* P;
    int y0, y1;
    const float* p;
    float *out0, *out1;   /* Ap | (r, pre) */
    double acc;
    int use_pre;
} slab;

/* ---- applyJTJ (o.t:2770-2830): for each unknown x00 of pixel k, sum over residual
 * instances r containing x00 of dr/dx00 * sum_{u in supp r} dr/du p_u. */
static void apply_px(const iw_problem* P, const float* p, int x, int y, float* ao, float* at) {
    const int N = P->W * P->H, k = y * P->W + x;
    float accO[2] = {0.f, 0.f}, accA = 0.f;
    for (int s = 0; s < 4; ++s) {
        for (int c = 0; c < 2; ++c) {
            /* instance centered at k: contains O_c(k) and A(k) */
            reg_res r = reg_residual(P, x, y, s, c);
            if (r.valid) {
                const int t = (y + SY[s]) * P->W + (x + SX[s]);
                const float Jp = r.dOc * p[2 * k + c] + r.dOsc * p[2 * t + c] + r.dA * p[2 * N + k];
                accO[c] += r.dOc * Jp;
                accA += r.dA * Jp;
            }
            /* instance centered at k - s: contains O_c(k) as its neighbour */
            const int jx = x - SX[s], jy = y - SY[s];
            reg_res q = reg_residual(P, jx, jy, s, c);
            if (q.valid) {
                const int j = jy * P->W + jx;
                const float Jp = q.dOc * p[2 * j + c] + q.dOsc * p[2 * k + c] + q.dA * p[2 * N + j];
                accO[c] += q.dOsc * Jp;
            }
        }
    }
    if (fit_valid(P, k)) {
        accO[0] += P->wf * (P->wf * p[2 * k]);
        accO[1] += P->wf * (P->wf * p[2 * k + 1]);
    }
    ao[0] = accO[0];
    ao[1] = accO[1];
    *at = accA;
}

/* ---- evalJTF (o.t:2870-2913): F_hat = sum dr/dx00 * r ; P_hat = sum (dr/dx00)^2 */
static void jtf_px(const iw_problem* P, int x, int y, float* F, float* D) {
    const int k = y * P->W + x;
    float FO[2] = {0.f, 0.f}, FA = 0.f, DO[2] = {0.f, 0.f}, DA = 0.f;
    for (int s = 0; s < 4; ++s) {
        for (int c = 0; c < 2; ++c) {
            reg_res r = reg_residual(P, x, y, s, c);
            if (r.valid) {
                FO[c] += r.dOc * r.value;
                DO[c] += r.dOc * r.dOc;
                FA += r.dA * r.value;
                DA += r.dA * r.dA;
            }
            reg_res q = reg_residual(P, x - SX[s], y - SY[s], s, c);
            if (q.valid) {
                FO[c] += q.dOsc * q.value;
                DO[c] += q.dOsc * q.dOsc;
            }
        }
    }
    if (fit_valid(P, k)) {
        for (int c = 0; c < 2; ++c) {
            const float e = P->wf * (P->O[2 * k + c] - P->C[2 * k + c]);
            FO[c] += P->wf * e;
            DO[c] += P->wf * P->wf;
        }
    }
    F[0] = FO[0]; F[1] = FO[1]; F[2] = FA;
    D[0] = DO[0]; D[1] = DO[1]; D[2] = DA;
}

static float cost_px(const iw_problem* P, int x, int y) {
    const int k = y * P->W + x;
    float sum = 0.f;
    for (int s = 0; s < 4; ++s)
        for (int c = 0; c < 2; ++c) {
            reg_res r = reg_residual(P, x, y, s, c);
            if (r.valid) sum += r.value * r.value;
        }
    if (fit_valid(P, k))
        for (int c = 0; c < 2; ++c) {
            const float e = P->wf * (P->O[2 * k + c] - P->C[2 * k + c]);
            sum += e * e;
        }
    return 0.5f * sum;
}

/* ---- slab workers (backend_cpu_mt: outer dimension split, per-thread sums) ---- */
static void* w_apply(void* v) {
    slab* S = (slab*)v;
    const iw_problem* P = S->P;
    const int N = P->W * P->H;
    double acc = 0.0;
    for (int y = S->y0; y < S->y1; ++y)
        for (int x = 0; x < P->W; ++x) {
            const int k = y * P->W + x;
            float ao[2] = {0.f, 0.f}, at = 0.f;
            if (!excluded(P, x, y)) {
                apply_px(P, S->p, x, y, ao, &at);
                acc += (double)S->p[2 * k] * ao[0] + (double)S->p[2 * k + 1] * ao[1] +
                       (double)S->p[2 * N + k] * at;
            }
            S->out0[2 * k] = ao[0];
            S->out0[2 * k + 1] = ao[1];
            S->out0[2 * N + k] = at;
        }
    S->acc = acc;
    return NULL;
}
static float guarded_invert(float d) { const float s = 1.f + sqrtf(d); return 1.f / (s * s); }
static void* w_jtf(void* v) {
    slab* S = (slab*)v;
    const iw_problem* P = S->P;
    const int N = P->W * P->H;
    double acc = 0.0;
    for (int y = S->y0; y < S->y1; ++y)
        for (int x = 0; x < P->W; ++x) {
            const int k = y * P->W + x;
            float r[3] = {0.f, 0.f, 0.f}, pre[3] = {0.f, 0.f, 0.f};
            if (!excluded(P, x, y)) {
                float F[3], D[3];
                jtf_px(P, x, y, F, D);
                for (int c = 0; c < 3; ++c) {
                    r[c] = -F[c];
                    pre[c] = guarded_invert(S->use_pre ? D[c] : 1.f);
                    acc += (double)r[c] * (pre[c] * r[c]);
                }
            }
            S->out0[2 * k] = r[0]; S->out0[2 * k + 1] = r[1]; S->out0[2 * N + k] = r[2];
            S->out1[2 * k] = pre[0]; S->out1[2 * k + 1] = pre[1]; S->out1[2 * N + k] = pre[2];
        }
    S->acc = acc;
    return NULL;
}
static void* w_cost(void* v) {
    slab* S = (slab*)v;
    const iw_problem* P = S->P;
    double acc = 0.0;
    for (int y = S->y0; y < S->y1; ++y)
        for (int x = 0; x < P->W; ++x)
            if (!excluded(P, x, y)) acc += cost_px(P, x, y);
    S->acc = acc;
    return NULL;
}

static double run_slabs(const iw_problem* P, int nthreads, void* (*fn)(void*), const float* p,
                        float* o0, float* o1) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > P->H) nthreads = P->H;
    slab* S = (slab*)calloc(nthreads, sizeof(slab));
    pthread_t* th = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        S[t].P = P;
        S[t].y0 = t * (P->H / nthreads);
        S[t].y1 = (t == nthreads - 1) ? P->H : (t + 1) * (P->H / nthreads);
        S[t].p = p; S[t].out0 = o0; S[t].out1 = o1; S[t].use_pre = 1;
    }
    if (nthreads == 1) fn(&S[0]);
    else {
        for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fn, &S[t]);
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    }
    double acc = 0.0;
    for (int t = 0; t < nthreads; ++t) acc += S[t].acc;   /* thread order (backend_cpu_mt.t:402-410) */
    free(S);
    free(th);
    return acc;
}

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
    iw_problem P = {W, H, O, A, U, C, M, wf, wr};
    const int N = W * H;
    const size_t n3 = (size_t)3 * N;
    float* r = (float*)calloc(n3, sizeof(float));
    float* pre = (float*)calloc(n3, sizeof(float));
    float* p = (float*)calloc(n3, sizeof(float));
    float* Ap = (float*)calloc(n3, sizeof(float));
    float* d = (float*)calloc(n3, sizeof(float));
    costs[0] = run_slabs(&P, nthreads, w_cost, NULL, NULL, NULL);
    for (int it = 0; it < nIter; ++it) {
        /* PCGInit1 */
        double alpha_num = run_slabs(&P, nthreads, w_jtf, NULL, r, pre);
        for (size_t e = 0; e < n3; ++e) { d[e] = 0.f; p[e] = pre[e] * r[e]; }
        for (int li = 0; li < lIter; ++li) {
            /* PCGStep1 */
            double alpha_den = run_slabs(&P, nthreads, w_apply, p, Ap, NULL);
            /* PCGStep2 (excluded elements hold r = pre = p = Ap = 0) */
            const float alpha = (float)(alpha_num / alpha_den);
            double beta_num = 0.0;
            for (size_t e = 0; e < n3; ++e) {
                d[e] = d[e] + alpha * p[e];
                r[e] = r[e] - alpha * Ap[e];
                const float z = pre[e] * r[e];
                beta_num += (double)z * r[e];
            }
            if (scalars) {
                scalars[((size_t)it * lIter + li) * 3 + 0] = alpha_num;
                scalars[((size_t)it * lIter + li) * 3 + 1] = alpha_den;
                scalars[((size_t)it * lIter + li) * 3 + 2] = beta_num;
            }
            /* PCGStep3 */
            const float beta = (float)(beta_num / alpha_num);
            for (size_t e = 0; e < n3; ++e) p[e] = pre[e] * r[e] + beta * p[e];
            alpha_num = beta_num;
        }
        /* PCGLinearUpdate (skips excluded pixels) */
        for (int k = 0; k < N; ++k) {
            if (M[k] != 0.f) continue;
            O[2 * k] += d[2 * k];
            O[2 * k + 1] += d[2 * k + 1];
            A[k] += d[2 * N + k];
        }
        costs[it + 1] = run_slabs(&P, nthreads, w_cost, NULL, NULL, NULL);
    }
    free(r); free(pre); free(p); free(Ap); free(d);
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

/* ------------------------------------------------ generic GN / LM (solver_impl.h) ---- */
/* Vector layout [Offset.xy * N | Angle * N]; an element is active iff its pixel's Mask
 * is 0. Model cost = 1/2 sum (F + J delta)^2 over the residuals of active pixels
 * (createmodelcost, API/src/o.t:2915-2943). */
#include "solver.h"
typedef struct {
    iw_problem P;
    float *O, *A, *prevO, *prevA;
    int nthreads;
} iw_ctx;

static double iwg_cost(void* v) {
    iw_ctx* c = (iw_ctx*)v;
    return run_slabs(&c->P, c->nthreads, w_cost, NULL, NULL, NULL);
}
static void iwg_jtf(void* v, float* r, float* diag) {
    iw_ctx* c = (iw_ctx*)v;
    const iw_problem* P = &c->P;
    const int N = P->W * P->H;
    for (int y = 0; y < P->H; ++y)
        for (int x = 0; x < P->W; ++x) {
            const int k = y * P->W + x;
            float F[3] = {0.f, 0.f, 0.f}, D[3] = {0.f, 0.f, 0.f};
            if (!excluded(P, x, y)) jtf_px(P, x, y, F, D);
            r[2 * k] = -F[0]; r[2 * k + 1] = -F[1]; r[2 * N + k] = -F[2];
            diag[2 * k] = D[0]; diag[2 * k + 1] = D[1]; diag[2 * N + k] = D[2];
        }
}
static double iwg_apply(void* v, const float* p, float* Ap) {
    iw_ctx* c = (iw_ctx*)v;
    return run_slabs(&c->P, c->nthreads, w_apply, p, Ap, NULL);
}
static double iwg_model(void* v, const float* d) {
    iw_ctx* c = (iw_ctx*)v;
    const iw_problem* P = &c->P;
    const int N = P->W * P->H;
    double acc = 0.0;
    for (int y = 0; y < P->H; ++y)
        for (int x = 0; x < P->W; ++x) {
            if (excluded(P, x, y)) continue;
            const int k = y * P->W + x;
            float sum = 0.f;
            for (int s = 0; s < 4; ++s)
                for (int ch = 0; ch < 2; ++ch) {
                    reg_res r = reg_residual(P, x, y, s, ch);
                    if (!r.valid) continue;
                    const int t = (y + SY[s]) * P->W + (x + SX[s]);
                    const float e = r.value + (r.dOc * d[2 * k + ch] + r.dOsc * d[2 * t + ch] + r.dA * d[2 * N + k]);
                    sum += e * e;
                }
            if (fit_valid(P, k))
                for (int ch = 0; ch < 2; ++ch) {
                    const float e = P->wf * (P->O[2 * k + ch] - P->C[2 * k + ch]) + P->wf * d[2 * k + ch];
                    sum += e * e;
                }
            acc += 0.5f * sum;
        }
    return acc;
}
static void iwg_update(void* v, const float* d) {
    iw_ctx* c = (iw_ctx*)v;
    const int N = c->P.W * c->P.H;
    for (int k = 0; k < N; ++k) {
        if (c->P.M[k] != 0.f) continue;
        c->O[2 * k] += d[2 * k];
        c->O[2 * k + 1] += d[2 * k + 1];
        c->A[k] += d[2 * N + k];
    }
}
static void iwg_save(void* v) {
    iw_ctx* c = (iw_ctx*)v;
    const int N = c->P.W * c->P.H;
    memcpy(c->prevO, c->O, sizeof(float) * 2 * N);
    memcpy(c->prevA, c->A, sizeof(float) * N);
}
static void iwg_revert(void* v) {
    iw_ctx* c = (iw_ctx*)v;
    const int N = c->P.W * c->P.H;
    for (int k = 0; k < N; ++k) {
        if (c->P.M[k] != 0.f) continue;
        c->O[2 * k] = c->prevO[2 * k];
        c->O[2 * k + 1] = c->prevO[2 * k + 1];
        c->A[k] = c->prevA[k];
    }
}

/* GN (lm = 0) or LM solve through the generic loop; returns completed steps. */
int oracle_iw_solve_generic(int W, int H, float* O, float* A, const float* U, const float* C, const float* M,
                            float wf, float wr, int lm, int nIter, int lIter, int nthreads, double* costs) {
    const int N = W * H;
    iw_ctx c = {{W, H, O, A, U, C, M, wf, wr}, O, A, NULL, NULL, nthreads};
    c.prevO = (float*)malloc(sizeof(float) * 2 * N);
    c.prevA = (float*)malloc(sizeof(float) * N);
    unsigned char* act = (unsigned char*)malloc((size_t)3 * N);
    for (int k = 0; k < N; ++k) act[2 * k] = act[2 * k + 1] = act[2 * N + k] = M[k] == 0.f;
    oracle_problem_float P = {3LL * N, act, 1, &c, iwg_cost, iwg_jtf, iwg_apply, iwg_model,
                              iwg_update, iwg_save, iwg_revert};
    oracle_params sp = oracle_default_params();
    sp.nIterations = nIter;
    sp.lIterations = lIter;
    const int k = oracle_solve_f32(&P, lm, &sp, costs);
    free(act); free(c.prevO); free(c.prevA);
    return k;
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
