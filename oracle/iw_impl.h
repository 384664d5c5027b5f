/*
 * oracle/iw_impl.h — TEST INFRASTRUCTURE ONLY (oracle/README.md): the image_warping
 * restatement (header comment of oracle/image_warping.c) in opt_float = REAL arithmetic.
 * Instantiated for REAL = float (the entry points oracle_iw_*) and REAL = double
 * (oracle_iw_*_double) by oracle/image_warping.c, which defines RCOS / RSIN / RSQRT as
 * the math functions of that precision (the reference casts the arguments of math
 * functions to opt_float, API/src/o.t:1960-1966, 2021-2028).
 *
 * doublePrecision (API/release/include/Opt.h:11-14): the unknowns (Offset, Angle), the
 * solver vectors and the parameters are opt_float = double; the known arrays UrShape,
 * Constraints and Mask stay float, as the harness passes them
 * (examples/shared/OptSolver.h:20-28). Arithmetic between two float array reads stays
 * float (the generated code emits the Terra operation on the loaded values, o.t:2418-2470):
 * UrShape differences are float subtractions promoted afterwards; Constraints are
 * promoted where they meet an Offset.
 *
 * OACC, the accumulator of every sum (rz, p.Ap, cost), is double for REAL = float and
 * long double for REAL = double (oracle/image_warping.c). The reference's reductions are
 * atomics in no fixed order (backend_cuda.t:366-495), so its fp64 trajectory is defined
 * only up to summation order; this trajectory (10 PCG iterations on the bench workload)
 * amplifies one rounding of a PCG scalar ~1e9-fold, so a double accumulator made the
 * "double oracle" itself move by up to 3.5e-7 between slab counts at 1024^2 (round 5,
 * DESIGN.md §5). The 80-bit sums are the fp64 truth the GPU paths are held to.
 */
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define FN(name) CAT(name, CAT(_, REAL))

typedef struct {
    int W, H;
    const REAL* O;    /* Offset, 2 per pixel (current unknowns) */
    const REAL* A;    /* Angle */
    const float* U;   /* UrShape, 2 per pixel */
    const float* C;   /* Constraints, 2 per pixel */
    const float* M;   /* Mask */
    REAL wf, wr;      /* w_fitSqrt, w_regSqrt */
} FN(iw_problem);

static int FN(inb)(const FN(iw_problem) * P, int x, int y) { return x >= 0 && x < P->W && y >= 0 && y < P->H; }
/* Image:get zero-fills out-of-bounds reads (o.t:856-862) */
static float FN(getM)(const FN(iw_problem) * P, int x, int y) { return FN(inb)(P, x, y) ? P->M[y * P->W + x] : 0.f; }
/* fmap.exclude: Exclude(Not(eq(Mask(0,0),0))) */
static int FN(excluded)(const FN(iw_problem) * P, int x, int y) { return FN(getM)(P, x, y) != 0.f; }

/* Residual template s (0..3: stencil dir, component c) centered at (x,y):
 *   valid = InBounds(x,y) [bbox of the center, usesbounds]  &  InBounds(x+sx,y+sy)
 *           & Mask(x+sx,y+sy)==0 & Mask(x,y)==0
 *   value = wr*((O - O_s) - Rotate2D(A, U - U_s))_c
 * Partials w.r.t. its support {O_c(x,y), O_c(x+s), A(x,y)}. */
typedef struct { int valid; REAL value, dOc, dOsc, dA; } FN(reg_res);

static FN(reg_res) FN(reg_residual)(const FN(iw_problem) * P, int x, int y, int s, int c) {
    FN(reg_res) r = {0, (REAL)0, (REAL)0, (REAL)0, (REAL)0};
    const int tx = x + SX[s], ty = y + SY[s];
    if (!FN(inb)(P, x, y) || !FN(inb)(P, tx, ty)) return r;
    if (FN(getM)(P, tx, ty) != 0.f || FN(getM)(P, x, y) != 0.f) return r;
    const int i = y * P->W + x, t = ty * P->W + tx;
    const REAL a = P->A[i];
    const REAL ca = RCOS(a), sa = RSIN(a);
    const REAL dx = (REAL)(P->U[2 * i] - P->U[2 * t]), dy = (REAL)(P->U[2 * i + 1] - P->U[2 * t + 1]);
    /* Rotate2D (lib.t): (cos*v0 - sin*v1, sin*v0 + cos*v1); its angle derivative */
    const REAL rot = c == 0 ? ca * dx - sa * dy : sa * dx + ca * dy;
    const REAL drot = c == 0 ? -sa * dx - ca * dy : ca * dx - sa * dy;
    r.valid = 1;
    r.value = P->wr * ((P->O[2 * i + c] - P->O[2 * t + c]) - rot);
    r.dOc = P->wr;
    r.dOsc = -P->wr;
    r.dA = -P->wr * drot;
    return r;
}
/* fit residual c at (x,y): wf*Select(All(Constraints>=0), O - C, 0) */
static int FN(fit_valid)(const FN(iw_problem) * P, int i) { return P->C[2 * i] >= 0.f && P->C[2 * i + 1] >= 0.f; }

typedef struct {
    const FN(iw_problem) * P;
    int y0, y1;
    const REAL* p;
    REAL *out0, *out1;   /* Ap | (r, pre) */
    OACC acc;
    int use_pre;
} FN(slab);

/* ---- applyJTJ (o.t:2770-2830): for each unknown x00 of pixel k, sum over residual
 * instances r containing x00 of dr/dx00 * sum_{u in supp r} dr/du p_u. */
static void FN(apply_px)(const FN(iw_problem) * P, const REAL* p, int x, int y, REAL* ao, REAL* at) {
    const int N = P->W * P->H, k = y * P->W + x;
    REAL accO[2] = {(REAL)0, (REAL)0}, accA = (REAL)0;
    for (int s = 0; s < 4; ++s) {
        for (int c = 0; c < 2; ++c) {
            /* instance centered at k: contains O_c(k) and A(k) */
            FN(reg_res) r = FN(reg_residual)(P, x, y, s, c);
            if (r.valid) {
                const int t = (y + SY[s]) * P->W + (x + SX[s]);
                const REAL Jp = r.dOc * p[2 * k + c] + r.dOsc * p[2 * t + c] + r.dA * p[2 * N + k];
                accO[c] += r.dOc * Jp;
                accA += r.dA * Jp;
            }
            /* instance centered at k - s: contains O_c(k) as its neighbour */
            const int jx = x - SX[s], jy = y - SY[s];
            FN(reg_res) q = FN(reg_residual)(P, jx, jy, s, c);
            if (q.valid) {
                const int j = jy * P->W + jx;
                const REAL Jp = q.dOc * p[2 * j + c] + q.dOsc * p[2 * k + c] + q.dA * p[2 * N + j];
                accO[c] += q.dOsc * Jp;
            }
        }
    }
    if (FN(fit_valid)(P, k)) {
        accO[0] += P->wf * (P->wf * p[2 * k]);
        accO[1] += P->wf * (P->wf * p[2 * k + 1]);
    }
    ao[0] = accO[0];
    ao[1] = accO[1];
    *at = accA;
}

/* ---- evalJTF (o.t:2870-2913): F_hat = sum dr/dx00 * r ; P_hat = sum (dr/dx00)^2 */
static void FN(jtf_px)(const FN(iw_problem) * P, int x, int y, REAL* F, REAL* D) {
    const int k = y * P->W + x;
    REAL FO[2] = {(REAL)0, (REAL)0}, FA = (REAL)0, DO[2] = {(REAL)0, (REAL)0}, DA = (REAL)0;
    for (int s = 0; s < 4; ++s) {
        for (int c = 0; c < 2; ++c) {
            FN(reg_res) r = FN(reg_residual)(P, x, y, s, c);
            if (r.valid) {
                FO[c] += r.dOc * r.value;
                DO[c] += r.dOc * r.dOc;
                FA += r.dA * r.value;
                DA += r.dA * r.dA;
            }
            FN(reg_res) q = FN(reg_residual)(P, x - SX[s], y - SY[s], s, c);
            if (q.valid) {
                FO[c] += q.dOsc * q.value;
                DO[c] += q.dOsc * q.dOsc;
            }
        }
    }
    if (FN(fit_valid)(P, k)) {
        for (int c = 0; c < 2; ++c) {
            const REAL e = P->wf * (P->O[2 * k + c] - (REAL)P->C[2 * k + c]);
            FO[c] += P->wf * e;
            DO[c] += P->wf * P->wf;
        }
    }
    F[0] = FO[0]; F[1] = FO[1]; F[2] = FA;
    D[0] = DO[0]; D[1] = DO[1]; D[2] = DA;
}

static REAL FN(cost_px)(const FN(iw_problem) * P, int x, int y) {
    const int k = y * P->W + x;
    REAL sum = (REAL)0;
    for (int s = 0; s < 4; ++s)
        for (int c = 0; c < 2; ++c) {
            FN(reg_res) r = FN(reg_residual)(P, x, y, s, c);
            if (r.valid) sum += r.value * r.value;
        }
    if (FN(fit_valid)(P, k))
        for (int c = 0; c < 2; ++c) {
            const REAL e = P->wf * (P->O[2 * k + c] - (REAL)P->C[2 * k + c]);
            sum += e * e;
        }
    return (REAL)0.5 * sum;
}

/* ---- slab workers (backend_cpu_mt: outer dimension split, per-thread sums) ---- */
static void* FN(w_apply)(void* v) {
    FN(slab)* S = (FN(slab)*)v;
    const FN(iw_problem)* P = S->P;
    const int N = P->W * P->H;
    OACC acc = 0.0;
    for (int y = S->y0; y < S->y1; ++y)
        for (int x = 0; x < P->W; ++x) {
            const int k = y * P->W + x;
            REAL ao[2] = {(REAL)0, (REAL)0}, at = (REAL)0;
            if (!FN(excluded)(P, x, y)) {
                FN(apply_px)(P, S->p, x, y, ao, &at);
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
static REAL FN(guarded_invert)(REAL d) { const REAL s = (REAL)1 + RSQRT(d); return (REAL)1 / (s * s); }
static void* FN(w_jtf)(void* v) {
    FN(slab)* S = (FN(slab)*)v;
    const FN(iw_problem)* P = S->P;
    const int N = P->W * P->H;
    OACC acc = 0.0;
    for (int y = S->y0; y < S->y1; ++y)
        for (int x = 0; x < P->W; ++x) {
            const int k = y * P->W + x;
            REAL r[3] = {(REAL)0, (REAL)0, (REAL)0}, pre[3] = {(REAL)0, (REAL)0, (REAL)0};
            if (!FN(excluded)(P, x, y)) {
                REAL F[3], D[3];
                FN(jtf_px)(P, x, y, F, D);
                for (int c = 0; c < 3; ++c) {
                    r[c] = -F[c];
                    pre[c] = FN(guarded_invert)(S->use_pre ? D[c] : (REAL)1);
                    acc += (double)r[c] * (pre[c] * r[c]);
                }
            }
            S->out0[2 * k] = r[0]; S->out0[2 * k + 1] = r[1]; S->out0[2 * N + k] = r[2];
            S->out1[2 * k] = pre[0]; S->out1[2 * k + 1] = pre[1]; S->out1[2 * N + k] = pre[2];
        }
    S->acc = acc;
    return NULL;
}
static void* FN(w_cost)(void* v) {
    FN(slab)* S = (FN(slab)*)v;
    const FN(iw_problem)* P = S->P;
    OACC acc = 0.0;
    for (int y = S->y0; y < S->y1; ++y)
        for (int x = 0; x < P->W; ++x)
            if (!FN(excluded)(P, x, y)) acc += FN(cost_px)(P, x, y);
    S->acc = acc;
    return NULL;
}

static OACC FN(run_slabs)(const FN(iw_problem) * P, int nthreads, void* (*fn)(void*), const REAL* p,
                            REAL* o0, REAL* o1) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > P->H) nthreads = P->H;
    FN(slab)* S = (FN(slab)*)calloc(nthreads, sizeof(FN(slab)));
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
    OACC acc = 0.0;
    for (int t = 0; t < nthreads; ++t) acc += S[t].acc;   /* thread order (backend_cpu_mt.t:402-410) */
    free(S);
    free(th);
    return acc;
}

/* Full GN solve in the reference's kernel order (O and A updated in place); see
 * oracle_iw_solve in image_warping.c for the arguments. */
static void FN(iw_solve)(int W, int H, REAL* O, REAL* A, const float* U, const float* C, const float* M,
                         REAL wf, REAL wr, int nIter, int lIter, int nthreads, double* costs, double* scalars) {
    FN(iw_problem) P = {W, H, O, A, U, C, M, wf, wr};
    const int N = W * H;
    const size_t n3 = (size_t)3 * N;
    REAL* r = (REAL*)calloc(n3, sizeof(REAL));
    REAL* pre = (REAL*)calloc(n3, sizeof(REAL));
    REAL* p = (REAL*)calloc(n3, sizeof(REAL));
    REAL* Ap = (REAL*)calloc(n3, sizeof(REAL));
    REAL* d = (REAL*)calloc(n3, sizeof(REAL));
    costs[0] = FN(run_slabs)(&P, nthreads, FN(w_cost), NULL, NULL, NULL);
    for (int it = 0; it < nIter; ++it) {
        /* PCGInit1 */
        OACC alpha_num = FN(run_slabs)(&P, nthreads, FN(w_jtf), NULL, r, pre);
        for (size_t e = 0; e < n3; ++e) { d[e] = (REAL)0; p[e] = pre[e] * r[e]; }
        for (int li = 0; li < lIter; ++li) {
            /* PCGStep1 */
            OACC alpha_den = FN(run_slabs)(&P, nthreads, FN(w_apply), p, Ap, NULL);
            /* PCGStep2 (excluded elements hold r = pre = p = Ap = 0) */
            const REAL alpha = (REAL)(alpha_num / alpha_den);
            OACC beta_num = 0.0;
            for (size_t e = 0; e < n3; ++e) {
                d[e] = d[e] + alpha * p[e];
                r[e] = r[e] - alpha * Ap[e];
                const REAL z = pre[e] * r[e];
                beta_num += (double)z * r[e];
            }
            if (scalars) {
                scalars[((size_t)it * lIter + li) * 3 + 0] = alpha_num;
                scalars[((size_t)it * lIter + li) * 3 + 1] = alpha_den;
                scalars[((size_t)it * lIter + li) * 3 + 2] = beta_num;
            }
            /* PCGStep3 */
            const REAL beta = (REAL)(beta_num / alpha_num);
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
        costs[it + 1] = FN(run_slabs)(&P, nthreads, FN(w_cost), NULL, NULL, NULL);
    }
    free(r); free(pre); free(p); free(Ap); free(d);
}

/* ------------------------------------------------ generic GN / LM (solver_impl.h) ---- */
/* Vector layout [Offset.xy * N | Angle * N]; an element is active iff its pixel's Mask
 * is 0. Model cost = 1/2 sum (F + J delta)^2 over the residuals of active pixels
 * (createmodelcost, API/src/o.t:2915-2943). */
typedef struct {
    FN(iw_problem) P;
    REAL *O, *A, *prevO, *prevA;
    int nthreads;
} FN(iw_ctx);

static double FN(iwg_cost)(void* v) {
    FN(iw_ctx)* c = (FN(iw_ctx)*)v;
    return FN(run_slabs)(&c->P, c->nthreads, FN(w_cost), NULL, NULL, NULL);
}
static void FN(iwg_jtf)(void* v, REAL* r, REAL* diag) {
    FN(iw_ctx)* c = (FN(iw_ctx)*)v;
    const FN(iw_problem)* P = &c->P;
    const int N = P->W * P->H;
    for (int y = 0; y < P->H; ++y)
        for (int x = 0; x < P->W; ++x) {
            const int k = y * P->W + x;
            REAL F[3] = {(REAL)0, (REAL)0, (REAL)0}, D[3] = {(REAL)0, (REAL)0, (REAL)0};
            if (!FN(excluded)(P, x, y)) FN(jtf_px)(P, x, y, F, D);
            r[2 * k] = -F[0]; r[2 * k + 1] = -F[1]; r[2 * N + k] = -F[2];
            diag[2 * k] = D[0]; diag[2 * k + 1] = D[1]; diag[2 * N + k] = D[2];
        }
}
static double FN(iwg_apply)(void* v, const REAL* p, REAL* Ap) {
    FN(iw_ctx)* c = (FN(iw_ctx)*)v;
    return FN(run_slabs)(&c->P, c->nthreads, FN(w_apply), p, Ap, NULL);
}
static double FN(iwg_model)(void* v, const REAL* d) {
    FN(iw_ctx)* c = (FN(iw_ctx)*)v;
    const FN(iw_problem)* P = &c->P;
    const int N = P->W * P->H;
    OACC acc = 0.0;
    for (int y = 0; y < P->H; ++y)
        for (int x = 0; x < P->W; ++x) {
            if (FN(excluded)(P, x, y)) continue;
            const int k = y * P->W + x;
            REAL sum = (REAL)0;
            for (int s = 0; s < 4; ++s)
                for (int ch = 0; ch < 2; ++ch) {
                    FN(reg_res) r = FN(reg_residual)(P, x, y, s, ch);
                    if (!r.valid) continue;
                    const int t = (y + SY[s]) * P->W + (x + SX[s]);
                    const REAL e = r.value + (r.dOc * d[2 * k + ch] + r.dOsc * d[2 * t + ch] + r.dA * d[2 * N + k]);
                    sum += e * e;
                }
            if (FN(fit_valid)(P, k))
                for (int ch = 0; ch < 2; ++ch) {
                    const REAL e = P->wf * (P->O[2 * k + ch] - (REAL)P->C[2 * k + ch]) + P->wf * d[2 * k + ch];
                    sum += e * e;
                }
            acc += (REAL)0.5 * sum;
        }
    return acc;
}
static void FN(iwg_update)(void* v, const REAL* d) {
    FN(iw_ctx)* c = (FN(iw_ctx)*)v;
    const int N = c->P.W * c->P.H;
    for (int k = 0; k < N; ++k) {
        if (c->P.M[k] != 0.f) continue;
        c->O[2 * k] += d[2 * k];
        c->O[2 * k + 1] += d[2 * k + 1];
        c->A[k] += d[2 * N + k];
    }
}
static void FN(iwg_save)(void* v) {
    FN(iw_ctx)* c = (FN(iw_ctx)*)v;
    const int N = c->P.W * c->P.H;
    memcpy(c->prevO, c->O, sizeof(REAL) * 2 * N);
    memcpy(c->prevA, c->A, sizeof(REAL) * N);
}
static void FN(iwg_revert)(void* v) {
    FN(iw_ctx)* c = (FN(iw_ctx)*)v;
    const int N = c->P.W * c->P.H;
    for (int k = 0; k < N; ++k) {
        if (c->P.M[k] != 0.f) continue;
        c->O[2 * k] = c->prevO[2 * k];
        c->O[2 * k + 1] = c->prevO[2 * k + 1];
        c->A[k] = c->prevA[k];
    }
}

/* GN (lm = 0) or LM solve through the generic loop; returns completed steps. */
static int FN(iw_solve_generic)(int W, int H, REAL* O, REAL* A, const float* U, const float* C, const float* M,
                                REAL wf, REAL wr, int lm, int nIter, int lIter, int nthreads, double* costs) {
    const int N = W * H;
    FN(iw_ctx) c = {{W, H, O, A, U, C, M, wf, wr}, O, A, NULL, NULL, nthreads};
    c.prevO = (REAL*)malloc(sizeof(REAL) * 2 * N);
    c.prevA = (REAL*)malloc(sizeof(REAL) * N);
    unsigned char* act = (unsigned char*)malloc((size_t)3 * N);
    for (int k = 0; k < N; ++k) act[2 * k] = act[2 * k + 1] = act[2 * N + k] = M[k] == 0.f;
    CAT(oracle_problem_, REAL) P = {3LL * N, act, 1, &c, FN(iwg_cost), FN(iwg_jtf), FN(iwg_apply), FN(iwg_model),
                                    FN(iwg_update), FN(iwg_save), FN(iwg_revert)};
    oracle_params sp = oracle_default_params();
    sp.nIterations = nIter;
    sp.lIterations = lIter;
    const int k = SOLVE_FN(&P, lm, &sp, costs);
    free(act); free(c.prevO); free(c.prevA);
    return k;
}

#undef FN
#undef CAT
#undef CAT2
