/*
 * oracle/optical_flow_impl.h — TEST INFRASTRUCTURE ONLY (oracle/README.md).
 * PINNED to the reference's own output: its end-to-end test's CUDA final cost for the
 * dogdance example (first solve, examples/test_final_cost.py:62, 0.52119255) is
 * reproduced within 2e-7 (tests/test_reference_costs.py); also checked by finite
 * differences + the GN quadratic identity (tests/test_oracle_optical_flow.py).
 *
 * Energy examples/optical_flow/optical_flow.t: unknown X (opt_float2), knowns I,
 * I_hat, I_hat_dx, I_hat_dy (float); UsePreconditioner(false); no Exclude.
 *   e_fit(k)   = wf (I_k - S(I_hat; i + X0, j + X1))
 *   e_reg(k,s) = InBounds(k+s) ? wr (X_k - X_{k+s}) : 0      s in 4-neighbours
 * S = Image:sample (API/src/o.t:863-876): x0 = floor, x1 = ceil, lerp (1-t) v0 + t v1,
 * zero outside the image (Image:get, o.t:856-862). d e_fit / d X_c = -wf S(I_hat_d{x,y})
 * at the same point (ad.sampledimage getpartials, o.t:3270-3280).
 * Gathers follow o.t:2770-2830 / 2870-2913 / 2915-2943 / 3119-3129 literally, in REAL
 * (opt_float) arithmetic; known arrays stay float (the harness converts only the
 * unknowns, examples/shared/OptSolver.h:20-28).
 * Instantiated for REAL = float and double by oracle/optical_flow.c.
 */
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define FN(name) CAT(name, CAT(_, REAL))

typedef struct {
    int W, H;
    REAL* X;
    const float *I, *Ih, *Ihx, *Ihy;
    REAL wf, wr;
    REAL* prev;
    REAL* G;   /* sampled (I_hat_dx, I_hat_dy) at the current X, 2 per pixel */
} FN(of_ctx);

static REAL FN(of_get)(const FN(of_ctx) * c, const float* im, int x, int y) {
    return (x >= 0 && x < c->W && y >= 0 && y < c->H) ? (REAL)im[(long long)y * c->W + x] : (REAL)0;
}
static REAL FN(of_lerp)(REAL v0, REAL v1, REAL t) { return ((REAL)1 - t) * v0 + t * v1; }
static REAL FN(of_sample)(const FN(of_ctx) * c, const float* im, REAL x, REAL y) {
    const int x0 = (int)floor((double)x), x1 = (int)ceil((double)x);
    const int y0 = (int)floor((double)y), y1 = (int)ceil((double)y);
    const REAL xn = x - (REAL)x0, yn = y - (REAL)y0;
    const REAL u = FN(of_lerp)(FN(of_get)(c, im, x0, y0), FN(of_get)(c, im, x1, y0), xn);
    const REAL b = FN(of_lerp)(FN(of_get)(c, im, x0, y1), FN(of_get)(c, im, x1, y1), xn);
    return FN(of_lerp)(u, b, yn);
}
#ifndef OF_DIRS
#define OF_DIRS
static const int OFX[4] = {1, -1, 0, 0};
static const int OFY[4] = {0, 0, 1, -1};
#endif
static int FN(of_in)(const FN(of_ctx) * c, int x, int y) { return x >= 0 && x < c->W && y >= 0 && y < c->H; }

/* fit residual at pixel k and its gradient direction g = (S(I_hat_dx), S(I_hat_dy)) */
static REAL FN(of_fit)(const FN(of_ctx) * c, const REAL* X, int x, int y, REAL* gx, REAL* gy) {
    const long long k = (long long)y * c->W + x;
    const REAL sx = (REAL)x + X[2 * k], sy = (REAL)y + X[2 * k + 1];
    if (gx) { *gx = FN(of_sample)(c, c->Ihx, sx, sy); *gy = FN(of_sample)(c, c->Ihy, sx, sy); }
    return c->wf * ((REAL)c->I[k] - FN(of_sample)(c, c->Ih, sx, sy));
}

static double FN(of_cost)(void* v) {
    FN(of_ctx)* c = (FN(of_ctx)*)v;
    OACC acc = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            const REAL ef = FN(of_fit)(c, c->X, x, y, NULL, NULL);
            REAL s2 = ef * ef;
            for (int s = 0; s < 4; ++s) {
                if (!FN(of_in)(c, x + OFX[s], y + OFY[s])) continue;
                const long long t = (long long)(y + OFY[s]) * c->W + (x + OFX[s]);
                for (int ch = 0; ch < 2; ++ch) {
                    const REAL e = c->wr * (c->X[2 * k + ch] - c->X[2 * t + ch]);
                    s2 += e * e;
                }
            }
            acc += (REAL)0.5 * s2;
        }
    return acc;
}

/* r = -J^T F, diag = sum (dr/dx)^2; also caches G for the apply (the Jacobian of the
 * fit term at the linearisation point) */
static void FN(of_jtf)(void* v, REAL* r, REAL* diag) {
    FN(of_ctx)* c = (FN(of_ctx)*)v;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            REAL g[2];
            const REAL ef = FN(of_fit)(c, c->X, x, y, &g[0], &g[1]);
            c->G[2 * k] = g[0];
            c->G[2 * k + 1] = g[1];
            for (int ch = 0; ch < 2; ++ch) {
                const REAL dfit = -c->wf * g[ch];
                REAL F = dfit * ef, D = dfit * dfit;
                for (int s = 0; s < 4; ++s) {
                    const int tx = x + OFX[s], ty = y + OFY[s];
                    if (FN(of_in)(c, tx, ty)) {   /* instance centred at k */
                        const long long t = (long long)ty * c->W + tx;
                        F += c->wr * (c->wr * (c->X[2 * k + ch] - c->X[2 * t + ch]));
                        D += c->wr * c->wr;
                    }
                    const int jx = x - OFX[s], jy = y - OFY[s];
                    if (FN(of_in)(c, jx, jy)) {   /* instance centred at k - s, k is its neighbour */
                        const long long j = (long long)jy * c->W + jx;
                        F += -c->wr * (c->wr * (c->X[2 * j + ch] - c->X[2 * k + ch]));
                        D += (-c->wr) * (-c->wr);
                    }
                }
                r[2 * k + ch] = -F;
                diag[2 * k + ch] = D;
            }
        }
}

static double FN(of_apply)(void* v, const REAL* p, REAL* Ap) {
    FN(of_ctx)* c = (FN(of_ctx)*)v;
    OACC dot = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            const REAL jx0 = -c->wf * c->G[2 * k], jx1 = -c->wf * c->G[2 * k + 1];
            const REAL Jp_fit = jx0 * p[2 * k] + jx1 * p[2 * k + 1];
            for (int ch = 0; ch < 2; ++ch) {
                REAL a = (ch ? jx1 : jx0) * Jp_fit;
                for (int s = 0; s < 4; ++s) {
                    const int tx = x + OFX[s], ty = y + OFY[s];
                    if (FN(of_in)(c, tx, ty)) {
                        const long long t = (long long)ty * c->W + tx;
                        a += c->wr * (c->wr * (p[2 * k + ch] - p[2 * t + ch]));
                    }
                    const int jx = x - OFX[s], jy = y - OFY[s];
                    if (FN(of_in)(c, jx, jy)) {
                        const long long j = (long long)jy * c->W + jx;
                        a += -c->wr * (c->wr * (p[2 * j + ch] - p[2 * k + ch]));
                    }
                }
                Ap[2 * k + ch] = a;
                dot += (double)p[2 * k + ch] * a;
            }
        }
    return dot;
}

static double FN(of_model)(void* v, const REAL* d) {
    FN(of_ctx)* c = (FN(of_ctx)*)v;
    OACC acc = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            REAL gx, gy;
            const REAL ef = FN(of_fit)(c, c->X, x, y, &gx, &gy);
            const REAL em = ef + ((-c->wf * gx) * d[2 * k] + (-c->wf * gy) * d[2 * k + 1]);
            REAL s2 = em * em;
            for (int s = 0; s < 4; ++s) {
                if (!FN(of_in)(c, x + OFX[s], y + OFY[s])) continue;
                const long long t = (long long)(y + OFY[s]) * c->W + (x + OFX[s]);
                for (int ch = 0; ch < 2; ++ch) {
                    const REAL e = c->wr * (c->X[2 * k + ch] - c->X[2 * t + ch]) +
                                   (c->wr * d[2 * k + ch] + (-c->wr) * d[2 * t + ch]);
                    s2 += e * e;
                }
            }
            acc += (REAL)0.5 * s2;
        }
    return acc;
}
static void FN(of_update)(void* v, const REAL* d) {
    FN(of_ctx)* c = (FN(of_ctx)*)v;
    for (long long e = 0; e < 2LL * c->W * c->H; ++e) c->X[e] += d[e];
}
static void FN(of_save)(void* v) {
    FN(of_ctx)* c = (FN(of_ctx)*)v;
    memcpy(c->prev, c->X, sizeof(REAL) * 2 * (size_t)c->W * c->H);
}
static void FN(of_revert)(void* v) {
    FN(of_ctx)* c = (FN(of_ctx)*)v;
    memcpy(c->X, c->prev, sizeof(REAL) * 2 * (size_t)c->W * c->H);
}

static FN(of_ctx) FN(of_make)(int W, int H, REAL* X, const float* I, const float* Ih, const float* Ihx,
                              const float* Ihy, float wf, float wr) {
    FN(of_ctx) c = {W, H, X, I, Ih, Ihx, Ihy, (REAL)wf, (REAL)wr, NULL, NULL};
    c.G = (REAL*)calloc(2 * (size_t)W * H, sizeof(REAL));
    return c;
}

#undef FN
#undef CAT
#undef CAT2
