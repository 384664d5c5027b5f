/*
 * oracle/sfs.c — CPU restatement of the reference's shape_from_shading solver.
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
#include <stdlib.h>
#include <string.h>
#include "solver.h"

typedef struct {
    int W, H;
    float* X;
    const float *D, *Im;
    const unsigned char *mR, *mC;
    float wp, ws, wg, fx, fy, ux, uy, L[9];
    /* precomputed */
    float *BI, *G00, *Gm0, *G0m, *VAL;
    float* prev;
} sfs_ctx;

static int sin_(const sfs_ctx* c, int x, int y) { return x >= 0 && x < c->W && y >= 0 && y < c->H; }
static float sget(const sfs_ctx* c, const float* im, int x, int y) {
    return sin_(c, x, y) ? im[(long long)y * c->W + x] : 0.f;
}
static float sgetu(const sfs_ctx* c, const unsigned char* im, int x, int y) {
    return sin_(c, x, y) ? (float)im[(long long)y * c->W + x] : 0.f;
}
static int DV(const sfs_ctx* c, int x, int y) { return sget(c, c->D, x, y) > 0.f; }
static int inbe(const sfs_ctx* c, int x, int y) { return x >= 1 && x < c->W - 1 && y >= 1 && y < c->H - 1; }

/* B_I(c) and its partials w.r.t. X(c), X(c-(1,0)), X(c-(0,1)) */
static void bi_eval(const sfs_ctx* c, const float* X, int x, int y, float* bi, float g[3]) {
    g[0] = g[1] = g[2] = 0.f;
    *bi = 0.f;
    if (!(inbe(c, x, y) && DV(c, x - 1, y) && DV(c, x, y) && DV(c, x, y - 1))) return;
    const float d = sget(c, X, x, y), a = sget(c, X, x - 1, y), b = sget(c, X, x, y - 1);
    const float fx = c->fx, fy = c->fy, ux = c->ux, uy = c->uy;
    const float i = (float)x, j = (float)y;
    const float nx = b * (d - a) / fy;
    const float ny = a * (d - b) / fx;
    const float nz = (nx * (ux - i) / fx) + (ny * (uy - j) / fy) - (a * b / (fx * fy));
    const float sq = nx * nx + ny * ny + nz * nz;
    const float inv = sq > 0.f ? 1.f / sqrtf(sq) : 1.f;
    const float Nx = inv * nx, Ny = inv * ny, Nz = inv * nz;
    const float* L = c->L;
    const float B = L[0] + L[1] * Ny + L[2] * Nz + L[3] * Nx + L[4] * Nx * Ny + L[5] * Ny * Nz +
                    L[6] * (-Nx * Nx - Ny * Ny + 2.f * Nz * Nz) + L[7] * Nz * Nx + L[8] * (Nx * Nx - Ny * Ny);
    const float I = sget(c, c->Im, x, y) * 0.5f + 0.25f * (sget(c, c->Im, x - 1, y) + sget(c, c->Im, x, y - 1));
    *bi = B - I;
    const float dBx = L[3] + L[4] * Ny + L[7] * Nz + 2.f * Nx * (L[8] - L[6]);
    const float dBy = L[1] + L[4] * Nx + L[5] * Nz - 2.f * Ny * (L[6] + L[8]);
    const float dBz = L[2] + L[5] * Ny + 4.f * L[6] * Nz + L[7] * Nx;
    const float dnx[3] = {b / fy, -b / fy, (d - a) / fy};
    const float dny[3] = {a / fx, (d - b) / fx, -a / fx};
    const float dab[3] = {0.f, b, a};
    for (int v = 0; v < 3; ++v) {
        const float dnz = dnx[v] * (ux - i) / fx + dny[v] * (uy - j) / fy - dab[v] / (fx * fy);
        const float dinv = sq > 0.f ? -(inv * inv * inv) * (nx * dnx[v] + ny * dny[v] + nz * dnz) : 0.f;
        const float dNx = dinv * nx + inv * dnx[v], dNy = dinv * ny + inv * dny[v], dNz = dinv * nz + inv * dnz;
        g[v] = dBx * dNx + dBy * dNy + dBz * dNz;
    }
}

static void sfs_precompute(sfs_ctx* c) {
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            float g[3];
            bi_eval(c, c->X, x, y, &c->BI[k], g);
            c->G00[k] = g[0]; c->Gm0[k] = g[1]; c->G0m[k] = g[2];
            const float xc = c->X[k];
            int v = inbe(c, x, y) && DV(c, x, y) && DV(c, x, y - 1) && DV(c, x, y + 1) && DV(c, x - 1, y) &&
                    DV(c, x + 1, y);
            const int ox[4] = {0, 0, -1, 1}, oy[4] = {-1, 1, 0, 0};
            for (int s = 0; s < 4 && v; ++s) v = fabsf(xc - sget(c, c->X, x + ox[s], y + oy[s])) < 0.01f;
            c->VAL[k] = v ? 1.f : 0.f;
        }
}

/* one residual template instance at centre (x,y): up to 3 components, up to 6 unknown
 * offsets with their partials */
typedef struct {
    int ncomp, nent;
    float val[3];
    int ox[6], oy[6];
    float d[6][3];
} res_t;

static void add_ent(res_t* r, int ox, int oy, const float* d) {
    for (int e = 0; e < r->nent; ++e)
        if (r->ox[e] == ox && r->oy[e] == oy) {
            for (int q = 0; q < r->ncomp; ++q) r->d[e][q] += d[q];
            return;
        }
    r->ox[r->nent] = ox; r->oy[r->nent] = oy;
    for (int q = 0; q < r->ncomp; ++q) r->d[r->nent][q] = d[q];
    r->nent++;
}

/* template t: 0 E_p, 1 E_g_h, 2 E_g_v, 3 E_s. Returns 0 if the instance is absent. */
static int eval_res(const sfs_ctx* c, int t, int x, int y, res_t* r) {
    memset(r, 0, sizeof(*r));
    r->ncomp = (t == 3) ? 3 : 1;
    if (!sin_(c, x, y)) return 0;
    const long long k = (long long)y * c->W + x;
    const float wp = sqrtf(c->wp), ws = sqrtf(c->ws), wg = sqrtf(c->wg);
    if (t == 0) {
        if (!DV(c, x, y)) return 0;
        r->val[0] = wp * (c->X[k] - c->D[k]);
        const float d[1] = {wp};
        add_ent(r, 0, 0, d);
        return 1;
    }
    if (t == 1 || t == 2) {
        if (!inbe(c, x, y)) return 0;
        const int sx = t == 1 ? 1 : 0, sy = t == 1 ? 0 : 1;
        const float m = t == 1 ? sgetu(c, c->mR, x, y) : sgetu(c, c->mC, x, y);
        const long long n = (long long)(y + sy) * c->W + (x + sx);
        r->val[0] = wg * (c->BI[k] - c->BI[n]) * m;
        const float e0[1] = {wg * m * c->G00[k]}, e1[1] = {wg * m * c->Gm0[k]}, e2[1] = {wg * m * c->G0m[k]};
        const float f0[1] = {-wg * m * c->G00[n]}, f1[1] = {-wg * m * c->Gm0[n]}, f2[1] = {-wg * m * c->G0m[n]};
        add_ent(r, 0, 0, e0);
        add_ent(r, -1, 0, e1);
        add_ent(r, 0, -1, e2);
        add_ent(r, sx, sy, f0);
        add_ent(r, sx - 1, sy, f1);
        add_ent(r, sx, sy - 1, f2);
        return 1;
    }
    /* E_s */
    if (c->VAL[k] != 1.f) return 0;
    const int ox[5] = {0, -1, 0, 1, 0}, oy[5] = {0, 0, -1, 0, 1};
    float px[5], py[5], xv[5];
    for (int s = 0; s < 5; ++s) {
        px[s] = ((float)(x + ox[s]) - c->ux) / c->fx;
        py[s] = ((float)(y + oy[s]) - c->uy) / c->fy;
        xv[s] = sget(c, c->X, x + ox[s], y + oy[s]);
    }
    float sx_ = 0.f, sy_ = 0.f, sz_ = 0.f;
    for (int s = 1; s < 5; ++s) { sx_ += px[s] * xv[s]; sy_ += py[s] * xv[s]; sz_ += xv[s]; }
    r->val[0] = ws * (4.f * (px[0] * xv[0]) - sx_);
    r->val[1] = ws * (4.f * (py[0] * xv[0]) - sy_);
    r->val[2] = ws * (4.f * xv[0] - sz_);
    for (int s = 0; s < 5; ++s) {
        const float co = s == 0 ? 4.f : -1.f;
        const float d[3] = {ws * co * px[s], ws * co * py[s], ws * co};
        add_ent(r, ox[s], oy[s], d);
    }
    return 1;
}

static int excl(const sfs_ctx* c, long long k) { return !(c->D[k] > 0.f); }

static double sfs_cost_fn(void* v) {
    sfs_ctx* c = (sfs_ctx*)v;
    double acc = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            if (excl(c, (long long)y * c->W + x)) continue;
            float s2 = 0.f;
            for (int t = 0; t < 4; ++t) {
                res_t r;
                if (!eval_res(c, t, x, y, &r)) continue;
                for (int q = 0; q < r.ncomp; ++q) s2 += r.val[q] * r.val[q];
            }
            acc += 0.5f * s2;
        }
    return acc;
}

static double sfs_model_fn(void* v, const float* dl) {
    sfs_ctx* c = (sfs_ctx*)v;
    double acc = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            if (excl(c, (long long)y * c->W + x)) continue;
            float s2 = 0.f;
            for (int t = 0; t < 4; ++t) {
                res_t r;
                if (!eval_res(c, t, x, y, &r)) continue;
                for (int q = 0; q < r.ncomp; ++q) {
                    float jd = 0.f;
                    for (int e = 0; e < r.nent; ++e) jd += r.d[e][q] * sget(c, dl, x + r.ox[e], y + r.oy[e]);
                    const float m = r.val[q] + jd;
                    s2 += m * m;
                }
            }
            acc += 0.5f * s2;
        }
    return acc;
}

/* the support offsets of each template (where X_k can sit relative to the centre) */
static const int NSUP[4] = {1, 5, 5, 5};
static const int SUPX[4][5] = {{0}, {0, -1, 0, 1, 1}, {0, -1, 0, 0, -1}, {0, -1, 0, 1, 0}};
static const int SUPY[4][5] = {{0}, {0, 0, -1, 0, -1}, {0, 0, -1, 1, 1}, {0, 0, -1, 0, 1}};

/* gather over the instances containing X_k: mode 0 J^T F + diag, mode 1 J^T J p */
static void gather(const sfs_ctx* c, int x, int y, const float* p, float* out0, float* out1, int mode) {
    float F = 0.f, Dg = 0.f, A = 0.f;
    for (int t = 0; t < 4; ++t)
        for (int s = 0; s < NSUP[t]; ++s) {
            const int o_x = SUPX[t][s], o_y = SUPY[t][s];
            const int cx = x - o_x, cy = y - o_y;
            res_t r;
            if (!eval_res(c, t, cx, cy, &r)) continue;
            int e = 0;
            while (e < r.nent && !(r.ox[e] == o_x && r.oy[e] == o_y)) ++e;
            if (e == r.nent) continue;
            for (int q = 0; q < r.ncomp; ++q) {
                const float dk = r.d[e][q];
                if (mode == 0) {
                    F += dk * r.val[q];
                    Dg += dk * dk;
                } else {
                    float jp = 0.f;
                    for (int u = 0; u < r.nent; ++u) jp += r.d[u][q] * sget(c, p, cx + r.ox[u], cy + r.oy[u]);
                    A += dk * jp;
                }
            }
        }
    if (mode == 0) { *out0 = F; *out1 = Dg; }
    else *out0 = A;
}

static void sfs_jtf_fn(void* v, float* r, float* diag) {
    sfs_ctx* c = (sfs_ctx*)v;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            float F = 0.f, D = 0.f;
            if (!excl(c, k)) gather(c, x, y, NULL, &F, &D, 0);
            r[k] = -F;
            diag[k] = D;
        }
}
static double sfs_apply_fn(void* v, const float* p, float* Ap) {
    sfs_ctx* c = (sfs_ctx*)v;
    double dot = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            float a = 0.f;
            if (!excl(c, k)) {
                gather(c, x, y, p, &a, NULL, 1);
                dot += (double)p[k] * a;
            }
            Ap[k] = a;
        }
    return dot;
}
static void sfs_update_fn(void* v, const float* d) {
    sfs_ctx* c = (sfs_ctx*)v;
    for (long long k = 0; k < (long long)c->W * c->H; ++k)
        if (!excl(c, k)) c->X[k] += d[k];
    sfs_precompute(c);
}
static void sfs_save_fn(void* v) {
    sfs_ctx* c = (sfs_ctx*)v;
    memcpy(c->prev, c->X, sizeof(float) * (size_t)c->W * c->H);
}
static void sfs_revert_fn(void* v) {
    sfs_ctx* c = (sfs_ctx*)v;
    for (long long k = 0; k < (long long)c->W * c->H; ++k)
        if (!excl(c, k)) c->X[k] = c->prev[k];
    sfs_precompute(c);
}

/* ------------------------------------------------------------- public API ---- */
/* prm: w_p, w_s, w_g, f_x, f_y, u_x, u_y, L_1..L_9 (16 floats, declaration order) */
static sfs_ctx make_ctx(int W, int H, float* X, const float* D, const float* Im, const unsigned char* mR,
                        const unsigned char* mC, const float* prm) {
    sfs_ctx c;
    memset(&c, 0, sizeof(c));
    c.W = W; c.H = H; c.X = X; c.D = D; c.Im = Im; c.mR = mR; c.mC = mC;
    c.wp = prm[0]; c.ws = prm[1]; c.wg = prm[2]; c.fx = prm[3]; c.fy = prm[4]; c.ux = prm[5]; c.uy = prm[6];
    for (int i = 0; i < 9; ++i) c.L[i] = prm[7 + i];
    const size_t N = (size_t)W * H;
    c.BI = calloc(N, sizeof(float)); c.G00 = calloc(N, sizeof(float)); c.Gm0 = calloc(N, sizeof(float));
    c.G0m = calloc(N, sizeof(float)); c.VAL = calloc(N, sizeof(float)); c.prev = calloc(N, sizeof(float));
    sfs_precompute(&c);
    return c;
}
static void free_ctx(sfs_ctx* c) {
    free(c->BI); free(c->G00); free(c->Gm0); free(c->G0m); free(c->VAL); free(c->prev);
}

/* precomputed arrays: out = [B_I | dB_I/dX(0,0) | dB_I/dX(-1,0) | dB_I/dX(0,-1) | valid], 5 N floats */
void oracle_sfs_precompute(int W, int H, float* X, const float* D, const float* Im, const unsigned char* mR,
                           const unsigned char* mC, const float* prm, float* out) {
    sfs_ctx c = make_ctx(W, H, X, D, Im, mR, mC, prm);
    const size_t N = (size_t)W * H;
    memcpy(out, c.BI, N * 4); memcpy(out + N, c.G00, N * 4); memcpy(out + 2 * N, c.Gm0, N * 4);
    memcpy(out + 3 * N, c.G0m, N * 4); memcpy(out + 4 * N, c.VAL, N * 4);
    free_ctx(&c);
}
double oracle_sfs_cost(int W, int H, float* X, const float* D, const float* Im, const unsigned char* mR,
                       const unsigned char* mC, const float* prm) {
    sfs_ctx c = make_ctx(W, H, X, D, Im, mR, mC, prm);
    const double v = sfs_cost_fn(&c);
    free_ctx(&c);
    return v;
}
void oracle_sfs_jtf(int W, int H, float* X, const float* D, const float* Im, const unsigned char* mR,
                    const unsigned char* mC, const float* prm, float* r, float* diag) {
    sfs_ctx c = make_ctx(W, H, X, D, Im, mR, mC, prm);
    sfs_jtf_fn(&c, r, diag);
    free_ctx(&c);
}
double oracle_sfs_apply(int W, int H, float* X, const float* D, const float* Im, const unsigned char* mR,
                        const unsigned char* mC, const float* prm, const float* p, float* Ap) {
    sfs_ctx c = make_ctx(W, H, X, D, Im, mR, mC, prm);
    const double v = sfs_apply_fn(&c, p, Ap);
    free_ctx(&c);
    return v;
}
double oracle_sfs_model_cost(int W, int H, float* X, const float* D, const float* Im, const unsigned char* mR,
                             const unsigned char* mC, const float* prm, const float* d) {
    sfs_ctx c = make_ctx(W, H, X, D, Im, mR, mC, prm);
    const double v = sfs_model_fn(&c, d);
    free_ctx(&c);
    return v;
}
int oracle_sfs_solve(int W, int H, float* X, const float* D, const float* Im, const unsigned char* mR,
                     const unsigned char* mC, const float* prm, int lm, int nIter, int lIter, double* costs) {
    sfs_ctx c = make_ctx(W, H, X, D, Im, mR, mC, prm);
    const long long n = (long long)W * H;
    unsigned char* act = malloc(n);
    for (long long k = 0; k < n; ++k) act[k] = !excl(&c, k);
    oracle_problem_float P = {n, act, 0, &c, sfs_cost_fn, sfs_jtf_fn, sfs_apply_fn, sfs_model_fn,
                              sfs_update_fn, sfs_save_fn, sfs_revert_fn};
    oracle_params sp = oracle_default_params();
    sp.nIterations = nIter;
    sp.lIterations = lIter;
    const int k = oracle_solve_f32(&P, lm, &sp, costs);
    free(act);
    free_ctx(&c);
    return k;
}
