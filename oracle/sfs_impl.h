/*
 * oracle/sfs_impl.h — TEST INFRASTRUCTURE ONLY (oracle/README.md): the shape_from_shading
 * restatement (header comment of oracle/sfs.c) in opt_float = REAL arithmetic; known
 * arrays (D_i, Im, edge masks) stay float, as the harness passes them
 * (examples/shared/OptSolver.h:20-28). Instantiated for REAL = float and double by
 * oracle/sfs.c. Constants are the energy's Lua numbers cast to opt_float; the three
 * weights are square-rooted in float, as the runtime passes float parameters.
 */
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define FN(name) CAT(name, CAT(_, REAL))

typedef struct {
    int W, H;
    REAL* X;
    const float *D, *Im;
    const unsigned char *mR, *mC;
    REAL wp, ws, wg, fx, fy, ux, uy, L[9];
    /* precomputed */
    REAL *BI, *G00, *Gm0, *G0m, *VAL;
    REAL* prev;
    int nthreads;   /* row slabs over pthreads (backend_cpu_mt.t:716-737); 0 or 1: one thread */
} FN(sfs_ctx);

static int FN(sin_)(const FN(sfs_ctx) * c, int x, int y) { return x >= 0 && x < c->W && y >= 0 && y < c->H; }
/* unknown-precision arrays (X, delta, p) and float known arrays (D_i, Im) */
static REAL FN(sget)(const FN(sfs_ctx) * c, const REAL* im, int x, int y) {
    return FN(sin_)(c, x, y) ? im[(long long)y * c->W + x] : (REAL)0;
}
static REAL FN(sgetk)(const FN(sfs_ctx) * c, const float* im, int x, int y) {
    return FN(sin_)(c, x, y) ? (REAL)im[(long long)y * c->W + x] : (REAL)0;
}
static REAL FN(sgetu)(const FN(sfs_ctx) * c, const unsigned char* im, int x, int y) {
    return FN(sin_)(c, x, y) ? (REAL)im[(long long)y * c->W + x] : (REAL)0;
}
static int FN(DV)(const FN(sfs_ctx) * c, int x, int y) { return FN(sgetk)(c, c->D, x, y) > (REAL)0; }
static int FN(inbe)(const FN(sfs_ctx) * c, int x, int y) { return x >= 1 && x < c->W - 1 && y >= 1 && y < c->H - 1; }

/* B_I(c) and its partials w.r.t. X(c), X(c-(1,0)), X(c-(0,1)) */
static void FN(bi_eval)(const FN(sfs_ctx)* c, const REAL* X, int x, int y, REAL* bi, REAL g[3]) {
    g[0] = g[1] = g[2] = (REAL)0.;
    *bi = (REAL)0.;
    if (!(FN(inbe)(c, x, y) && FN(DV)(c, x - 1, y) && FN(DV)(c, x, y) && FN(DV)(c, x, y - 1))) return;
    const REAL d = FN(sget)(c, X, x, y), a = FN(sget)(c, X, x - 1, y), b = FN(sget)(c, X, x, y - 1);
    const REAL fx = c->fx, fy = c->fy, ux = c->ux, uy = c->uy;
    const REAL i = (REAL)x, j = (REAL)y;
    const REAL nx = b * (d - a) / fy;
    const REAL ny = a * (d - b) / fx;
    const REAL nz = (nx * (ux - i) / fx) + (ny * (uy - j) / fy) - (a * b / (fx * fy));
    const REAL sq = nx * nx + ny * ny + nz * nz;
    const REAL inv = sq > (REAL)0. ? (REAL)1. / (REAL)sqrt((double)sq) : (REAL)1.;
    const REAL Nx = inv * nx, Ny = inv * ny, Nz = inv * nz;
    const REAL* L = c->L;
    const REAL B = L[0] + L[1] * Ny + L[2] * Nz + L[3] * Nx + L[4] * Nx * Ny + L[5] * Ny * Nz +
                    L[6] * (-Nx * Nx - Ny * Ny + (REAL)2. * Nz * Nz) + L[7] * Nz * Nx + L[8] * (Nx * Nx - Ny * Ny);
    const REAL I = FN(sgetk)(c, c->Im, x, y) * (REAL)0.5 + (REAL)0.25 * (FN(sgetk)(c, c->Im, x - 1, y) + FN(sgetk)(c, c->Im, x, y - 1));
    *bi = B - I;
    const REAL dBx = L[3] + L[4] * Ny + L[7] * Nz + (REAL)2. * Nx * (L[8] - L[6]);
    const REAL dBy = L[1] + L[4] * Nx + L[5] * Nz - (REAL)2. * Ny * (L[6] + L[8]);
    const REAL dBz = L[2] + L[5] * Ny + (REAL)4. * L[6] * Nz + L[7] * Nx;
    const REAL dnx[3] = {b / fy, -b / fy, (d - a) / fy};
    const REAL dny[3] = {a / fx, (d - b) / fx, -a / fx};
    const REAL dab[3] = {(REAL)0., b, a};
    for (int v = 0; v < 3; ++v) {
        const REAL dnz = dnx[v] * (ux - i) / fx + dny[v] * (uy - j) / fy - dab[v] / (fx * fy);
        const REAL dinv = sq > (REAL)0. ? -(inv * inv * inv) * (nx * dnx[v] + ny * dny[v] + nz * dnz) : (REAL)0.;
        const REAL dNx = dinv * nx + inv * dnx[v], dNy = dinv * ny + inv * dny[v], dNz = dinv * nz + inv * dnz;
        g[v] = dBx * dNx + dBy * dNy + dBz * dNz;
    }
}

static void FN(pre_rows)(FN(sfs_ctx)* c, int y0, int y1) {
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            REAL g[3];
            FN(bi_eval)(c, c->X, x, y, &c->BI[k], g);
            c->G00[k] = g[0]; c->Gm0[k] = g[1]; c->G0m[k] = g[2];
            const REAL xc = c->X[k];
            int v = FN(inbe)(c, x, y) && FN(DV)(c, x, y) && FN(DV)(c, x, y - 1) && FN(DV)(c, x, y + 1) && FN(DV)(c, x - 1, y) &&
                    FN(DV)(c, x + 1, y);
            const int ox[4] = {0, 0, -1, 1}, oy[4] = {-1, 1, 0, 0};
            for (int s = 0; s < 4 && v; ++s) v = fabs(xc - FN(sget)(c, c->X, x + ox[s], y + oy[s])) < (REAL)0.01;
            c->VAL[k] = v ? (REAL)1. : (REAL)0.;
        }
}

/* one residual template instance at centre (x,y): up to 3 components, up to 6 unknown
 * offsets with their partials */
typedef struct {
    int ncomp, nent;
    REAL val[3];
    int ox[6], oy[6];
    REAL d[6][3];
} FN(res_t);

static void FN(add_ent)(FN(res_t)* r, int ox, int oy, const REAL* d) {
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
static int FN(eval_res)(const FN(sfs_ctx)* c, int t, int x, int y, FN(res_t)* r) {
    memset(r, 0, sizeof(*r));
    r->ncomp = (t == 3) ? 3 : 1;
    if (!FN(sin_)(c, x, y)) return 0;
    const long long k = (long long)y * c->W + x;
    const REAL wp = (REAL)sqrtf((float)c->wp), ws = (REAL)sqrtf((float)c->ws), wg = (REAL)sqrtf((float)c->wg);
    if (t == 0) {
        if (!FN(DV)(c, x, y)) return 0;
        r->val[0] = wp * (c->X[k] - c->D[k]);
        const REAL d[1] = {wp};
        FN(add_ent)(r, 0, 0, d);
        return 1;
    }
    if (t == 1 || t == 2) {
        if (!FN(inbe)(c, x, y)) return 0;
        const int sx = t == 1 ? 1 : 0, sy = t == 1 ? 0 : 1;
        const REAL m = t == 1 ? FN(sgetu)(c, c->mR, x, y) : FN(sgetu)(c, c->mC, x, y);
        const long long n = (long long)(y + sy) * c->W + (x + sx);
        r->val[0] = wg * (c->BI[k] - c->BI[n]) * m;
        const REAL e0[1] = {wg * m * c->G00[k]}, e1[1] = {wg * m * c->Gm0[k]}, e2[1] = {wg * m * c->G0m[k]};
        const REAL f0[1] = {-wg * m * c->G00[n]}, f1[1] = {-wg * m * c->Gm0[n]}, f2[1] = {-wg * m * c->G0m[n]};
        FN(add_ent)(r, 0, 0, e0);
        FN(add_ent)(r, -1, 0, e1);
        FN(add_ent)(r, 0, -1, e2);
        FN(add_ent)(r, sx, sy, f0);
        FN(add_ent)(r, sx - 1, sy, f1);
        FN(add_ent)(r, sx, sy - 1, f2);
        return 1;
    }
    /* E_s */
    if (c->VAL[k] != (REAL)1.) return 0;
    const int ox[5] = {0, -1, 0, 1, 0}, oy[5] = {0, 0, -1, 0, 1};
    REAL px[5], py[5], xv[5];
    for (int s = 0; s < 5; ++s) {
        px[s] = ((REAL)(x + ox[s]) - c->ux) / c->fx;
        py[s] = ((REAL)(y + oy[s]) - c->uy) / c->fy;
        xv[s] = FN(sget)(c, c->X, x + ox[s], y + oy[s]);
    }
    REAL sx_ = (REAL)0., sy_ = (REAL)0., sz_ = (REAL)0.;
    for (int s = 1; s < 5; ++s) { sx_ += px[s] * xv[s]; sy_ += py[s] * xv[s]; sz_ += xv[s]; }
    r->val[0] = ws * ((REAL)4. * (px[0] * xv[0]) - sx_);
    r->val[1] = ws * ((REAL)4. * (py[0] * xv[0]) - sy_);
    r->val[2] = ws * ((REAL)4. * xv[0] - sz_);
    for (int s = 0; s < 5; ++s) {
        const REAL co = s == 0 ? (REAL)4. : -(REAL)1.;
        const REAL d[3] = {ws * co * px[s], ws * co * py[s], ws * co};
        FN(add_ent)(r, ox[s], oy[s], d);
    }
    return 1;
}

static int FN(excl)(const FN(sfs_ctx)* c, long long k) { return !(c->D[k] > (REAL)0.); }

static double FN(cost_rows)(FN(sfs_ctx)* c, int y0, int y1) {
    OACC acc = 0.0;
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < c->W; ++x) {
            if (FN(excl)(c, (long long)y * c->W + x)) continue;
            REAL s2 = (REAL)0.;
            for (int t = 0; t < 4; ++t) {
                FN(res_t) r;
                if (!FN(eval_res)(c, t, x, y, &r)) continue;
                for (int q = 0; q < r.ncomp; ++q) s2 += r.val[q] * r.val[q];
            }
            acc += (REAL)0.5 * s2;
        }
    return acc;
}

static double FN(model_rows)(FN(sfs_ctx)* c, const REAL* dl, int y0, int y1) {
    OACC acc = 0.0;
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < c->W; ++x) {
            if (FN(excl)(c, (long long)y * c->W + x)) continue;
            REAL s2 = (REAL)0.;
            for (int t = 0; t < 4; ++t) {
                FN(res_t) r;
                if (!FN(eval_res)(c, t, x, y, &r)) continue;
                for (int q = 0; q < r.ncomp; ++q) {
                    REAL jd = (REAL)0.;
                    for (int e = 0; e < r.nent; ++e) jd += r.d[e][q] * FN(sget)(c, dl, x + r.ox[e], y + r.oy[e]);
                    const REAL m = r.val[q] + jd;
                    s2 += m * m;
                }
            }
            acc += (REAL)0.5 * s2;
        }
    return acc;
}

/* the support offsets of each template (where X_k can sit relative to the centre) */
#ifndef SFS_SUPPORT
#define SFS_SUPPORT
static const int NSUP[4] = {1, 5, 5, 5};
static const int SUPX[4][5] = {{0}, {0, -1, 0, 1, 1}, {0, -1, 0, 0, -1}, {0, -1, 0, 1, 0}};
static const int SUPY[4][5] = {{0}, {0, 0, -1, 0, -1}, {0, 0, -1, 1, 1}, {0, 0, -1, 0, 1}};
#endif

/* FN(gather) over the instances containing X_k: mode 0 J^T F + diag, mode 1 J^T J p */
static void FN(gather)(const FN(sfs_ctx)* c, int x, int y, const REAL* p, REAL* out0, REAL* out1, int mode) {
    REAL F = (REAL)0., Dg = (REAL)0., A = (REAL)0.;
    for (int t = 0; t < 4; ++t)
        for (int s = 0; s < NSUP[t]; ++s) {
            const int o_x = SUPX[t][s], o_y = SUPY[t][s];
            const int cx = x - o_x, cy = y - o_y;
            FN(res_t) r;
            if (!FN(eval_res)(c, t, cx, cy, &r)) continue;
            int e = 0;
            while (e < r.nent && !(r.ox[e] == o_x && r.oy[e] == o_y)) ++e;
            if (e == r.nent) continue;
            for (int q = 0; q < r.ncomp; ++q) {
                const REAL dk = r.d[e][q];
                if (mode == 0) {
                    F += dk * r.val[q];
                    Dg += dk * dk;
                } else {
                    REAL jp = (REAL)0.;
                    for (int u = 0; u < r.nent; ++u) jp += r.d[u][q] * FN(sget)(c, p, cx + r.ox[u], cy + r.oy[u]);
                    A += dk * jp;
                }
            }
        }
    if (mode == 0) { *out0 = F; *out1 = Dg; }
    else *out0 = A;
}

static void FN(jtf_rows)(FN(sfs_ctx)* c, REAL* r, REAL* diag, int y0, int y1) {
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            REAL F = (REAL)0., D = (REAL)0.;
            if (!FN(excl)(c, k)) FN(gather)(c, x, y, NULL, &F, &D, 0);
            r[k] = -F;
            diag[k] = D;
        }
}
static double FN(apply_rows)(FN(sfs_ctx)* c, const REAL* p, REAL* Ap, int y0, int y1) {
    OACC dot = 0.0;
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < c->W; ++x) {
            const long long k = (long long)y * c->W + x;
            REAL a = (REAL)0.;
            if (!FN(excl)(c, k)) {
                FN(gather)(c, x, y, p, &a, NULL, 1);
                dot += (double)p[k] * a;
            }
            Ap[k] = a;
        }
    return dot;
}
/* ---- row slabs over threads, per-thread partial sums added in thread order
 * (backend_cpu_mt.t:350-414, 716-737); one thread is the whole image in row order ---- */
typedef struct {
    FN(sfs_ctx) * c;
    int op, y0, y1;
    const REAL* in;
    REAL *o0, *o1;
    OACC acc;
} FN(sjob);
static void* FN(sjob_run)(void* v) {
    FN(sjob)* j = (FN(sjob)*)v;
    switch (j->op) {
        case 0: FN(pre_rows)(j->c, j->y0, j->y1); break;
        case 1: j->acc = FN(cost_rows)(j->c, j->y0, j->y1); break;
        case 2: j->acc = FN(model_rows)(j->c, j->in, j->y0, j->y1); break;
        case 3: FN(jtf_rows)(j->c, j->o0, j->o1, j->y0, j->y1); break;
        default: j->acc = FN(apply_rows)(j->c, j->in, j->o0, j->y0, j->y1); break;
    }
    return NULL;
}
static double FN(spar)(FN(sfs_ctx)* c, int op, const REAL* in, REAL* o0, REAL* o1) {
    int nt = c->nthreads < 1 ? 1 : c->nthreads;
    if (nt > c->H) nt = c->H;
    FN(sjob)* J = (FN(sjob)*)calloc(nt, sizeof(FN(sjob)));
    pthread_t* th = (pthread_t*)calloc(nt, sizeof(pthread_t));
    for (int t = 0; t < nt; ++t) {
        J[t].c = c; J[t].op = op; J[t].in = in; J[t].o0 = o0; J[t].o1 = o1;
        J[t].y0 = t * (c->H / nt);
        J[t].y1 = t == nt - 1 ? c->H : (t + 1) * (c->H / nt);
    }
    if (nt == 1) FN(sjob_run)(&J[0]);
    else {
        for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, FN(sjob_run), &J[t]);
        for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
    }
    OACC acc = 0.0;
    for (int t = 0; t < nt; ++t) acc += J[t].acc;
    free(J);
    free(th);
    return acc;
}
static void FN(sfs_precompute)(FN(sfs_ctx)* c) { FN(spar)(c, 0, NULL, NULL, NULL); }
static double FN(sfs_cost_fn)(void* v) { return FN(spar)((FN(sfs_ctx)*)v, 1, NULL, NULL, NULL); }
static double FN(sfs_model_fn)(void* v, const REAL* dl) { return FN(spar)((FN(sfs_ctx)*)v, 2, dl, NULL, NULL); }
static void FN(sfs_jtf_fn)(void* v, REAL* r, REAL* diag) { FN(spar)((FN(sfs_ctx)*)v, 3, NULL, r, diag); }
static double FN(sfs_apply_fn)(void* v, const REAL* p, REAL* Ap) { return FN(spar)((FN(sfs_ctx)*)v, 4, p, Ap, NULL); }

static void FN(sfs_update_fn)(void* v, const REAL* d) {
    FN(sfs_ctx)* c = (FN(sfs_ctx)*)v;
    for (long long k = 0; k < (long long)c->W * c->H; ++k)
        if (!FN(excl)(c, k)) c->X[k] += d[k];
    FN(sfs_precompute)(c);
}
static void FN(sfs_save_fn)(void* v) {
    FN(sfs_ctx)* c = (FN(sfs_ctx)*)v;
    memcpy(c->prev, c->X, sizeof(REAL) * (size_t)c->W * c->H);
}
static void FN(sfs_revert_fn)(void* v) {
    FN(sfs_ctx)* c = (FN(sfs_ctx)*)v;
    for (long long k = 0; k < (long long)c->W * c->H; ++k)
        if (!FN(excl)(c, k)) c->X[k] = c->prev[k];
    FN(sfs_precompute)(c);
}

#undef FN
#undef CAT
#undef CAT2
