/*
 * oracle/pie_impl.h — TEST INFRASTRUCTURE ONLY (oracle/README.md): the
 * poisson_image_editing restatement (header comment of oracle/poisson.c) in
 * opt_float = REAL arithmetic, instantiated for float and double by oracle/poisson.c.
 * doublePrecision (API/release/include/Opt.h:11-14): the unknown X and the solver
 * vectors in double; the known arrays T and M stay float, so T_k - T_{k+s} is a float
 * subtraction promoted afterwards (the Terra operation on the loaded values,
 * API/src/o.t:2418-2470).
 */
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define FN(name) CAT(name, CAT(_, REAL))

typedef struct {
    int W, H;
    REAL* X;           /* 4 per pixel, updated in place */
    const float* T;
    const float* M;
    REAL* prev;
} FN(pie_ctx);

static int FN(pin)(const FN(pie_ctx)* c, int x, int y) { return x >= 0 && x < c->W && y >= 0 && y < c->H; }
static int FN(pact)(const FN(pie_ctx)* c, int k) { return c->M[k] == 0.f; }
/* residual channel ch centred at (x,y) toward s; valid if both in bounds */
static REAL FN(pres)(const FN(pie_ctx)* c, const REAL* X, int x, int y, int s, int ch) {
    const int k = y * c->W + x, j = (y + PY[s]) * c->W + (x + PX[s]);
    return (X[4 * k + ch] - X[4 * j + ch]) - (c->T[4 * k + ch] - c->T[4 * j + ch]);
}

static double FN(pie_cost_fn)(void* v) {
    FN(pie_ctx)* c = (FN(pie_ctx)*)v;
    OACC acc = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            if (!FN(pact)(c, y * c->W + x)) continue;
            REAL s2 = (REAL)0;
            for (int s = 0; s < 4; ++s) {
                if (!FN(pin)(c, x + PX[s], y + PY[s])) continue;
                for (int ch = 0; ch < 4; ++ch) { const REAL e = FN(pres)(c, c->X, x, y, s, ch); s2 += e * e; }
            }
            acc += (REAL)0.5 * s2;
        }
    return acc;
}

static void FN(pie_jtf_fn)(void* v, REAL* r, REAL* diag) {
    FN(pie_ctx)* c = (FN(pie_ctx)*)v;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const int k = y * c->W + x;
            for (int ch = 0; ch < 4; ++ch) {
                REAL F = (REAL)0, D = (REAL)0;
                if (FN(pact)(c, k)) {
                    for (int s = 0; s < 4; ++s) {
                        if (FN(pin)(c, x + PX[s], y + PY[s])) { F += FN(pres)(c, c->X, x, y, s, ch); D += (REAL)1; }
                        if (FN(pin)(c, x - PX[s], y - PY[s])) { F += -(REAL)1 * FN(pres)(c, c->X, x - PX[s], y - PY[s], s, ch); D += (REAL)1; }
                    }
                }
                r[4 * k + ch] = -F;
                diag[4 * k + ch] = D;
            }
        }
}

static double FN(pie_apply_fn)(void* v, const REAL* p, REAL* Ap) {
    FN(pie_ctx)* c = (FN(pie_ctx)*)v;
    OACC dot = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const int k = y * c->W + x;
            for (int ch = 0; ch < 4; ++ch) {
                REAL a = (REAL)0;
                if (FN(pact)(c, k)) {
                    for (int s = 0; s < 4; ++s) {
                        const int tx = x + PX[s], ty = y + PY[s], jx = x - PX[s], jy = y - PY[s];
                        if (FN(pin)(c, tx, ty)) {
                            const int t = ty * c->W + tx;
                            const REAL pt = FN(pact)(c, t) ? p[4 * t + ch] : (REAL)0;
                            a += (REAL)1 * (p[4 * k + ch] - pt);
                        }
                        if (FN(pin)(c, jx, jy)) {
                            const int j = jy * c->W + jx;
                            const REAL pj = FN(pact)(c, j) ? p[4 * j + ch] : (REAL)0;
                            a += -(REAL)1 * (pj - p[4 * k + ch]);
                        }
                    }
                    dot += (double)p[4 * k + ch] * a;
                }
                Ap[4 * k + ch] = a;
            }
        }
    return dot;
}

static double FN(pie_model_fn)(void* v, const REAL* d) {
    FN(pie_ctx)* c = (FN(pie_ctx)*)v;
    OACC acc = 0.0;
    for (int y = 0; y < c->H; ++y)
        for (int x = 0; x < c->W; ++x) {
            const int k = y * c->W + x;
            if (!FN(pact)(c, k)) continue;
            REAL s2 = (REAL)0;
            for (int s = 0; s < 4; ++s) {
                const int tx = x + PX[s], ty = y + PY[s];
                if (!FN(pin)(c, tx, ty)) continue;
                const int t = ty * c->W + tx;
                for (int ch = 0; ch < 4; ++ch) {
                    const REAL dt = FN(pact)(c, t) ? d[4 * t + ch] : (REAL)0;
                    const REAL e = FN(pres)(c, c->X, x, y, s, ch) + (d[4 * k + ch] - dt);
                    s2 += e * e;
                }
            }
            acc += (REAL)0.5 * s2;
        }
    return acc;
}
static void FN(pie_update_fn)(void* v, const REAL* d) {
    FN(pie_ctx)* c = (FN(pie_ctx)*)v;
    for (int k = 0; k < c->W * c->H; ++k)
        if (FN(pact)(c, k)) for (int ch = 0; ch < 4; ++ch) c->X[4 * k + ch] += d[4 * k + ch];
}
static void FN(pie_save_fn)(void* v) {
    FN(pie_ctx)* c = (FN(pie_ctx)*)v;
    memcpy(c->prev, c->X, sizeof(REAL) * 4 * c->W * c->H);
}
static void FN(pie_revert_fn)(void* v) {
    FN(pie_ctx)* c = (FN(pie_ctx)*)v;
    for (int k = 0; k < c->W * c->H; ++k)
        if (FN(pact)(c, k)) for (int ch = 0; ch < 4; ++ch) c->X[4 * k + ch] = c->prev[4 * k + ch];
}


#undef FN
#undef CAT
#undef CAT2
