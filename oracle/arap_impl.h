/*
 * oracle/arap_impl.h — TEST INFRASTRUCTURE ONLY (oracle/README.md): the
 * arap_mesh_deformation restatement (header comment of oracle/arap.c) in opt_float =
 * REAL arithmetic (tgmath: cos / sin / sqrt at REAL's width); known arrays stay float.
 * Instantiated for REAL = float and double by oracle/arap.c.
 */
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define FN(name) CAT(name, CAT(_, REAL))

typedef struct {
    int N, E;
    REAL *O, *A;
    const float *U, *C;
    const int *v0, *v1;
    REAL wf, wr;
    REAL *prevO, *prevA;
} FN(arap_ctx);

/* R(a) and dR/da_j (row-major 3x3) */
static void FN(rot)(const REAL* a, REAL R[9], REAL dR[3][9]) {
    const REAL ca = cos(a[0]), cb = cos(a[1]), cg = cos(a[2]);
    const REAL sa = sin(a[0]), sb = sin(a[1]), sg = sin(a[2]);
    R[0] = cg * cb;  R[1] = -sg * ca + cg * sb * sa; R[2] = sg * sa + cg * sb * ca;
    R[3] = sg * cb;  R[4] = cg * ca + sg * sb * sa;  R[5] = -cg * sa + sg * sb * ca;
    R[6] = -sb;      R[7] = cb * sa;                 R[8] = cb * ca;
    if (!dR) return;
    /* d/dalpha */
    dR[0][0] = (REAL)0.; dR[0][1] = sg * sa + cg * sb * ca; dR[0][2] = sg * ca - cg * sb * sa;
    dR[0][3] = (REAL)0.; dR[0][4] = -cg * sa + sg * sb * ca; dR[0][5] = -cg * ca - sg * sb * sa;
    dR[0][6] = (REAL)0.; dR[0][7] = cb * ca; dR[0][8] = -cb * sa;
    /* d/dbeta */
    dR[1][0] = -cg * sb; dR[1][1] = cg * cb * sa; dR[1][2] = cg * cb * ca;
    dR[1][3] = -sg * sb; dR[1][4] = sg * cb * sa; dR[1][5] = sg * cb * ca;
    dR[1][6] = -cb;      dR[1][7] = -sb * sa;     dR[1][8] = -sb * ca;
    /* d/dgamma */
    dR[2][0] = -sg * cb; dR[2][1] = -cg * ca - sg * sb * sa; dR[2][2] = cg * sa - sg * sb * ca;
    dR[2][3] = cg * cb;  dR[2][4] = -sg * ca + cg * sb * sa; dR[2][5] = sg * sa + cg * sb * ca;
    dR[2][6] = (REAL)0.;      dR[2][7] = (REAL)0.;                     dR[2][8] = (REAL)0.;
}
static void FN(mv)(const REAL M[9], const REAL* v, REAL* o) {
    o[0] = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
    o[1] = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
    o[2] = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
}
static int FN(fit_valid)(const FN(arap_ctx)* c, int v) { return c->C[3 * v] >= -999999.9f; }

/* edge residual (3 comps) and the columns dR_j d (partial w.r.t. Angle_j(v0) = -wr * col_j) */
static void FN(edge_res)(const FN(arap_ctx)* c, int e, REAL r[3], REAL col[3][3]) {
    const int a = c->v0[e], b = c->v1[e];
    REAL R[9], dR[3][9], d[3], Rd[3];
    FN(rot)(&c->A[3 * a], R, col ? dR : NULL);
    for (int k = 0; k < 3; ++k) d[k] = c->U[3 * a + k] - c->U[3 * b + k];
    FN(mv)(R, d, Rd);
    for (int k = 0; k < 3; ++k) r[k] = c->wr * ((c->O[3 * a + k] - c->O[3 * b + k]) - Rd[k]);
    if (col)
        for (int j = 0; j < 3; ++j) FN(mv)(dR[j], d, col[j]);
}

static double FN(arap_cost_fn)(void* v) {
    FN(arap_ctx)* c = (FN(arap_ctx)*)v;
    OACC acc = 0.0;
    for (int i = 0; i < c->N; ++i) {
        if (!FN(fit_valid)(c, i)) continue;
        REAL s = (REAL)0.;
        for (int k = 0; k < 3; ++k) {
            const REAL e = c->wf * (c->O[3 * i + k] - c->C[3 * i + k]);
            s += e * e;
        }
        acc += (REAL)0.5 * s;
    }
    for (int e = 0; e < c->E; ++e) {
        REAL r[3];
        FN(edge_res)(c, e, r, NULL);
        acc += (REAL)0.5 * (r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    }
    return acc;
}

static void FN(arap_jtf_fn)(void* v, REAL* r, REAL* diag) {
    FN(arap_ctx)* c = (FN(arap_ctx)*)v;
    const int N = c->N;
    REAL* rO = r; REAL* rA = r + 3 * N;
    REAL* dO = diag; REAL* dA = diag + 3 * N;
    memset(r, 0, sizeof(REAL) * 6 * N);
    memset(diag, 0, sizeof(REAL) * 6 * N);
    for (int i = 0; i < N; ++i)   /* centred fit (PCGInit1) */
        if (FN(fit_valid)(c, i))
            for (int k = 0; k < 3; ++k) {
                const REAL e = c->wf * (c->O[3 * i + k] - c->C[3 * i + k]);
                rO[3 * i + k] = -(c->wf * e);
                dO[3 * i + k] = c->wf * c->wf;
            }
    for (int e = 0; e < c->E; ++e) {   /* graph scatter (PCGInit1_Graph) */
        const int a = c->v0[e], b = c->v1[e];
        REAL res[3], col[3][3];
        FN(edge_res)(c, e, res, col);
        for (int k = 0; k < 3; ++k) {
            rO[3 * a + k] += -(REAL)1. * (c->wr * res[k]);
            dO[3 * a + k] += c->wr * c->wr;
            rO[3 * b + k] += -(REAL)1. * (-c->wr * res[k]);
            dO[3 * b + k] += (-c->wr) * (-c->wr);
        }
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) {
                const REAL pj = -c->wr * col[j][k];
                rA[3 * a + j] += -(REAL)1. * (pj * res[k]);
                dA[3 * a + j] += pj * pj;
            }
    }
}

static double FN(arap_apply_fn)(void* v, const REAL* p, REAL* Ap) {
    FN(arap_ctx)* c = (FN(arap_ctx)*)v;
    const int N = c->N;
    const REAL* pO = p; const REAL* pA = p + 3 * N;
    REAL* aO = Ap; REAL* aA = Ap + 3 * N;
    memset(Ap, 0, sizeof(REAL) * 6 * N);
    OACC dot = 0.0;
    for (int i = 0; i < N; ++i)   /* centred fit (PCGStep1) */
        if (FN(fit_valid)(c, i))
            for (int k = 0; k < 3; ++k) {
                aO[3 * i + k] = c->wf * (c->wf * pO[3 * i + k]);
                dot += (double)pO[3 * i + k] * aO[3 * i + k];
            }
    for (int e = 0; e < c->E; ++e) {   /* graph scatter (PCGStep1_Graph) */
        const int a = c->v0[e], b = c->v1[e];
        REAL res[3], col[3][3];
        FN(edge_res)(c, e, res, col);
        REAL gdot = (REAL)0.;
        for (int k = 0; k < 3; ++k) {
            REAL jp = c->wr * pO[3 * a + k] + (-c->wr) * pO[3 * b + k];
            for (int j = 0; j < 3; ++j) jp += (-c->wr * col[j][k]) * pA[3 * a + j];
            aO[3 * a + k] += c->wr * jp;
            aO[3 * b + k] += -c->wr * jp;
            for (int j = 0; j < 3; ++j) aA[3 * a + j] += (-c->wr * col[j][k]) * jp;
            gdot += jp * jp;
        }
        dot += gdot;
    }
    return dot;
}

static double FN(arap_model_fn)(void* v, const REAL* d) {
    FN(arap_ctx)* c = (FN(arap_ctx)*)v;
    const int N = c->N;
    const REAL* dO = d; const REAL* dA = d + 3 * N;
    OACC acc = 0.0;
    for (int i = 0; i < N; ++i) {
        if (!FN(fit_valid)(c, i)) continue;
        REAL s = (REAL)0.;
        for (int k = 0; k < 3; ++k) {
            const REAL e = c->wf * (c->O[3 * i + k] - c->C[3 * i + k]) + c->wf * dO[3 * i + k];
            s += e * e;
        }
        acc += (REAL)0.5 * s;
    }
    for (int e = 0; e < c->E; ++e) {
        const int a = c->v0[e], b = c->v1[e];
        REAL res[3], col[3][3];
        FN(edge_res)(c, e, res, col);
        REAL s = (REAL)0.;
        for (int k = 0; k < 3; ++k) {
            REAL jd = c->wr * dO[3 * a + k] + (-c->wr) * dO[3 * b + k];
            for (int j = 0; j < 3; ++j) jd += (-c->wr * col[j][k]) * dA[3 * a + j];
            const REAL m = res[k] + jd;
            s += m * m;
        }
        acc += (REAL)0.5 * s;
    }
    return acc;
}
static void FN(arap_update_fn)(void* v, const REAL* d) {
    FN(arap_ctx)* c = (FN(arap_ctx)*)v;
    for (int i = 0; i < 3 * c->N; ++i) { c->O[i] += d[i]; c->A[i] += d[3 * c->N + i]; }
}
static void FN(arap_save_fn)(void* v) {
    FN(arap_ctx)* c = (FN(arap_ctx)*)v;
    memcpy(c->prevO, c->O, sizeof(REAL) * 3 * c->N);
    memcpy(c->prevA, c->A, sizeof(REAL) * 3 * c->N);
}
static void FN(arap_revert_fn)(void* v) {
    FN(arap_ctx)* c = (FN(arap_ctx)*)v;
    memcpy(c->O, c->prevO, sizeof(REAL) * 3 * c->N);
    memcpy(c->A, c->prevA, sizeof(REAL) * 3 * c->N);
}


#undef FN
#undef CAT
#undef CAT2
