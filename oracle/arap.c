/*
 * oracle/arap.c — CPU restatement of the reference's arap_mesh_deformation solver.
 * TEST INFRASTRUCTURE ONLY (oracle/README.md). PINNED to the reference's own output:
 * its end-to-end test's CUDA final cost for the small_armadillo example
 * (examples/test_final_cost.py:55-66, 7183.464843) is reproduced within 1.2e-7
 * (tests/test_reference_costs.py); also checked against an independent float64 numpy
 * restatement with finite differences (tests/test_oracle_arap.py).
 *
 * Energy examples/arap_mesh_deformation/arap_mesh_deformation.t:
 *   unknowns Offset, Angle (float3 per vertex); knowns UrShape, Constraints (float3);
 *   graph G (edges v0 -> v1, int32); UsePreconditioner(true)
 *   e_fit(v) = Constraints(v).x >= -999999.9 ? w_fit (Offset(v) - Constraints(v)) : 0
 *   e_reg(e) = w_reg ((Offset(v0) - Offset(v1)) - Rotate3D(Angle(v0), UrShape(v0) - UrShape(v1)))
 * Rotate3D / Matrix3x3Mul: API/src/lib.t:46-98.
 * The fit term is a centred function over vertices (PCGInit1 / PCGStep1 / computeCost,
 * solverGPUGaussNewton.t:521-632, 971-997); the regulariser a graph function whose
 * J^T F, diag, J^T J p and cost are scattered per edge (createjtfgraph o.t:2969-2994,
 * createjtjgraph o.t:2833-2867, PCGInit1_Graph / PCGInit1_Finish / PCGStep1_Graph
 * solverGPUGaussNewton.t:570-602, 1188-1233). Here the edge scatters run sequentially
 * in edge order (the reference's float atomics have no fixed order).
 * Vector layout [Offset.xyz * N | Angle.xyz * N].
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "solver.h"

typedef struct {
    int N, E;
    float *O, *A;
    const float *U, *C;
    const int *v0, *v1;
    float wf, wr;
    float *prevO, *prevA;
} arap_ctx;

/* R(a) and dR/da_j (row-major 3x3) */
static void rot(const float* a, float R[9], float dR[3][9]) {
    const float ca = cosf(a[0]), cb = cosf(a[1]), cg = cosf(a[2]);
    const float sa = sinf(a[0]), sb = sinf(a[1]), sg = sinf(a[2]);
    R[0] = cg * cb;  R[1] = -sg * ca + cg * sb * sa; R[2] = sg * sa + cg * sb * ca;
    R[3] = sg * cb;  R[4] = cg * ca + sg * sb * sa;  R[5] = -cg * sa + sg * sb * ca;
    R[6] = -sb;      R[7] = cb * sa;                 R[8] = cb * ca;
    if (!dR) return;
    /* d/dalpha */
    dR[0][0] = 0.f; dR[0][1] = sg * sa + cg * sb * ca; dR[0][2] = sg * ca - cg * sb * sa;
    dR[0][3] = 0.f; dR[0][4] = -cg * sa + sg * sb * ca; dR[0][5] = -cg * ca - sg * sb * sa;
    dR[0][6] = 0.f; dR[0][7] = cb * ca; dR[0][8] = -cb * sa;
    /* d/dbeta */
    dR[1][0] = -cg * sb; dR[1][1] = cg * cb * sa; dR[1][2] = cg * cb * ca;
    dR[1][3] = -sg * sb; dR[1][4] = sg * cb * sa; dR[1][5] = sg * cb * ca;
    dR[1][6] = -cb;      dR[1][7] = -sb * sa;     dR[1][8] = -sb * ca;
    /* d/dgamma */
    dR[2][0] = -sg * cb; dR[2][1] = -cg * ca - sg * sb * sa; dR[2][2] = cg * sa - sg * sb * ca;
    dR[2][3] = cg * cb;  dR[2][4] = -sg * ca + cg * sb * sa; dR[2][5] = sg * sa + cg * sb * ca;
    dR[2][6] = 0.f;      dR[2][7] = 0.f;                     dR[2][8] = 0.f;
}
static void mv(const float M[9], const float* v, float* o) {
    o[0] = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
    o[1] = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
    o[2] = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
}
static int fit_valid(const arap_ctx* c, int v) { return c->C[3 * v] >= -999999.9f; }

/* edge residual (3 comps) and the columns dR_j d (partial w.r.t. Angle_j(v0) = -wr * col_j) */
static void edge_res(const arap_ctx* c, int e, float r[3], float col[3][3]) {
    const int a = c->v0[e], b = c->v1[e];
    float R[9], dR[3][9], d[3], Rd[3];
    rot(&c->A[3 * a], R, col ? dR : NULL);
    for (int k = 0; k < 3; ++k) d[k] = c->U[3 * a + k] - c->U[3 * b + k];
    mv(R, d, Rd);
    for (int k = 0; k < 3; ++k) r[k] = c->wr * ((c->O[3 * a + k] - c->O[3 * b + k]) - Rd[k]);
    if (col)
        for (int j = 0; j < 3; ++j) mv(dR[j], d, col[j]);
}

static double arap_cost_fn(void* v) {
    arap_ctx* c = (arap_ctx*)v;
    double acc = 0.0;
    for (int i = 0; i < c->N; ++i) {
        if (!fit_valid(c, i)) continue;
        float s = 0.f;
        for (int k = 0; k < 3; ++k) {
            const float e = c->wf * (c->O[3 * i + k] - c->C[3 * i + k]);
            s += e * e;
        }
        acc += 0.5f * s;
    }
    for (int e = 0; e < c->E; ++e) {
        float r[3];
        edge_res(c, e, r, NULL);
        acc += 0.5f * (r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    }
    return acc;
}

static void arap_jtf_fn(void* v, float* r, float* diag) {
    arap_ctx* c = (arap_ctx*)v;
    const int N = c->N;
    float* rO = r; float* rA = r + 3 * N;
    float* dO = diag; float* dA = diag + 3 * N;
    memset(r, 0, sizeof(float) * 6 * N);
    memset(diag, 0, sizeof(float) * 6 * N);
    for (int i = 0; i < N; ++i)   /* centred fit (PCGInit1) */
        if (fit_valid(c, i))
            for (int k = 0; k < 3; ++k) {
                const float e = c->wf * (c->O[3 * i + k] - c->C[3 * i + k]);
                rO[3 * i + k] = -(c->wf * e);
                dO[3 * i + k] = c->wf * c->wf;
            }
    for (int e = 0; e < c->E; ++e) {   /* graph scatter (PCGInit1_Graph) */
        const int a = c->v0[e], b = c->v1[e];
        float res[3], col[3][3];
        edge_res(c, e, res, col);
        for (int k = 0; k < 3; ++k) {
            rO[3 * a + k] += -1.f * (c->wr * res[k]);
            dO[3 * a + k] += c->wr * c->wr;
            rO[3 * b + k] += -1.f * (-c->wr * res[k]);
            dO[3 * b + k] += (-c->wr) * (-c->wr);
        }
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) {
                const float pj = -c->wr * col[j][k];
                rA[3 * a + j] += -1.f * (pj * res[k]);
                dA[3 * a + j] += pj * pj;
            }
    }
}

static double arap_apply_fn(void* v, const float* p, float* Ap) {
    arap_ctx* c = (arap_ctx*)v;
    const int N = c->N;
    const float* pO = p; const float* pA = p + 3 * N;
    float* aO = Ap; float* aA = Ap + 3 * N;
    memset(Ap, 0, sizeof(float) * 6 * N);
    double dot = 0.0;
    for (int i = 0; i < N; ++i)   /* centred fit (PCGStep1) */
        if (fit_valid(c, i))
            for (int k = 0; k < 3; ++k) {
                aO[3 * i + k] = c->wf * (c->wf * pO[3 * i + k]);
                dot += (double)pO[3 * i + k] * aO[3 * i + k];
            }
    for (int e = 0; e < c->E; ++e) {   /* graph scatter (PCGStep1_Graph) */
        const int a = c->v0[e], b = c->v1[e];
        float res[3], col[3][3];
        edge_res(c, e, res, col);
        float gdot = 0.f;
        for (int k = 0; k < 3; ++k) {
            float jp = c->wr * pO[3 * a + k] + (-c->wr) * pO[3 * b + k];
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

static double arap_model_fn(void* v, const float* d) {
    arap_ctx* c = (arap_ctx*)v;
    const int N = c->N;
    const float* dO = d; const float* dA = d + 3 * N;
    double acc = 0.0;
    for (int i = 0; i < N; ++i) {
        if (!fit_valid(c, i)) continue;
        float s = 0.f;
        for (int k = 0; k < 3; ++k) {
            const float e = c->wf * (c->O[3 * i + k] - c->C[3 * i + k]) + c->wf * dO[3 * i + k];
            s += e * e;
        }
        acc += 0.5f * s;
    }
    for (int e = 0; e < c->E; ++e) {
        const int a = c->v0[e], b = c->v1[e];
        float res[3], col[3][3];
        edge_res(c, e, res, col);
        float s = 0.f;
        for (int k = 0; k < 3; ++k) {
            float jd = c->wr * dO[3 * a + k] + (-c->wr) * dO[3 * b + k];
            for (int j = 0; j < 3; ++j) jd += (-c->wr * col[j][k]) * dA[3 * a + j];
            const float m = res[k] + jd;
            s += m * m;
        }
        acc += 0.5f * s;
    }
    return acc;
}
static void arap_update_fn(void* v, const float* d) {
    arap_ctx* c = (arap_ctx*)v;
    for (int i = 0; i < 3 * c->N; ++i) { c->O[i] += d[i]; c->A[i] += d[3 * c->N + i]; }
}
static void arap_save_fn(void* v) {
    arap_ctx* c = (arap_ctx*)v;
    memcpy(c->prevO, c->O, sizeof(float) * 3 * c->N);
    memcpy(c->prevA, c->A, sizeof(float) * 3 * c->N);
}
static void arap_revert_fn(void* v) {
    arap_ctx* c = (arap_ctx*)v;
    memcpy(c->O, c->prevO, sizeof(float) * 3 * c->N);
    memcpy(c->A, c->prevA, sizeof(float) * 3 * c->N);
}

/* ------------------------------------------------------------- public API ---- */
#define CTX arap_ctx c = {N, E, O, A, U, C, v0, v1, wf, wr, NULL, NULL}
double oracle_arap_cost(int N, int E, float* O, float* A, const float* U, const float* C, const int* v0,
                        const int* v1, float wf, float wr) {
    CTX;
    return arap_cost_fn(&c);
}
void oracle_arap_jtf(int N, int E, float* O, float* A, const float* U, const float* C, const int* v0,
                     const int* v1, float wf, float wr, float* r, float* diag) {
    CTX;
    arap_jtf_fn(&c, r, diag);
}
double oracle_arap_apply(int N, int E, float* O, float* A, const float* U, const float* C, const int* v0,
                         const int* v1, float wf, float wr, const float* p, float* Ap) {
    CTX;
    return arap_apply_fn(&c, p, Ap);
}
double oracle_arap_model_cost(int N, int E, float* O, float* A, const float* U, const float* C, const int* v0,
                              const int* v1, float wf, float wr, const float* d) {
    CTX;
    return arap_model_fn(&c, d);
}
int oracle_arap_solve(int N, int E, float* O, float* A, const float* U, const float* C, const int* v0,
                      const int* v1, float wf, float wr, int lm, int nIter, int lIter, double* costs) {
    CTX;
    c.prevO = malloc(sizeof(float) * 3 * N);
    c.prevA = malloc(sizeof(float) * 3 * N);
    unsigned char* act = malloc(6 * (size_t)N);
    memset(act, 1, 6 * (size_t)N);
    oracle_problem_float P = {6LL * N, act, 1, &c, arap_cost_fn, arap_jtf_fn, arap_apply_fn, arap_model_fn,
                              arap_update_fn, arap_save_fn, arap_revert_fn};
    oracle_params sp = oracle_default_params();
    sp.nIterations = nIter;
    sp.lIterations = lIter;
    const int k = oracle_solve_f32(&P, lm, &sp, costs);
    free(act); free(c.prevO); free(c.prevA);
    return k;
}
