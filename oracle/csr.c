/*
 * oracle/csr.c — CPU restatement of the reference's CSR linear algebra for the
 * materialized-Jacobian path. TEST INFRASTRUCTURE ONLY (oracle/README.md).
 *
 * PINNED: API/src/linalg_cpu_test.t:49-176 holds known-answer vectors for every
 * function below (3x4 A, A^T, A x = {60, 63, 77}, A^T A); tests/test_oracle_csr.py
 * checks this restatement against them.
 *
 * Restated from API/src/linalg_cpu.t (the single-threaded CPU backend of the fork; the
 * CUDA backend calls cuSPARSE for the same products, API/src/backend_cuda.t:541-654):
 *   computeNnzPatternAT  :203-297   computeNnzPatternATA :300-440
 *   computeATA           :447-508   computeAT            :512-551
 *   applyAtoVector       :560-600
 * and the solver glue cusparseOuter / cusparseInner / PCGStep1_Finish
 * (API/src/solverGPUGaussNewton.t:1532-1757, :646-663).
 * Compiled with -ffp-contract=off (float products and sums rounded one by one).
 */
#include "csr.h"
#include <stdlib.h>
#include <string.h>

void oracle_csr_pattern_at(int nColsA, int nRowsA, int nnzA, const int* rowPtrA, const int* colIndA,
                           int* rowPtrAT, int* colIndAT) {
    const int nRowsAT = nColsA;
    int* cnt = calloc(nRowsAT > 0 ? nRowsAT : 1, sizeof(int));
    int* next = calloc(nRowsAT > 0 ? nRowsAT : 1, sizeof(int));
    (void)nnzA;
    /* a) count the entries of every row of A^T */
    for (int ri = 0; ri < nRowsA; ++ri)
        for (int k = rowPtrA[ri]; k < rowPtrA[ri + 1]; ++k) cnt[colIndA[k]] += 1;
    /* b) offsets */
    rowPtrAT[0] = 0;
    for (int r = 0; r < nRowsAT; ++r) rowPtrAT[r + 1] = rowPtrAT[r] + cnt[r];
    /* c) second traversal in row order of A: column indices of A^T come out sorted */
    for (int ri = 0; ri < nRowsA; ++ri)
        for (int k = rowPtrA[ri]; k < rowPtrA[ri + 1]; ++k) {
            const int r = colIndA[k];
            colIndAT[rowPtrAT[r] + next[r]] = ri;
            next[r] += 1;
        }
    free(cnt);
    free(next);
}

/* getEntry: A(row, col) by a scan of the row (0 if absent) */
static float get_entry(int row, int col, const int* rowPtrA, const int* colIndA, const float* valA) {
    for (int k = rowPtrA[row]; k < rowPtrA[row + 1]; ++k)
        if (colIndA[k] == col) return valA[k];
    return 0.f;
}

void oracle_csr_at(int nColsA, int nRowsA, int nnzA, const float* valA, const int* rowPtrA, const int* colIndA,
                   float* valAT, const int* rowPtrAT, const int* colIndAT) {
    (void)nRowsA;
    memset(valAT, 0, sizeof(float) * (size_t)(nnzA > 0 ? nnzA : 0));
    for (int r = 0; r < nColsA; ++r)
        for (int k = rowPtrAT[r]; k < rowPtrAT[r + 1]; ++k) valAT[k] = get_entry(colIndAT[k], r, rowPtrA, colIndA, valA);
}

static int cmp_int(const void* a, const void* b) {
    const int x = *(const int*)a, y = *(const int*)b;
    return (x > y) - (x < y);
}

int oracle_csr_pattern_ata(int nUnknowns, int nResiduals, int nnzA, const int* rowPtrA, const int* colIndA,
                           int* rowPtrATA, int* colIndATA) {
    int* rowPtrAT = malloc(sizeof(int) * (nUnknowns + 1));
    int* colIndAT = malloc(sizeof(int) * (nnzA > 0 ? nnzA : 1));
    oracle_csr_pattern_at(nUnknowns, nResiduals, nnzA, rowPtrA, colIndA, rowPtrAT, colIndAT);
    unsigned char* seen = calloc(nUnknowns > 0 ? nUnknowns : 1, 1);
    int* list = malloc(sizeof(int) * (nUnknowns > 0 ? nUnknowns : 1));
    int nnz = 0;
    rowPtrATA[0] = 0;
    for (int i = 0; i < nUnknowns; ++i) {
        int nl = 0;
        for (int k = rowPtrAT[i]; k < rowPtrAT[i + 1]; ++k) {
            const int ra = colIndAT[k];
            for (int j = rowPtrA[ra]; j < rowPtrA[ra + 1]; ++j) {
                const int c = colIndA[j];
                if (!seen[c]) { seen[c] = 1; list[nl++] = c; }
            }
        }
        qsort(list, nl, sizeof(int), cmp_int);   /* uniquelist:sortInPlace */
        if (colIndATA) memcpy(colIndATA + rowPtrATA[i], list, sizeof(int) * nl);
        rowPtrATA[i + 1] = rowPtrATA[i] + nl;
        nnz += nl;
        for (int q = 0; q < nl; ++q) seen[list[q]] = 0;
    }
    free(rowPtrAT); free(colIndAT); free(seen); free(list);
    return nnz;
}

void oracle_csr_ata(int nUnknowns, int nResiduals, int nnzA, int nnzATA, const float* valA, const int* rowPtrA,
                    const int* colIndA, const float* valAT, const int* rowPtrAT, const int* colIndAT,
                    float* valATA, const int* rowPtrATA, const int* colIndATA) {
    (void)nResiduals; (void)nnzA;
    memset(valATA, 0, sizeof(float) * (size_t)(nnzATA > 0 ? nnzATA : 0));
    for (int i = 0; i < nUnknowns; ++i) {
        const int oAT = rowPtrAT[i], nAT = rowPtrAT[i + 1] - oAT;
        const int oATA = rowPtrATA[i], nATA = rowPtrATA[i + 1] - oATA;
        for (int k = 0; k < nAT; ++k) {
            const float t = valAT[oAT + k];
            const int ra = colIndAT[oAT + k];
            const int oA = rowPtrA[ra], nA = rowPtrA[ra + 1] - oA;
            int ci = 0;
            for (int l = 0; l < nATA; ++l)
                if (ci < nA && colIndATA[oATA + l] == colIndA[oA + ci]) {
                    valATA[oATA + l] = valATA[oATA + l] + t * valA[oA + ci];
                    ++ci;
                }
        }
    }
}

void oracle_csr_spmv(int nColsA, int nRowsA, int nnzA, const float* valA, const int* rowPtrA, const int* colIndA,
                     const float* valInVec, float* valOutVec) {
    (void)nColsA; (void)nnzA;
    for (int k = 0; k < nRowsA; ++k) {
        float tmp = 0.f;
        for (int l = rowPtrA[k]; l < rowPtrA[k + 1]; ++l) tmp = tmp + valInVec[colIndA[l]] * valA[l];
        valOutVec[k] = tmp;
    }
}

/* ------------------------------------------------------------ materialized apply */
void oracle_mat_init(oracle_mat* m, long long nres, long long nnz, int n, int fused, const unsigned char* act,
                     void (*dump)(void*, int*, int*, float*), void* fctx) {
    memset(m, 0, sizeof(*m));
    m->nres = nres; m->nnz = nnz; m->n = n; m->fused = fused; m->act = act; m->dump = dump; m->fctx = fctx;
    m->rowPtr = malloc(sizeof(int) * (nres + 1));
    m->colInd = malloc(sizeof(int) * (nnz > 0 ? nnz : 1));
    m->val = malloc(sizeof(float) * (nnz > 0 ? nnz : 1));
    m->rowPtrT = malloc(sizeof(int) * (n + 1));
    m->colIndT = malloc(sizeof(int) * (nnz > 0 ? nnz : 1));
    m->valT = malloc(sizeof(float) * (nnz > 0 ? nnz : 1));
    m->Jp = malloc(sizeof(float) * (nres > 0 ? nres : 1));
    m->rowPtrATA = malloc(sizeof(int) * (n + 1));
}
void oracle_mat_free(oracle_mat* m) {
    free(m->rowPtr); free(m->colInd); free(m->val); free(m->rowPtrT); free(m->colIndT); free(m->valT);
    free(m->Jp); free(m->rowPtrATA); free(m->colIndATA); free(m->valATA);
    memset(m, 0, sizeof(*m));
}
void oracle_mat_build(oracle_mat* m) {
    m->dump(m->fctx, m->rowPtr, m->colInd, m->val);
    if (!m->patterns) {   /* section 1 of cusparseOuter (:1563-1620): once per solve */
        if (m->fused) {
            m->nnzATA = oracle_csr_pattern_ata(m->n, (int)m->nres, (int)m->nnz, m->rowPtr, m->colInd, m->rowPtrATA, NULL);
            m->colIndATA = malloc(sizeof(int) * (m->nnzATA > 0 ? m->nnzATA : 1));
            m->valATA = malloc(sizeof(float) * (m->nnzATA > 0 ? m->nnzATA : 1));
            oracle_csr_pattern_ata(m->n, (int)m->nres, (int)m->nnz, m->rowPtr, m->colInd, m->rowPtrATA, m->colIndATA);
        }
        oracle_csr_pattern_at(m->n, (int)m->nres, (int)m->nnz, m->rowPtr, m->colInd, m->rowPtrT, m->colIndT);
        m->patterns = 1;
    }
    oracle_csr_at(m->n, (int)m->nres, (int)m->nnz, m->val, m->rowPtr, m->colInd, m->valT, m->rowPtrT, m->colIndT);
    if (m->fused)
        oracle_csr_ata(m->n, (int)m->nres, (int)m->nnz, m->nnzATA, m->val, m->rowPtr, m->colInd, m->valT, m->rowPtrT,
                       m->colIndT, m->valATA, m->rowPtrATA, m->colIndATA);
}
double oracle_mat_apply(oracle_mat* m, const float* p, float* Ap) {
    if (m->fused) {
        oracle_csr_spmv(m->n, m->n, m->nnzATA, m->valATA, m->rowPtrATA, m->colIndATA, p, Ap);
    } else {
        oracle_csr_spmv(m->n, (int)m->nres, (int)m->nnz, m->val, m->rowPtr, m->colInd, p, m->Jp);
        oracle_csr_spmv((int)m->nres, m->n, (int)m->nnz, m->valT, m->rowPtrT, m->colIndT, m->Jp, Ap);
    }
    double d = 0.0;
    for (int e = 0; e < m->n; ++e) {
        if (!m->act[e]) { Ap[e] = 0.f; continue; }
        d += (double)p[e] * Ap[e];
    }
    return d;
}
