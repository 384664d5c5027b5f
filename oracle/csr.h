/* oracle/csr.h — TEST INFRASTRUCTURE ONLY (oracle/README.md): CPU restatement of the
 * reference's CSR linear algebra (API/src/linalg_cpu.t) and of the materialized-Jacobian
 * PCG apply (cusparseOuter / cusparseInner, API/src/solverGPUGaussNewton.t:1532-1757). */
#pragma once

/* linalg_cpu.t:203-297 computeNnzPatternAT — argument order as the reference
 * (number of columns of A first). */
void oracle_csr_pattern_at(int nColsA, int nRowsA, int nnzA, const int* rowPtrA, const int* colIndA,
                           int* rowPtrAT, int* colIndAT);
/* linalg_cpu.t:512-551 computeAT (values via getEntry) */
void oracle_csr_at(int nColsA, int nRowsA, int nnzA, const float* valA, const int* rowPtrA, const int* colIndA,
                   float* valAT, const int* rowPtrAT, const int* colIndAT);
/* linalg_cpu.t:300-440 computeNnzPatternATA: fills rowPtrATA (nUnknowns+1); returns
 * nnz(A^T A); writes colIndATA when non-NULL. */
int oracle_csr_pattern_ata(int nUnknowns, int nResiduals, int nnzA, const int* rowPtrA, const int* colIndA,
                           int* rowPtrATA, int* colIndATA);
/* linalg_cpu.t:447-508 computeATA */
void oracle_csr_ata(int nUnknowns, int nResiduals, int nnzA, int nnzATA, const float* valA, const int* rowPtrA,
                    const int* colIndA, const float* valAT, const int* rowPtrAT, const int* colIndAT,
                    float* valATA, const int* rowPtrATA, const int* colIndATA);
/* linalg_cpu.t:560-600 applyAtoVector: valOutVec = A valInVec */
void oracle_csr_spmv(int nColsA, int nRowsA, int nnzA, const float* valA, const int* rowPtrA, const int* colIndA,
                     const float* valInVec, float* valOutVec);

/* The materialized apply over a family's J assembly. */
typedef struct {
    long long nres, nnz;
    int n;                                  /* unknowns */
    int fused;
    const unsigned char* act;               /* active unknowns (not excluded) */
    void (*dump)(void* fctx, int* rowPtr, int* colInd, float* val);
    void* fctx;
    int *rowPtr, *colInd, *rowPtrT, *colIndT, *rowPtrATA, *colIndATA;
    float *val, *valT, *valATA, *Jp;
    int nnzATA, patterns;
} oracle_mat;
void oracle_mat_init(oracle_mat* m, long long nres, long long nnz, int n, int fused, const unsigned char* act,
                     void (*dump)(void*, int*, int*, float*), void* fctx);
void oracle_mat_free(oracle_mat* m);
/* cusparseOuter: J at the current unknowns, patterns once, J^T (+ J^T J) values */
void oracle_mat_build(oracle_mat* m);
/* cusparseInner + PCGStep1_Finish: Ap = J^T J p or J^T (J p); Ap = 0 on excluded
 * unknowns; returns sum p.Ap over the active ones (accumulated in double). */
double oracle_mat_apply(oracle_mat* m, const float* p, float* Ap);
