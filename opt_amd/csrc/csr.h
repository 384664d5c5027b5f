// csr.h — the materialized-Jacobian path (reference useMaterializedJTJ / useFusedJTJ,
// API/release/include/Opt.h:32-34): J assembled in CSR once per GN/LM step, its
// transpose and (fused) J^T J formed on the device, and the PCG apply done as sparse
// matrix-vector products.
//
// Reference: cusparseOuter / cusparseInner (API/src/solverGPUGaussNewton.t:1532-1757)
// over cuSPARSE csrgemm / csr2csc / csrmv (API/src/backend_cuda.t:541-654), with the
// CPU restatement in API/src/linalg_cpu.t:203-682 (computeNnzPatternAT, computeAT,
// computeNnzPatternATA, computeATA, applyAtoVector) whose unit test
// (API/src/linalg_cpu_test.t) is the golden vector set these kernels are checked on.
//
// MI355X design: no sparse library. The transpose is a stable radix sort of the
// column indices (hipCUB) — rows of A stay ascending inside every row of A^T, exactly
// the csr2csc / computeNnzPatternAT order — which also yields a gather map, so the
// per-step value transpose is one coalesced gather. The A^T A pattern is built once
// per plan (one thread per row, sorted-unique merge of the A rows the A^T row
// touches); its values are recomputed every step in the reference's summation order
// (rows of A ascending), so they match the CPU restatement bit for bit. The SpMV
// gives each row a group of G lanes (G = power of two near the mean row length, <= 16)
// so a wavefront streams 64 consecutive (value, column) pairs per load; the PCG
// variant masks excluded unknowns and reduces p.Ap deterministically
// (PCGStep1_Finish, solverGPUGaussNewton.t:646-663).
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <string>
#include "common.h"

namespace optamd {

void* dmalloc(size_t bytes);
void dfree(void* p);

// Device scratch that grows on demand.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void* need(size_t n) {
        if (n > bytes) {
            dfree(p);
            p = dmalloc(n);
            bytes = n;
        }
        return p;
    }
    void release() { dfree(p); p = nullptr; bytes = 0; }
    ~DevBuf() { release(); }
};

// Rows of A^T A up to this length take the one-thread-per-row pattern path; longer
// rows switch the whole pattern build to candidate lists + a segmented radix sort.
constexpr int kMaxAtaRow = 64;

// A^T pattern and gather map. rowPtrT: cols+1; colIndT: nnz (the rows of A, ascending
// inside each row of A^T); perm: nnz, perm[j] = position in A of the j-th entry of A^T.
void csr_transpose_pattern(int rows, int cols, long long nnz, const int* rowPtr, const int* colInd,
                           int* rowPtrT, int* colIndT, int* perm, DevBuf& scratch, hipStream_t s);
// valT[j] = val[perm[j]] (computeAT, linalg_cpu.t:512-551).
template <typename T>
void csr_gather(long long nnz, const int* perm, const T* val, T* valT, hipStream_t s);
// Pattern of A^T A (computeNnzPatternATA, linalg_cpu.t:300-440): rowPtrATA (cols+1)
// always, colIndATA (sorted) when non-null. Returns nnz(A^T A); -1 if a count exceeds
// 2^31-1 (int32 CSR).
long long csr_ata_pattern(int cols, const int* rowPtrA, const int* colIndA, const int* rowPtrT,
                          const int* colIndT, int* rowPtrATA, int* colIndATA, DevBuf& scratch, hipStream_t s);
// Values of A^T A on that pattern (computeATA, linalg_cpu.t:447-508): every entry summed
// over the rows of A in ascending order, no FMA contraction.
template <typename T>
void csr_ata_values(int cols, const int* rowPtrA, const int* colIndA, const T* valA, const int* rowPtrT,
                    const int* colIndT, const T* valT, const int* rowPtrATA, const int* colIndATA, T* valATA,
                    hipStream_t s);
// y = A x (applyAtoVector, linalg_cpu.t:560-600; cusparseScsrmv backend_cuda.t:627-634).
template <typename T>
void csr_spmv(int rows, long long nnz, const int* rowPtr, const int* colInd, const T* val, const T* x, T* y,
              hipStream_t s);

// PCG apply with rows = unknowns: y[e] = active(e) ? (A x)[e] : 0 and sum pv.y into rs
// (PCGStep1 + PCGStep1_Finish); returns at entry once *stop is set.
struct PcgMask {
    VecLayout L;
    const uint8_t* flags;     // bit0: active pixel
    long long pix_lo, pix_hi;
    const int* stop;
};
int csr_pcg_blocks(int rows);
template <typename T>
void csr_spmv_pcg(int rows, long long nnz, const int* rowPtr, const int* colInd, const T* val, const T* x, T* y,
                  const T* pv, const PcgMask& m, ReduceSlot rs, hipStream_t s);

// The solver-side holder: J (filled by the family's dump_j), J^T (pattern once, values
// every step), J^T J (fused only), and the apply.
template <typename T>
class MaterializedJacobian {
public:
    MaterializedJacobian(long long nres, long long nnz, long long nunk, bool fused) : fused_(fused) {
        if (nres >= (1LL << 31) - 1 || nnz >= (1LL << 31) - 1 || nunk >= (1LL << 31) - 1) {
            fprintf(stderr, "[opt_amd] materialized Jacobian: %lld residuals / %lld nonzeros exceed int32 CSR\n",
                    nres, nnz);
            exit(1);
        }
        rows_ = (int)nres;
        cols_ = (int)nunk;
        nnz_ = nnz;
        rowPtrJ_ = (int*)dmalloc(sizeof(int) * (rows_ + 1));
        colIndJ_ = (int*)dmalloc(sizeof(int) * std::max(nnz_, 1LL));
        valJ_ = (T*)dmalloc(sizeof(T) * std::max(nnz_, 1LL));
        rowPtrT_ = (int*)dmalloc(sizeof(int) * (cols_ + 1));
        colIndT_ = (int*)dmalloc(sizeof(int) * std::max(nnz_, 1LL));
        perm_ = (int*)dmalloc(sizeof(int) * std::max(nnz_, 1LL));
        valT_ = (T*)dmalloc(sizeof(T) * std::max(nnz_, 1LL));
        if (!fused_) Jp_ = (T*)dmalloc(sizeof(T) * std::max(rows_, 1));
        else rowPtrATA_ = (int*)dmalloc(sizeof(int) * (cols_ + 1));
    }
    ~MaterializedJacobian() {
        for (void* v : {(void*)rowPtrJ_, (void*)colIndJ_, (void*)valJ_, (void*)rowPtrT_, (void*)colIndT_, (void*)perm_,
                        (void*)valT_, (void*)Jp_, (void*)rowPtrATA_, (void*)colIndATA_, (void*)valATA_})
            dfree(v);
    }
    int* rowPtrJ() { return rowPtrJ_; }
    int* colIndJ() { return colIndJ_; }
    T* valJ() { return valJ_; }
    int rows() const { return rows_; }
    int cols() const { return cols_; }
    long long nnz() const { return nnz_; }
    long long nnz_jtj() const { return nnz_ata_; }
    bool fused() const { return fused_; }
    int blocks() const { return csr_pcg_blocks(cols_); }
    const char* apply_name() const { return fused_ ? "J^TJp" : "J^T"; }

    // After the family filled J: the patterns once (section 1 of cusparseOuter,
    // :1563-1620), then J^T values (+ J^T J values when fused) (section 2, :1623-1656).
    template <class Timer>
    void build(Timer&& tb, hipStream_t s) {
        if (!patterns_) {
            tb("JT alloc", true);
            csr_transpose_pattern(rows_, cols_, nnz_, rowPtrJ_, colIndJ_, rowPtrT_, colIndT_, perm_, scratch_, s);
            tb("JT alloc", false);
            if (fused_) {
                tb("J^TJ alloc", true);
                nnz_ata_ = csr_ata_pattern(cols_, rowPtrJ_, colIndJ_, rowPtrT_, colIndT_, rowPtrATA_, nullptr,
                                           scratch_, s);
                if (nnz_ata_ < 0) {
                    fprintf(stderr, "[opt_amd] materialized J^T J: more than 2^31 nonzeros\n");
                    exit(1);
                }
                colIndATA_ = (int*)dmalloc(sizeof(int) * std::max(nnz_ata_, 1LL));
                valATA_ = (T*)dmalloc(sizeof(T) * std::max(nnz_ata_, 1LL));
                csr_ata_pattern(cols_, rowPtrJ_, colIndJ_, rowPtrT_, colIndT_, rowPtrATA_, colIndATA_, scratch_, s);
                tb("J^TJ alloc", false);
            }
            scratch_.release();
            patterns_ = true;
        }
        tb("J_transpose", true);
        csr_gather<T>(nnz_, perm_, valJ_, valT_, s);
        tb("J_transpose", false);
        if (fused_) {
            tb("JTJ multiply", true);
            csr_ata_values<T>(cols_, rowPtrJ_, colIndJ_, valJ_, rowPtrT_, colIndT_, valT_, rowPtrATA_, colIndATA_,
                              valATA_, s);
            tb("JTJ multiply", false);
        }
    }
    // Ap = J^T J p (fused) or J^T (J p), masked to the active unknowns, p.Ap into rs
    // (cusparseInner :1660-1757 + PCGStep1_Finish :646-663).
    template <class Timer>
    void apply(const T* p, T* Ap, const PcgMask& m, ReduceSlot rs, Timer&& tb, hipStream_t s) {
        if (fused_) {
            tb("J^TJp", true);
            csr_spmv_pcg<T>(cols_, nnz_ata_, rowPtrATA_, colIndATA_, valATA_, p, Ap, p, m, rs, s);
            tb("J^TJp", false);
        } else {
            tb("Jp", true);
            csr_spmv<T>(rows_, nnz_, rowPtrJ_, colIndJ_, valJ_, p, Jp_, s);
            tb("Jp", false);
            tb("J^T", true);
            csr_spmv_pcg<T>(cols_, nnz_, rowPtrT_, colIndT_, valT_, Jp_, Ap, p, m, rs, s);
            tb("J^T", false);
        }
    }

private:
    bool fused_ = false, patterns_ = false;
    int rows_ = 0, cols_ = 0;
    long long nnz_ = 0, nnz_ata_ = 0;
    int *rowPtrJ_ = nullptr, *colIndJ_ = nullptr, *rowPtrT_ = nullptr, *colIndT_ = nullptr, *perm_ = nullptr;
    int *rowPtrATA_ = nullptr, *colIndATA_ = nullptr;
    T *valJ_ = nullptr, *valT_ = nullptr, *valATA_ = nullptr, *Jp_ = nullptr;
    DevBuf scratch_;
};

}  // namespace optamd
