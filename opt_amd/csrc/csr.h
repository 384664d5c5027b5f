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
// (rows of A ascending), so they match the CPU restatement bit for bit. The solver's
// SpMVs run over a SELL-64 copy of each operator (slices of 64 rows = one wavefront,
// column-major inside the slice): lane r owns row r, every load instruction is one
// contiguous segment, and each row is summed in column order with rounded products —
// bitwise the reference CPU backend's applyAtoVector. The PCG variant masks excluded
// unknowns and reduces p.Ap deterministically (PCGStep1_Finish,
// solverGPUGaussNewton.t:646-663).
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

// SELL-64 (the solver's SpMV layout): rows in slices of 64 = one wavefront, slice
// width = its longest row, entries column-major inside a slice so lane r of the wave
// reads row r and every load instruction is one contiguous 256-B (fp32) segment. Built
// once per pattern; pos[] maps every slot to its CSR position (-1: padding, value 0).
struct SellMatrix {
    int rows = 0, nslices = 0;
    long long padded = 0;
    int* sliceOff = nullptr;   // nslices + 1
    int* col = nullptr;        // padded
    int* pos = nullptr;        // padded
    void release() {
        dfree(sliceOff); dfree(col); dfree(pos);
        sliceOff = col = pos = nullptr;
        rows = nslices = 0;
        padded = 0;
    }
    ~SellMatrix() { release(); }
};
void sell_build(int rows, const int* rowPtr, const int* colInd, SellMatrix& S, DevBuf& scratch, hipStream_t s);
// pos[q] <- perm[pos[q]]: slots of A^T addressed directly into A's value array
void sell_compose(SellMatrix& S, const int* perm, hipStream_t s);
template <typename T>
void sell_values(const SellMatrix& S, const T* csrVal, T* sellVal, hipStream_t s);
// computeATA straight into the SELL layout of the A^T A pattern (bitwise computeATA)
template <typename T>
void ata_values_sell(int cols, const int* rowPtrA, const int* colIndA, const T* valA, const int* rowPtrT,
                     const int* colIndT, const T* valT, const int* rowPtrATA, const int* colIndATA,
                     const SellMatrix& S, T* sellVal, hipStream_t s);
int sell_blocks(const SellMatrix& S);

// A^T A product map (the solver's per-step J^T J): for every slot of the A^T A SELL-64
// copy, the position pairs (p1, p2) into A's values with slot = sum_m A[p1_m] A[p2_m],
// rows of A ascending — computeATA's products in its order, so the result is bitwise
// computeATA. Stored like the SELL copy itself: the 64 slots of a slice column (group
// g) keep their pair lists column-major at gbase[g], padded with (-1, -1), so the
// per-step kernel streams the map with coalesced loads and writes the SELL values
// directly.
struct AtaProducts {
    long long n = 0, npairs = 0, padded = 0;
    long long* off = nullptr;     // build only
    int2* pairs = nullptr;        // npairs (padded, grouped)
    long long* gbase = nullptr;   // padded / 64 + 1
    void release() {
        dfree(off); dfree(pairs); dfree(gbase);
        off = nullptr; pairs = nullptr; gbase = nullptr;
        n = npairs = padded = 0;
    }
    ~AtaProducts() { release(); }
};
void ata_products_build(int cols, const int* rowPtrA, const int* colIndA, const int* rowPtrT, const int* colIndT,
                        const int* perm, const int* rowPtrATA, const int* colIndATA, long long nnzATA,
                        const SellMatrix& S, AtaProducts& P, DevBuf& scratch, hipStream_t s);
template <typename T>
void ata_values_products(const AtaProducts& P, const T* valA, T* out, hipStream_t s);
template <typename T>
void sell_spmv(const SellMatrix& S, const T* val, const T* x, T* y, hipStream_t s);
template <typename T>
void sell_spmv_pcg(const SellMatrix& S, const T* val, const T* x, T* y, const T* pv, const PcgMask& m, ReduceSlot rs,
                   hipStream_t s);

// The solver-side holder: J (filled by the family's dump_j), J^T (pattern once, values
// every step), J^T J (fused only), the SELL-64 copies the SpMVs stream, and the apply.
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
        const long long nz = std::max(nnz_, 1LL);
        rowPtrJ_ = (int*)dmalloc(sizeof(int) * (rows_ + 1));
        colIndJ_ = (int*)dmalloc(sizeof(int) * nz);
        valJ_ = (T*)dmalloc(sizeof(T) * nz);
        rowPtrT_ = (int*)dmalloc(sizeof(int) * (cols_ + 1));
        colIndT_ = (int*)dmalloc(sizeof(int) * nz);
        perm_ = (int*)dmalloc(sizeof(int) * nz);
        if (fused_) {
            rowPtrATA_ = (int*)dmalloc(sizeof(int) * (cols_ + 1));
        } else {
            Jp_ = (T*)dmalloc(sizeof(T) * std::max(rows_, 1));
        }
    }
    ~MaterializedJacobian() {
        for (void* v : {(void*)rowPtrJ_, (void*)colIndJ_, (void*)valJ_, (void*)rowPtrT_, (void*)colIndT_, (void*)perm_,
                        (void*)valT_, (void*)Jp_, (void*)rowPtrATA_, (void*)colIndATA_, (void*)svJ_, (void*)svT_,
                        (void*)svA_})
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
    int blocks() const { return sell_blocks(fused_ ? sA_ : sT_); }
    const char* apply_name() const { return fused_ ? "J^TJp" : "J^T"; }

    // After the family filled J: the patterns once (section 1 of cusparseOuter,
    // :1563-1620), then J^T values (+ J^T J values when fused) (section 2, :1623-1656).
    template <class Timer>
    void build(Timer&& tb, hipStream_t s) {
        if (!patterns_) {
            tb("JT alloc", true);
            csr_transpose_pattern(rows_, cols_, nnz_, rowPtrJ_, colIndJ_, rowPtrT_, colIndT_, perm_, scratch_, s);
            if (!fused_) {
                sell_build(rows_, rowPtrJ_, colIndJ_, sJ_, scratch_, s);
                sell_build(cols_, rowPtrT_, colIndT_, sT_, scratch_, s);
                sell_compose(sT_, perm_, s);   // J^T slots read J's values directly
                svJ_ = (T*)dmalloc(sizeof(T) * std::max(sJ_.padded, 1LL));
                svT_ = (T*)dmalloc(sizeof(T) * std::max(sT_.padded, 1LL));
            }
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
                csr_ata_pattern(cols_, rowPtrJ_, colIndJ_, rowPtrT_, colIndT_, rowPtrATA_, colIndATA_, scratch_, s);
                sell_build(cols_, rowPtrATA_, colIndATA_, sA_, scratch_, s);
                ata_products_build(cols_, rowPtrJ_, colIndJ_, rowPtrT_, colIndT_, perm_, rowPtrATA_, colIndATA_,
                                   nnz_ata_, sA_, prod_, scratch_, s);
                svA_ = (T*)dmalloc(sizeof(T) * std::max(sA_.padded, 1LL));
                OPT_HIP_CHECK(hipMemsetAsync(svA_, 0, sizeof(T) * std::max(sA_.padded, 1LL), s));   // padding
                tb("J^TJ alloc", false);
            }
            scratch_.release();
            patterns_ = true;
        }
        if (fused_) {   // J^T J straight from J's values (the product map holds the transpose)
            tb("JTJ multiply", true);
            ata_values_products<T>(prod_, valJ_, svA_, s);
            tb("JTJ multiply", false);
        } else {
            tb("J_transpose", true);
            sell_values<T>(sJ_, valJ_, svJ_, s);
            sell_values<T>(sT_, valJ_, svT_, s);
            tb("J_transpose", false);
        }
    }
    // Ap = J^T J p (fused) or J^T (J p), masked to the active unknowns, p.Ap into rs
    // (cusparseInner :1660-1757 + PCGStep1_Finish :646-663).
    template <class Timer>
    void apply(const T* p, T* Ap, const PcgMask& m, ReduceSlot rs, Timer&& tb, hipStream_t s) {
        if (fused_) {
            tb("J^TJp", true);
            sell_spmv_pcg<T>(sA_, svA_, p, Ap, p, m, rs, s);
            tb("J^TJp", false);
        } else {
            tb("Jp", true);
            sell_spmv<T>(sJ_, svJ_, p, Jp_, s);
            tb("Jp", false);
            tb("J^T", true);
            sell_spmv_pcg<T>(sT_, svT_, Jp_, Ap, p, m, rs, s);
            tb("J^T", false);
        }
    }

private:
    bool fused_ = false, patterns_ = false;
    int rows_ = 0, cols_ = 0;
    long long nnz_ = 0, nnz_ata_ = 0;
    int *rowPtrJ_ = nullptr, *colIndJ_ = nullptr, *rowPtrT_ = nullptr, *colIndT_ = nullptr, *perm_ = nullptr;
    int *rowPtrATA_ = nullptr, *colIndATA_ = nullptr;
    T *valJ_ = nullptr, *valT_ = nullptr, *Jp_ = nullptr;
    SellMatrix sJ_, sT_, sA_;
    AtaProducts prod_;
    T *svJ_ = nullptr, *svT_ = nullptr, *svA_ = nullptr;
    DevBuf scratch_;
};

}  // namespace optamd
