// csr.hip — device CSR kernels of the materialized-Jacobian path (see csr.h for the
// reference functions each one replaces and the design).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include "csr.h"
#include "stencil_driver.h"

namespace optamd {
namespace csr {

constexpr int kGrid = 4096;   // grid-stride cap for the flat kernels

inline int grid_for(long long n, int per_block = kBlock) {
    return (int)std::max<long long>(1, std::min<long long>((n + per_block - 1) / per_block, kGrid));
}

// rowOf[k] = row of the k-th nonzero; iota[k] = k
__global__ __launch_bounds__(kBlock) void expand_rows(int rows, const int* __restrict__ rowPtr,
                                                      int* __restrict__ rowOf, int* __restrict__ iota) {
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += gridDim.x * blockDim.x)
        for (int k = rowPtr[r]; k < rowPtr[r + 1]; ++k) {
            rowOf[k] = r;
            iota[k] = k;
        }
}

// colIndT[j] = row of A of the j-th entry of A^T
__global__ __launch_bounds__(kBlock) void gather_int(long long n, const int* __restrict__ perm,
                                                     const int* __restrict__ src, int* __restrict__ dst) {
    for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (long long)gridDim.x * blockDim.x)
        dst[j] = src[perm[j]];
}

// rowPtrT[c] = first position of the sorted column keys >= c (c = 0..cols)
__global__ __launch_bounds__(kBlock) void lower_bounds(int cols, long long n, const int* __restrict__ keys,
                                                       int* __restrict__ rowPtrT) {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c <= cols; c += gridDim.x * blockDim.x) {
        long long lo = 0, hi = n;
        while (lo < hi) {
            const long long mid = (lo + hi) >> 1;
            if (keys[mid] < c) lo = mid + 1;
            else hi = mid;
        }
        rowPtrT[c] = (int)lo;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void gather_val(long long n, const int* __restrict__ perm,
                                                     const T* __restrict__ val, T* __restrict__ valT) {
    for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (long long)gridDim.x * blockDim.x)
        valT[j] = val[perm[j]];
}

// One A^T A row: the sorted unique union of the columns of the A rows in A^T row i.
// FILL = false: count (counts[i]); FILL = true: write them at rowPtrATA[i].
template <bool FILL>
__global__ __launch_bounds__(kBlock) void ata_rows(int cols, const int* __restrict__ rowPtrA,
                                                   const int* __restrict__ colIndA, const int* __restrict__ rowPtrT,
                                                   const int* __restrict__ colIndT, int* __restrict__ counts,
                                                   int* __restrict__ colIndATA, int* __restrict__ overflow) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += gridDim.x * blockDim.x) {
        int buf[kMaxAtaRow];
        int n = 0;
        bool over = false;
        for (int k = rowPtrT[i]; k < rowPtrT[i + 1] && !over; ++k) {
            const int r = colIndT[k];
            for (int j = rowPtrA[r]; j < rowPtrA[r + 1]; ++j) {
                const int c = colIndA[j];
                int pos = n;
                while (pos > 0 && buf[pos - 1] > c) --pos;
                if (pos > 0 && buf[pos - 1] == c) continue;
                if (n == kMaxAtaRow) { over = true; break; }
                for (int q = n; q > pos; --q) buf[q] = buf[q - 1];
                buf[pos] = c;
                ++n;
            }
        }
        if (over) { *overflow = 1; n = 0; }
        if (!FILL) {
            counts[i] = n;
        } else {
            int* out = colIndATA + counts[i];   // counts = rowPtrATA here
            for (int q = 0; q < n; ++q) out[q] = buf[q];
        }
    }
}

// General A^T A pattern (rows of any length): candidate columns of every row, a
// segmented radix sort, then the distinct values.
__global__ __launch_bounds__(kBlock) void cand_counts(int cols, const int* __restrict__ rowPtrA,
                                                      const int* __restrict__ rowPtrT,
                                                      const int* __restrict__ colIndT, long long* __restrict__ cnt) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += gridDim.x * blockDim.x) {
        long long c = 0;
        for (int k = rowPtrT[i]; k < rowPtrT[i + 1]; ++k) c += rowPtrA[colIndT[k] + 1] - rowPtrA[colIndT[k]];
        cnt[i] = c;
    }
}
__global__ __launch_bounds__(kBlock) void cand_fill(int cols, const int* __restrict__ rowPtrA,
                                                    const int* __restrict__ colIndA, const int* __restrict__ rowPtrT,
                                                    const int* __restrict__ colIndT, const long long* __restrict__ off,
                                                    int* __restrict__ cand, int* __restrict__ seg) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += gridDim.x * blockDim.x) {
        long long o = off[i];
        seg[i] = (int)o;
        if (i == cols - 1) seg[cols] = (int)off[cols];
        for (int k = rowPtrT[i]; k < rowPtrT[i + 1]; ++k) {
            const int r = colIndT[k];
            for (int j = rowPtrA[r]; j < rowPtrA[r + 1]; ++j) cand[o++] = colIndA[j];
        }
    }
}
template <bool FILL>
__global__ __launch_bounds__(kBlock) void cand_unique(int cols, const int* __restrict__ seg,
                                                      const int* __restrict__ sorted, int* __restrict__ counts,
                                                      int* __restrict__ colIndATA) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += gridDim.x * blockDim.x) {
        int n = 0;
        int* out = FILL ? colIndATA + counts[i] : nullptr;
        for (int k = seg[i]; k < seg[i + 1]; ++k)
            if (k == seg[i] || sorted[k] != sorted[k - 1]) {
                if (FILL) out[n] = sorted[k];
                ++n;
            }
        if (!FILL) counts[i] = n;
    }
}

__global__ __launch_bounds__(kBlock) void sum_counts(int n, const int* __restrict__ counts,
                                                     unsigned long long* __restrict__ total) {
    unsigned long long s = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += (unsigned)counts[i];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) atomicAdd(total, s);
}

// computeATA (linalg_cpu.t:447-508): row i of A^T A accumulates, for every entry k of
// A^T row i in order (rows r of A ascending), valT[k] * A(r, c) into column c; the
// column is located by the reference's forward merge over the sorted row.
template <typename T>
__global__ __launch_bounds__(kBlock) void ata_values(int cols, const int* __restrict__ rowPtrA,
                                                     const int* __restrict__ colIndA, const T* __restrict__ valA,
                                                     const int* __restrict__ rowPtrT, const int* __restrict__ colIndT,
                                                     const T* __restrict__ valT, const int* __restrict__ rowPtrATA,
                                                     const int* __restrict__ colIndATA, T* __restrict__ valATA) {
#pragma clang fp contract(off)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += gridDim.x * blockDim.x) {
        const int b = rowPtrATA[i], n = rowPtrATA[i + 1] - b;
        for (int l = 0; l < n; ++l) valATA[b + l] = (T)0;
        for (int k = rowPtrT[i]; k < rowPtrT[i + 1]; ++k) {
            const T t = valT[k];
            const int r = colIndT[k];
            int ci = rowPtrA[r];
            const int ce = rowPtrA[r + 1];
            for (int l = 0; l < n && ci < ce; ++l) {
                if (colIndATA[b + l] == colIndA[ci]) {
                    valATA[b + l] = valATA[b + l] + t * valA[ci];
                    ++ci;
                }
            }
        }
    }
}

template <typename T>
__device__ __forceinline__ T group_sum(T v, int G) {
    for (int off = G >> 1; off > 0; off >>= 1) v += __shfl_xor(v, off, G);
    return v;
}

// y = A x with G lanes per row.
template <typename T, int G>
__global__ __launch_bounds__(kBlock) void spmv(int rows, const int* __restrict__ rowPtr,
                                               const int* __restrict__ colInd, const T* __restrict__ val,
                                               const T* __restrict__ x, T* __restrict__ y) {
    const int lg = threadIdx.x & (G - 1);
    const long long ngroups = (long long)gridDim.x * (kBlock / G);
    for (long long r = ((long long)blockIdx.x * kBlock + threadIdx.x) / G; r < rows; r += ngroups) {
        const int b = rowPtr[r], e = rowPtr[r + 1];
        T acc = 0;
        for (int k = b + lg; k < e; k += G) acc += val[k] * x[colInd[k]];
        acc = group_sum(acc, G);
        if (lg == 0) y[r] = acc;
    }
}

// PCG variant: masked output + sum pv.y (deterministic block reduction).
template <typename T, int G>
__global__ __launch_bounds__(kBlock) void spmv_pcg(int rows, const int* __restrict__ rowPtr,
                                                   const int* __restrict__ colInd, const T* __restrict__ val,
                                                   const T* __restrict__ x, T* __restrict__ y,
                                                   const T* __restrict__ pv, PcgMask m, ReduceSlot rs) {
    if (stopped(m.stop)) return;
    const int lg = threadIdx.x & (G - 1);
    const long long ngroups = (long long)gridDim.x * (kBlock / G);
    T dot = 0;
    for (long long r = ((long long)blockIdx.x * kBlock + threadIdx.x) / G; r < rows; r += ngroups) {
        const int b = rowPtr[r], e = rowPtr[r + 1];
        T acc = 0;
        for (int k = b + lg; k < e; k += G) acc += val[k] * x[colInd[k]];
        acc = group_sum(acc, G);
        if (lg == 0) {
            const long long px = m.L.pix(r);
            const bool act = px >= m.pix_lo && px < m.pix_hi && (m.flags[px] & 1);
            if (!act) acc = 0;
            y[r] = acc;
            dot += pv[r] * acc;
        }
    }
    double v[1] = {(double)dot};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

inline int group_for(long long rows, long long nnz) {
    const double avg = rows > 0 ? (double)nnz / (double)rows : 1.0;
    int G = 1;
    while (G < 16 && G < avg) G <<= 1;
    return G;
}

}  // namespace csr

void csr_transpose_pattern(int rows, int cols, long long nnz, const int* rowPtr, const int* colInd, int* rowPtrT,
                           int* colIndT, int* perm, DevBuf& scratch, hipStream_t s) {
    if (nnz == 0) {
        OPT_HIP_CHECK(hipMemsetAsync(rowPtrT, 0, sizeof(int) * (cols + 1), s));
        return;
    }
    int* rowOf = (int*)dmalloc(sizeof(int) * nnz);
    int* iota = (int*)dmalloc(sizeof(int) * nnz);
    int* keys = (int*)dmalloc(sizeof(int) * nnz);
    hipLaunchKernelGGL(csr::expand_rows, dim3(csr::grid_for(rows)), dim3(kBlock), 0, s, rows, rowPtr, rowOf, iota);
    int bits = 1;
    while ((1LL << bits) < cols) ++bits;
    size_t need = 0;
    OPT_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, colInd, keys, iota, perm, (int)nnz, 0, bits, s));
    void* tmp = scratch.need(need);
    // stable: equal columns keep ascending positions, i.e. ascending rows of A
    OPT_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, need, colInd, keys, iota, perm, (int)nnz, 0, bits, s));
    hipLaunchKernelGGL(csr::gather_int, dim3(csr::grid_for(nnz)), dim3(kBlock), 0, s, nnz, (const int*)perm,
                       (const int*)rowOf, colIndT);
    hipLaunchKernelGGL(csr::lower_bounds, dim3(csr::grid_for(cols + 1LL)), dim3(kBlock), 0, s, cols, nnz,
                       (const int*)keys, rowPtrT);
    OPT_HIP_CHECK(hipGetLastError());
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    dfree(rowOf);
    dfree(iota);
    dfree(keys);
}

template <typename T>
void csr_gather(long long nnz, const int* perm, const T* val, T* valT, hipStream_t s) {
    if (nnz == 0) return;
    hipLaunchKernelGGL((csr::gather_val<T>), dim3(csr::grid_for(nnz)), dim3(kBlock), 0, s, nnz, perm, val, valT);
    OPT_HIP_CHECK(hipGetLastError());
}

// Rows longer than kMaxAtaRow: the general path. Same result (sorted unique columns).
static long long ata_pattern_general(int cols, const int* rowPtrA, const int* colIndA, const int* rowPtrT,
                                     const int* colIndT, int* rowPtrATA, int* colIndATA, DevBuf& scratch,
                                     hipStream_t s) {
    const dim3 g(csr::grid_for(cols)), b(kBlock);
    long long* off = (long long*)dmalloc(sizeof(long long) * (cols + 1));
    OPT_HIP_CHECK(hipMemsetAsync(off + cols, 0, sizeof(long long), s));
    hipLaunchKernelGGL(csr::cand_counts, g, b, 0, s, cols, rowPtrA, rowPtrT, colIndT, off);
    size_t need = 0;
    OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, off, off, cols + 1, s));
    OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scratch.need(need), need, off, off, cols + 1, s));
    long long total = 0;
    OPT_HIP_CHECK(hipMemcpyAsync(&total, off + cols, sizeof(total), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    if (total >= (1LL << 31) - 1) { dfree(off); return -1; }
    int* cand = (int*)dmalloc(sizeof(int) * std::max(total, 1LL));
    int* sorted = (int*)dmalloc(sizeof(int) * std::max(total, 1LL));
    int* seg = (int*)dmalloc(sizeof(int) * (cols + 1));
    hipLaunchKernelGGL(csr::cand_fill, g, b, 0, s, cols, rowPtrA, colIndA, rowPtrT, colIndT, (const long long*)off,
                       cand, seg);
    int bits = 1;
    while ((1LL << bits) < cols) ++bits;
    need = 0;
    OPT_HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, need, cand, sorted, (int)total, cols, seg,
                                                             seg + 1, 0, bits, s));
    OPT_HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortKeys(scratch.need(need), need, cand, sorted, (int)total,
                                                             cols, seg, seg + 1, 0, bits, s));
    long long nnz = 0;
    if (!colIndATA) {
        OPT_HIP_CHECK(hipMemsetAsync(rowPtrATA + cols, 0, sizeof(int), s));
        hipLaunchKernelGGL((csr::cand_unique<false>), g, b, 0, s, cols, (const int*)seg, (const int*)sorted, rowPtrATA,
                           (int*)nullptr);
        need = 0;
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, rowPtrATA, rowPtrATA, cols + 1, s));
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scratch.need(need), need, rowPtrATA, rowPtrATA, cols + 1, s));
    } else {
        hipLaunchKernelGGL((csr::cand_unique<true>), g, b, 0, s, cols, (const int*)seg, (const int*)sorted, rowPtrATA,
                           colIndATA);
    }
    int last = 0;
    OPT_HIP_CHECK(hipMemcpyAsync(&last, rowPtrATA + cols, sizeof(int), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipGetLastError());
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    nnz = last;
    for (void* v : {(void*)off, (void*)cand, (void*)sorted, (void*)seg}) dfree(v);
    return nnz;
}

long long csr_ata_pattern(int cols, const int* rowPtrA, const int* colIndA, const int* rowPtrT, const int* colIndT,
                          int* rowPtrATA, int* colIndATA, DevBuf& scratch, hipStream_t s) {
    int* flag = (int*)dmalloc(sizeof(int) + sizeof(unsigned long long) * 2);
    unsigned long long* total = (unsigned long long*)((char*)flag + sizeof(unsigned long long));
    OPT_HIP_CHECK(hipMemsetAsync(flag, 0, sizeof(int) + sizeof(unsigned long long) * 2, s));
    const dim3 g(csr::grid_for(cols)), b(kBlock);
    long long nnz = 0;
    // Fast path: one thread per row, sorted-unique insertion into a kMaxAtaRow buffer.
    // Counts go into rowPtrATA[0..cols) (exclusive scan over cols+1 entries after); in
    // the fill call they are recounted into a temporary to detect the same overflow.
    int* counts = colIndATA ? (int*)dmalloc(sizeof(int) * (cols + 1)) : rowPtrATA;
    OPT_HIP_CHECK(hipMemsetAsync(counts + cols, 0, sizeof(int), s));
    hipLaunchKernelGGL((csr::ata_rows<false>), g, b, 0, s, cols, rowPtrA, colIndA, rowPtrT, colIndT, counts,
                       (int*)nullptr, flag);
    hipLaunchKernelGGL(csr::sum_counts, g, b, 0, s, cols, (const int*)counts, total);
    int hflag = 0;
    unsigned long long htotal = 0;
    OPT_HIP_CHECK(hipMemcpyAsync(&hflag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipMemcpyAsync(&htotal, total, sizeof(htotal), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    if (colIndATA) dfree(counts);
    if (hflag) {
        dfree(flag);
        return ata_pattern_general(cols, rowPtrA, colIndA, rowPtrT, colIndT, rowPtrATA, colIndATA, scratch, s);
    }
    if (htotal >= (1ULL << 31) - 1) { dfree(flag); return -1; }
    if (!colIndATA) {
        size_t need = 0;
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, rowPtrATA, rowPtrATA, cols + 1, s));
        void* tmp = scratch.need(need);
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, need, rowPtrATA, rowPtrATA, cols + 1, s));
        nnz = (long long)htotal;
    } else {
        hipLaunchKernelGGL((csr::ata_rows<true>), g, b, 0, s, cols, rowPtrA, colIndA, rowPtrT, colIndT, rowPtrATA,
                           colIndATA, flag);
        int last = 0;
        OPT_HIP_CHECK(hipMemcpyAsync(&last, rowPtrATA + cols, sizeof(int), hipMemcpyDeviceToHost, s));
        OPT_HIP_CHECK(hipStreamSynchronize(s));
        nnz = last;
    }
    OPT_HIP_CHECK(hipGetLastError());
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    dfree(flag);
    return nnz;
}

template <typename T>
void csr_ata_values(int cols, const int* rowPtrA, const int* colIndA, const T* valA, const int* rowPtrT,
                    const int* colIndT, const T* valT, const int* rowPtrATA, const int* colIndATA, T* valATA,
                    hipStream_t s) {
    hipLaunchKernelGGL((csr::ata_values<T>), dim3(csr::grid_for(cols)), dim3(kBlock), 0, s, cols, rowPtrA, colIndA,
                       valA, rowPtrT, colIndT, valT, rowPtrATA, colIndATA, valATA);
    OPT_HIP_CHECK(hipGetLastError());
}

template <typename T>
void csr_spmv(int rows, long long nnz, const int* rowPtr, const int* colInd, const T* val, const T* x, T* y,
              hipStream_t s) {
    if (rows == 0) return;
    const int G = csr::group_for(rows, nnz);
    const dim3 g(csr::grid_for((long long)rows * G)), b(kBlock);
#define SPMV(GG) hipLaunchKernelGGL((csr::spmv<T, GG>), g, b, 0, s, rows, rowPtr, colInd, val, x, y)
    switch (G) {
        case 1: SPMV(1); break;
        case 2: SPMV(2); break;
        case 4: SPMV(4); break;
        case 8: SPMV(8); break;
        default: SPMV(16); break;
    }
#undef SPMV
    OPT_HIP_CHECK(hipGetLastError());
}

int csr_pcg_blocks(int rows) { return csr::grid_for((long long)rows * 16); }

template <typename T>
void csr_spmv_pcg(int rows, long long nnz, const int* rowPtr, const int* colInd, const T* val, const T* x, T* y,
                  const T* pv, const PcgMask& m, ReduceSlot rs, hipStream_t s) {
    // the grid is fixed by csr_pcg_blocks (the reduction slot's block count)
    const int G = csr::group_for(rows, nnz);
    const dim3 g(csr_pcg_blocks(rows)), b(kBlock);
#define SPMV(GG) hipLaunchKernelGGL((csr::spmv_pcg<T, GG>), g, b, 0, s, rows, rowPtr, colInd, val, x, y, pv, m, rs)
    switch (G) {
        case 1: SPMV(1); break;
        case 2: SPMV(2); break;
        case 4: SPMV(4); break;
        case 8: SPMV(8); break;
        default: SPMV(16); break;
    }
#undef SPMV
    OPT_HIP_CHECK(hipGetLastError());
}

#define INST(T)                                                                                                  \
    template void csr_gather<T>(long long, const int*, const T*, T*, hipStream_t);                              \
    template void csr_ata_values<T>(int, const int*, const int*, const T*, const int*, const int*, const T*,     \
                                    const int*, const int*, T*, hipStream_t);                                    \
    template void csr_spmv<T>(int, long long, const int*, const int*, const T*, const T*, T*, hipStream_t);      \
    template void csr_spmv_pcg<T>(int, long long, const int*, const int*, const T*, const T*, T*, const T*,      \
                                  const PcgMask&, ReduceSlot, hipStream_t);
INST(float)
INST(double)
#undef INST

}  // namespace optamd
