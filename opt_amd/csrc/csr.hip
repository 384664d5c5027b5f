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
// A^T row i in order (rows r of A ascending), valT[k] * A(r, c) into column c.
// Same sums with the row held in registers: the row's columns and accumulators are
// WMAX-wide register arrays (unrolled compare-select, no dynamic indexing); every
// product t * A(r, c) is rounded and added to its column's accumulator in the order of
// the reference loop, so the result is bitwise that of computeATA. Rows longer than
// WMAX take the merge loop above. sliceOff != nullptr writes the SELL-64 layout of the
// A^T A pattern (sell_* below) instead of CSR.
template <typename T, int WMAX>
__global__ __launch_bounds__(kBlock) void ata_values_reg(int cols, const int* __restrict__ rowPtrA,
                                                         const int* __restrict__ colIndA, const T* __restrict__ valA,
                                                         const int* __restrict__ rowPtrT,
                                                         const int* __restrict__ colIndT, const T* __restrict__ valT,
                                                         const int* __restrict__ rowPtrATA,
                                                         const int* __restrict__ colIndATA, T* __restrict__ valATA,
                                                         const int* __restrict__ sliceOff) {
#pragma clang fp contract(off)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += gridDim.x * blockDim.x) {
        const int b = rowPtrATA[i], n = rowPtrATA[i + 1] - b;
        // output position of the row's l-th entry
        const long long ob = sliceOff ? (long long)sliceOff[i >> 6] + (i & 63) : b;
        const int os = sliceOff ? 64 : 1;
        if (n > WMAX) {
            for (int l = 0; l < n; ++l) valATA[ob + (long long)l * os] = (T)0;
            for (int k = rowPtrT[i]; k < rowPtrT[i + 1]; ++k) {
                const T t = valT[k];
                const int r = colIndT[k];
                int ci = rowPtrA[r];
                const int ce = rowPtrA[r + 1];
                for (int l = 0; l < n && ci < ce; ++l) {
                    if (colIndATA[b + l] == colIndA[ci]) {
                        const long long o = ob + (long long)l * os;
                        valATA[o] = valATA[o] + t * valA[ci];
                        ++ci;
                    }
                }
            }
            continue;
        }
        int cix[WMAX];
        T acc[WMAX];
#pragma unroll
        for (int l = 0; l < WMAX; ++l) {
            cix[l] = l < n ? colIndATA[b + l] : -1;
            acc[l] = (T)0;
        }
        for (int k = rowPtrT[i]; k < rowPtrT[i + 1]; ++k) {
            const T t = valT[k];
            const int r = colIndT[k];
            for (int j = rowPtrA[r]; j < rowPtrA[r + 1]; ++j) {
                const int c = colIndA[j];
                const T v = t * valA[j];
#pragma unroll
                for (int l = 0; l < WMAX; ++l)
                    if (cix[l] == c) acc[l] = acc[l] + v;
            }
        }
#pragma unroll
        for (int l = 0; l < WMAX; ++l)
            if (l < n) valATA[ob + (long long)l * os] = acc[l];
    }
}

// ---- A^T A product map: for every A^T A entry, the (J(r,i), J(r,c)) position pairs
// whose products sum to it, rows r ascending (computeATA's order). Built once per
// pattern; the per-step values are then pure gathers (no dependent index chains).
template <int WMAX, bool FILL>
__global__ __launch_bounds__(kBlock) void prod_map(int cols, const int* __restrict__ rowPtrA,
                                                   const int* __restrict__ colIndA, const int* __restrict__ rowPtrT,
                                                   const int* __restrict__ colIndT, const int* __restrict__ perm,
                                                   const int* __restrict__ rowPtrATA,
                                                   const int* __restrict__ colIndATA, long long* __restrict__ cnt,
                                                   int2* __restrict__ pairs, int* __restrict__ cursor) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < cols; i += gridDim.x * blockDim.x) {
        const int b = rowPtrATA[i], n = rowPtrATA[i + 1] - b;
        if (n <= WMAX) {
            int cix[WMAX], cur[WMAX];
            long long o[WMAX];
#pragma unroll
            for (int l = 0; l < WMAX; ++l) {
                cix[l] = l < n ? colIndATA[b + l] : -1;
                cur[l] = 0;
                o[l] = (FILL && l < n) ? cnt[b + l] : 0;
            }
            for (int k = rowPtrT[i]; k < rowPtrT[i + 1]; ++k) {
                const int r = colIndT[k], p1 = perm[k];
                for (int j = rowPtrA[r]; j < rowPtrA[r + 1]; ++j) {
                    const int c = colIndA[j];
#pragma unroll
                    for (int l = 0; l < WMAX; ++l)
                        if (cix[l] == c) {
                            if (FILL) pairs[o[l] + cur[l]] = make_int2(p1, j);
                            ++cur[l];
                        }
                }
            }
            if (!FILL) {
#pragma unroll
                for (int l = 0; l < WMAX; ++l)
                    if (l < n) cnt[b + l] = cur[l];
            }
        } else {   // long rows: cursors in global memory (this thread owns the row)
            for (int l = 0; l < n; ++l) cursor[b + l] = 0;
            for (int k = rowPtrT[i]; k < rowPtrT[i + 1]; ++k) {
                const int r = colIndT[k], p1 = perm[k];
                for (int j = rowPtrA[r]; j < rowPtrA[r + 1]; ++j) {
                    const int c = colIndA[j];
                    int lo = 0, hi = n - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (colIndATA[b + mid] < c) lo = mid + 1;
                        else hi = mid;
                    }
                    if (FILL) pairs[cnt[b + lo] + cursor[b + lo]] = make_int2(p1, j);
                    ++cursor[b + lo];
                }
            }
            if (!FILL)
                for (int l = 0; l < n; ++l) cnt[b + l] = cursor[b + l];
        }
    }
}
// SELL layout of the product map: the slots of the A^T A SELL copy come in groups of
// 64 (one slice column); group g stores its pairs column-major, pair m of lane l at
// gbase[g] + 64 m + l, padded to the group's deepest list with (-1, -1).
__global__ __launch_bounds__(kBlock) void pair_depth(long long padded, const int* __restrict__ pos,
                                                     const long long* __restrict__ off, long long* __restrict__ depth) {
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < padded;
         q += (long long)gridDim.x * blockDim.x) {
        const int k = pos[q];
        int c = k >= 0 ? (int)(off[k + 1] - off[k]) : 0;
        for (int o = 32; o > 0; o >>= 1) c = max(c, __shfl_xor(c, o, 64));
        if ((q & 63) == 0) depth[q >> 6] = 64LL * c;
    }
}
__global__ __launch_bounds__(kBlock) void pair_fill(long long padded, const int* __restrict__ pos,
                                                    const long long* __restrict__ off, const int2* __restrict__ pairs,
                                                    const long long* __restrict__ gbase, int2* __restrict__ out) {
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < padded;
         q += (long long)gridDim.x * blockDim.x) {
        const long long g = q >> 6, b = gbase[g];
        const int d = (int)((gbase[g + 1] - b) >> 6), lane = (int)(q & 63);
        const int k = pos[q];
        const int c = k >= 0 ? (int)(off[k + 1] - off[k]) : 0;
        for (int m = 0; m < d; ++m) out[b + 64LL * m + lane] = m < c ? pairs[off[k] + m] : make_int2(-1, -1);
    }
}
// Per step: every SELL slot of A^T A = its products summed in order (bitwise computeATA).
template <typename T>
__global__ __launch_bounds__(kBlock) void ata_from_pairs(long long padded, const long long* __restrict__ gbase,
                                                         const int2* __restrict__ pairs, const T* __restrict__ valA,
                                                         T* __restrict__ out) {
#pragma clang fp contract(off)
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < padded;
         q += (long long)gridDim.x * blockDim.x) {
        const long long g = q >> 6, b = gbase[g];
        const int d = (int)((gbase[g + 1] - b) >> 6), lane = (int)(q & 63);
        const int2* pr = pairs + b + lane;
        T acc = 0;
        int m = 0;
        for (; m + 2 <= d; m += 2) {
            const int2 a0 = pr[64 * m], a1 = pr[64 * (m + 1)];
            const T x0 = a0.x >= 0 ? valA[a0.x] : (T)0, y0 = a0.x >= 0 ? valA[a0.y] : (T)0;
            const T x1 = a1.x >= 0 ? valA[a1.x] : (T)0, y1 = a1.x >= 0 ? valA[a1.y] : (T)0;
            if (a0.x >= 0) acc = acc + x0 * y0;
            if (a1.x >= 0) acc = acc + x1 * y1;
        }
        if (m < d) {
            const int2 a0 = pr[64 * m];
            if (a0.x >= 0) acc = acc + valA[a0.x] * valA[a0.y];
        }
        out[q] = acc;
    }
}

// ---- SELL-64: rows in slices of one wavefront, column-major inside a slice --------
__global__ __launch_bounds__(kBlock) void sell_widths(int rows, int nslices, const int* __restrict__ rowPtr,
                                                      long long* __restrict__ off) {
    for (int sl = blockIdx.x * blockDim.x + threadIdx.x; sl < nslices; sl += gridDim.x * blockDim.x) {
        int w = 0;
        const int r1 = min(rows, sl * 64 + 64);
        for (int r = sl * 64; r < r1; ++r) w = max(w, rowPtr[r + 1] - rowPtr[r]);
        off[sl] = 64LL * w;
    }
}
__global__ __launch_bounds__(kBlock) void sell_fill(int rows, int nslices, const int* __restrict__ rowPtr,
                                                    const int* __restrict__ colInd, const long long* __restrict__ off,
                                                    int* __restrict__ sliceOff, int* __restrict__ col,
                                                    int* __restrict__ pos) {
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < 64LL * nslices;
         t += (long long)gridDim.x * blockDim.x) {
        const int sl = (int)(t >> 6), lane = (int)(t & 63), r = (int)t;
        const long long o = off[sl];
        const int w = (int)((off[sl + 1] - o) >> 6);
        if (lane == 0) sliceOff[sl] = (int)o;
        if (t == 0) sliceOff[nslices] = (int)off[nslices];
        const int b = r < rows ? rowPtr[r] : 0, len = r < rows ? rowPtr[r + 1] - b : 0;
        for (int j = 0; j < w; ++j) {
            const long long q = o + (long long)j * 64 + lane;
            col[q] = j < len ? colInd[b + j] : 0;
            pos[q] = j < len ? b + j : -1;
        }
    }
}
template <typename T>
__global__ __launch_bounds__(kBlock) void sell_gather(long long n, const int* __restrict__ pos,
                                                      const T* __restrict__ val, T* __restrict__ out) {
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
        const int k = pos[q];
        out[q] = k >= 0 ? val[k] : (T)0;
    }
}
__global__ __launch_bounds__(kBlock) void compose(long long n, const int* __restrict__ pos,
                                                  const int* __restrict__ perm, int* __restrict__ out) {
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
        const int k = pos[q];
        out[q] = k >= 0 ? perm[k] : -1;
    }
}

// y = A x over SELL-64: one lane per row, one wavefront per slice; every row summed in
// column order with rounded products (applyAtoVector's order: bitwise its result).
// PCG: y masked to the active unknowns and sum pv.y reduced (PCGStep1_Finish).
template <typename T, bool PCG>
__global__ __launch_bounds__(kBlock) void sell_spmv(int rows, int nslices, const int* __restrict__ sliceOff,
                                                    const int* __restrict__ col, const T* __restrict__ val,
                                                    const T* __restrict__ x, T* __restrict__ y,
                                                    const T* __restrict__ pv, PcgMask m, ReduceSlot rs) {
#pragma clang fp contract(off)
    if (PCG && stopped(m.stop)) return;
    const int lane = threadIdx.x & 63;
    const int nwaves = gridDim.x * (kBlock / 64);
    T dot = 0;
    // plain interleaved slices: an XCD-contiguous split measured slower here (the +-W
    // neighbours are only 2W elements away and stay L2/MALL-resident either way)
    for (int sl = __builtin_amdgcn_readfirstlane((blockIdx.x * kBlock + threadIdx.x) >> 6); sl < nslices;
         sl += nwaves) {
        const int o = sliceOff[sl], w = (sliceOff[sl + 1] - o) >> 6;
        const int* c = col + o + lane;
        const T* v = val + o + lane;
        T acc = 0;
        int j = 0;
        for (; j + 4 <= w; j += 4) {
            const int c0 = c[64 * j], c1 = c[64 * (j + 1)], c2 = c[64 * (j + 2)], c3 = c[64 * (j + 3)];
            const T v0 = v[64 * j], v1 = v[64 * (j + 1)], v2 = v[64 * (j + 2)], v3 = v[64 * (j + 3)];
            const T x0 = x[c0], x1 = x[c1], x2 = x[c2], x3 = x[c3];
            acc = acc + x0 * v0;
            acc = acc + x1 * v1;
            acc = acc + x2 * v2;
            acc = acc + x3 * v3;
        }
        for (; j < w; ++j) acc = acc + x[c[64 * j]] * v[64 * j];
        const int r = sl * 64 + lane;
        if (r < rows) {
            if (PCG) {
                int k = 0;   // element -> pixel (32-bit: the vector is < 2^31 long)
                while (k + 1 < m.L.nimg && r >= m.L.off[k + 1]) ++k;
                const long long px = (r - (int)m.L.off[k]) / m.L.ch[k];
                const bool act = px >= m.pix_lo && px < m.pix_hi && (m.flags[px] & 1);
                if (!act) acc = 0;
                dot += pv[r] * acc;
            }
            y[r] = acc;
        }
    }
    if (PCG) {
        double d[1] = {(double)dot};
        block_reduce_publish<1>(d, rs, blockIdx.x);
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
#pragma clang fp contract(off)
    const int lg = threadIdx.x & (G - 1);
    const long long ngroups = (long long)gridDim.x * (kBlock / G);
    for (long long r = ((long long)blockIdx.x * kBlock + threadIdx.x) / G; r < rows; r += ngroups) {
        const int b = rowPtr[r], e = rowPtr[r + 1];
        T acc = 0;
        for (int k = b + lg; k < e; k += G) acc = acc + x[colInd[k]] * val[k];
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
    hipLaunchKernelGGL((csr::ata_values_reg<T, 16>), dim3(csr::grid_for(cols)), dim3(kBlock), 0, s, cols, rowPtrA,
                       colIndA, valA, rowPtrT, colIndT, valT, rowPtrATA, colIndATA, valATA, (const int*)nullptr);
    OPT_HIP_CHECK(hipGetLastError());
}

template <typename T>
void csr_spmv(int rows, long long nnz, const int* rowPtr, const int* colInd, const T* val, const T* x, T* y,
              hipStream_t s) {
    // one lane per row, entries in order with rounded products: bitwise applyAtoVector
    if (rows == 0) return;
    (void)nnz;
    hipLaunchKernelGGL((csr::spmv<T, 1>), dim3(csr::grid_for(rows)), dim3(kBlock), 0, s, rows, rowPtr, colInd, val, x,
                       y);
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

// ---- SELL-64 host side ------------------------------------------------------------
void sell_build(int rows, const int* rowPtr, const int* colInd, SellMatrix& S, DevBuf& scratch, hipStream_t s) {
    S.release();
    S.rows = rows;
    S.nslices = (rows + 63) / 64;
    long long* off = (long long*)dmalloc(sizeof(long long) * (S.nslices + 1));
    OPT_HIP_CHECK(hipMemsetAsync(off + S.nslices, 0, sizeof(long long), s));
    hipLaunchKernelGGL(csr::sell_widths, dim3(csr::grid_for(S.nslices)), dim3(kBlock), 0, s, rows, S.nslices, rowPtr,
                       off);
    size_t need = 0;
    OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, off, off, S.nslices + 1, s));
    OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scratch.need(need), need, off, off, S.nslices + 1, s));
    OPT_HIP_CHECK(hipMemcpyAsync(&S.padded, off + S.nslices, sizeof(long long), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    if (S.padded >= (1LL << 31) - 1) {
        fprintf(stderr, "[opt_amd] SELL-64 layout of %d rows exceeds 2^31 padded entries\n", rows);
        exit(1);
    }
    S.sliceOff = (int*)dmalloc(sizeof(int) * (S.nslices + 1));
    S.col = (int*)dmalloc(sizeof(int) * std::max(S.padded, 1LL));
    S.pos = (int*)dmalloc(sizeof(int) * std::max(S.padded, 1LL));
    hipLaunchKernelGGL(csr::sell_fill, dim3(csr::grid_for(64LL * S.nslices)), dim3(kBlock), 0, s, rows, S.nslices,
                       rowPtr, colInd, (const long long*)off, S.sliceOff, S.col, S.pos);
    OPT_HIP_CHECK(hipGetLastError());
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    dfree(off);
}
void sell_compose(SellMatrix& S, const int* perm, hipStream_t s) {
    if (S.padded == 0) return;
    hipLaunchKernelGGL(csr::compose, dim3(csr::grid_for(S.padded)), dim3(kBlock), 0, s, S.padded, (const int*)S.pos,
                       perm, S.pos);
    OPT_HIP_CHECK(hipGetLastError());
}
template <typename T>
void sell_values(const SellMatrix& S, const T* csrVal, T* sellVal, hipStream_t s) {
    if (S.padded == 0) return;
    hipLaunchKernelGGL((csr::sell_gather<T>), dim3(csr::grid_for(S.padded)), dim3(kBlock), 0, s, S.padded,
                       (const int*)S.pos, csrVal, sellVal);
    OPT_HIP_CHECK(hipGetLastError());
}
template <typename T>
void ata_values_sell(int cols, const int* rowPtrA, const int* colIndA, const T* valA, const int* rowPtrT,
                     const int* colIndT, const T* valT, const int* rowPtrATA, const int* colIndATA,
                     const SellMatrix& S, T* sellVal, hipStream_t s) {
    if (S.padded == 0) return;
    OPT_HIP_CHECK(hipMemsetAsync(sellVal, 0, sizeof(T) * S.padded, s));   // padding stays 0
    hipLaunchKernelGGL((csr::ata_values_reg<T, 16>), dim3(csr::grid_for(cols)), dim3(kBlock), 0, s, cols, rowPtrA,
                       colIndA, valA, rowPtrT, colIndT, valT, rowPtrATA, colIndATA, sellVal,
                       (const int*)S.sliceOff);
    OPT_HIP_CHECK(hipGetLastError());
}
void ata_products_build(int cols, const int* rowPtrA, const int* colIndA, const int* rowPtrT, const int* colIndT,
                        const int* perm, const int* rowPtrATA, const int* colIndATA, long long nnzATA,
                        const SellMatrix& S, AtaProducts& P, DevBuf& scratch, hipStream_t s) {
    P.release();
    P.n = nnzATA;
    P.off = (long long*)dmalloc(sizeof(long long) * (nnzATA + 1));
    int* cursor = (int*)dmalloc(sizeof(int) * std::max(nnzATA, 1LL));
    OPT_HIP_CHECK(hipMemsetAsync(P.off, 0, sizeof(long long) * (nnzATA + 1), s));
    const dim3 g(csr::grid_for(cols)), b(kBlock);
    hipLaunchKernelGGL((csr::prod_map<16, false>), g, b, 0, s, cols, rowPtrA, colIndA, rowPtrT, colIndT, perm,
                       rowPtrATA, colIndATA, P.off, (int2*)nullptr, cursor);
    size_t need = 0;
    OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, P.off, P.off, nnzATA + 1, s));
    OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scratch.need(need), need, P.off, P.off, nnzATA + 1, s));
    OPT_HIP_CHECK(hipMemcpyAsync(&P.npairs, P.off + nnzATA, sizeof(long long), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    P.pairs = (int2*)dmalloc(sizeof(int2) * std::max(P.npairs, 1LL));
    hipLaunchKernelGGL((csr::prod_map<16, true>), g, b, 0, s, cols, rowPtrA, colIndA, rowPtrT, colIndT, perm,
                       rowPtrATA, colIndATA, P.off, P.pairs, cursor);
    OPT_HIP_CHECK(hipGetLastError());
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    dfree(cursor);
    // regroup into the SELL layout of the A^T A copy (see pair_fill)
    const long long G = S.padded / 64;
    P.padded = S.padded;
    P.gbase = (long long*)dmalloc(sizeof(long long) * (G + 1));
    OPT_HIP_CHECK(hipMemsetAsync(P.gbase + G, 0, sizeof(long long), s));
    hipLaunchKernelGGL(csr::pair_depth, dim3(csr::grid_for(S.padded)), dim3(kBlock), 0, s, S.padded,
                       (const int*)S.pos, (const long long*)P.off, P.gbase);
    need = 0;
    OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, P.gbase, P.gbase, G + 1, s));
    OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scratch.need(need), need, P.gbase, P.gbase, G + 1, s));
    long long total = 0;
    OPT_HIP_CHECK(hipMemcpyAsync(&total, P.gbase + G, sizeof(total), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    int2* sp = (int2*)dmalloc(sizeof(int2) * std::max(total, 1LL));
    hipLaunchKernelGGL(csr::pair_fill, dim3(csr::grid_for(S.padded)), dim3(kBlock), 0, s, S.padded,
                       (const int*)S.pos, (const long long*)P.off, (const int2*)P.pairs, (const long long*)P.gbase, sp);
    OPT_HIP_CHECK(hipGetLastError());
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    dfree(P.pairs);
    dfree(P.off);
    P.off = nullptr;
    P.pairs = sp;
    P.npairs = total;
}
template <typename T>
void ata_values_products(const AtaProducts& P, const T* valA, T* out, hipStream_t s) {
    if (P.padded == 0) return;
    hipLaunchKernelGGL((csr::ata_from_pairs<T>), dim3(csr::grid_for(P.padded)), dim3(kBlock), 0, s, P.padded,
                       (const long long*)P.gbase, (const int2*)P.pairs, valA, out);
    OPT_HIP_CHECK(hipGetLastError());
}

int sell_blocks(const SellMatrix& S) { return csr::grid_for((long long)S.nslices, kBlock / 64); }
template <typename T>
void sell_spmv(const SellMatrix& S, const T* val, const T* x, T* y, hipStream_t s) {
    if (S.rows == 0) return;
    hipLaunchKernelGGL((csr::sell_spmv<T, false>), dim3(sell_blocks(S)), dim3(kBlock), 0, s, S.rows, S.nslices,
                       (const int*)S.sliceOff, (const int*)S.col, val, x, y, (const T*)nullptr, PcgMask{},
                       ReduceSlot{});
    OPT_HIP_CHECK(hipGetLastError());
}
template <typename T>
void sell_spmv_pcg(const SellMatrix& S, const T* val, const T* x, T* y, const T* pv, const PcgMask& m, ReduceSlot rs,
                   hipStream_t s) {
    hipLaunchKernelGGL((csr::sell_spmv<T, true>), dim3(sell_blocks(S)), dim3(kBlock), 0, s, S.rows, S.nslices,
                       (const int*)S.sliceOff, (const int*)S.col, val, x, y, pv, m, rs);
    OPT_HIP_CHECK(hipGetLastError());
}

#define INST(T)                                                                                                  \
    template void csr_gather<T>(long long, const int*, const T*, T*, hipStream_t);                              \
    template void csr_ata_values<T>(int, const int*, const int*, const T*, const int*, const int*, const T*,     \
                                    const int*, const int*, T*, hipStream_t);                                    \
    template void csr_spmv<T>(int, long long, const int*, const int*, const T*, const T*, T*, hipStream_t);      \
    template void csr_spmv_pcg<T>(int, long long, const int*, const int*, const T*, const T*, T*, const T*,      \
                                  const PcgMask&, ReduceSlot, hipStream_t);                                   \
    template void sell_values<T>(const SellMatrix&, const T*, T*, hipStream_t);                                 \
    template void ata_values_sell<T>(int, const int*, const int*, const T*, const int*, const int*, const T*,    \
                                     const int*, const int*, const SellMatrix&, T*, hipStream_t);                \
    template void sell_spmv<T>(const SellMatrix&, const T*, const T*, T*, hipStream_t);                         \
    template void ata_values_products<T>(const AtaProducts&, const T*, T*, hipStream_t);                        \
    template void sell_spmv_pcg<T>(const SellMatrix&, const T*, const T*, T*, const T*, const PcgMask&,          \
                                   ReduceSlot, hipStream_t);
INST(float)
INST(double)
#undef INST

}  // namespace optamd
