// pcg_kernels.h — family-independent PCG vector kernels over the flat unknown
// vector (reference kernels.PCGStep2 / PCGStep3 / PCGLinearUpdate,
// API/src/solverGPUGaussNewton.t:665-731, 814-859). These are pure HBM streams:
// 16-byte vector loads per lane, a grid capped at a few blocks per CU with a
// grid-stride loop, and the deterministic block->last-arriver reduction.
#pragma once
#include "common.h"

namespace optamd {

template <typename T> struct V4 { T a, b, c, d; };

template <typename T>
__device__ __forceinline__ V4<T> ld4(const T* p) { return *reinterpret_cast<const V4<T>*>(p); }
template <typename T>
__device__ __forceinline__ void st4(T* p, const V4<T>& v) { *reinterpret_cast<V4<T>*>(p) = v; }
// Streaming (nontemporal) forms for once-touched vectors: +12-15 % on MI355X for the
// 3-read/1-write PCG update shape at 1-8 K blocks (tools/streambench.hip).
template <typename T>
__device__ __forceinline__ V4<T> ld4nt(const T* p) {
    V4<T> v;
    v.a = __builtin_nontemporal_load(p); v.b = __builtin_nontemporal_load(p + 1);
    v.c = __builtin_nontemporal_load(p + 2); v.d = __builtin_nontemporal_load(p + 3);
    return v;
}
template <typename T>
__device__ __forceinline__ void st4nt(T* p, const V4<T>& v) {
    __builtin_nontemporal_store(v.a, p); __builtin_nontemporal_store(v.b, p + 1);
    __builtin_nontemporal_store(v.c, p + 2); __builtin_nontemporal_store(v.d, p + 3);
}

// PCGStep2 of iteration i, residual half (alpha = rz[i] / pAp[i]):
//   r -= alpha Ap;  z = pre r (or r when UsePreconditioner(false),
//   solverGPUGaussNewton.t:705-708);  rz[i+1] = sum z.r.
// The delta half (delta += alpha p) runs inside the next apply kernel, which reads
// p anyway; z is not stored: the next apply rebuilds p = z + beta p from r and pre.
// Excluded unknowns hold Ap = r = pre = 0, so the flat stream leaves them 0.
template <typename T>
__global__ __launch_bounds__(kBlock) void pcg_residual_kernel(
    long long n, const T* __restrict__ Ap, const T* __restrict__ pre, T* __restrict__ r,
    const double* __restrict__ sc, int i_num, int i_den, int use_pre, ReduceSlot rs) {
    const T alpha = (T)(sc[i_num] / sc[i_den]);
    T acc = 0;
    const long long n4 = n / 4;
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    // two independent 16-B groups per thread per trip keep 6 loads in flight
    for (; q + stride < n4; q += 2 * stride) {
        const long long e0 = q * 4, e1 = (q + stride) * 4;
        V4<T> a0 = ld4nt(Ap + e0), w0 = ld4nt(pre + e0), r0 = ld4nt(r + e0);
        V4<T> a1 = ld4nt(Ap + e1), w1 = ld4nt(pre + e1), r1 = ld4nt(r + e1);
        r0.a -= alpha * a0.a; r0.b -= alpha * a0.b; r0.c -= alpha * a0.c; r0.d -= alpha * a0.d;
        r1.a -= alpha * a1.a; r1.b -= alpha * a1.b; r1.c -= alpha * a1.c; r1.d -= alpha * a1.d;
        st4nt(r + e0, r0);
        st4nt(r + e1, r1);
        if (use_pre)
            acc += (w0.a * r0.a * r0.a + w0.b * r0.b * r0.b + w0.c * r0.c * r0.c + w0.d * r0.d * r0.d) +
                   (w1.a * r1.a * r1.a + w1.b * r1.b * r1.b + w1.c * r1.c * r1.c + w1.d * r1.d * r1.d);
        else
            acc += (r0.a * r0.a + r0.b * r0.b + r0.c * r0.c + r0.d * r0.d) +
                   (r1.a * r1.a + r1.b * r1.b + r1.c * r1.c + r1.d * r1.d);
    }
    for (; q < n4; q += stride) {
        const long long e = q * 4;
        V4<T> av = ld4(Ap + e), wv = ld4(pre + e), rv = ld4(r + e);
        rv.a -= alpha * av.a; rv.b -= alpha * av.b; rv.c -= alpha * av.c; rv.d -= alpha * av.d;
        st4(r + e, rv);
        if (use_pre)
            acc += wv.a * rv.a * rv.a + wv.b * rv.b * rv.b + wv.c * rv.c * rv.c + wv.d * rv.d * rv.d;
        else
            acc += rv.a * rv.a + rv.b * rv.b + rv.c * rv.c + rv.d * rv.d;
    }
    // tail (n not a multiple of 4): block 0
    if (blockIdx.x == 0) {
        for (long long e = n4 * 4 + threadIdx.x; e < n; e += blockDim.x) {
            const T rr = r[e] - alpha * Ap[e];
            r[e] = rr;
            acc += use_pre ? pre[e] * rr * rr : rr * rr;
        }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// Grid for the flat streams: enough blocks for ~8 per CU, never more than the work.
inline int flat_grid(long long n, int vec = 4) {
    long long need = (n / vec + kBlock - 1) / kBlock;
    if (need < 1) need = 1;
    return (int)std::min<long long>(need, 2048);
}

}  // namespace optamd
