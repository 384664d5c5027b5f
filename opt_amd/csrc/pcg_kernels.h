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

// Step2 of iteration i (alpha = rz[i] / pAp[i]):
//   delta (+)= alpha p;  r -= alpha Ap;  z = pre r (or r when UsePreconditioner(false),
//   solverGPUGaussNewton.t:705-708);  rz[i+1] = sum z.r.
// z is not stored: the next apply kernel rebuilds p = z + beta p from r and pre.
// Excluded unknowns hold p = Ap = r = pre = 0, so the flat stream leaves them 0.
template <typename T, bool FIRST>
__global__ __launch_bounds__(kBlock) void pcg_step2_kernel(
    long long n, const T* __restrict__ p, const T* __restrict__ Ap, const T* __restrict__ pre,
    T* __restrict__ r, T* __restrict__ delta, const double* __restrict__ sc, int i_num, int i_den,
    int use_pre, ReduceSlot rs) {
    const T alpha = (T)(sc[i_num] / sc[i_den]);
    T acc = 0;
    const long long n4 = n / 4;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += stride) {
        const long long e = q * 4;
        V4<T> pv = ld4(p + e), av = ld4(Ap + e), rv = ld4(r + e), wv = ld4(pre + e);
        V4<T> dv;
        if (FIRST) {
            dv = {alpha * pv.a, alpha * pv.b, alpha * pv.c, alpha * pv.d};
        } else {
            dv = ld4(delta + e);
            dv.a += alpha * pv.a; dv.b += alpha * pv.b; dv.c += alpha * pv.c; dv.d += alpha * pv.d;
        }
        rv.a -= alpha * av.a; rv.b -= alpha * av.b; rv.c -= alpha * av.c; rv.d -= alpha * av.d;
        st4(delta + e, dv);
        st4(r + e, rv);
        if (use_pre)
            acc += wv.a * rv.a * rv.a + wv.b * rv.b * rv.b + wv.c * rv.c * rv.c + wv.d * rv.d * rv.d;
        else
            acc += rv.a * rv.a + rv.b * rv.b + rv.c * rv.c + rv.d * rv.d;
    }
    // tail (n not a multiple of 4): handled by block 0
    if (blockIdx.x == 0) {
        for (long long e = n4 * 4 + threadIdx.x; e < n; e += blockDim.x) {
            T d = FIRST ? alpha * p[e] : delta[e] + alpha * p[e];
            T rr = r[e] - alpha * Ap[e];
            delta[e] = d;
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
