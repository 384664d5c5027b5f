// graph_util.h — content fingerprint of a graph's vertex arrays.
//
// Both graph paths (arap.hip, generic.hip) build per-vertex incidence lists once and reuse
// them across Steps. The reference re-reads the edge arrays in every kernel
// (problemparams are re-read on every Step, solverGPUGaussNewton.t:2001), so a caller may
// pass different edges at any Step — possibly at the address of a freed earlier array
// (allocators reuse addresses). A pointer comparison is therefore not enough: every bind
// hashes the arrays' contents on the device (one streaming pass per array)
// and the incidence lists are rebuilt when the hash changes.
#pragma once
#include <algorithm>
#include "common.h"

namespace optamd {

// splitmix64's finaliser of (position, value, salt): a full 64-bit mix per entry, so two
// different edge lists collide with probability ~2^-64 (a 32-bit mix per entry would leave
// ~2^-32 once two or more entries change).
__device__ __forceinline__ unsigned long long fp_mix(unsigned v, unsigned e, unsigned long long salt) {
    unsigned long long x = (((unsigned long long)e << 32) | v) ^ salt;
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// Position-keyed sum of 64-bit mixes (order-independent, so the block sums can meet in
// one place): 16-byte loads, a streaming pass at HBM rate.
// VEC = false: an array that is not 16-byte aligned, read as four 4-byte loads.
template <bool VEC>
static __global__ void graph_fingerprint_kernel(const int* __restrict__ v, int E, unsigned long long salt,
                                                unsigned long long* parts) {
    unsigned long long h = 0;
    const int n4 = E / 4;
    const int4* v4 = reinterpret_cast<const int4*>(v);
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += gridDim.x * blockDim.x) {
        const int4 w = VEC ? v4[q] : int4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
        const unsigned e = 4u * (unsigned)q;
        h += fp_mix((unsigned)w.x, e, salt) + fp_mix((unsigned)w.y, e + 1, salt) +
             fp_mix((unsigned)w.z, e + 2, salt) + fp_mix((unsigned)w.w, e + 3, salt);
    }
    if (blockIdx.x == 0 && (int)threadIdx.x < E - 4 * n4)   // the tail
        h += fp_mix((unsigned)v[4 * n4 + threadIdx.x], 4u * n4 + threadIdx.x, salt);
    for (int off = 32; off > 0; off >>= 1) h += __shfl_down(h, off, 64);
    __shared__ unsigned long long part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
    __syncthreads();
    // one partial per block (a single hot atomic costs ~12 ns per add: 4096 blocks would
    // serialise ~50 us on it); graph_fingerprint_sum adds them up
    if (threadIdx.x == 0) parts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}
static __global__ void graph_fingerprint_sum(const unsigned long long* __restrict__ parts, int n,
                                             unsigned long long* out) {
    unsigned long long h = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) h += parts[i];
    for (int off = 32; off > 0; off >>= 1) h += __shfl_down(h, off, 64);
    __shared__ unsigned long long part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) *out += part[0] + part[1] + part[2] + part[3];   // integer sum: order-free
}

constexpr int kFingerprintGrid = 2048;   // blocks per array (one partial each)
// Fingerprint of n vertex arrays of E entries each; `d` is device scratch of
// 1 + kFingerprintGrid words (synchronises `s`).
inline unsigned long long graph_fingerprint(const int* const* arrays, int n, int E, hipStream_t s,
                                            unsigned long long* d) {
    const int grid = std::max(1, std::min((E / 4 + 255) / 256, kFingerprintGrid));
    OPT_HIP_CHECK(hipMemsetAsync(d, 0, sizeof(unsigned long long), s));
    for (int k = 0; k < n; ++k)
        if (E > 0) {
            const unsigned long long salt = 0x9E3779B97F4A7C15ull * (unsigned long long)(k + 1);
            if ((reinterpret_cast<uintptr_t>(arrays[k]) & 15) == 0)
                hipLaunchKernelGGL(graph_fingerprint_kernel<true>, dim3(grid), dim3(256), 0, s, arrays[k], E, salt,
                                   d + 1);
            else
                hipLaunchKernelGGL(graph_fingerprint_kernel<false>, dim3(grid), dim3(256), 0, s, arrays[k], E, salt,
                                   d + 1);
            hipLaunchKernelGGL(graph_fingerprint_sum, dim3(1), dim3(256), 0, s, (const unsigned long long*)(d + 1),
                               grid, d);
        }
    unsigned long long h = 0;
    OPT_HIP_CHECK(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    return h ^ ((unsigned long long)E << 1) ^ (unsigned long long)n;
}

}  // namespace optamd
