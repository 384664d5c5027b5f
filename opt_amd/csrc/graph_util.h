// graph_util.h — content fingerprint of a graph's vertex arrays.
//
// Both graph paths (arap.hip, generic.hip) build per-vertex incidence lists once and reuse
// them across Steps. The reference re-reads the edge arrays in every kernel
// (problemparams are re-read on every Step, solverGPUGaussNewton.t:2001), so a caller may
// pass different edges at any Step — possibly at the address of a freed earlier array
// (allocators reuse addresses). A pointer comparison is therefore not enough: every bind
// hashes the arrays' contents on the device (one streaming pass, ~10 µs per 6 M edges)
// and the incidence lists are rebuilt when the hash changes.
#pragma once
#include <algorithm>
#include "common.h"

namespace optamd {

static __global__ void graph_fingerprint_kernel(const int* __restrict__ v, int E, unsigned long long salt,
                                         unsigned long long* out) {
    unsigned long long h = 0;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < E; e += gridDim.x * blockDim.x) {
        unsigned long long x = ((unsigned long long)(unsigned)e << 32 | (unsigned)v[e]) ^ salt;
        x += 0x9E3779B97F4A7C15ull;   // splitmix64 finaliser
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        h += x ^ (x >> 31);
    }
    for (int off = 32; off > 0; off >>= 1) h += __shfl_down(h, off, 64);
    __shared__ unsigned long long part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, part[0] + part[1] + part[2] + part[3]);   // a sum: order-independent
}

// Fingerprint of n vertex arrays of E entries each; `d` is 8 bytes of device scratch
// (synchronises `s`).
inline unsigned long long graph_fingerprint(const int* const* arrays, int n, int E, hipStream_t s,
                                            unsigned long long* d) {
    OPT_HIP_CHECK(hipMemsetAsync(d, 0, sizeof(unsigned long long), s));
    const int grid = std::max(1, std::min((E + 255) / 256, 1024));   // one atomic per block
    for (int k = 0; k < n; ++k)
        if (E > 0)
            hipLaunchKernelGGL(graph_fingerprint_kernel, dim3(grid), dim3(256), 0, s, arrays[k], E,
                               0x5851F42D4C957F2Dull * (unsigned long long)(k + 1), d);
    unsigned long long h = 0;
    OPT_HIP_CHECK(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, s));
    OPT_HIP_CHECK(hipStreamSynchronize(s));
    return h ^ ((unsigned long long)E << 1) ^ (unsigned long long)n;
}

}  // namespace optamd
