// streambench.hip — HBM stream microbenchmark for the shapes of the PCG vector
// kernels (3 reads + 1 write with a reduction, like pcg r-update), to pick the
// launch/unroll/cache-policy of the flat kernels on MI355X. Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct F4 { float a, b, c, d; };

__device__ __forceinline__ F4 ld(const float* p) { return *reinterpret_cast<const F4*>(p); }
__device__ __forceinline__ void st(float* p, F4 v) { *reinterpret_cast<F4*>(p) = v; }
__device__ __forceinline__ F4 ldnt(const float* p) {
    F4 v;
    v.a = __builtin_nontemporal_load(p); v.b = __builtin_nontemporal_load(p + 1);
    v.c = __builtin_nontemporal_load(p + 2); v.d = __builtin_nontemporal_load(p + 3);
    return v;
}
__device__ __forceinline__ void stnt(float* p, F4 v) {
    __builtin_nontemporal_store(v.a, p); __builtin_nontemporal_store(v.b, p + 1);
    __builtin_nontemporal_store(v.c, p + 2); __builtin_nontemporal_store(v.d, p + 3);
}

__global__ void copy_k(long long n4, const float* __restrict__ a, float* __restrict__ b) {
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x)
        st(b + 4 * q, ld(a + 4 * q));
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void upd_k(long long n4, const float* __restrict__ Ap, const float* __restrict__ pre,
                                             float* __restrict__ r, float alpha, float* out) {
    float acc = 0.f;
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    for (; q + (U - 1) * stride < n4; q += U * stride) {
        F4 a[U], w[U], x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long e = 4 * (q + u * stride);
            a[u] = NT ? ldnt(Ap + e) : ld(Ap + e);
            w[u] = NT ? ldnt(pre + e) : ld(pre + e);
            x[u] = NT ? ldnt(r + e) : ld(r + e);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long e = 4 * (q + u * stride);
            x[u].a -= alpha * a[u].a; x[u].b -= alpha * a[u].b; x[u].c -= alpha * a[u].c; x[u].d -= alpha * a[u].d;
            if (NT) stnt(r + e, x[u]); else st(r + e, x[u]);
            acc += w[u].a * x[u].a * x[u].a + w[u].b * x[u].b * x[u].b + w[u].c * x[u].c * x[u].c + w[u].d * x[u].d * x[u].d;
        }
    }
    for (; q < n4; q += stride) {
        const long long e = 4 * q;
        F4 a = ld(Ap + e), w = ld(pre + e), x = ld(r + e);
        x.a -= alpha * a.a; x.b -= alpha * a.b; x.c -= alpha * a.c; x.d -= alpha * a.d;
        st(r + e, x);
        acc += w.a * x.a * x.a + w.b * x.b * x.b + w.c * x.c * x.c + w.d * x.d * x.d;
    }
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    const long long n = 3LL * 4096 * 4096;
    float *a, *b, *c, *out;
    CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&c, n * 4)); CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 0, n * 4)); CK(hipMemset(b, 0, n * 4)); CK(hipMemset(c, 0, n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const long long n4 = n / 4;
    auto run = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(e0));
        const int reps = 20;
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-34s %8.1f us  %7.0f GB/s\n", name, 1000.0 * ms / reps, bytes / (ms / reps * 1e-3) / 1e9);
        return 0;
    };
    const double cb = 2.0 * n * 4, ub = 4.0 * n * 4;
    for (int grid : {1024, 2048, 4096, 8192, (int)((n4 + 255) / 256)}) {
        char nm[64];
        snprintf(nm, 64, "copy grid=%d", grid);
        run(nm, cb, [&] { hipLaunchKernelGGL(copy_k, dim3(grid), dim3(256), 0, 0, n4, a, b); });
        snprintf(nm, 64, "upd U1 grid=%d", grid);
        run(nm, ub, [&] { hipLaunchKernelGGL((upd_k<1, false>), dim3(grid), dim3(256), 0, 0, n4, a, b, c, 0.5f, out); });
        snprintf(nm, 64, "upd U2 grid=%d", grid);
        run(nm, ub, [&] { hipLaunchKernelGGL((upd_k<2, false>), dim3(grid), dim3(256), 0, 0, n4, a, b, c, 0.5f, out); });
        snprintf(nm, 64, "upd U4 grid=%d", grid);
        run(nm, ub, [&] { hipLaunchKernelGGL((upd_k<4, false>), dim3(grid), dim3(256), 0, 0, n4, a, b, c, 0.5f, out); });
        snprintf(nm, 64, "upd U2 NT grid=%d", grid);
        run(nm, ub, [&] { hipLaunchKernelGGL((upd_k<2, true>), dim3(grid), dim3(256), 0, 0, n4, a, b, c, 0.5f, out); });
    }
    return 0;
}
