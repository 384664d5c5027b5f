// fetchcal.hip — calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE against known byte counts
// for the access widths the solver kernels use (1, 4, 8, 16 B per lane reads; 4, 8 B
// per lane writes), on arrays far larger than the 256 MiB Infinity Cache. Run under
// `rocprofv3 --pmc FETCH_SIZE` (and separately WRITE_SIZE); the program prints the
// bytes each kernel moves so the ratio can be read per kernel. Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename V>
__global__ __launch_bounds__(256) void read_k(long long n, const V* __restrict__ a, float* out) {
    float acc = 0.f;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const V v = a[i];
        const float* f = reinterpret_cast<const float*>(&v);
        if constexpr (sizeof(V) >= 4) for (int k = 0; k < (int)(sizeof(V) / 4); ++k) acc += f[k];
        else acc += (float)*reinterpret_cast<const unsigned char*>(&v);
    }
    if (acc == 12345.f) out[0] = acc;
}
template <typename V>
__global__ __launch_bounds__(256) void write_k(long long n, V* __restrict__ a) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        V v;
        float* f = reinterpret_cast<float*>(&v);
        for (int k = 0; k < (int)(sizeof(V) / 4); ++k) f[k] = (float)i;
        a[i] = v;
    }
}
struct F2 { float x, y; };
struct alignas(8) F2a { float x, y; };
struct alignas(16) F4a { float x, y, z, w; };

int main() {
    const size_t bytes = 1ull << 30;   // 1 GiB
    char* a;
    float* out;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 1, bytes));
    const int grid = 256 * 32;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(read_k<unsigned char>, grid, 256, 0, 0, (long long)bytes, (const unsigned char*)a, out);
        hipLaunchKernelGGL(read_k<float>, grid, 256, 0, 0, (long long)(bytes / 4), (const float*)a, out);
        hipLaunchKernelGGL(read_k<F2a>, grid, 256, 0, 0, (long long)(bytes / 8), (const F2a*)a, out);
        hipLaunchKernelGGL(read_k<F4a>, grid, 256, 0, 0, (long long)(bytes / 16), (const F4a*)a, out);
        hipLaunchKernelGGL(write_k<float>, grid, 256, 0, 0, (long long)(bytes / 4), (float*)a);
        hipLaunchKernelGGL(write_k<F2a>, grid, 256, 0, 0, (long long)(bytes / 8), (F2a*)a);
        hipLaunchKernelGGL(write_k<F4a>, grid, 256, 0, 0, (long long)(bytes / 16), (F4a*)a);
    }
    CK(hipDeviceSynchronize());
    printf("each kernel moves %zu bytes (%.1f KiB)\n", bytes, bytes / 1024.0);
    return 0;
}
