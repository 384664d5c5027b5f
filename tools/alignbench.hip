// alignbench.hip — isolates the memory pattern of the image_warping stencil kernels:
// each wavefront walks T rows of a 64-lane column strip reading p(f2)+pt(f)+angle(f)
// +U(f2)+flags(u8) and writing Ap(f2)+Apt(f). Compares 62-output overlapped strips
// (x = 62s-1+lane, lanes 1..62 store) with 64-output aligned strips (x = 64s+lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int STRIP, bool COMPUTE>
__global__ __launch_bounds__(256) void walk(int W, int H, int rows, int nstrips, const float2* __restrict__ p,
                                            const float* __restrict__ pt, const float* __restrict__ ang,
                                            const float2* __restrict__ U, const uint8_t* __restrict__ fl,
                                            float2* __restrict__ Ap, float* __restrict__ Apt) {
    const int b = blockIdx.x;
    const int strip = b % nstrips, rb = b / nstrips;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int x = (STRIP == 62) ? strip * 62 - 1 + lane : strip * 64 + lane;
    const bool out = (STRIP == 62) ? (lane >= 1 && lane <= 62 && x < W) : (x < W);
    const int xc = x < 0 ? 0 : (x >= W ? W - 1 : x);
    const int y0 = (rb * 4 + w) * rows;
    float acc = 0.f;
    for (int y = y0; y < y0 + rows && y < H; ++y) {
        const long long i = (long long)y * W + xc;
        const float2 pp = p[i];
        const float q = pt[i], a = ang[i];
        const float2 u = U[i];
        const int f = fl[i];
        float r0 = pp.x * u.x + a, r1 = pp.y * u.y + q;
        if (COMPUTE) {
#pragma unroll
            for (int k = 0; k < 40; ++k) { r0 = r0 * 0.999f + r1; r1 = r1 * 0.998f - r0; }
        }
        if (out) {
            Ap[i] = make_float2(r0, r1);
            Apt[i] = (float)f + r0 * r1;
        }
        acc += r0;
    }
    if (acc == 1234.5f) Apt[0] = acc;
}

int main() {
    const int W = 4096, H = 4096;
    const long long N = (long long)W * H;
    float2 *p, *U, *Ap; float *pt, *ang, *Apt; uint8_t* fl;
    CK(hipMalloc(&p, N * 8)); CK(hipMalloc(&U, N * 8)); CK(hipMalloc(&Ap, N * 8));
    CK(hipMalloc(&pt, N * 4)); CK(hipMalloc(&ang, N * 4)); CK(hipMalloc(&Apt, N * 4)); CK(hipMalloc(&fl, N));
    CK(hipMemset(p, 0, N * 8)); CK(hipMemset(U, 0, N * 8)); CK(hipMemset(pt, 0, N * 4)); CK(hipMemset(ang, 0, N * 4));
    CK(hipMemset(fl, 1, N));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double bytes = 37.0 * N;
    for (int rows : {8, 16, 32}) {
        auto run = [&](const char* nm, auto kern, int strip) {
            const int nstrips = (W + strip - 1) / strip;
            const int nrb = (H + 4 * rows - 1) / (4 * rows);
            const int nb = nstrips * nrb;
            for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, 0, W, H, rows, nstrips, p, pt, ang, U, fl, Ap, Apt);
            CK(hipEventRecord(e0));
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, 0, W, H, rows, nstrips, p, pt, ang, U, fl, Ap, Apt);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            printf("rows=%2d %-22s %8.1f us %7.0f GB/s\n", rows, nm, ms * 1000 / 20, bytes / (ms / 20 * 1e-3) / 1e9);
            return 0;
        };
        run("62-overlap", walk<62, false>, 62);
        run("64-aligned", walk<64, false>, 64);
        run("62-overlap+alu", walk<62, true>, 62);
        run("64-aligned+alu", walk<64, true>, 64);
    }
    return 0;
}
