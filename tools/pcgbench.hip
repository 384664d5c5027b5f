// pcgbench.hip — memory-pattern microbenchmark for iw_pcg (round 5): the odd pass's loads
// (flag u8, UrShape f2, angle f, r f2 + f, angle pre f, p f2 + f: 41 B/px) and stores
// (r f2 + f, p f2 + f: 24 B/px) at 4096^2 with (almost) no arithmetic, in four traversals:
//   strip60   iw_pcg's: a wave walks a 60-column strip (x = 60 s - 2 + lane), rows y0-2 .. y1+1
//             loaded, rows y0 .. y1-1 stored at lanes 2..61; 4 waves stacked per block
//   strip64   aligned 64-column strips, every lane stores, rows y0-1 .. y1 loaded
//   side64    four waves side by side over 256 columns walking the same rows
//   flat      grid-stride over pixels, each loaded and stored once
//   pad60     strip60 with every array in a strip-padded layout (a row = nstrips x 64 slots,
//             column x at slot 64 (x / 60) + x % 60): a wave's 60 outputs start 256-B aligned
//   pad60u    pad60 for the solver's own vectors, UrShape and the angle in the image layout
//   pad60f    pad60 with every lane storing: lanes 0, 1, 62, 63 fill the block's unused slots
//             60..63 (junk no one reads), so each store covers whole 128-B lines
//   pad60fu   pad60f, UrShape and the angle in the image layout
//   aos60     strip60 with records: (u.x, u.y, angle, pre) as one 16-B record, (r, p) as one
//             24-B record read and another written (fewer, wider arrays: fewer partial lines
//             per byte at the strip edges); flags u8
//   aos60p    aos60 with the (r, p) record padded to 32 B (dwordx4 twice; 73 B/px moved)
//   edge64    aligned 64-column strips (rows y0-2 .. y1+1) plus, per row and array, one more
//             load with lanes 0..3 active for the columns x0-2, x0-1, x0+64, x0+65
//   pair124   two pixels per lane: 124-column strips, x = 124 s - 2 + 2 lane (+0 / +1)
//   shiftK    strip64 with every window shifted by K columns (x = 64 s + K + lane): the cost of
//             a window's byte alignment alone (K = 2: 8 B, 8: 32 B, 16: 64 B, 32: 128 B)
//   side60    (round 6) strip60 with the block's four waves side by side over four adjacent
//             60-column strips walking the same rows: iw_pcg's geometry since round 6
// `pcgbench r06` runs the round-6 set, each walk also with its occupancy capped by dynamic LDS
// at iw_pcg's 3 waves per SIMD (48 KB per block: 3 blocks per CU).
// Not part of the library.  hipcc --offload-arch=gfx950 -O3 -o tools/pcgbench tools/pcgbench.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Arr {
    const uint8_t* f; const float2* u; const float* ang; const float2* rxy; const float* rt; const float* pre;
    const float2* pxy; const float* pt;
    float2* oxy; float* ot; float2* qxy; float* qt;
};

struct Row { float2 u, r, p; float a, rt, w, pt; int f; };

__device__ __forceinline__ Row ld(const Arr& A, long long i, long long iu) {
    Row q;
    q.f = A.f[i]; q.u = A.u[iu]; q.a = A.ang[iu]; q.r = A.rxy[i]; q.rt = A.rt[i]; q.w = A.pre[i];
    q.p = A.pxy[i]; q.pt = A.pt[i];
    return q;
}
__device__ __forceinline__ Row ld(const Arr& A, long long i) { return ld(A, i, i); }
__device__ __forceinline__ float mix(const Row& q) {
    return q.u.x + q.u.y + q.a + q.r.x + q.r.y + q.rt + q.w + q.p.x + q.p.y + q.pt + (float)q.f;
}

template <int MODE, int PF>   // MODE 0 strip60, 1 strip64, 2 side64, 3 pad60, 4 pad60u, 5 pad60f, 6 pad60fu; PF rows in flight
__global__ __launch_bounds__(256) void walk(Arr A, int W, int H, int rows, int nstrips) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int strip, y0;
    if (MODE == 2 || MODE == 7) {
        const int ng = (nstrips + 3) / 4;
        strip = (t % ng) * 4 + w;
        y0 = (t / ng) * rows;
    } else {
        strip = t % nstrips;
        y0 = ((t / nstrips) * 4 + w) * rows;
    }
    constexpr bool S60 = MODE == 0 || MODE >= 3;
    constexpr bool PADL = MODE >= 3 && MODE <= 6;   // the strip-padded layouts
    const int x = S60 ? strip * 60 - 2 + lane : strip * 64 + lane;
    const bool out = S60 ? (lane >= 2 && lane < 62 && x < W) : x < W;
    const int xc = x < 0 ? 0 : (x >= W ? W - 1 : x);
    const int y1 = min(y0 + rows, H);
    if (y0 >= y1 || strip >= nstrips) return;
    const int lo = S60 ? 2 : 1;   // halo rows above / below
    const int pw = nstrips * 64;  // padded row (MODE 3 / 4)
    const int xs = (xc / 60) * 64 + xc % 60;
    auto idx = [&](int y) {
        const int yc = y < 0 ? 0 : (y >= H ? H - 1 : y);
        return PADL ? (long long)yc * pw + xs : (long long)yc * W + xc;
    };
    auto idu = [&](int y) {
        const int yc = y < 0 ? 0 : (y >= H ? H - 1 : y);
        return (MODE == 3 || MODE == 5) ? (long long)yc * pw + xs : (long long)yc * W + xc;
    };
    Row q[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) q[k] = ld(A, idx(y0 - lo + k), idu(y0 - lo + k));
    float acc = 0.f;
    for (int y = y0 - lo; y < y1 + lo; ++y) {
        const Row c = q[0];
#pragma unroll
        for (int k = 0; k + 1 < PF; ++k) q[k] = q[k + 1];
        q[PF - 1] = ld(A, idx(min(y + PF, y1 + lo - 1)), idu(min(y + PF, y1 + lo - 1)));
        const float v = mix(c);
        acc += v;
        const int ys = y - (lo - 1) - 1;   // the row stored this trip (one behind the loads)
        if (MODE == 5 || MODE == 6) {   // full-line stores: every lane, a bijection lane -> slot
            if (ys >= y0 && ys < y1) {
                const int sl = (lane >= 2 && lane < 62) ? lane - 2 : (lane < 2 ? 60 + lane : lane);
                const long long i = (long long)ys * pw + 64 * strip + sl;
                A.oxy[i] = make_float2(v, acc); A.ot[i] = v * 2.f;
                A.qxy[i] = make_float2(acc, v); A.qt[i] = acc;
            }
        } else if (out && ys >= y0 && ys < y1) {
            const long long i = idx(ys);
            A.oxy[i] = make_float2(v, acc); A.ot[i] = v * 2.f;
            A.qxy[i] = make_float2(acc, v); A.qt[i] = acc;
        }
    }
}

template <int PAD>
__global__ __launch_bounds__(256) void aos60(const uint8_t* F, const float4* SA, const float* RP, float* RPo, int W,
                                             int H, int rows, int nstrips) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int strip = t % nstrips, y0 = ((t / nstrips) * 4 + w) * rows;
    const int x = strip * 60 - 2 + lane;
    const bool out = lane >= 2 && lane < 62 && x < W;
    const int xc = x < 0 ? 0 : (x >= W ? W - 1 : x);
    const int y1 = min(y0 + rows, H);
    if (y0 >= y1) return;
    constexpr int RS = PAD ? 8 : 6;   // floats per (r, p) record
    auto idx = [&](int y) { const int yc = y < 0 ? 0 : (y >= H ? H - 1 : y); return (long long)yc * W + xc; };
    struct Q { float4 sa; float2 a, b, c; float4 d, e; int f; };
    auto ld = [&](long long i) {
        Q q;
        q.f = F[i]; q.sa = SA[i];
        if (PAD) { q.d = *(const float4*)(RP + RS * i); q.e = *(const float4*)(RP + RS * i + 4); }
        else { q.a = *(const float2*)(RP + RS * i); q.b = *(const float2*)(RP + RS * i + 2); q.c = *(const float2*)(RP + RS * i + 4); }
        return q;
    };
    float acc = 0.f;
    Q q = ld(idx(y0 - 2));
    for (int y = y0 - 2; y < y1 + 2; ++y) {
        const Q c = q;
        q = ld(idx(min(y + 1, y1 + 1)));
        const float v = PAD ? c.sa.x + c.sa.y + c.sa.z + c.sa.w + c.d.x + c.d.y + c.d.z + c.e.x + c.e.y + c.e.z + (float)c.f
                            : c.sa.x + c.sa.y + c.sa.z + c.sa.w + c.a.x + c.a.y + c.b.x + c.b.y + c.c.x + c.c.y + (float)c.f;
        acc += v;
        const int ys = y - 2;
        if (out && ys >= y0 && ys < y1) {
            const long long i = idx(ys);
            if (PAD) {
                *(float4*)(RPo + RS * i) = make_float4(v, acc, v, 0.f);
                *(float4*)(RPo + RS * i + 4) = make_float4(acc, v, acc, 0.f);
            } else {
                *(float2*)(RPo + RS * i) = make_float2(v, acc);
                *(float2*)(RPo + RS * i + 2) = make_float2(v, acc);
                *(float2*)(RPo + RS * i + 4) = make_float2(v, acc);
            }
        }
    }
}

__global__ __launch_bounds__(256) void edge64(Arr A, int W, int H, int rows, int nstrips) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int strip = t % nstrips, y0 = ((t / nstrips) * 4 + w) * rows;
    const int x = strip * 64 + lane;
    const int y1 = min(y0 + rows, H);
    if (y0 >= y1) return;
    const int ex = strip * 64 + (lane < 2 ? lane - 2 : 62 + lane);   // lanes 0..3: x0-2, x0-1, x0+64, x0+65
    const int exc = ex < 0 ? 0 : (ex >= W ? W - 1 : ex);
    auto idx = [&](int y, int xx) { const int yc = y < 0 ? 0 : (y >= H ? H - 1 : y); return (long long)yc * W + xx; };
    float acc = 0.f;
    Row q = ld(A, idx(y0 - 2, x));
    Row e = q;
    if (lane < 4) e = ld(A, idx(y0 - 2, exc));
    for (int y = y0 - 2; y < y1 + 2; ++y) {
        const Row c = q, ce = e;
        q = ld(A, idx(min(y + 1, y1 + 1), x));
        if (lane < 4) e = ld(A, idx(min(y + 1, y1 + 1), exc));
        const float v = mix(c) + mix(ce);
        acc += v;
        const int ys = y - 2;
        if (ys >= y0 && ys < y1) {
            const long long i = idx(ys, x);
            A.oxy[i] = make_float2(v, acc); A.ot[i] = v * 2.f;
            A.qxy[i] = make_float2(acc, v); A.qt[i] = acc;
        }
    }
}

struct Row2 { float4 u, r, p; float2 a, rt, w, pt; unsigned short f; };
__global__ __launch_bounds__(256) void pair124(Arr A, int W, int H, int rows, int nstrips) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int strip = t % nstrips, y0 = ((t / nstrips) * 4 + w) * rows;
    const int x = strip * 124 - 2 + 2 * lane;
    const bool out = lane >= 1 && lane < 63 && x < W;
    const int xc = x < 0 ? 0 : (x >= W ? W - 2 : x);
    const int y1 = min(y0 + rows, H);
    if (y0 >= y1) return;
    auto idx = [&](int y) { const int yc = y < 0 ? 0 : (y >= H ? H - 1 : y); return (long long)yc * W + xc; };
    auto ld2 = [&](long long i) {
        Row2 q;
        q.f = *(const unsigned short*)(A.f + i);
        q.u = *(const float4*)(A.u + i); q.a = *(const float2*)(A.ang + i);
        q.r = *(const float4*)(A.rxy + i); q.rt = *(const float2*)(A.rt + i); q.w = *(const float2*)(A.pre + i);
        q.p = *(const float4*)(A.pxy + i); q.pt = *(const float2*)(A.pt + i);
        return q;
    };
    float acc = 0.f;
    Row2 q = ld2(idx(y0 - 2));
    for (int y = y0 - 2; y < y1 + 2; ++y) {
        const Row2 c = q;
        q = ld2(idx(min(y + 1, y1 + 1)));
        const float v = c.u.x + c.u.w + c.a.x + c.a.y + c.r.x + c.r.w + c.rt.y + c.w.x + c.p.z + c.pt.y + (float)c.f;
        acc += v;
        const int ys = y - 2;
        if (out && ys >= y0 && ys < y1) {
            const long long i = idx(ys);
            *(float4*)(A.oxy + i) = make_float4(v, acc, v, acc); *(float2*)(A.ot + i) = make_float2(v, v);
            *(float4*)(A.qxy + i) = make_float4(acc, v, acc, v); *(float2*)(A.qt + i) = make_float2(acc, acc);
        }
    }
}

template <int K>
__global__ __launch_bounds__(256) void shifted(Arr A, int W, int H, int rows, int nstrips) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int strip = t % nstrips, y0 = ((t / nstrips) * 4 + w) * rows;
    const int x = strip * 64 + K + lane;
    const bool out = x < W;
    const int xc = x >= W ? W - 1 : x;
    const int y1 = min(y0 + rows, H);
    if (y0 >= y1) return;
    auto idx = [&](int y) { const int yc = y < 0 ? 0 : (y >= H ? H - 1 : y); return (long long)yc * W + xc; };
    float acc = 0.f;
    Row q = ld(A, idx(y0 - 1));
    for (int y = y0 - 1; y < y1 + 1; ++y) {
        const Row c = q;
        q = ld(A, idx(min(y + 1, y1)));
        const float v = mix(c);
        acc += v;
        const int ys = y - 1;
        if (out && ys >= y0 && ys < y1) {
            const long long i = idx(ys);
            A.oxy[i] = make_float2(v, acc); A.ot[i] = v * 2.f;
            A.qxy[i] = make_float2(acc, v); A.qt[i] = acc;
        }
    }
}

__global__ __launch_bounds__(256) void flat(Arr A, long long n) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const Row c = ld(A, i);
        const float v = mix(c);
        A.oxy[i] = make_float2(v, v); A.ot[i] = v;
        A.qxy[i] = make_float2(v, 1.f); A.qt[i] = v;
    }
}

template <typename K, typename... Args>
static float timeit_lds(K k, int grid, unsigned lds, Args... a) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, a...);
    (void)hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, a...);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return 1000.f * ms / reps;
}
template <typename K, typename... Args>
static float timeit(K k, int grid, Args... a) { return timeit_lds(k, grid, 0u, a...); }

int main(int argc, char** argv) {
    const bool r06 = argc > 1 && argv[1][0] == 'r';
    const int W = 4096, H = 4096;
    const long long N = (long long)W * H;
    Arr A;
    void* p;
    const long long NP = (long long)((W + 59) / 60) * 64 * H;   // padded layout
    CK(hipMalloc(&p, NP)); CK(hipMemset(p, 1, NP)); A.f = (const uint8_t*)p;
    size_t f2 = 8 * NP, f1 = 4 * NP;
    void* bufs[12];
    size_t sz[12] = {4 * f2, f1, 4 * f2, f1, f1, f2, f1, 4 * f2, f1, f2, f1, 2 * f2};
    for (int k = 0; k < 12; ++k) { CK(hipMalloc(&bufs[k], sz[k])); CK(hipMemset(bufs[k], 0, sz[k])); }
    A.u = (const float2*)bufs[0]; A.ang = (const float*)bufs[1]; A.rxy = (const float2*)bufs[2];
    A.rt = (const float*)bufs[3]; A.pre = (const float*)bufs[4]; A.pxy = (const float2*)bufs[5];
    A.pt = (const float*)bufs[6]; A.oxy = (float2*)bufs[7]; A.ot = (float*)bufs[8]; A.qxy = (float2*)bufs[9];
    A.qt = (float*)bufs[10];
    const double bytes = 65.0 * N;
    auto rep = [&](const char* name, float us) { printf("%-28s %8.1f us  %6.0f GB/s (65 B/px)\n", name, us, bytes / us / 1e3); };
    if (r06) {   // iw_pcg's geometries at its occupancy (3 waves per SIMD: 48 KB of LDS per block)
        const unsigned cap = 48 * 1024;
        for (int rows : {32}) {
            const int n60 = (W + 59) / 60, n64 = W / 64, rb = (H + 4 * rows - 1) / (4 * rows);
            const int g60 = (n60 + 3) / 4 * (H / rows), g64 = (n64 / 4) * (H / rows);
            for (int k = 0; k < 2; ++k) {
                const unsigned l = k ? cap : 0u;
                const char* o = k ? " occ3" : " free";
                char nm[64];
                snprintf(nm, 64, "strip60 pf1%s", o); rep(nm, timeit_lds(walk<0, 1>, n60 * rb, l, A, W, H, rows, n60));
                snprintf(nm, 64, "strip60 pf2%s", o); rep(nm, timeit_lds(walk<0, 2>, n60 * rb, l, A, W, H, rows, n60));
                snprintf(nm, 64, "side60 pf1%s", o); rep(nm, timeit_lds(walk<7, 1>, g60, l, A, W, H, rows, n60));
                snprintf(nm, 64, "side60 pf2%s", o); rep(nm, timeit_lds(walk<7, 2>, g60, l, A, W, H, rows, n60));
                snprintf(nm, 64, "strip64 pf1%s", o); rep(nm, timeit_lds(walk<1, 1>, n64 * rb, l, A, W, H, rows, n64));
                snprintf(nm, 64, "side64 pf1%s", o); rep(nm, timeit_lds(walk<2, 1>, g64, l, A, W, H, rows, n64));
                snprintf(nm, 64, "side64 pf2%s", o); rep(nm, timeit_lds(walk<2, 2>, g64, l, A, W, H, rows, n64));
            }
        }
        for (int g : {2048, 8192}) {
            char nm[64];
            snprintf(nm, 64, "flat grid=%d", g); rep(nm, timeit(flat, g, A, N));
        }
        return 0;
    }
    for (int rows : {16, 32}) {
        const int n60 = (W + 59) / 60, n64 = W / 64, rb = (H + 4 * rows - 1) / (4 * rows);
        char nm[64];
        snprintf(nm, 64, "strip60 rows=%d pf1", rows); rep(nm, timeit(walk<0, 1>, n60 * rb, A, W, H, rows, n60));
        snprintf(nm, 64, "strip60 rows=%d pf2", rows); rep(nm, timeit(walk<0, 2>, n60 * rb, A, W, H, rows, n60));
        snprintf(nm, 64, "strip60 rows=%d pf3", rows); rep(nm, timeit(walk<0, 3>, n60 * rb, A, W, H, rows, n60));
        snprintf(nm, 64, "strip64 rows=%d pf1", rows); rep(nm, timeit(walk<1, 1>, n64 * rb, A, W, H, rows, n64));
        snprintf(nm, 64, "strip64 rows=%d pf2", rows); rep(nm, timeit(walk<1, 2>, n64 * rb, A, W, H, rows, n64));
        snprintf(nm, 64, "side64 rows=%d pf2", rows); rep(nm, timeit(walk<2, 2>, (n64 / 4) * (H / rows), A, W, H, rows, n64));
        snprintf(nm, 64, "pad60 rows=%d pf1", rows); rep(nm, timeit(walk<3, 1>, n60 * rb, A, W, H, rows, n60));
        snprintf(nm, 64, "pad60u rows=%d pf1", rows); rep(nm, timeit(walk<4, 1>, n60 * rb, A, W, H, rows, n60));
        snprintf(nm, 64, "pad60f rows=%d pf1", rows); rep(nm, timeit(walk<5, 1>, n60 * rb, A, W, H, rows, n60));
        snprintf(nm, 64, "pad60f rows=%d pf2", rows); rep(nm, timeit(walk<5, 2>, n60 * rb, A, W, H, rows, n60));
        snprintf(nm, 64, "pad60fu rows=%d pf1", rows); rep(nm, timeit(walk<6, 1>, n60 * rb, A, W, H, rows, n60));
        snprintf(nm, 64, "edge64 rows=%d", rows); rep(nm, timeit(edge64, n64 * rb, A, W, H, rows, n64));
        {
            const float* rp = (const float*)bufs[2];   // 8 NP floats each: room for 32-B records
            float* rpo = (float*)bufs[7];
            snprintf(nm, 64, "aos60 rows=%d", rows);
            rep(nm, timeit(aos60<0>, n60 * rb, A.f, (const float4*)bufs[11], rp, rpo, W, H, rows, n60));
            snprintf(nm, 64, "aos60p rows=%d", rows);
            rep(nm, timeit(aos60<1>, n60 * rb, A.f, (const float4*)bufs[11], rp, rpo, W, H, rows, n60));
        }
        const int n124 = (W + 123) / 124;
        snprintf(nm, 64, "pair124 rows=%d", rows); rep(nm, timeit(pair124, n124 * rb, A, W, H, rows, n124));
    }
    {
        const int rows = 32, n64 = W / 64, rb = (H + 4 * rows - 1) / (4 * rows);
        rep("shift0 rows=32", timeit(shifted<0>, n64 * rb, A, W, H, rows, n64));
        rep("shift2 rows=32", timeit(shifted<2>, n64 * rb, A, W, H, rows, n64));
        rep("shift8 rows=32", timeit(shifted<8>, n64 * rb, A, W, H, rows, n64));
        rep("shift16 rows=32", timeit(shifted<16>, n64 * rb, A, W, H, rows, n64));
        rep("shift32 rows=32", timeit(shifted<32>, n64 * rb, A, W, H, rows, n64));
    }
    for (int g : {1024, 2048, 8192}) {
        char nm[64];
        snprintf(nm, 64, "flat grid=%d", g); rep(nm, timeit(flat, g, A, N));
    }
    return 0;
}
