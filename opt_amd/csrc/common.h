// common.h — shared HIP plumbing for libopt_amd: fail-stop error checks, the image
// domain descriptor, DPP lane shifts and the deterministic device-wide reduction.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

// Fail-stop on any HIP error, as the reference's `cd` macro does
// (API/src/backend_cuda.t:26-40): print the call and exit.
#define OPT_HIP_CHECK(call)                                                         \
    do {                                                                            \
        hipError_t e_ = (call);                                                     \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "[opt_amd] HIP error %d (%s) in %s at %s:%d\n", (int)e_,\
                    hipGetErrorString(e_), #call, __FILE__, __LINE__);              \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

namespace optamd {

#define OPTAMD_HAVE_KBLOCK
constexpr int kWave = 64;           // CDNA wavefront
constexpr int kBlock = 256;         // 4 waves per workgroup
constexpr int kMaxReduce = 4;       // scalars one kernel may reduce at once

// A 2-D image domain as one rank sees it. Global size W x H; this rank owns rows
// [y_lo, y_hi) and holds rows [y_mem0, y_mem0 + mem_rows) in memory (owned rows plus
// halo rows on multi-GPU slabs; identical to the owned rows on one GPU). Row-major,
// x fastest, as the reference's IndexSpace:indextype (API/src/o.t:564-579).
struct Domain {
    int W, H;
    int y_lo, y_hi;
    int y_mem0, mem_rows;
    int edges = 0;   // graph domains (W = vertex count, H = 1): directed edge count
    __host__ __device__ long long npix_mem() const { return (long long)W * mem_rows; }
    __host__ __device__ long long off(int x, int yg) const {
        return (long long)(yg - y_mem0) * W + x;
    }
};

// Element -> pixel map of the unknown vector [img0 (ch0 x N) | img1 (ch1 x N) | ...]
// (reference UnknownType contiguous allocation, o.t:1056-1100).
struct VecLayout {
    int nimg;
    int ch[4];
    long long off[5];
    long long N;       // pixels in memory
    // local element index -> pixel: channel counts 1..4 by shifts / a constant divide
    // (no 64-bit integer division in the flat PCG kernels)
    __host__ __device__ static long long div_ch(long long l, int c) {
        switch (c) {
            case 1: return l;
            case 2: return l >> 1;
            case 3: return l < (1LL << 32) ? (long long)((unsigned)l / 3u) : l / 3;
            case 4: return l >> 2;
            default: return l / c;
        }
    }
    __host__ __device__ long long locate(long long e, int* img, long long* local) const {
        int k = 0;
        while (k + 1 < nimg && e >= off[k + 1]) ++k;
        *img = k;
        *local = e - off[k];
        return div_ch(*local, ch[k]);
    }
    __host__ __device__ long long pix(long long e) const {
        int k;
        long long l;
        return locate(e, &k, &l);
    }
};

// ---- DPP whole-wave lane shifts (gfx9 family: wave_shr:1 / wave_shl:1) ----------
// from_left(v, e):  lane l gets v of lane l-1, lane 0 gets e.
// from_right(v, e): lane l gets v of lane l+1, lane 63 gets e.
__device__ __forceinline__ float from_left(float v, float e) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(e), __float_as_int(v),
                                                      0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float from_right(float v, float e) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(e), __float_as_int(v),
                                                      0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ int from_left_i(int v, int e) {
    return __builtin_amdgcn_update_dpp(e, v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int from_right_i(int v, int e) {
    return __builtin_amdgcn_update_dpp(e, v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ double from_left(double v, double e) {
    int2 vi = *reinterpret_cast<int2*>(&v), ei = *reinterpret_cast<int2*>(&e);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(ei.x, vi.x, 0x138, 0xf, 0xf, false);
    r.y = __builtin_amdgcn_update_dpp(ei.y, vi.y, 0x138, 0xf, 0xf, false);
    return *reinterpret_cast<double*>(&r);
}
__device__ __forceinline__ double from_right(double v, double e) {
    int2 vi = *reinterpret_cast<int2*>(&v), ei = *reinterpret_cast<int2*>(&e);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(ei.x, vi.x, 0x130, 0xf, 0xf, false);
    r.y = __builtin_amdgcn_update_dpp(ei.y, vi.y, 0x130, 0xf, 0xf, false);
    return *reinterpret_cast<double*>(&r);
}

// The same shifts with 0 shifted into the end lane by the hardware (bound_ctrl): no
// register has to be set to the edge value first (one instruction per shift, not two)
__device__ __forceinline__ float from_left0(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_right0(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ int from_left0_i(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, true); }
__device__ __forceinline__ int from_right0_i(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, true); }
__device__ __forceinline__ double from_left0(double v) {
    int2 vi = *reinterpret_cast<int2*>(&v);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(0, vi.x, 0x138, 0xf, 0xf, true);
    r.y = __builtin_amdgcn_update_dpp(0, vi.y, 0x138, 0xf, 0xf, true);
    return *reinterpret_cast<double*>(&r);
}
__device__ __forceinline__ double from_right0(double v) {
    int2 vi = *reinterpret_cast<int2*>(&v);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(0, vi.x, 0x130, 0xf, 0xf, true);
    r.y = __builtin_amdgcn_update_dpp(0, vi.y, 0x130, 0xf, 0xf, true);
    return *reinterpret_cast<double*>(&r);
}

#include "reduce_dev.h"   // ReduceSlot, wave_sum, block_reduce_publish (also pasted into generated kernels)

// XCD-aware bijective remap of a linear block id (cdna_hip_programming.md §5.5 T1):
// blocks b and b+8 share an XCD, so consecutive remapped ids land on one XCD's L2
// and neighbouring tiles share their halo lines there.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

template <typename T> struct Vec2 { T x, y; };

// Tuning knob read from the environment (measurement sweeps), `dflt` when unset.
inline int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

// Persistent tile loops: a grid of at most kMaxTileBlocks blocks (a multiple of 8)
// walks `ntiles` tiles; the blocks of one XCD (b % 8) take a contiguous range of tiles
// so neighbouring tiles' halos meet in that XCD's L2, and every block arrives at the
// reduction tickets once instead of once per tile.
constexpr int kMaxTileBlocks = 2048;
__host__ __device__ inline int tile_blocks(int ntiles) {
    const int nb = ntiles < kMaxTileBlocks ? ntiles : kMaxTileBlocks;
    return ((nb + 7) / 8) * 8;
}
struct TileRange { int first, end, step; };
// 64 x 4 pixel tiles of a Domain's owned rows (one pixel per thread of a 256-thread block)
struct PixGeom { int x, y; bool ok; long long i; };
__host__ __device__ inline int pix_tiles(const Domain& d) { return ((d.W + 63) / 64) * ((d.y_hi - d.y_lo + 3) / 4); }
__device__ __forceinline__ PixGeom tile_pix(const Domain& d, int tile) {
    const int ntx = (d.W + 63) / 64;
    PixGeom g;
    g.x = (tile % ntx) * 64 + (threadIdx.x & 63);
    g.y = d.y_lo + (tile / ntx) * 4 + (threadIdx.x >> 6);
    g.ok = g.x < d.W && g.y < d.y_hi;
    g.i = g.ok ? d.off(g.x, g.y) : 0;
    return g;
}
__device__ __forceinline__ TileRange tile_range(int ntiles) {
    const int nb = gridDim.x, b = blockIdx.x, xcd = b % 8, slot = b / 8, nslots = nb / 8;
    const int lo = (int)((long long)ntiles * xcd / 8), hi = (int)((long long)ntiles * (xcd + 1) / 8);
    return TileRange{lo + slot, hi, nslots};
}

}  // namespace optamd
