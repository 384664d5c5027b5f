// sfs.hip — kernels for the shape_from_shading energy
// (reference examples/shape_from_shading/shape_from_shading.t):
//
//   unknown X (depth), knowns D_i, Im (float), edgeMaskR / edgeMaskC (uint8)
//   params w_p, w_s, w_g (square-rooted by the energy), f_x, f_y, u_x, u_y, L_1..L_9
//   Exclude(D_i <= 0); no UsePreconditioner (default false, o.t:258)
//   ComputedArray B_I = Select(InBoundsExpanded(0,0,1) & DV(-1,0) DV(0,0) DV(0,-1), B - I, 0)
//     with its gradient images w.r.t. X(0,0), X(-1,0), X(0,-1) (o.t:1686-1716), and
//   ComputedArray valid (comparisons only, so no gradient images)
//   E_p   = DV ? w_p (X - D_i) : 0
//   E_g_h = InBoundsExpanded(0,0,1) ? w_g (B_I(0,0) - B_I(1,0)) edgeMaskR : 0
//   E_g_v = InBoundsExpanded(0,0,1) ? w_g (B_I(0,0) - B_I(0,1)) edgeMaskC : 0
//   E_s   = valid == 1 ? w_s (4 p(0,0) - p(-1,0) - p(0,-1) - p(1,0) - p(0,1)) : 0  (3-vector)
//
// sfs_precompute materialises B_I, its three gradient images and valid once per
// precompute point (init, after an update, after a revert: solverGPUGaussNewton.t:1876,
// 2242, 2284). The gathers (J^T F + diag, J^T J p) visit, for each unknown, every
// residual instance containing it — centred anywhere, including excluded centres — as
// the reference's residualsincludingX00 does (o.t:2723-2733); cost and model cost sum
// only non-excluded centres (computeCost, :971-997). The E_s partial w.r.t. X(q) is
// w_s c (px(q), py(q), 1) with px, py functions of q alone, so it is formed in registers.
// One thread per unknown, 64 x 4 pixel blocks; the 5x5 neighbourhood reads are L1/L2 hits.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cmath>
#include <cstring>
#include "plan.h"
#include "stencil_plan.h"

namespace optamd {
namespace sfs {

template <typename T>
struct Args {
    Domain dom;
    T* X;
    const float* D;
    const float* Im;
    const uint8_t* mR;
    const uint8_t* mC;
    // precomputed images (unknown precision)
    T *BI, *G00, *Gm0, *G0m;
    uint8_t* valid;
    uint8_t* flags;     // bit0: unknown active (D_i > 0)
    T wp, ws, wg, fx, fy, ux, uy;
    T L[9];
};

__device__ __forceinline__ PixGeom pix(const Domain& d) {
    PixGeom g;
    g.x = blockIdx.x * 64 + (threadIdx.x & 63);
    g.y = d.y_lo + blockIdx.y * 4 + (threadIdx.x >> 6);
    g.ok = g.x < d.W && g.y < d.y_hi;
    g.i = g.ok ? d.off(g.x, g.y) : 0;
    return g;
}
// Inside the image AND held in this rank's memory rows. On a row slab the tile loaders
// reach past the owned rows by the tile remainder + the halo; rows beyond the memory slab
// never feed an owned output, so they read as zero instead of past the allocation.
__device__ __forceinline__ bool in_mem(const Domain& d, int y) {
    return y >= d.y_mem0 && y < d.y_mem0 + d.mem_rows;
}
__device__ __forceinline__ bool inside(const Domain& d, int x, int y) {
    return x >= 0 && x < d.W && y >= 0 && y < d.H && in_mem(d, y);
}
__device__ __forceinline__ bool inbe(const Domain& d, int x, int y) {
    return x >= 1 && x < d.W - 1 && y >= 1 && y < d.H - 1 && in_mem(d, y);
}
template <typename V>
__device__ __forceinline__ V get(const V* a, const Domain& d, int x, int y) {
    return inside(d, x, y) ? a[d.off(x, y)] : (V)0;
}
template <typename T>
__device__ __forceinline__ bool DV(const Args<T>& a, int x, int y) { return get(a.D, a.dom, x, y) > 0.f; }

// ---------------------------------------------------------------- precompute
// B_I and its three gradient images at (x, y) from X(0,0) = d, X(-1,0) = A, X(0,-1) = B
// and Im at (0,0), (-1,0), (0,-1) (shape_from_shading.t:26-52; o.t:1686-1716).
template <typename T>
__device__ __forceinline__ void shade_px(const Args<T>& a, int x, int y, T d, T A, T B, float Im0, float Iml,
                                         float Imu, T* bi, T* g0, T* g1, T* g2) {
    const T fx = a.fx, fy = a.fy, ux = a.ux, uy = a.uy;
    const T i = (T)x, j = (T)y;
    const T nx = B * (d - A) / fy;
    const T ny = A * (d - B) / fx;
    const T nz = (nx * (ux - i) / fx) + (ny * (uy - j) / fy) - (A * B / (fx * fy));
    const T sq = nx * nx + ny * ny + nz * nz;
    const T inv = sq > (T)0 ? (T)1 / sqrt(sq) : (T)1;
    const T Nx = inv * nx, Ny = inv * ny, Nz = inv * nz;
    const T* L = a.L;
    const T Bv = L[0] + L[1] * Ny + L[2] * Nz + L[3] * Nx + L[4] * Nx * Ny + L[5] * Ny * Nz +
                 L[6] * (-Nx * Nx - Ny * Ny + (T)2 * Nz * Nz) + L[7] * Nz * Nx + L[8] * (Nx * Nx - Ny * Ny);
    const T I = (T)Im0 * (T)0.5 + (T)0.25 * ((T)Iml + (T)Imu);
    *bi = Bv - I;
    const T dBx = L[3] + L[4] * Ny + L[7] * Nz + (T)2 * Nx * (L[8] - L[6]);
    const T dBy = L[1] + L[4] * Nx + L[5] * Nz - (T)2 * Ny * (L[6] + L[8]);
    const T dBz = L[2] + L[5] * Ny + (T)4 * L[6] * Nz + L[7] * Nx;
    // partials of the normal (divisions by the constants done once as reciprocals:
    // these feed the gradient images only, never the energy value)
    const T rfx = (T)1 / fx, rfy = (T)1 / fy, rfxy = (T)1 / (fx * fy);
    const T cx_ = (ux - i) * rfx, cy_ = (uy - j) * rfy;
    const T dnx[3] = {B * rfy, -B * rfy, (d - A) * rfy};
    const T dny[3] = {A * rfx, (d - B) * rfx, -A * rfx};
    const T dab[3] = {(T)0, B, A};
    T gv[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) {
        const T dnz = dnx[v] * cx_ + dny[v] * cy_ - dab[v] * rfxy;
        const T dinv = sq > (T)0 ? -(inv * inv * inv) * (nx * dnx[v] + ny * dny[v] + nz * dnz) : (T)0;
        const T dNx = dinv * nx + inv * dnx[v], dNy = dinv * ny + inv * dny[v], dNz = dinv * nz + inv * dnz;
        gv[v] = dBx * dNx + dBy * dNy + dBz * dNz;
    }
    *g0 = gv[0]; *g1 = gv[1]; *g2 = gv[2];
}

template <typename T>
__global__ __launch_bounds__(kBlock) void sfs_precompute(Args<T> a) {
    const PixGeom g = pix(a.dom);
    if (!g.ok) return;
    const int x = g.x, y = g.y, W = a.dom.W;
    const long long i0 = g.i;
    // inbe: the 3x3 neighbourhood is inside the image and in memory, plain offsets
    const bool ib = inbe(a.dom, x, y);
    const float* D = a.D;
    T bi = 0, g0 = 0, g1 = 0, g2 = 0;
    if (ib && D[i0 - 1] > 0.f && D[i0] > 0.f && D[i0 - W] > 0.f)
        shade_px(a, x, y, a.X[i0], a.X[i0 - 1], a.X[i0 - W], a.Im[i0], a.Im[i0 - 1], a.Im[i0 - W], &bi, &g0, &g1,
                 &g2);
    a.BI[g.i] = bi; a.G00[g.i] = g0; a.Gm0[g.i] = g1; a.G0m[g.i] = g2;
    bool v = ib && D[i0] > 0.f && D[i0 - W] > 0.f && D[i0 + W] > 0.f && D[i0 - 1] > 0.f && D[i0 + 1] > 0.f;
    if (v) {
        const T xc = a.X[i0];
        v = fabs(xc - a.X[i0 - W]) < (T)0.01 && fabs(xc - a.X[i0 + W]) < (T)0.01 &&
            fabs(xc - a.X[i0 - 1]) < (T)0.01 && fabs(xc - a.X[i0 + 1]) < (T)0.01;
    }
    a.valid[g.i] = v;
}

// The same per-pixel values from register strips: a wave owns 62 output columns (lanes
// 1..62 of a 64-column window; lane 0 / 63 only feed their neighbours through DPP) and
// walks `rows` rows with X and D of rows y-1, y, y+1 and Im of rows y-1, y in
// registers: three loads per pixel instead of thirteen.
constexpr int kPreOut = 62;
template <typename T>
__global__ __launch_bounds__(kBlock) void sfs_precompute_strip(Args<T> a, int nstrips, int rows) {
    const Domain& d = a.dom;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = xcd_remap(blockIdx.x, gridDim.x) * (kBlock / kWave) + (threadIdx.x >> 6);   // XCD-contiguous
    const int strip = wave % nstrips, rb = wave / nstrips;
    const int x = strip * kPreOut - 1 + lane;
    const int y0 = d.y_lo + rb * rows, y1 = min(y0 + rows, d.y_hi);
    if (y0 >= y1) return;
    const bool out_lane = lane >= 1 && lane <= kPreOut && x < d.W;
    auto ldX = [&](int y) { return inside(d, x, y) ? a.X[d.off(x, y)] : (T)0; };
    auto ldD = [&](int y) { return inside(d, x, y) ? a.D[d.off(x, y)] : 0.f; };
    auto ldI = [&](int y) { return inside(d, x, y) ? a.Im[d.off(x, y)] : 0.f; };
    T Xu = ldX(y0 - 1), Xc = ldX(y0);
    float Du = ldD(y0 - 1), Dc = ldD(y0), Iu = ldI(y0 - 1), Ic = ldI(y0);
    for (int y = y0; y < y1; ++y) {
        const T Xd = ldX(y + 1);
        const float Dd = ldD(y + 1), Id = ldI(y + 1);
        const T Xl = from_left(Xc, (T)0), Xr = from_right(Xc, (T)0);
        const float Dl = from_left(Dc, 0.f), Dr = from_right(Dc, 0.f), Il = from_left(Ic, 0.f);
        if (out_lane) {
            const bool ib = inbe(d, x, y);
            T bi = 0, g0 = 0, g1 = 0, g2 = 0;
            if (ib && Dl > 0.f && Dc > 0.f && Du > 0.f) shade_px(a, x, y, Xc, Xl, Xu, Ic, Il, Iu, &bi, &g0, &g1, &g2);
            const long long i = d.off(x, y);
            a.BI[i] = bi; a.G00[i] = g0; a.Gm0[i] = g1; a.G0m[i] = g2;
            bool v = ib && Dc > 0.f && Du > 0.f && Dd > 0.f && Dl > 0.f && Dr > 0.f;
            if (v)
                v = fabs(Xc - Xu) < (T)0.01 && fabs(Xc - Xd) < (T)0.01 && fabs(Xc - Xl) < (T)0.01 &&
                    fabs(Xc - Xr) < (T)0.01;
            a.valid[i] = v;
        }
        Xu = Xc; Xc = Xd; Du = Dc; Dc = Dd; Iu = Ic; Ic = Id;
    }
}

// ------------------------------------------------------- residual instances
// Used by the cost / model cost at centres c with inbe(c) (shading) or valid(c) == 1
// (smoothness, which implies inbe): every stencil point is then inside the image and in
// this rank's memory rows, so the reads are plain offsets from the centre's index i
// (row stride W), no per-read bounds tests.
//
// J p of the shading residual of direction sx (1: E_g_h, n = i + 1; 0: E_g_v, n = i + W)
// at centre i, entries in the oracle's order (0,0), (-1,0), (0,-1), (s), and (1,-1) for
// E_g_h / (-1,1) for E_g_v; each coefficient is the partial of w_g m (B_I(c) - B_I(c+s))
// through the gradient images (the two X(c) partials combined).
template <typename T>
__device__ __forceinline__ T shade_jp(const Args<T>& a, const T* p, long long i, long long n, int W, int sx, T m) {
    const T wg = a.wg;
    T jp = (wg * m * a.G00[i] + (sx ? -wg * m * a.Gm0[n] : -wg * m * a.G0m[n])) * p[i];
    jp += (wg * m * a.Gm0[i]) * p[i - 1];
    jp += (wg * m * a.G0m[i]) * p[i - W];
    jp += (-wg * m * a.G00[n]) * p[n];
    if (sx) jp += (-wg * m * a.G0m[n]) * p[n - W];   // X(c + (1,-1))
    else jp += (-wg * m * a.Gm0[n]) * p[n - 1];      // X(c + (-1,1))
    return jp;
}

// px / py of columns x-1..x+1 and rows y-1..y+1 (p(0,0) of shape_from_shading.t:26-31,
// divisions as the reference writes them)
template <typename T>
struct PTab {
    T x[3], y[3];
    __device__ __forceinline__ void init(const Args<T>& a, int x0, int y0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            x[j] = ((T)(x0 + j - 1) - a.ux) / a.fx;
            y[j] = ((T)(y0 + j - 1) - a.uy) / a.fy;
        }
    }
};
// The five points of E_s in the oracle's order: centre, (-1,0), (0,-1), (1,0), (0,1).
// E_s partial w.r.t. X(q) = w_s co (px(q), py(q), 1); J p of the instance at i.
template <typename T>
__device__ __forceinline__ void smooth_jp(const Args<T>& a, const PTab<T>& tb, const T* p, long long i, int W,
                                          T out[3]) {
    const int XI[5] = {1, 0, 1, 2, 1}, YI[5] = {1, 1, 0, 1, 2};
    const long long o[5] = {i, i - 1, i - W, i + 1, i + W};
    out[0] = out[1] = out[2] = 0;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const T px = tb.x[XI[s]], py = tb.y[YI[s]];
        const T co = s == 0 ? (T)4 : (T)-1;
        const T pv = p[o[s]];
        out[0] += a.ws * co * px * pv;
        out[1] += a.ws * co * py * pv;
        out[2] += a.ws * co * pv;
    }
}
// E_s value at i (oracle order: 4 p(0,0) - (the four neighbours in the order above))
template <typename T>
__device__ __forceinline__ void smooth_val(const Args<T>& a, const PTab<T>& tb, const T* X, long long i, int W,
                                           T out[3]) {
    const int XI[5] = {1, 0, 1, 2, 1}, YI[5] = {1, 1, 0, 1, 2};
    const long long o[5] = {i, i - 1, i - W, i + 1, i + W};
    T sx = 0, sy = 0, sz = 0, x0 = 0, y0 = 0, z0 = 0;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const T px = tb.x[XI[s]], py = tb.y[YI[s]];
        const T xv = X[o[s]];
        if (s == 0) { x0 = px * xv; y0 = py * xv; z0 = xv; }
        else { sx += px * xv; sy += py * xv; sz += xv; }
    }
    out[0] = a.ws * ((T)4 * x0 - sx);
    out[1] = a.ws * ((T)4 * y0 - sy);
    out[2] = a.ws * ((T)4 * z0 - sz);
}


// ------------------------------------------------------------------- J^T J p
// The shading residuals are w_g m(c) (B_I(c) - B_I(c+s)), so their Jacobian factors
// through the directional derivative of the computed array,
//   D(q) = J_{B_I}(q) p = G00(q) p(q) + Gm0(q) p(q-x) + G0m(q) p(q-y),
// and J_g^T J_g p collapses to a chain of 3-point stencils:
//   V_h(c) = w_g m_R(c) u_h(c),  u_h(c) = [inbe(c)] w_g m_R(c) (D(c) - D(c+x))   (same for v, +y)
//   W(q)   = V_h(q) - V_h(q-x) + V_v(q) - V_v(q-y)
//   (J_g^T J_g p)(k) = G00(k) W(k) + Gm0(k+x) W(k+x) + G0m(k+y) W(k+y).
// The smoothness term is w_s^2 P(k).L(valid * L(Q))(k) with Q(q) = (px, py, 1)(q) p(q),
// L = 4 centre - 4 neighbours; the fit term w_p^2 p(k). This is the reference's
// per-unknown gather (o.t:2770-2830) re-associated; each residual is evaluated once.
// A block owns a 64 x 8 tile; p and the gradient images are staged in LDS with a
// 2 / 1-pixel ring, all tile loads issued before the first wait.
constexpr int TX = 64, TY = 8;
constexpr int PW = TX + 4, PH = TY + 4;    // p: origin (x0-2, y0-2)
constexpr int GW = TX + 3, GH = TY + 3;    // gradient images and D: origin (x0-1, y0-1)
constexpr int CW = TX + 2, CH = TY + 2;    // residual centres (V, u_s): origin (x0-1, y0-1)

// One tile's global data in registers: issued for tile t+1 right after tile t's copy
// has gone to LDS, so its latency overlaps tile t's three compute phases.
template <typename T, bool JTF>
struct SfsTileRegs {
    static constexpr int NP = (PW * PH + kBlock - 1) / kBlock;
    static constexpr int NG = (GW * GH + kBlock - 1) / kBlock;
    static constexpr int NC = (CW * CH + kBlock - 1) / kBlock;
    static constexpr int NK = TX * TY / kBlock;
    T P[NP], G0[NG], G1[NG], G2[NG], BI[JTF ? NG : 1];
    int MR[NC], MC[NC], V[NC], F[NK];
    T Dg[NK];   // apply: the LM diagonal; J^T F: D_i
    __device__ __forceinline__ void load(const Args<T>& a, const T* p, const T* dadd, int x0, int y0) {
        const Domain& d = a.dom;
        const int t = threadIdx.x;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int i = t + j * kBlock, rx = i % PW, ry = i / PW, gx = x0 - 2 + rx, gy = y0 - 2 + ry;
            P[j] = (i < PW * PH && inside(d, gx, gy)) ? p[d.off(gx, gy)] : (T)0;
        }
#pragma unroll
        for (int j = 0; j < NG; ++j) {
            const int i = t + j * kBlock, rx = i % GW, ry = i / GW, gx = x0 - 1 + rx, gy = y0 - 1 + ry;
            const bool in = i < GW * GH && inside(d, gx, gy);
            const long long o = in ? d.off(gx, gy) : 0;
            G0[j] = in ? a.G00[o] : (T)0;
            G1[j] = in ? a.Gm0[o] : (T)0;
            G2[j] = in ? a.G0m[o] : (T)0;
            if (JTF) BI[j] = in ? a.BI[o] : (T)0;
        }
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const int i = t + j * kBlock, rx = i % CW, ry = i / CW, gx = x0 - 1 + rx, gy = y0 - 1 + ry;
            const bool in = i < CW * CH && inbe(d, gx, gy);
            const long long o = in ? d.off(gx, gy) : 0;
            MR[j] = in ? a.mR[o] : 0;
            MC[j] = in ? a.mC[o] : 0;
            V[j] = in ? a.valid[o] : 0;
        }
#pragma unroll
        for (int j = 0; j < NK; ++j) {
            const int i = t + j * kBlock, gx = x0 + (i % TX), gy = y0 + i / TX;
            const bool own = gx < d.W && gy < d.y_hi;
            const long long k = own ? d.off(gx, gy) : 0;
            if (JTF) {
                Dg[j] = own ? (T)a.D[k] : (T)0;
                F[j] = own && a.D[k] > 0.f;
            } else {
                F[j] = own ? a.flags[k] : 0;
                Dg[j] = (own && dadd) ? dadd[k] : (T)0;
            }
        }
    }
};

// JTF = true: the same tile pipeline evaluates r = -J^T F and diag(J^T J) (evalJTF,
// o.t:2870-2913): "p" is X, the directional derivative D is replaced by B_I itself
// (the shading residual values), the smoothness Q by P X, the fit term by w_p (X - D_i);
// it also writes the flag byte. Ap / dadd / reduction unused.
template <typename T, bool JTF>
__global__ __launch_bounds__(kBlock) void sfs_tiles(Args<T> a, const T* __restrict__ p, T* __restrict__ Ap,
                                                    T* __restrict__ diag, const T* __restrict__ dadd,
                                                    const int* stop, ReduceSlot rs) {
    if (stop && *stop) return;
    __shared__ T sP[PH][PW];
    __shared__ T sG00[GH][GW], sGm0[GH][GW], sG0m[GH][GW], sD[GH][GW];
    __shared__ T sVh[CH][CW], sVv[CH][CW], sUs[3][CH][CW];
    __shared__ uint8_t sMR[CH][CW], sMC[CH][CW], sV[CH][CW];
    __shared__ T sPX[PW], sPY[PH];
    using R = SfsTileRegs<T, JTF>;
    const Domain& d = a.dom;
    const int t = threadIdx.x;
    const int ntx = (d.W + TX - 1) / TX, nty = (d.y_hi - d.y_lo + TY - 1) / TY;
    const TileRange tr = tile_range(ntx * nty);
    const T wg = a.wg, ws = a.ws;
    T dot = 0;
    R r;
    if (tr.first < tr.end) r.load(a, p, dadd, (tr.first % ntx) * TX, d.y_lo + (tr.first / ntx) * TY);
    for (int tile = tr.first; tile < tr.end; tile += tr.step) {
        const int x0 = (tile % ntx) * TX, y0 = d.y_lo + (tile / ntx) * TY;
        if (t < PW) sPX[t] = ((T)(x0 - 2 + t) - a.ux) / a.fx;
        else if (t < PW + PH) sPY[t - PW] = ((T)(y0 - 2 + (t - PW)) - a.uy) / a.fy;
#pragma unroll
        for (int j = 0; j < R::NP; ++j) {
            const int i = t + j * kBlock;
            if (i < PW * PH) sP[i / PW][i % PW] = r.P[j];
        }
#pragma unroll
        for (int j = 0; j < R::NG; ++j) {
            const int i = t + j * kBlock;
            if (i < GW * GH) {
                sG00[i / GW][i % GW] = r.G0[j]; sGm0[i / GW][i % GW] = r.G1[j]; sG0m[i / GW][i % GW] = r.G2[j];
                if (JTF) sD[i / GW][i % GW] = r.BI[j];
            }
        }
#pragma unroll
        for (int j = 0; j < R::NC; ++j) {
            const int i = t + j * kBlock;
            if (i < CW * CH) { sMR[i / CW][i % CW] = r.MR[j]; sMC[i / CW][i % CW] = r.MC[j]; sV[i / CW][i % CW] = r.V[j]; }
        }
        int F[R::NK];
        T Dg[R::NK];
#pragma unroll
        for (int j = 0; j < R::NK; ++j) { F[j] = r.F[j]; Dg[j] = r.Dg[j]; }
        const int next = tile + tr.step;
        if (next < tr.end) r.load(a, p, dadd, (next % ntx) * TX, d.y_lo + (next / ntx) * TY);
        __syncthreads();
        // D over the G region (G coords = P coords - 1); J^T F: B_I, staged above
        if (!JTF)
            for (int i = t; i < GW * GH; i += kBlock) {
                const int cx = i % GW, cy = i / GW;
                sD[cy][cx] = sG00[cy][cx] * sP[cy + 1][cx + 1] + sGm0[cy][cx] * sP[cy + 1][cx] + sG0m[cy][cx] * sP[cy][cx + 1];
            }
        // u_s over the centre region (C coords = G coords)
        for (int i = t; i < CW * CH; i += kBlock) {
            const int cx = i % CW, cy = i / CW, px = cx + 1, py = cy + 1;
            T q0 = 0, q1 = 0, q2 = 0;
            if (sV[cy][cx] == 1) {
                constexpr int OX[5] = {0, -1, 0, 1, 0}, OY[5] = {0, 0, -1, 0, 1};
#pragma unroll
                for (int sIdx = 0; sIdx < 5; ++sIdx) {
                    const T qx = sPX[px + OX[sIdx]], qy = sPY[py + OY[sIdx]];
                    const T co = sIdx == 0 ? (T)4 : (T)-1;
                    const T pv = sP[py + OY[sIdx]][px + OX[sIdx]];
                    q0 += ws * co * qx * pv;
                    q1 += ws * co * qy * pv;
                    q2 += ws * co * pv;
                }
            }
            sUs[0][cy][cx] = q0; sUs[1][cy][cx] = q1; sUs[2][cy][cx] = q2;
        }
        __syncthreads();
        // V_h, V_v over the centre region (masks are 0 outside InBoundsExpanded(0,0,1))
        for (int i = t; i < CW * CH; i += kBlock) {
            const int cx = i % CW, cy = i / CW;
            const T mh = (T)sMR[cy][cx], mv = (T)sMC[cy][cx];
            const T dc = sD[cy][cx];
            sVh[cy][cx] = wg * mh * (wg * mh * (dc - sD[cy][cx + 1]));
            sVv[cy][cx] = wg * mv * (wg * mv * (dc - sD[cy + 1][cx]));
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < R::NK; ++j) {
            const int i = t + j * kBlock, kx = i % TX, ky = i / TX;
            const int gx = x0 + kx, gy = y0 + ky;
            if (gx < d.W && gy < d.y_hi) {
                const long long k = d.off(gx, gy);
                T acc = 0, dg = 0;
                if (F[j] & 1) {
                    const int cx = kx + 1, cy = ky + 1;   // k in C / G coords
                    const T pk = sP[ky + 2][kx + 2];
                    auto W = [&](int qx, int qy) {
                        return (sVh[qy][qx] - sVh[qy][qx - 1]) + (sVv[qy][qx] - sVv[qy - 1][qx]);
                    };
                    const T shade = sG00[cy][cx] * W(cx, cy) + sGm0[cy][cx + 1] * W(cx + 1, cy) +
                                    sG0m[cy + 1][cx] * W(cx, cy + 1);
                    T l[3];
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        l[c] = (T)4 * sUs[c][cy][cx] -
                               (sUs[c][cy][cx - 1] + sUs[c][cy - 1][cx] + sUs[c][cy][cx + 1] + sUs[c][cy + 1][cx]);
                    const T qx = sPX[kx + 2], qy = sPY[ky + 2];
                    const T fit = JTF ? a.wp * (a.wp * (pk - Dg[j])) : a.wp * (a.wp * pk);
                    acc = fit + shade + ws * (qx * l[0] + qy * l[1] + l[2]);
                    if (JTF) {
                        // diag: squared partials of every residual containing X_k
                        auto sq = [](T v) { return v * v; };
                        const T mh0 = wg * (T)sMR[cy][cx], mv0 = wg * (T)sMC[cy][cx];
                        dg = a.wp * a.wp;
                        dg += sq(mh0 * (sG00[cy][cx] - sGm0[cy][cx + 1])) + sq(wg * (T)sMR[cy][cx + 1] * sGm0[cy][cx + 1]) +
                              sq(wg * (T)sMR[cy + 1][cx] * sG0m[cy + 1][cx]) + sq(wg * (T)sMR[cy][cx - 1] * sG00[cy][cx]) +
                              sq(wg * (T)sMR[cy + 1][cx - 1] * sG0m[cy + 1][cx]);
                        dg += sq(mv0 * (sG00[cy][cx] - sG0m[cy + 1][cx])) + sq(wg * (T)sMC[cy][cx + 1] * sGm0[cy][cx + 1]) +
                              sq(wg * (T)sMC[cy + 1][cx] * sG0m[cy + 1][cx]) + sq(wg * (T)sMC[cy - 1][cx] * sG00[cy][cx]) +
                              sq(wg * (T)sMC[cy - 1][cx + 1] * sGm0[cy][cx + 1]);
                        const T nv = (T)16 * (T)(sV[cy][cx] == 1) + (T)(sV[cy][cx - 1] == 1) + (T)(sV[cy - 1][cx] == 1) +
                                     (T)(sV[cy][cx + 1] == 1) + (T)(sV[cy + 1][cx] == 1);
                        dg += ws * ws * (qx * qx + qy * qy + (T)1) * nv;
                    } else {
                        if (dadd) acc += Dg[j] * pk;
                        dot += pk * acc;
                    }
                }
                if (JTF) {
                    Ap[k] = -acc;   // r
                    diag[k] = dg;
                    a.flags[k] = (uint8_t)(F[j] & 1);
                } else {
                    Ap[k] = acc;
                }
            }
        }
        __syncthreads();   // the next tile overwrites the LDS
    }
    if (JTF) return;
    double v[1] = {(double)dot};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// --------------------------------------------------- register-strip apply
// The same re-associated chain as sfs_tiles (D -> V_h, V_v -> W -> shade; u_s -> L), but
// with no LDS: a wavefront owns a 64-column strip and walks its rows top to bottom,
// keeping the few rows each stage needs in registers; horizontal neighbours are DPP
// lane shifts. The chain reaches two columns to either side, so a strip computes 64
// columns and stores the middle 60 (strips overlap by 4 columns, re-read from L2). Row r
// is loaded while row r-1 is processed; after loading row r the wave forms D(r), V_h(r),
// then V_v(r-1), W(r-1), u_s(r-1), and stores row k = r-2. Same floating-point
// operations in the same order as the tile kernel.
constexpr int kStripOut = 60;
template <typename T>
struct SRow {   // raw loads of row r (+ flags / LM diagonal of the output row r-2)
    T p, g0, g1, g2, dg, bi;
    T rr, w;        // SUMS: r and the preconditioner of the output row r-2
    int mr, mc, v, f;
};
// JTF: p is X, bi = B_I(r), dg = D_i and f = [D_i > 0] of the output row r-2.
template <typename T, bool JTF = false, bool SUMS = false>
__device__ __forceinline__ SRow<T> strip_row(const Args<T>& a, const T* __restrict__ p, const T* __restrict__ dadd,
                                             int gx, int r, const T* __restrict__ rv = nullptr,
                                             const T* __restrict__ wv = nullptr) {
    const Domain& d = a.dom;
    SRow<T> s;
    const bool in = inside(d, gx, r);
    const long long o = in ? d.off(gx, r) : 0;
    s.p = in ? p[o] : (T)0;
    s.g0 = in ? a.G00[o] : (T)0;
    s.g1 = in ? a.Gm0[o] : (T)0;
    s.g2 = in ? a.G0m[o] : (T)0;
    s.bi = (JTF && in) ? a.BI[o] : (T)0;
    const bool ib = inbe(d, gx, r);
    s.mr = ib ? a.mR[o] : 0;
    s.mc = ib ? a.mC[o] : 0;
    s.v = ib ? a.valid[o] : 0;
    const int rk = r - 2;
    const bool own = gx >= 0 && gx < d.W && rk >= d.y_lo && rk < d.y_hi;
    const long long ok = own ? d.off(gx, rk) : 0;
    if (JTF) {
        s.dg = own ? (T)a.D[ok] : (T)0;
        s.f = own && a.D[ok] > 0.f;
    } else {
        s.f = own ? a.flags[ok] : 0;
        s.dg = (own && dadd) ? dadd[ok] : (T)0;
    }
    if (SUMS) {
        s.rr = own ? rv[ok] : (T)0;
        s.w = (own && wv) ? wv[ok] : (T)1;
    }
    return s;
}
// JTF = true: r = -J^T F, diag(J^T J) and the flag byte (evalJTF, o.t:2870-2913) by the
// same chain with D replaced by B_I, p by X and the fit term by w_p (X - D_i), as
// sfs_tiles<T, true> does (same operations in the same order); Ap is r, dadd is diag.
// SUMS (the generic driver's fused PCGStep2+3, Op::apply_sums): instead of p.Ap alone,
// sc[rs.out + 0..3] = {p.Ap, r.W Ap, Ap.W Ap, r.W r}, products in T summed in fp64 per
// lane, W = the preconditioner wv (null: 1), r = rv of the output pixels.
template <typename T, bool JTF = false, bool SUMS = false>
__global__ __launch_bounds__(kBlock) void sfs_strip(Args<T> a, const T* __restrict__ p, T* __restrict__ Ap,
                                                    const T* __restrict__ dadd, const int* stop, ReduceSlot rs,
                                                    int nstrips, int rows, int bb0 = 0, int bn0 = 1 << 30,
                                                    int bb1 = 0, const T* __restrict__ rv = nullptr,
                                                    const T* __restrict__ wv = nullptr) {
    if (stop && *stop) return;
    const Domain& d = a.dom;
    const int lane = threadIdx.x & (kWave - 1);
    // this launch's blocks: local b < bn0 -> bb0 + b, else bb1 + b - bn0 (whole slab: the
    // identity; the slab plans launch interior and boundary block ranges separately)
    // XCD-contiguous block order: neighbouring strips (which share halo columns) and row
    // blocks run on the same XCD's L2; the reduction stays indexed by gb, so the sums are
    // bitwise those of blockIdx order (round 4, same box: LM step 3.36-3.37 -> 3.29-3.30 ms,
    // in-loop apply 131 -> 128 us; profiles/r04_sfs_xcd_ab.json)
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int gb = lb < bn0 ? bb0 + lb : bb1 + lb - bn0;
    const int wave = gb * (kBlock / kWave) + (threadIdx.x >> 6);
    const int strip = wave % nstrips, rb = wave / nstrips;
    const int gx = strip * kStripOut - 2 + lane;
    const int y0 = d.y_lo + rb * rows, y1 = min(y0 + rows, d.y_hi);
    const bool out_lane = lane >= 2 && lane < 2 + kStripOut && gx < d.W;
    const T wg = a.wg, ws = a.ws;
    const T qxc = ((T)gx - a.ux) / a.fx, qxl = ((T)(gx - 1) - a.ux) / a.fx, qxr = ((T)(gx + 1) - a.ux) / a.fx;
    T dot = 0;
    double papd = 0, rapd = 0, apapd = 0, rwrd = 0;
    if (y0 < y1) {
        T p_m2 = 0, p_m1 = 0, D_m1 = 0, Vh_m1 = 0, Vv_m2 = 0, W_k = 0;
        T g0_m2 = 0, g1_m2 = 0, g0_m1 = 0, g1_m1 = 0, g2_m1 = 0, qy_m1 = 0, qy_m2 = 0;
        T us_k[3] = {0, 0, 0}, us_km1[3] = {0, 0, 0};
        int mc_m1 = 0, v_m1 = 0;
        // JTF's diagonal: masks / valid of rows k-1 (m3), k (m2), k+1 (m1)
        int mr_m2 = 0, mc_m2 = 0, mc_m3 = 0, v_m2 = 0, v_m3 = 0, mr_m1 = 0;
        SRow<T> nx = strip_row<T, JTF, SUMS>(a, p, dadd, gx, y0 - 2, rv, wv);
        for (int r = y0 - 2; r <= y1 + 1; ++r) {
            const SRow<T> cur = nx;
            if (r + 1 <= y1 + 1) nx = strip_row<T, JTF, SUMS>(a, p, dadd, gx, r + 1, rv, wv);
            const T qy = ((T)r - a.uy) / a.fy;
            // row r: D (J^T F: the shading residual values B_I), V_h
            const T D = JTF ? cur.bi : cur.g0 * cur.p + cur.g1 * from_left(cur.p, (T)0) + cur.g2 * p_m1;
            const T mh = (T)cur.mr;
            const T Vh = wg * mh * (wg * mh * (D - from_right(D, (T)0)));
            // row r-1: V_v, W, u_s
            const T mv = (T)mc_m1;
            const T Vv = wg * mv * (wg * mv * (D_m1 - D));
            const T W1 = (Vh_m1 - from_left(Vh_m1, (T)0)) + (Vv - Vv_m2);
            T us[3] = {0, 0, 0};
            {
                const T pl = from_left(p_m1, (T)0), pr = from_right(p_m1, (T)0);
                if (v_m1 == 1) {
                    const T qv[5] = {qxc, qxl, qxc, qxr, qxc};
                    const T qw[5] = {qy_m1, qy_m1, qy_m2, qy_m1, qy};
                    const T pv[5] = {p_m1, pl, p_m2, pr, cur.p};
#pragma unroll
                    for (int sI = 0; sI < 5; ++sI) {
                        const T co = sI == 0 ? (T)4 : (T)-1;
                        us[0] += ws * co * qv[sI] * pv[sI];
                        us[1] += ws * co * qw[sI] * pv[sI];
                        us[2] += ws * co * pv[sI];
                    }
                }
            }
            // row k = r - 2: output
            const int k = r - 2;
            const T gw = g1_m2 * W_k;
            const T shade = g0_m2 * W_k + from_right(gw, (T)0) + g2_m1 * W1;
            T l[3];
#pragma unroll
            for (int c = 0; c < 3; ++c)
                l[c] = (T)4 * us_k[c] - (from_left(us_k[c], (T)0) + us_km1[c] + from_right(us_k[c], (T)0) + us[c]);
            // J^T F's diagonal operands of row k: masks of rows k-1..k+1 and their lane
            // neighbours (evaluated by every lane: the DPP shifts need the whole wave)
            T dgk = 0;
            if constexpr (JTF) {
                auto sq = [](T v) { return v * v; };
                const T Gm0r = from_right(g1_m2, (T)0);   // Gm0(k + x)
                const T mh0 = wg * (T)mr_m2, mv0 = wg * (T)mc_m2;
                dgk = a.wp * a.wp;
                dgk += sq(mh0 * (g0_m2 - Gm0r)) + sq(wg * (T)from_right_i(mr_m2, 0) * Gm0r) +
                       sq(wg * (T)mr_m1 * g2_m1) + sq(wg * (T)from_left_i(mr_m2, 0) * g0_m2) +
                       sq(wg * (T)from_left_i(mr_m1, 0) * g2_m1);
                dgk += sq(mv0 * (g0_m2 - g2_m1)) + sq(wg * (T)from_right_i(mc_m2, 0) * Gm0r) +
                       sq(wg * (T)mc_m1 * g2_m1) + sq(wg * (T)mc_m3 * g0_m2) +
                       sq(wg * (T)from_right_i(mc_m3, 0) * Gm0r);
                const T nv = (T)16 * (T)(v_m2 == 1) + (T)(from_left_i(v_m2, 0) == 1) + (T)(v_m3 == 1) +
                             (T)(from_right_i(v_m2, 0) == 1) + (T)(v_m1 == 1);
                dgk += ws * ws * (qxc * qxc + qy_m2 * qy_m2 + (T)1) * nv;
            }
            if (k >= y0 && out_lane) {
                const long long i = d.off(gx, k);
                T acc = 0;
                if (cur.f & 1) {
                    const T pk = p_m2;
                    const T fit = JTF ? a.wp * (a.wp * (pk - cur.dg)) : a.wp * (a.wp * pk);
                    acc = fit + shade + ws * (qxc * l[0] + qy_m2 * l[1] + l[2]);
                    if (!JTF) {
                        if (dadd) acc += cur.dg * pk;
                        if (SUMS) papd += (double)(pk * acc);
                        else dot += pk * acc;
                    }
                }
                if (SUMS) {   // inactive pixels: Ap = 0 (r is 0 there too)
                    // fp64 products and sums, as step23's direct rz (w r r in fp64) and
                    // iw_apply_res's wdot3: the identity r.W r - 2 a r.W Ap + a^2 Ap.W Ap
                    // cancels, so both sides must be rounded alike
                    const double w_ = (double)cur.w, r_ = (double)cur.rr, ap_ = (double)acc;
                    rapd += w_ * r_ * ap_;
                    apapd += w_ * ap_ * ap_;
                    rwrd += w_ * r_ * r_;
                }
                if constexpr (JTF) {
                    Ap[i] = -acc;   // r
                    ((T*)dadd)[i] = (cur.f & 1) ? dgk : (T)0;
                    a.flags[i] = (uint8_t)(cur.f & 1);
                } else {
                    Ap[i] = acc;
                }
            }
            // roll the window
            p_m2 = p_m1; p_m1 = cur.p;
            D_m1 = D; Vh_m1 = Vh; Vv_m2 = Vv; W_k = W1;
            g0_m2 = g0_m1; g1_m2 = g1_m1; g0_m1 = cur.g0; g1_m1 = cur.g1; g2_m1 = cur.g2;
            qy_m2 = qy_m1; qy_m1 = qy;
#pragma unroll
            for (int c = 0; c < 3; ++c) { us_km1[c] = us_k[c]; us_k[c] = us[c]; }
            mc_m3 = mc_m2; mc_m2 = mc_m1; v_m3 = v_m2; v_m2 = v_m1; mr_m2 = mr_m1;
            mc_m1 = cur.mc; v_m1 = cur.v; mr_m1 = cur.mr;
        }
    }
    if (JTF) return;
    if constexpr (SUMS) {
        double v[4] = {papd, rapd, apapd, rwrd};
        block_reduce_publish<4>(v, rs, gb);
    } else {
        double v[1] = {(double)dot};
        block_reduce_publish<1>(v, rs, gb);
    }
}

// ------------------------------------------------------- cost / model cost
template <typename T>
__global__ __launch_bounds__(kBlock) void sfs_cost(Args<T> a, const T* __restrict__ delta, ReduceSlot rs) {
    const TileRange tr = tile_range(pix_tiles(a.dom));
    const int W = a.dom.W;
    T acc = 0;
    for (int tile = tr.first; tile < tr.end; tile += tr.step) {
    const PixGeom g = tile_pix(a.dom, tile);
    if (g.ok && a.D[g.i] > 0.f) {
        const int x = g.x, y = g.y;
        const long long i = g.i;
        T s2 = 0;
        {   // E_p
            T e = a.wp * (a.X[i] - (T)a.D[i]);
            if (delta) e += a.wp * delta[i];
            s2 += e * e;
        }
        if (inbe(a.dom, x, y)) {
            const T bi = a.BI[i];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int sx = t == 0 ? 1 : 0;
                const T m = (T)(t == 0 ? a.mR[i] : a.mC[i]);
                const long long n = sx ? i + 1 : i + W;
                T e = a.wg * (bi - a.BI[n]) * m;
                if (delta) e += shade_jp(a, delta, i, n, W, sx, m);
                s2 += e * e;
            }
        }
        if (a.valid[i] == 1) {
            PTab<T> tb;
            tb.init(a, x, y);
            T v[3];
            smooth_val(a, tb, a.X, i, W, v);
            if (delta) {
                T jd[3];
                smooth_jp(a, tb, delta, i, W, jd);
                v[0] += jd[0]; v[1] += jd[1]; v[2] += jd[2];
            }
            s2 += v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        }
        acc += (T)0.5 * s2;
    }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// Register-strip form of the cost / model cost: a wavefront owns 64 columns (the middle
// 62 are its output; neighbours at x +- 1 are DPP lane shifts of the rows in registers)
// and walks rows y0..y1 keeping rows y-1, y, y+1. Every value, the order of the sums and
// the expressions are sfs_cost's (the shading J delta term as shade_jp, the smoothness
// term as smooth_val / smooth_jp); the strip only replaces the per-pixel neighbour loads
// by register / lane reads and forms the PTab quotients once per column and per row.
constexpr int kCostOut = 62;
template <typename T, bool DELTA>
struct CRow {
    T x, dl, bi, g0, g1, g2;
    float D;
    int mr, mc, v;
};
template <typename T, bool DELTA>
__device__ __forceinline__ CRow<T, DELTA> cost_row(const Args<T>& a, const T* __restrict__ delta, int gx, int r) {
    const Domain& d = a.dom;
    CRow<T, DELTA> q;
    const bool in = inside(d, gx, r);
    const long long o = in ? d.off(gx, r) : 0;
    q.x = in ? a.X[o] : (T)0;
    q.bi = in ? a.BI[o] : (T)0;
    q.D = in ? a.D[o] : 0.f;
    if (DELTA) {
        q.dl = in ? delta[o] : (T)0;
        q.g0 = in ? a.G00[o] : (T)0;
        q.g1 = in ? a.Gm0[o] : (T)0;
        q.g2 = in ? a.G0m[o] : (T)0;
    } else {
        q.dl = q.g0 = q.g1 = q.g2 = (T)0;
    }
    const bool ib = inbe(d, gx, r);
    q.mr = ib ? a.mR[o] : 0;
    q.mc = ib ? a.mC[o] : 0;
    q.v = ib ? a.valid[o] : 0;
    return q;
}
template <typename T, bool DELTA>
__global__ __launch_bounds__(kBlock) void sfs_cost_strip(Args<T> a, const T* __restrict__ delta, ReduceSlot rs,
                                                         int nstrips, int rows) {
    const Domain& d = a.dom;
    const int lane = threadIdx.x & (kWave - 1);
    const int lb = xcd_remap(blockIdx.x, gridDim.x);   // XCD-contiguous, as sfs_strip
    const int wave = lb * (kBlock / kWave) + (threadIdx.x >> 6);
    const int strip = wave % nstrips, rb = wave / nstrips;
    const int gx = strip * kCostOut - 1 + lane;
    const int y0 = d.y_lo + rb * rows, y1 = min(y0 + rows, d.y_hi);
    const bool out_lane = lane >= 1 && lane < 1 + kCostOut && gx < d.W;
    const T wp = a.wp, wg = a.wg, ws = a.ws;
    // PTab of the column: px(x-1), px(x), px(x+1)
    const T qxl = ((T)(gx - 1) - a.ux) / a.fx, qxc = ((T)gx - a.ux) / a.fx, qxr = ((T)(gx + 1) - a.ux) / a.fx;
    T acc = 0;
    if (y0 < y1) {
        CRow<T, DELTA> up = cost_row<T, DELTA>(a, delta, gx, y0 - 1);
        CRow<T, DELTA> cur = cost_row<T, DELTA>(a, delta, gx, y0);
        CRow<T, DELTA> dn = cost_row<T, DELTA>(a, delta, gx, y0 + 1);
        T qyu = ((T)(y0 - 1) - a.uy) / a.fy, qyc = ((T)y0 - a.uy) / a.fy;
        for (int y = y0; y < y1; ++y) {
            const CRow<T, DELTA> nx = cost_row<T, DELTA>(a, delta, gx, y + 2);
            const T qyd = ((T)(y + 1) - a.uy) / a.fy;
            // neighbour values by lane shifts (every lane, before the divergent branch)
            const T xl = from_left(cur.x, (T)0), xr = from_right(cur.x, (T)0);
            const T bir = from_right(cur.bi, (T)0);
            T dll = 0, dlr = 0, dlur = 0, dldl = 0, g0r = 0, g1r = 0, g2r = 0;
            if (DELTA) {
                dll = from_left(cur.dl, (T)0); dlr = from_right(cur.dl, (T)0);
                dlur = from_right(up.dl, (T)0); dldl = from_left(dn.dl, (T)0);
                g0r = from_right(cur.g0, (T)0); g1r = from_right(cur.g1, (T)0); g2r = from_right(cur.g2, (T)0);
            }
            if (out_lane && cur.D > 0.f) {
                T s2 = 0;
                {   // E_p
                    T e = wp * (cur.x - (T)cur.D);
                    if (DELTA) e += wp * cur.dl;
                    s2 += e * e;
                }
                if (inbe(d, gx, y)) {
                    const T bi = cur.bi;
                    {   // E_g_h: n = c + (1, 0)
                        const T m = (T)cur.mr;
                        T e = wg * (bi - bir) * m;
                        if (DELTA) {
                            T jp = (wg * m * cur.g0 + -wg * m * g1r) * cur.dl;
                            jp += (wg * m * cur.g1) * dll;
                            jp += (wg * m * cur.g2) * up.dl;
                            jp += (-wg * m * g0r) * dlr;
                            jp += (-wg * m * g2r) * dlur;
                            e += jp;
                        }
                        s2 += e * e;
                    }
                    {   // E_g_v: n = c + (0, 1)
                        const T m = (T)cur.mc;
                        T e = wg * (bi - dn.bi) * m;
                        if (DELTA) {
                            T jp = (wg * m * cur.g0 + -wg * m * dn.g2) * cur.dl;
                            jp += (wg * m * cur.g1) * dll;
                            jp += (wg * m * cur.g2) * up.dl;
                            jp += (-wg * m * dn.g0) * dn.dl;
                            jp += (-wg * m * dn.g1) * dldl;
                            e += jp;
                        }
                        s2 += e * e;
                    }
                }
                if (cur.v == 1) {   // E_s: centre, (-1,0), (0,-1), (1,0), (0,1)
                    const T px[5] = {qxc, qxl, qxc, qxr, qxc}, py[5] = {qyc, qyc, qyu, qyc, qyd};
                    const T xv[5] = {cur.x, xl, up.x, xr, dn.x};
                    T sx = 0, sy = 0, sz = 0, x0 = 0, y0v = 0, z0 = 0;
#pragma unroll
                    for (int sI = 0; sI < 5; ++sI) {
                        if (sI == 0) { x0 = px[0] * xv[0]; y0v = py[0] * xv[0]; z0 = xv[0]; }
                        else { sx += px[sI] * xv[sI]; sy += py[sI] * xv[sI]; sz += xv[sI]; }
                    }
                    T v3[3] = {ws * ((T)4 * x0 - sx), ws * ((T)4 * y0v - sy), ws * ((T)4 * z0 - sz)};
                    if (DELTA) {
                        const T pv[5] = {cur.dl, dll, up.dl, dlr, dn.dl};
                        T jd[3] = {0, 0, 0};
#pragma unroll
                        for (int sI = 0; sI < 5; ++sI) {
                            const T co = sI == 0 ? (T)4 : (T)-1;
                            jd[0] += ws * co * px[sI] * pv[sI];
                            jd[1] += ws * co * py[sI] * pv[sI];
                            jd[2] += ws * co * pv[sI];
                        }
                        v3[0] += jd[0]; v3[1] += jd[1]; v3[2] += jd[2];
                    }
                    s2 += v3[0] * v3[0] + v3[1] * v3[1] + v3[2] * v3[2];
                }
                acc += (T)0.5 * s2;
            }
            up = cur; cur = dn; dn = nx;
            qyu = qyc; qyc = qyd;
        }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, lb);   // slot of the logical block: the sums of blockIdx order
}

}  // namespace sfs

template <typename TT>
class ShapeFromShadingOp {
public:
    using T = TT;
    static constexpr const char* kName = "shape_from_shading";
    static constexpr const char* kApplyName = "sfs_strip";
    static constexpr bool kSlabs = true;
    ShapeFromShadingOp(const ProblemSpec& spec, const StateOptions& opts, Domain dom) : dom_(dom), opts_(opts) {
        idx_X_ = spec.unknown(0)->index;
        idx_D_ = spec.array(0)->index;
        idx_Im_ = spec.array(1)->index;
        idx_mR_ = spec.array(2)->index;
        idx_mC_ = spec.array(3)->index;
        static const char* names[16] = {"w_p", "w_s", "w_g", "f_x", "f_y", "u_x", "u_y", "L_1", "L_2",
                                        "L_3", "L_4", "L_5", "L_6", "L_7", "L_8", "L_9"};
        std::vector<DeclParam> ps = spec.params;
        std::sort(ps.begin(), ps.end(), [](auto& x, auto& y) { return x.index < y.index; });
        for (int k = 0; k < 16; ++k) {
            idx_p_[k] = k < (int)ps.size() ? ps[k].index : -1;
            for (auto& p : ps)
                if (p.name == names[k]) idx_p_[k] = p.index;
        }
        const long long N = dom_.npix_mem();
        for (T** v : {&BI_, &G00_, &Gm0_, &G0m_}) {
            *v = (T*)dmalloc(sizeof(T) * N);
            OPT_HIP_CHECK(hipMemset(*v, 0, sizeof(T) * N));
        }
        valid_ = (uint8_t*)dmalloc(N);
        OPT_HIP_CHECK(hipMemset(valid_, 0, N));
        if (opts.host_buffers) {
            dX_ = (T*)dmalloc(sizeof(T) * N);
            dD_ = (float*)dmalloc(sizeof(float) * N);
            dIm_ = (float*)dmalloc(sizeof(float) * N);
            dmR_ = (uint8_t*)dmalloc(N);
            dmC_ = (uint8_t*)dmalloc(N);
        }
    }
    ~ShapeFromShadingOp() {
        for (T* v : {BI_, G00_, Gm0_, G0m_, dX_}) dfree(v);
        dfree(valid_); dfree(dD_); dfree(dIm_); dfree(dmR_); dfree(dmC_);
    }
    VecLayout layout() const {
        VecLayout L{};
        L.nimg = 1;
        L.ch[0] = 1;
        L.off[0] = 0;
        L.off[1] = dom_.npix_mem();
        L.N = dom_.npix_mem();
        return L;
    }
    int halo() const { return 2; }
    int stencil_blocks() const { return std::max(grid().x * grid().y, tile_grid().x * tile_grid().y); }
    void bind(void** params, hipStream_t s) {
        auto pf = [&](int k) { return (T)*(const float*)params[idx_p_[k]]; };
        // w_p, w_s, w_g enter the energy as sqrt(Param) (shape_from_shading.t:4-6)
        a_.wp = std::sqrt(pf(0));
        a_.ws = std::sqrt(pf(1));
        a_.wg = std::sqrt(pf(2));
        a_.fx = pf(3); a_.fy = pf(4); a_.ux = pf(5); a_.uy = pf(6);
        for (int k = 0; k < 9; ++k) a_.L[k] = pf(7 + k);
        userX_ = (T*)params[idx_X_];
        const long long N = dom_.npix_mem();
        if (!opts_.host_buffers) {
            a_.X = userX_;
            a_.D = (const float*)params[idx_D_];
            a_.Im = (const float*)params[idx_Im_];
            a_.mR = (const uint8_t*)params[idx_mR_];
            a_.mC = (const uint8_t*)params[idx_mC_];
        } else {
            OPT_HIP_CHECK(hipMemcpyAsync(dX_, userX_, sizeof(T) * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dD_, params[idx_D_], sizeof(float) * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dIm_, params[idx_Im_], sizeof(float) * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dmR_, params[idx_mR_], N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dmC_, params[idx_mC_], N, hipMemcpyHostToDevice, s));
            a_.X = dX_; a_.D = dD_; a_.Im = dIm_; a_.mR = dmR_; a_.mC = dmC_;
        }
        a_.BI = BI_; a_.G00 = G00_; a_.Gm0 = Gm0_; a_.G0m = G0m_; a_.valid = valid_;
        a_.dom = dom_;
    }
    void unbind(hipStream_t s) {
        if (opts_.host_buffers)
            OPT_HIP_CHECK(hipMemcpyAsync(userX_, dX_, sizeof(T) * dom_.npix_mem(), hipMemcpyDeviceToHost, s));
    }
    T* unknown(int k) { return k == 0 ? a_.X : nullptr; }
    void precompute(hipStream_t s) {
        if (pre_strip_) {
            const int nstrips = (dom_.W + sfs::kPreOut - 1) / sfs::kPreOut;
            const int rows = pre_rows_;
            const int nrb = (dom_.y_hi - dom_.y_lo + rows - 1) / rows;
            const int blocks = (nstrips * nrb + kBlock / kWave - 1) / (kBlock / kWave);
            hipLaunchKernelGGL((sfs::sfs_precompute_strip<T>), dim3(blocks), dim3(kBlock), 0, s, a_, nstrips, rows);
        } else {
            hipLaunchKernelGGL((sfs::sfs_precompute<T>), grid(), dim3(kBlock), 0, s, a_);
        }
        OPT_HIP_CHECK(hipGetLastError());
    }
    void computed_planes(std::vector<HaloPlane>& v) const {
        for (T* im : {BI_, G00_, Gm0_, G0m_}) v.push_back({(void*)im, sizeof(T) * dom_.W});
        v.push_back({(void*)valid_, (size_t)dom_.W});
    }
    void jtf(T* r, T* diag, uint8_t* flags, hipStream_t s) {
        a_.flags = flags;
        if (jtf_strip_) {   // register strips (the apply's chain on B_I and X)
            const int nstrips = (dom_.W + sfs::kStripOut - 1) / sfs::kStripOut;
            const int nrb = (dom_.y_hi - dom_.y_lo + strip_rows_ - 1) / strip_rows_;
            const int blocks = (nstrips * nrb + kBlock / kWave - 1) / (kBlock / kWave);
            hipLaunchKernelGGL((sfs::sfs_strip<T, true>), dim3(blocks), dim3(kBlock), 0, s, a_, (const T*)a_.X, r,
                               (const T*)diag, (const int*)nullptr, ReduceSlot{}, nstrips, strip_rows_, 0, 1 << 30, 0,
                               (const T*)nullptr, (const T*)nullptr);
        } else {
            hipLaunchKernelGGL((sfs::sfs_tiles<T, true>), tile_grid(), dim3(kBlock), 0, s, a_, (const T*)a_.X, r, diag,
                               (const T*)nullptr, (const int*)nullptr, ReduceSlot{});
        }
        OPT_HIP_CHECK(hipGetLastError());
    }
    void apply(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s) {
        apply_split(0, p, Ap, dadd, stop, rs, s);
    }
    // the same launch with the timer's events attached (StencilPlan's HasApplyExt)
    void apply_ext(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s,
                   hipEvent_t e0, hipEvent_t e1) {
        const int nstrips = (dom_.W + sfs::kStripOut - 1) / sfs::kStripOut;
        int i0 = 0, i1 = 0, blocks = 0;
        split_ranges(&i0, &i1, &blocks);
        rs.nblocks = blocks;
        hipExtLaunchKernelGGL((sfs::sfs_strip<T>), dim3(blocks), dim3(kBlock), 0, s, e0, e1, 0, a_, p, Ap, dadd,
                              stop, rs, nstrips, strip_rows_, 0, 1 << 30, 0, (const T*)nullptr, (const T*)nullptr);
        OPT_HIP_CHECK(hipGetLastError());
    }
    // Row slabs: part 1 launches the blocks whose waves read no halo row (strip rows
    // [y0 - 2, y1 + 1] inside the owned rows), part 2 the rest; together they are the
    // whole launch block for block (same partial per block: bitwise the same sums).
    bool split_ranges(int* i0, int* i1, int* blocks) const {
        const int nstrips = (dom_.W + sfs::kStripOut - 1) / sfs::kStripOut;
        const int rows = strip_rows_;
        const int nrb = (dom_.y_hi - dom_.y_lo + rows - 1) / rows;
        *blocks = (nstrips * nrb + kBlock / kWave - 1) / (kBlock / kWave);
        int rb_a = 0, rb_b = nrb;   // interior row blocks [rb_a, rb_b)
        while (rb_a < nrb && dom_.y_lo + rb_a * rows - 2 < dom_.y_lo) ++rb_a;
        while (rb_b > rb_a && std::min(dom_.y_lo + rb_b * rows, dom_.y_hi) + 1 >= dom_.y_hi) --rb_b;
        const int w4 = kBlock / kWave;
        *i0 = (nstrips * rb_a + w4 - 1) / w4;   // first block with only interior waves
        *i1 = (nstrips * rb_b) / w4;            // one past the last
        return *i1 > *i0;
    }
    bool can_split() const {
        int i0, i1, b;
        return split_ranges(&i0, &i1, &b);
    }
    void apply_split(int part, const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s) {
        const int nstrips = (dom_.W + sfs::kStripOut - 1) / sfs::kStripOut;
        int i0 = 0, i1 = 0, blocks = 0;
        split_ranges(&i0, &i1, &blocks);
        rs.nblocks = blocks;   // the reduction spans every block of the slab
        int grid = blocks, bb0 = 0, bn0 = 1 << 30, bb1 = 0;
        if (part == 1) { grid = i1 - i0; bb0 = i0; }
        if (part == 2) { grid = i0 + (blocks - i1); bb0 = 0; bn0 = i0; bb1 = i1; }
        if (grid <= 0) return;
        hipLaunchKernelGGL((sfs::sfs_strip<T>), dim3(grid), dim3(kBlock), 0, s, a_, p, Ap, dadd, stop, rs, nstrips,
                           strip_rows_, bb0, bn0, bb1, (const T*)nullptr, (const T*)nullptr);
        OPT_HIP_CHECK(hipGetLastError());
    }
    // The apply with the fused PCG step's four sums (StencilPlan's HasApplySums): part as
    // apply_split; r and w (the preconditioner, null without one) of the output pixels;
    // events attached to the launch when e0 is given.
    void apply_sums(int part, const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, const T* r,
                    const T* w, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
        const int nstrips = (dom_.W + sfs::kStripOut - 1) / sfs::kStripOut;
        int i0 = 0, i1 = 0, blocks = 0;
        split_ranges(&i0, &i1, &blocks);
        rs.nblocks = blocks;
        int grid = blocks, bb0 = 0, bn0 = 1 << 30, bb1 = 0;
        if (part == 1) { grid = i1 - i0; bb0 = i0; }
        if (part == 2) { grid = i0 + (blocks - i1); bb0 = 0; bn0 = i0; bb1 = i1; }
        if (grid <= 0) return;
        if (e0)
            hipExtLaunchKernelGGL((sfs::sfs_strip<T, false, true>), dim3(grid), dim3(kBlock), 0, s, e0, e1, 0, a_, p,
                                  Ap, dadd, stop, rs, nstrips, strip_rows_, bb0, bn0, bb1, r, w);
        else
            hipLaunchKernelGGL((sfs::sfs_strip<T, false, true>), dim3(grid), dim3(kBlock), 0, s, a_, p, Ap, dadd, stop,
                               rs, nstrips, strip_rows_, bb0, bn0, bb1, r, w);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void cost(ReduceSlot rs, hipStream_t s) {
        if (cost_strip_) {
            launch_cost_strip<false>(nullptr, rs, s);
            return;
        }
        rs.nblocks = tile_blocks(pix_tiles(dom_));
        hipLaunchKernelGGL((sfs::sfs_cost<T>), dim3(rs.nblocks), dim3(kBlock), 0, s, a_, (const T*)nullptr, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    template <bool DELTA>
    void launch_cost_strip(const T* delta, ReduceSlot rs, hipStream_t s) {
        const int nstrips = (dom_.W + sfs::kCostOut - 1) / sfs::kCostOut;
        const int nrb = (dom_.y_hi - dom_.y_lo + cost_rows_ - 1) / cost_rows_;
        rs.nblocks = (nstrips * nrb + kBlock / kWave - 1) / (kBlock / kWave);
        hipLaunchKernelGGL((sfs::sfs_cost_strip<T, DELTA>), dim3(rs.nblocks), dim3(kBlock), 0, s, a_, delta, rs,
                           nstrips, cost_rows_);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void model_cost(const T* delta, ReduceSlot rs, hipStream_t s) {
        if (cost_strip_) {
            launch_cost_strip<true>(delta, rs, s);
            return;
        }
        rs.nblocks = tile_blocks(pix_tiles(dom_));
        hipLaunchKernelGGL((sfs::sfs_cost<T>), dim3(rs.nblocks), dim3(kBlock), 0, s, a_, delta, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }

private:
    dim3 grid() const { return dim3((dom_.W + 63) / 64, (dom_.y_hi - dom_.y_lo + 3) / 4); }
    dim3 tile_grid() const {
        const int nt = ((dom_.W + sfs::TX - 1) / sfs::TX) * ((dom_.y_hi - dom_.y_lo + sfs::TY - 1) / sfs::TY);
        return dim3(tile_blocks(nt));
    }
    Domain dom_;
    StateOptions opts_;
    int idx_X_, idx_D_, idx_Im_, idx_mR_, idx_mC_, idx_p_[16];
    sfs::Args<T> a_{};
    // rows per strip wave (apply and J^T F strips). Measured at 4096^2 (sfs_strip, LM step):
    // 12 rows 113.9 us / 3.44 ms, 16: 110-111 / 3.42, 20: 105 / 3.41, 24: 108 / 3.45,
    // 36: 118 / 3.51 — 20 rows make the 69 x 205 strip waves ~2 full resident rounds at
    // 7 waves per SIMD (16 rows: 2.46 rounds, a partly idle last one)
    // A row slab of the multi-GPU split fills less of the chip: below 4096 strip waves at 20
    // rows, 12-row waves (LM step at 4096 x 512: 20 rows 0.748 ms, 16 0.736, 12 0.704,
    // 8 0.712; 4096 x 1024: 1.033 / 1.028 / 1.016 / 1.091; 4096 x 2048: 20 rows best,
    // 1.711 ms; tools/sweep_sfs_rows.py)
    const bool small_dom_ =
        (long long)((dom_.W + sfs::kStripOut - 1) / sfs::kStripOut) * ((dom_.y_hi - dom_.y_lo + 19) / 20) < 4096;
    int strip_rows_ = env_int("OPT_AMD_SFS_ROWS", 0) > 0 ? env_int("OPT_AMD_SFS_ROWS", 0) : (small_dom_ ? 12 : 20);
    // the once-per-Step strips (cost, model cost, precompute): 12 rows per wave (round 6:
    // 4096 x 512 slab, 32 / 16 / 12 / 8 rows: LM step 0.705 / 0.674 / 0.657 / 0.666 ms —
    // cost 32.8 -> 19.5, model cost 33.3 -> 22.1, precompute 48.8 -> 29.1 us at 12,
    // tools/r06_slab.sh with VARIANTS=sfsrows; whole 4096^2 image, same box: 3.177 / 3.202
    // -> 3.146 / 3.161 ms, tools/r06_sfs_ab.sh)
    int cost_rows_ = env_int("OPT_AMD_SFS_COST_ROWS", 0) > 0 ? env_int("OPT_AMD_SFS_COST_ROWS", 0) : 12;
    bool cost_strip_ = env_int("OPT_AMD_SFS_COST_STRIP", 1) != 0;   // 0: the per-pixel sfs_cost
    bool jtf_strip_ = env_int("OPT_AMD_SFS_JTF_STRIP", 1) != 0;     // 0: the LDS-tile J^T F
    bool pre_strip_ = env_int("OPT_AMD_SFS_PRE_STRIP", 1) != 0;     // 0: the per-pixel precompute
    int pre_rows_ = env_int("OPT_AMD_SFS_PRE_ROWS", 0) > 0 ? env_int("OPT_AMD_SFS_PRE_ROWS", 0) : 12;
    T *BI_ = nullptr, *G00_ = nullptr, *Gm0_ = nullptr, *G0m_ = nullptr;
    uint8_t* valid_ = nullptr;
    T* userX_ = nullptr;
    T* dX_ = nullptr;
    float *dD_ = nullptr, *dIm_ = nullptr;
    uint8_t *dmR_ = nullptr, *dmC_ = nullptr;
};

std::unique_ptr<Plan> make_sfs_plan(const ProblemSpec& spec, const StateOptions& opts, const unsigned* dims,
                                    std::string* err) {
    unsigned W = 0, H = 0;
    for (auto& d : spec.dims) {
        if (d.name == spec.unknown(0)->dims[0]) W = dims[d.index];
        if (d.name == spec.unknown(0)->dims[1]) H = dims[d.index];
    }
    if (W == 0 || H == 0) { *err = "shape_from_shading: zero-sized domain"; return nullptr; }
    if (spec.params.size() < 16) { *err = "shape_from_shading: expects 16 scalar parameters"; return nullptr; }
    Domain dom{(int)W, (int)H, 0, (int)H, 0, (int)H};
    if (opts.double_precision)
        return make_stencil_plan<ShapeFromShadingOp<double>>(spec, opts, dom, err);
    return make_stencil_plan<ShapeFromShadingOp<float>>(spec, opts, dom, err);
}

}  // namespace optamd
