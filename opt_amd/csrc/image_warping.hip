// image_warping.hip — MI355X kernels and GN driver for the image_warping energy
// (reference examples/image_warping/image_warping.t):
//
//   unknowns  Offset O (float2 per pixel), Angle t (float)      -> 3 unknowns / px
//   knowns    UrShape U (float2), Constraints C (float2), Mask M (float)
//   params    w_fitSqrt wf, w_regSqrt wr
//   Exclude(M != 0); UsePreconditioner(true)
//   for s in {(1,0),(-1,0),(0,1),(0,-1)}:
//       e_reg(k,s) = valid(k,s) ? wr * ((O_k - O_{k+s}) - R(t_k)(U_k - U_{k+s})) : 0
//       valid(k,s) = InBounds(k+s) & M_{k+s}==0 & M_k==0
//   e_fit(k) = wf * (C_k.x >= 0 & C_k.y >= 0 ? O_k - C_k : 0)
//
// Kernel map onto the reference's generated kernels (solverGPUGaussNewton.t):
//   iw_jtf          PCGInit1 (:521-563) with evalJTF (o.t:2870-2913), CERES
//                   guardedInvert (:478-507); also writes the per-pixel flag byte
//   iw_apply<MODE>  PCGStep1 (:607-632) with applyJTJ (o.t:2770-2830); MODE 1/2 fuse
//                   the previous iteration's PCGStep3 (:814-845): p = z + beta p
//   pcg_step2       PCGStep2 (:665-731)                     (pcg_kernels.h)
//   iw_update       PCGLinearUpdate (:854-859)
//   iw_cost         computeCost (:971-997) with cost (o.t:3119-3129)
//
// Geometry (all stencil kernels): a wavefront owns a vertical strip of 64 columns,
// x = 62*strip - 1 + lane, and writes lanes 1..62; it walks T rows top to bottom
// keeping rows y-1, y, y+1 in registers (plus one row of prefetch). Vertical
// neighbours therefore cost no reload, horizontal neighbours are one DPP
// wave_shr/wave_shl move, and every residual instance is evaluated exactly once:
// each lane computes its pixel's outgoing residuals (+x, -x, +y) and the residual
// of the pixel below pointing up, and receives the rest from its lane neighbours
// (DPP) or from the previous row (registers). The reference's generated gather
// recomputes each residual (incl. sin/cos of the neighbour's angle) from both ends.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstring>
#include <string>
#include "plan.h"
#include "pcg_kernels.h"
#include "stencil_plan.h"

namespace optamd {
namespace iw {
// Contraction inside one expression only (a * b + c as written): with the default
// cross-statement fusion the backend's choice of which product joins an fma depended on
// the surrounding code, so two instantiations of the same arithmetic (round 5's trial of
// a strip-blocked layout against the image layout) rounded a few pixels differently
#pragma clang fp contract(on)

constexpr int kStrip = 64;   // columns per wavefront strip (aligned: x = 64*strip + lane)

// Rows per wave of the stencil kernels: 32 while that still gives >= 2048 tiles of
// 4 waves (4096^2: 64 strips x 32 row blocks, two resident rounds at 4 waves per SIMD);
// a row slab of the multi-GPU split (4096 x 512 at 8 ranks) would otherwise fill a
// quarter of the chip, so shorter waves down to 16 rows keep the tile count up.
// Measured on one GPU at each rank's slab shape (GN step, rows 32 / 16 / 8 / 4; round 4's
// loop): 4096 x 512 0.89 / 0.73 / 0.70 / 0.76 ms, 4096 x 1024 1.33 / 1.17 / 1.21 / 1.40,
// 4096 x 2048 2.33 / 2.21 / 2.31 / 2.78. Round 6 (iw_pcg, one rank's interior 4096 x 512
// slab alone, tools/slab_rank.py): rows 8 / 16 / 24 0.580 / 0.566 / 0.561 ms — the radius-2
// pass loads rows y0 - 2 .. y1 + 1, 50 % more rows than it outputs at 8 rows — so the floor
// is 16 (this rule: 16, 16, 16).
inline int rows_for(int nstrips, int nrows) {
    int rows = 32;
    while (rows > 16 && (long long)nstrips * ((nrows + 4 * rows - 1) / (4 * rows)) < 2048) rows /= 2;
    return rows;
}
// Row slabs (round 6): a slab whose 16-row tiles are less than one resident round of iw_pcg
// costs one wave's walk per pass (latency, not bandwidth: DESIGN.md §4), so the waves take
// the fewest rows (>= 8) whose side-by-side tiles (ngroups x row chunks, 4 waves each) still
// fit ONE round at the one-row form's 4 waves per SIMD (rows < 16 run without row pairs).
// 16 when none does. Rank 3 of the 8-way 4096^2 split: rows 10, 0.582 -> 0.555 ms per GN
// step (tools/r06_slab.sh u2).
inline int rows_one_round(int ngroups, int nrows, int ncu) {
    const long long slots = 4LL * 4 * ncu;   // waves: 4 SIMDs x 4 waves per CU
    for (int r = 8; r < 16; ++r)
        if ((long long)ngroups * ((nrows + r - 1) / r) * 4 <= slots) return r;
    return 16;
}

template <typename T>
struct Args {
    Domain dom;
    const T* O;        // Offset (2 per px)
    const T* A;        // Angle
    const float* U;    // UrShape (float2)
    const float* C;    // Constraints (float2)
    const float* M;    // Mask
    uint8_t* flags;    // bit0 active (inside, Mask==0), bit1 fit constraint valid,
                       // bits 2-4 number of valid rigidity edges (0..4)
    T wf, wr;
    int use_pre;
    int nstrips, nrowblocks, rows;   // rows per wavefront
    // tiles (strip, row block) of this launch: local tile t < tn0 -> tb0 + t, else
    // tb1 + t - tn0 (whole domain: 0, nstrips * nrowblocks, 0; the slab plans launch the
    // interior row blocks and the two boundary row blocks separately to overlap the halo)
    int tb0, tn0, tb1;
    // side != 0 (geom): the block's four waves walk the SAME rows over four adjacent strips
    // (tile = row chunk x group of 4 strips) instead of four stacked row ranges of one strip
    int side;
    // alt != 0 (iw_pcg): waves of odd row chunks ((y0 - y_lo) / rows odd) walk their rows
    // bottom to top, so the two waves on either side of every chunk boundary read the shared
    // halo rows at the same time (both at their start or both at their end)
    int alt;
    // rev != 0 (round 6, OPT_AMD_IW_MALL_REV): the launch takes its tiles in reverse order
    // (logical tile gridDim - 1 - remapped block), so it starts where the previous kernel of
    // the Step ended, on the vectors that kernel wrote last and that still sit in the 256 MB
    // Infinity Cache. Each tile keeps its reduction slot (g.tile): the sums are bitwise the same.
    int rev;
    // REC layout (round 5; the fused loop's iw_jtf_apply / iw_pcg / iw_update with REC): the
    // PCG vectors of iteration i as ONE record per pixel, [r.x r.y | p.x p.y | r.t p.t]
    // (6 T: three aligned pairs), and the per-Step static data as the record
    // S = [u.x u.y angle pre_t] (4 T), both in the image's pixel order. A wave's row is then
    // read from 3 wide arrays (flags, S, the record) instead of 8 narrow ones, and each row
    // segment of a 60-column strip shares a cache line with its neighbours only at its two
    // ends: the same bytes measured 253 against 299 us in a load/store-only walk
    // (tools/pcgbench.hip, aos60 vs strip60). The delta stays in the unknown layout (own
    // pixels only). Off by default: the solver's passes did not gain (ImageWarpingPlan::rec_on_).
    T* S;
    // Jacobi preconditioner of the two Offset channels: diag(J^T J) there is
    // 2 wr^2 (#valid edges) + wf^2 [fit], so pre = 1/(1+sqrt(diag))^2 takes one of ten
    // values (host-computed once per step; 0.25 everywhere for UsePreconditioner(false)).
    // Only the angle channel's preconditioner is stored per pixel.
    T preO[2][5];
};

// In the kernels the same ten values live in LDS, entry fit | nv << 1 (IW_PRE_TABLE).
__shared__ float iw_ptab_f[16];
__shared__ double iw_ptab_d[16];
template <typename T> __device__ __forceinline__ T* iw_ptab();
template <> __device__ __forceinline__ float* iw_ptab<float>() { return iw_ptab_f; }
template <> __device__ __forceinline__ double* iw_ptab<double>() { return iw_ptab_d; }

template <typename T>
__device__ __forceinline__ T pre_offset(const Args<T>&, int f) {
    return (f & 1) ? iw_ptab<T>()[(f >> 1) & 15] : (T)0;
}
template <typename T>
__device__ __forceinline__ T pre_entry(const Args<T>& a, int k) {
    return k < 10 ? a.preO[k & 1][k >> 1] : (T)0;
}
// Every kernel that calls pre_offset starts with IW_PRE_TABLE(a). Indexed by a per-lane
// value, a.preO itself compiles to a vector-memory load from the kernel arguments, and
// vmcnt retires in order: the wait for that load drained every row prefetch issued before
// it, once per row (4.45 -> 4.26 ms per GN step at 4096^2, in-loop pass 409 -> 390 us).
// LDS reads wait on lgkmcnt instead.
#define IW_PRE_TABLE(a)                                                           \
    if (threadIdx.x < 16) iw_ptab<T>()[threadIdx.x] = pre_entry(a, threadIdx.x); \
    __syncthreads();

// ---------------------------------------------------------------- helpers
// Element access of the once-touched PCG vectors; NT: streaming (nontemporal) form.
template <bool NT, typename T>
__device__ __forceinline__ T ld_v(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st_v(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ void sc_of(float t, float* c, float* s) { sincosf(t, s, c); }
__device__ __forceinline__ void sc_of(double t, double* c, double* s) { sincos(t, s, c); }
// a b + c with one rounding: the delta accumulation delta += alpha p is written as an
// explicit fma everywhere, so deferring some of its terms to a later pass (iw_apply_res
// E, iw_update E2) keeps every delta bitwise
__device__ __forceinline__ float fmad(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }

// A rounded value the compiler may not see through: p_0 = pre r_0 is a product that the
// reference stores (PCGInit1) and reads back (PCGStep1); used in place, the compiler would
// contract it into the apply's subtractions (fma(pre, r, -p_t)) and the apply would act on
// an unrounded p_0. Every kernel that forms p_0 from r_0 passes it through opaque(), so
// iw_jtf_apply's Ap_0 and iw_pcg's recomputed Ap_0 act on the same rounded p_0.
template <typename T>
__device__ __forceinline__ T opaque(T v) {
    asm("" : "+v"(v));
    return v;
}

struct WaveGeom {
    int x, ex, lane, y0, y1, tile;
    bool out_lane, edge_lane;
};
template <typename T>
__device__ __forceinline__ WaveGeom geom(const Args<T>& a) {
    WaveGeom g;
    int lt = xcd_remap(blockIdx.x, gridDim.x);
    if (a.rev) lt = (int)gridDim.x - 1 - lt;
    const int t = lt < a.tn0 ? a.tb0 + lt : a.tb1 + (lt - a.tn0);
    g.tile = t;
    g.lane = threadIdx.x & (kWave - 1);
    // the wave index as a wave-uniform (SGPR) value: every row index, bound and row base
    // derived from it is then scalar arithmetic, not per-lane VALU work
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    int strip, ychunk;
    if (a.side) {
        const int ng = (a.nstrips + kBlock / kWave - 1) / (kBlock / kWave);
        strip = (t % ng) * (kBlock / kWave) + w;
        ychunk = t / ng;
    } else {
        strip = t % a.nstrips;
        ychunk = (t / a.nstrips) * (kBlock / kWave) + w;
    }
    g.x = strip * kStrip + g.lane;
    // lane 0 fetches the column left of the strip, lane 63 the column right of it
    g.edge_lane = (g.lane == 0) || (g.lane == kWave - 1);
    g.ex = g.lane == 0 ? g.x - 1 : g.x + 1;
    g.y0 = a.dom.y_lo + ychunk * a.rows;
    g.y1 = min(g.y0 + a.rows, a.dom.y_hi);
    g.out_lane = g.x < a.dom.W;
    return g;
}

// inside the image AND present in this rank's memory
__device__ __forceinline__ bool present(const Domain& d, int x, int y) {
    return x >= 0 && x < d.W && y >= 0 && y < d.H && y >= d.y_mem0 && y < d.y_mem0 + d.mem_rows;
}

// Linearised residual of the edge j -> t applied to p:
//   a  = dR(t_j)/dt (U_j - U_t)
//   Jp = valid ? wr (p_j - p_t - a p_tj) : 0
template <typename T>
__device__ __forceinline__ void jedge(T pjx, T pjy, T pjt, T cj, T sj, float ujx, float ujy,
                                      T ptx, T pty, float utx, float uty, bool v, T wr,
                                      T& Jx, T& Jy, T& ax, T& ay) {
    const T dx = (T)(ujx - utx), dy = (T)(ujy - uty);
    ax = -sj * dx - cj * dy;
    ay = cj * dx - sj * dy;
    Jx = v ? wr * (pjx - ptx - ax * pjt) : (T)0;
    Jy = v ? wr * (pjy - pty - ay * pjt) : (T)0;
}

// Residual value of the edge j -> t at the current unknowns, plus its angle partial
// direction a (d e / d t_j = -wr a).
template <typename T>
__device__ __forceinline__ void eedge(T ojx, T ojy, T cj, T sj, float ujx, float ujy, T otx,
                                      T oty, float utx, float uty, bool v, T wr, T& ex, T& ey,
                                      T& ax, T& ay) {
    const T dx = (T)(ujx - utx), dy = (T)(ujy - uty);
    const T rx = cj * dx - sj * dy, ry = sj * dx + cj * dy;
    ax = -sj * dx - cj * dy;
    ay = cj * dx - sj * dy;
    ex = v ? wr * (ojx - otx - rx) : (T)0;
    ey = v ? wr * (ojy - oty - ry) : (T)0;
}

// wr^2 |a|^2 for the edge j -> t, a = dR(t_j)/dt (U_j - U_t): the edge's term of the angle
// channel's diag(J^T J) at pixel j (evalJTF's preconditioner, o.t:2870-2913). Every rounding
// is explicit (fmas, opaque products), so iw_jtf / iw_jtf_apply, which store the angle
// preconditioner from it, and iw_pcg, which recomputes it (PRC), form bitwise the same
// value whatever the surrounding code lets the compiler contract.
template <typename T>
__device__ __forceinline__ T diag_a2(T cj, T sj, float ujx, float ujy, float utx, float uty, T wr2) {
    const T dx = (T)(ujx - utx), dy = (T)(ujy - uty);
    const T ax = fmad(-sj, dx, -opaque(cj * dy));
    const T ay = fmad(cj, dx, -opaque(sj * dy));
    return opaque(wr2 * fmad(ax, ax, opaque(ay * ay)));
}

// the angle channel's preconditioner from its diag(J^T J) (CERES guardedInvert form,
// PCGInit1 :543-550), one expression for every kernel that forms it
template <typename T>
__device__ __forceinline__ T pre_angle(T dt) {
    const T st = (T)1 + sqrt(dt);
    return (T)1 / (st * st);
}

// Accumulation of the fused passes' sums: fp64 products summed in fp64 (the identity's
// terms cancel, so their rounding is amplified by rz_{i-1} / rz_i; round 2 measured fp32
// products ~1e-7 of rz off, enough to matter there)
typedef double acc_t;
// alpha = rz / pAp of the fused loop, 0 when pAp is not positive. The reference divides
// unguarded (solverGPUGaussNewton.t:696), which far past convergence meets 0 / 0 or x / 0
// once p and Ap underflow: NaN unknowns. The fused loop takes a zero step there instead
// (bitwise the plain division whenever pAp > 0).
template <typename T>
__device__ __forceinline__ T pcg_alpha(double rz, double pap) {
    return pap > 0.0 ? (T)(rz / pap) : (T)0;
}
// a0 b0 + a1 b1 + a2 b2 at the accumulation precision: p.Ap of the fused passes. Its
// products must be formed as rz's are (wdot3): far past convergence (hundreds of PCG
// iterations on a small problem) p and Ap reach ~1e-40, their fp32 products underflow to 0
// while rz's fp64 products do not, and alpha = rz / pAp blew up (a 9x7 image at 400
// iterations: energy 1.6e20; test_pcg_far_past_convergence_stays_finite)
template <typename T>
__device__ __forceinline__ acc_t dot3(T a0, T b0, T a1, T b1, T a2, T b2) {
    return (double)a0 * (double)b0 + (double)a1 * (double)b1 + (double)a2 * (double)b2;
}
// w0 a0 b0 + w1 a1 b1 + w2 a2 b2 at the accumulation precision. Every caller passes
// w1 == w0 (the Offset channels share one preconditioner value), so the fp64 form
// factors it: w0 (a0 b0 + a1 b1) + w2 a2 b2 — five fp64 operations instead of eight
// (measured round 4: the same step time either way, `profiles/r04_arap_ab.json` "iw")
template <typename T>
__device__ __forceinline__ acc_t wdot3(T w0, T a0, T b0, T w1, T a1, T b1, T w2, T a2, T b2) {
    (void)w1;
    return (double)w0 * ((double)a0 * (double)b0 + (double)a1 * (double)b1) + (double)w2 * ((double)a2 * (double)b2);
}

// ------------------------------------------------------------ row records
// Every stencil kernel keeps rows y-1, y, y+1 finished in registers and has row y+2
// in flight: a raw row is issued as pure loads (no arithmetic on
// the loaded values, so no s_waitcnt there) and finished — combined, masked,
// sin/cos — only after the current row has been computed, so each load has at least
// a full row of compute to land. The strip's two outside neighbours (x0-1 for lane
// 0, x0+64 for lane 63) travel with the row as a second, 2-lane "edge" record that
// becomes the boundary operand of the DPP lane shifts.
template <typename T>
struct PRaw {          // apply kernels: raw loads of one row (+ its edge pixel)
    T v0, v1, v2;      // MODE 0: p | MODE 1,2: r
    T w0, w1, w2;      // MODE 1,2: angle-channel pre (w2)
    T q0, q1, q2;      // MODE 2: p_old
    T d0, d1, d2;      // MODE 2 with delta: delta
    T ang;
    float2 u;
    int f, in;
    // edge pixel
    T ev0, ev1, ev2, ew0, ew1, ew2, eq0, eq1, eq2, eang;
    float2 eu;
    int ef, ein;
};
template <typename T>
struct PRow {          // finished row
    T px, py, pt;      // p (x, y, angle channel)
    T c, s;            // cos / sin of the current angle
    float ux, uy;
    int act, fit;
    T dx, dy, dt;      // delta after this iteration's update (MODE 2 with delta)
    T rx, ry, rt, ww0, ww2;   // MODE 1: r_0 and PCGStep2's weights (iw_apply<SUMS>)
    // edge pixel seen by this lane (lane 0: left of the strip, lane 63: right of it)
    T epx, epy;        // its p (x, y)
    float eux, euy;
    int eact;
    T ejx, ejy;        // its residual pointing at this lane: J(edge -> this pixel)
};

template <typename T, int MODE, bool NT = false>
__device__ __forceinline__ void raw_p(const T* pin, const T* r, const T* pre, long long i, long long N,
                                      T& v0, T& v1, T& v2, T& w0, T& w1, T& w2, T& q0, T& q1, T& q2) {
    if (MODE == 0) {
        v0 = ld_v<NT>(pin + 2 * i); v1 = ld_v<NT>(pin + 2 * i + 1); v2 = ld_v<NT>(pin + 2 * N + i);
    } else {
        v0 = ld_v<NT>(r + 2 * i); v1 = ld_v<NT>(r + 2 * i + 1); v2 = ld_v<NT>(r + 2 * N + i);
        w2 = ld_v<NT>(pre + i);   // angle-channel preconditioner; Offset channels come from the flags
        if (MODE == 2) { q0 = ld_v<NT>(pin + 2 * i); q1 = ld_v<NT>(pin + 2 * i + 1); q2 = ld_v<NT>(pin + 2 * N + i); }
    }
}

// NT: the row's own pixels use streaming loads of the PCG vectors (each is read by
// exactly one lane of one wave, apart from the row-block boundary rows); the edge
// pixels, re-read by the neighbouring strip, stay cached.
template <typename T, int MODE, int DM, bool NT = false>
__device__ __forceinline__ PRaw<T> raw_prow(const Args<T>& a, const WaveGeom& g, int y, const T* pin,
                                            const T* r, const T* pre, const T* delta) {
    PRaw<T> q;
    const long long N = a.dom.npix_mem();
    q.in = present(a.dom, g.x, y);
    const long long i = q.in ? a.dom.off(g.x, y) : 0;
    q.f = a.flags[i];
    q.u = reinterpret_cast<const float2*>(a.U)[i];
    q.ang = a.A[i];
    raw_p<T, MODE, NT>(pin, r, pre, i, N, q.v0, q.v1, q.v2, q.w0, q.w1, q.w2, q.q0, q.q1, q.q2);
    if (MODE == 2 && DM == 2) {
        q.d0 = ld_v<NT>(delta + 2 * i); q.d1 = ld_v<NT>(delta + 2 * i + 1); q.d2 = ld_v<NT>(delta + 2 * N + i);
    }
    q.ein = 0;
    if (g.edge_lane) {
        q.ein = present(a.dom, g.ex, y);
        const long long e = q.ein ? a.dom.off(g.ex, y) : 0;
        q.ef = a.flags[e];
        q.eu = reinterpret_cast<const float2*>(a.U)[e];
        q.eang = a.A[e];
        raw_p<T, MODE>(pin, r, pre, e, N, q.ev0, q.ev1, q.ev2, q.ew0, q.ew1, q.ew2, q.eq0, q.eq1, q.eq2);
    }
    return q;
}

template <typename T, int MODE>
__device__ __forceinline__ void make_p(const Args<T>& a, int f, T beta, T v0, T v1, T v2, T w2,
                                       T q0, T q1, T q2, T& px, T& py, T& pt) {
    const T w0 = pre_offset(a, f), w1 = w0;
    if (MODE == 0) {
        px = v0; py = v1; pt = v2;
    } else if (MODE == 1) {
        px = w0 * v0; py = w1 * v1; pt = w2 * v2;
    } else {
        T zx = v0, zy = v1, zt = v2;
        if (a.use_pre) { zx = w0 * v0; zy = w1 * v1; zt = w2 * v2; }
        px = zx + beta * q0;
        py = zy + beta * q1;
        pt = zt + beta * q2;
    }
}

template <typename T, int MODE, int DM>
__device__ __forceinline__ PRow<T> finish_prow(const Args<T>& a, const PRaw<T>& q, T beta, T alpha) {
    PRow<T> o;
    const int f = q.in ? q.f : 0;
    o.act = f & 1;
    o.fit = (f >> 1) & 1;
    o.ux = q.in ? q.u.x : 0.f;
    o.uy = q.in ? q.u.y : 0.f;
    sc_of(q.in ? q.ang : (T)0, &o.c, &o.s);
    make_p<T, MODE>(a, f, beta, q.v0, q.v1, q.v2, q.w2, q.q0, q.q1, q.q2, o.px, o.py, o.pt);
    if (MODE == 1) {
        o.rx = q.v0; o.ry = q.v1; o.rt = q.v2;
        o.ww0 = a.use_pre ? pre_offset(a, f) : (T)1;
        o.ww2 = a.use_pre ? q.w2 : (T)1;
    }
    if (MODE == 2 && DM == 1) { o.dx = alpha * q.q0; o.dy = alpha * q.q1; o.dt = alpha * q.q2; }
    if (MODE == 2 && DM == 2) {
        o.dx = fmad(alpha, q.q0, q.d0); o.dy = fmad(alpha, q.q1, q.d1); o.dt = fmad(alpha, q.q2, q.d2);
    }
    if (!o.act) { o.px = 0; o.py = 0; o.pt = 0; }
    // edge pixel: its p, and the residual it sends to this lane's pixel
    const int ef = q.ein ? q.ef : 0;
    o.eact = ef & 1;
    o.eux = q.ein ? q.eu.x : 0.f;
    o.euy = q.ein ? q.eu.y : 0.f;
    T ec, es, ept, ax, ay;
    sc_of(q.ein ? q.eang : (T)0, &ec, &es);
    make_p<T, MODE>(a, ef, beta, q.ev0, q.ev1, q.ev2, q.ew2, q.eq0, q.eq1, q.eq2, o.epx, o.epy, ept);
    if (!o.eact) { o.epx = 0; o.epy = 0; ept = 0; }
    jedge(o.epx, o.epy, ept, ec, es, o.eux, o.euy, o.px, o.py, o.ux, o.uy, o.eact && o.act, a.wr,
          o.ejx, o.ejy, ax, ay);
    return o;
}

// ------------------------------------------------------------- apply kernel
// MODE 0: Ap = JtJ p for the given p.
// MODE 1: p = pre*r (first PCG iteration; PCGInit1's p), Ap = JtJ p, writes p.
// MODE 2: p = z + beta p_old with z = pre*r, beta = sc[ib_num]/sc[ib_den] (the previous
//         iteration's PCGStep3, :814-845), Ap = JtJ p, writes p; and the previous
//         iteration's delta update (PCGStep2's delta += alpha p, :680), alpha =
//         sc[ia_num]/sc[ia_den]: DM 1 delta = alpha p_old, DM 2 delta += alpha p_old.
// Always: sc[rs.out] = sum p.Ap over active pixels (the alpha denominator).
// (Measured: even waves walking bottom-up so both waves at a shared row-block boundary
// read its halo rows at the same moment — 4.43 ms per GN step either way, the in-loop
// apply 296-298 us either way; every wave walks top-down.)
// LMX (MODE 0 only, the generic LM driver): Ap += dadd p (the CtC term of
// PCGStep1's LM variant, :617-622) and the whole grid returns at entry once the
// device-side zeta test has set *stop.
// NT bit 0: streaming loads of the PCG vectors (raw_prow); bit 1: streaming stores.
// SUMS (MODE 1): iteration 0 of iw_apply_res's loop when PCGInit1 is not fused with it
// (row slabs): sc[rs.out + 0..2] = {p.Ap, r.W Ap, Ap.W Ap} in fp64, as iw_jtf_apply sums them.
template <typename T, int MODE, int DM, bool LMX = false, int NT = 0, bool SUMS = false>
__global__ __launch_bounds__(kBlock) void iw_apply(Args<T> a, const T* __restrict__ pin,
                                                   const T* __restrict__ r,
                                                   const T* __restrict__ pre, T* __restrict__ pout,
                                                   T* __restrict__ Ap, T* __restrict__ delta,
                                                   const double* __restrict__ sc, int ib_num,
                                                   int ib_den, int ia_num, int ia_den, ReduceSlot rs,
                                                   const T* __restrict__ dadd = nullptr,
                                                   const int* stop = nullptr) {
    if (LMX && stop && *stop) return;
    IW_PRE_TABLE(a);
    const WaveGeom g = geom(a);
    const T beta = (MODE == 2) ? (T)(sc[ib_num] / sc[ib_den]) : (T)0;
    const T alpha = (MODE == 2 && DM != 0) ? (T)(sc[ia_num] / sc[ia_den]) : (T)0;
    const T wr = a.wr, wf2 = a.wf * a.wf;
    const long long N = a.dom.npix_mem();
    T dot = 0;
    acc_t papd = 0, rapd = 0, apapd = 0;
    if (g.y0 < g.y1) {
        PRow<T> up = finish_prow<T, MODE, DM>(a, raw_prow<T, MODE, DM, (NT & 1) != 0>(a, g, g.y0 - 1, pin, r, pre, delta), beta, alpha);
        PRow<T> cur = finish_prow<T, MODE, DM>(a, raw_prow<T, MODE, DM, (NT & 1) != 0>(a, g, g.y0, pin, r, pre, delta), beta, alpha);
        PRow<T> dn = finish_prow<T, MODE, DM>(a, raw_prow<T, MODE, DM, (NT & 1) != 0>(a, g, g.y0 + 1, pin, r, pre, delta), beta, alpha);
        // carries from the row above: J(up->cur) and J(cur->up) with its angle term
        T in_up_x, in_up_y, my_x, my_y, thm, ax, ay;
        jedge(up.px, up.py, up.pt, up.c, up.s, up.ux, up.uy, cur.px, cur.py, cur.ux, cur.uy,
              up.act && cur.act, wr, in_up_x, in_up_y, ax, ay);
        jedge(cur.px, cur.py, cur.pt, cur.c, cur.s, cur.ux, cur.uy, up.px, up.py, up.ux, up.uy,
              up.act && cur.act, wr, my_x, my_y, ax, ay);
        thm = -wr * (ax * my_x + ay * my_y);
        for (int y = g.y0; y < g.y1; ++y) {
            // row y+2 in flight during row y (a second row in flight, y+3, was measured
            // slower: more VGPRs, fewer waves); the last trip re-reads the halo row y1 (an
            // L2 hit) instead of fetching row y1 + 1, which nothing needs
            const PRaw<T> nx = raw_prow<T, MODE, DM, (NT & 1) != 0>(a, g, min(y + 2, g.y1), pin, r, pre, delta);
            // horizontal neighbours; the strip's outside columns enter at lanes 0 / 63
            const T lpx = from_left(cur.px, cur.epx), lpy = from_left(cur.py, cur.epy);
            const T rpx = from_right(cur.px, cur.epx), rpy = from_right(cur.py, cur.epy);
            const float lux = from_left(cur.ux, cur.eux), luy = from_left(cur.uy, cur.euy);
            const float rux = from_right(cur.ux, cur.eux), ruy = from_right(cur.uy, cur.euy);
            const int lact = from_left_i(cur.act, cur.eact), ract = from_right_i(cur.act, cur.eact);
            T jpx_x, jpx_y, apx_x, apx_y, jmx_x, jmx_y, amx_x, amx_y;
            T jpy_x, jpy_y, apy_x, apy_y, jdn_x, jdn_y, adn_x, adn_y;
            jedge(cur.px, cur.py, cur.pt, cur.c, cur.s, cur.ux, cur.uy, rpx, rpy, rux, ruy,
                  cur.act && ract, wr, jpx_x, jpx_y, apx_x, apx_y);
            jedge(cur.px, cur.py, cur.pt, cur.c, cur.s, cur.ux, cur.uy, lpx, lpy, lux, luy,
                  cur.act && lact, wr, jmx_x, jmx_y, amx_x, amx_y);
            jedge(cur.px, cur.py, cur.pt, cur.c, cur.s, cur.ux, cur.uy, dn.px, dn.py, dn.ux, dn.uy,
                  cur.act && dn.act, wr, jpy_x, jpy_y, apy_x, apy_y);
            jedge(dn.px, dn.py, dn.pt, dn.c, dn.s, dn.ux, dn.uy, cur.px, cur.py, cur.ux, cur.uy,
                  cur.act && dn.act, wr, jdn_x, jdn_y, adn_x, adn_y);
            // residuals of the lane neighbours pointing at this pixel
            const T inpx_x = from_right(jmx_x, cur.ejx), inpx_y = from_right(jmx_y, cur.ejy);
            const T inmx_x = from_left(jpx_x, cur.ejx), inmx_y = from_left(jpx_y, cur.ejy);
            T aox = wr * ((jpx_x + jmx_x + jpy_x + my_x) - (inpx_x + inmx_x + jdn_x + in_up_x));
            T aoy = wr * ((jpx_y + jmx_y + jpy_y + my_y) - (inpx_y + inmx_y + jdn_y + in_up_y));
            if (cur.fit) { aox += wf2 * cur.px; aoy += wf2 * cur.py; }
            T aot = thm - wr * ((apx_x * jpx_x + apx_y * jpx_y) + (amx_x * jmx_x + amx_y * jmx_y) +
                                (apy_x * jpy_x + apy_y * jpy_y));
            if (!cur.act) { aox = 0; aoy = 0; aot = 0; }
            if (g.out_lane) {
                const long long i = a.dom.off(g.x, y);
                if (LMX && dadd) {
                    aox += dadd[2 * i] * cur.px; aoy += dadd[2 * i + 1] * cur.py; aot += dadd[2 * N + i] * cur.pt;
                }
                if (Ap) {   // null in the last PCG iteration: nothing reads that Ap
                    st_v<(NT & 2) != 0>(Ap + 2 * i, aox); st_v<(NT & 2) != 0>(Ap + 2 * i + 1, aoy);
                    st_v<(NT & 2) != 0>(Ap + 2 * N + i, aot);
                }
                if (MODE != 0) {
                    st_v<(NT & 2) != 0>(pout + 2 * i, cur.px); st_v<(NT & 2) != 0>(pout + 2 * i + 1, cur.py);
                    st_v<(NT & 2) != 0>(pout + 2 * N + i, cur.pt);
                }
                if (MODE == 2 && DM != 0) {
                    const bool on = cur.act;
                    st_v<(NT & 2) != 0>(delta + 2 * i, on ? cur.dx : (T)0); st_v<(NT & 2) != 0>(delta + 2 * i + 1, on ? cur.dy : (T)0);
                    st_v<(NT & 2) != 0>(delta + 2 * N + i, on ? cur.dt : (T)0);
                }
                if (SUMS) {
                    papd += dot3(cur.px, aox, cur.py, aoy, cur.pt, aot);
                    rapd += wdot3(cur.ww0, cur.rx, aox, cur.ww0, cur.ry, aoy, cur.ww2, cur.rt, aot);
                    apapd += wdot3(cur.ww0, aox, aox, cur.ww0, aoy, aoy, cur.ww2, aot, aot);
                } else {
                    dot += cur.px * aox + cur.py * aoy + cur.pt * aot;
                }
            }
            // roll the window; the raw row is finished only now
            in_up_x = jpy_x; in_up_y = jpy_y;
            my_x = jdn_x; my_y = jdn_y;
            thm = -wr * (adn_x * jdn_x + adn_y * jdn_y);
            up = cur; cur = dn;
            dn = finish_prow<T, MODE, DM>(a, nx, beta, alpha);
        }
    }
    if constexpr (SUMS) {
        double v[3] = {(double)papd, (double)rapd, (double)apapd};
        block_reduce_publish<3>(v, rs, g.tile);
    } else {
        double v[1] = {(double)dot};
        block_reduce_publish<1>(v, rs, g.tile);   // partials by tile: split launches share the slot
    }
}

// ------------------------------------------ apply with the residual update fused
// PCG iteration i >= 1 as ONE pass (iw_apply<2> + the previous iteration's iw_residual):
//   r_i   = r_{i-1} - alpha_{i-1} Ap_{i-1}                       (PCGStep2's r update, :690)
//   p_i   = z_i + beta_i p_{i-1},  z_i = pre r_i                  (PCGStep3, :814-845)
//   delta = delta + alpha_{i-1} p_{i-1}                          (PCGStep2's delta update, :680)
//   Ap_i  = J^T J p_i                                            (PCGStep1, :607-632)
// r_i is formed wherever the stencil needs it (own pixel, vertical window, edge pixel)
// from r_{i-1} and Ap_{i-1}, so the separate residual pass — which re-read r, Ap, pre and
// the flags and wrote r — is gone. Its reduction rz_i = r_i.(pre r_i) is still summed
// here, directly, for alpha_i and as the next expansion's base; what this pass cannot
// have is rz_i before it forms p_i, so beta_i's numerator comes from the exact identity
//   r_i.W r_i = r_{i-1}.W r_{i-1} - 2 alpha r_{i-1}.W Ap_{i-1} + alpha^2 Ap_{i-1}.W Ap_{i-1}
// (W = pre, or 1 without a preconditioner: PCGStep2's weighting, :705-708), whose two
// new sums the previous pass reduced beside p.Ap. All four sums accumulate in fp64 per
// lane, so the identity's value agrees with the direct sum to ~1e-10 relative (stored in
// slot `rzx_out`; the reference's own float-atomic sums move by ~1e-7 run to run).
// Reductions: sc[rs.out + 0..3] = {rz_i, p_i.Ap_i, r_i.W Ap_i, Ap_i.W Ap_i}.
// DM 1: delta = alpha p_{i-1} (i == 1), DM 2: delta += alpha p_{i-1}. rout / Apout null
// in the last iteration (nothing reads r_L or Ap_L).
// Scalar slots of iteration j (ImageWarpingPlan: kScBase + kSlots * j): rz, pAp, rAp, ApAp, rz by the identity
constexpr int kSlots = 5;
// 32-bit byte offsets from a uniform base: global_load / global_store with an SGPR base and
// a VGPR offset, no 64-bit address arithmetic per access (the plan takes these kernels
// only when 3 N sizeof(T) < 2^32). Vec2 = the two interleaved Offset channels of a pixel.
template <typename T>
using vec2_t = T __attribute__((ext_vector_type(2)));
template <bool NT, typename V, typename T>
__device__ __forceinline__ V ldb(const T* base, unsigned off) {
    const V* p = reinterpret_cast<const V*>(reinterpret_cast<const char*>(base) + off);
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, typename V, typename T>
__device__ __forceinline__ void stb(T* base, unsigned off, V v) {
    V* p = reinterpret_cast<V*>(reinterpret_cast<char*>(base) + off);
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// iw_apply_res addresses an unknown-layout vector (3 N values), UrShape (8 B per pixel)
// and the flags through 32-bit byte offsets: the plan runs it only when these fit
template <typename T>
constexpr bool offsets_fit_32(long long npix) {
    return 3 * npix * (long long)sizeof(T) < (1LL << 32) && 8 * npix < (1LL << 32);
}
static_assert(offsets_fit_32<float>(4096LL * 4096) && offsets_fit_32<double>(4096LL * 4096), "headline sizes");
static_assert(!offsets_fit_32<double>(180000000LL) && offsets_fit_32<float>(357000000LL) &&
              !offsets_fit_32<float>(358000000LL), "fp64 bound ~179 M px, fp32 ~358 M px");
// iw_jtf_apply's strips: 60 output columns per wavefront, x = 60 strip - 2 + lane. J^T F
// is valid at lanes 1..62 (lanes 0 / 63 lack a lane neighbour), the apply at lanes 2..61:
// no edge record at all (round 3's 62-column form carried one for J^T F at lanes 0 / 63,
// which cost a second sincos per lane, five more loads per row and 21 VGPRs: 146 VGPRs,
// 3 waves per SIMD)
constexpr int kFStrip = 60;
template <typename T>
__device__ __forceinline__ WaveGeom geom_fused(const Args<T>& a) {
    WaveGeom g;
    int lt = xcd_remap(blockIdx.x, gridDim.x);
    if (a.rev) lt = (int)gridDim.x - 1 - lt;   // Args::rev
    const int t = lt < a.tn0 ? a.tb0 + lt : a.tb1 + (lt - a.tn0);   // the launch's tile ranges (geom)
    g.tile = t;
    g.lane = threadIdx.x & (kWave - 1);
    // the wave index as a wave-uniform (SGPR) value: every row index, bound and row base
    // derived from it is then scalar arithmetic, not per-lane VALU work
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    int strip, y0;
    if (a.side) {   // the block's waves: four adjacent strips over the same rows (Args::side)
        const int ng = (a.nstrips + kBlock / kWave - 1) / (kBlock / kWave);
        strip = (t % ng) * (kBlock / kWave) + w;
        y0 = a.dom.y_lo + (t / ng) * a.rows;
    } else {
        strip = t % a.nstrips;
        y0 = a.dom.y_lo + ((t / a.nstrips) * (kBlock / kWave) + w) * a.rows;
    }
    g.x = strip * kFStrip - 2 + g.lane;
    g.edge_lane = false;
    g.ex = g.x;
    g.y0 = y0;
    g.y1 = strip < a.nstrips ? min(g.y0 + a.rows, a.dom.y_hi) : g.y0;
    g.out_lane = g.lane >= 2 && g.lane < 2 + kFStrip && g.x < a.dom.W;
    return g;
}
// REC byte offsets of pixel i: the record's pairs r.xy, p.xy, (r.t, p.t) and the S record
template <typename T>
struct ROff {
    unsigned r, p, t, s;
    __device__ __forceinline__ ROff(unsigned i) : r(i * 6u * (unsigned)sizeof(T)), p(r + 2u * (unsigned)sizeof(T)),
        t(r + 4u * (unsigned)sizeof(T)), s(i * 4u * (unsigned)sizeof(T)) {}
};
// the plan takes the REC layout only when its 32-bit byte offsets fit
template <typename T>
constexpr bool offsets_fit_rec(long long npix) {
    return 6 * npix * (long long)sizeof(T) < (1LL << 32);
}
typedef float vec4f_t __attribute__((ext_vector_type(4)));
// S = [u.x u.y angle pre_t]: one 16-B load in fp32, two in fp64
__device__ __forceinline__ void ld_srec(const float* S, unsigned off, vec2_t<float>& u, float& ang, float& pre) {
    const vec4f_t v = ldb<false, vec4f_t>(S, off);
    u.x = v.x; u.y = v.y; ang = v.z; pre = v.w;
}
__device__ __forceinline__ void ld_srec(const double* S, unsigned off, vec2_t<float>& u, double& ang, double& pre) {
    const vec2_t<double> a = ldb<false, vec2_t<double>>(S, off), b = ldb<false, vec2_t<double>>(S, off + 16u);
    u.x = (float)a.x; u.y = (float)a.y; ang = b.x; pre = b.y;
}
template <bool NT>
__device__ __forceinline__ void st_srec(float* S, unsigned off, float ux, float uy, float ang, float pre) {
    vec4f_t v; v.x = ux; v.y = uy; v.z = ang; v.w = pre;
    stb<NT>(S, off, v);
}
template <bool NT>
__device__ __forceinline__ void st_srec(double* S, unsigned off, float ux, float uy, double ang, double pre) {
    vec2_t<double> a, b; a.x = ux; a.y = uy; b.x = ang; b.y = pre;
    stb<NT>(S, off, a); stb<NT>(S, off + 16u, b);
}

template <typename T>
struct RRaw {
    vec2_t<T> r, ap, q, d, q2;  // r_{i-1}, Ap_{i-1}, p_{i-1}, delta, p_{i-2} (Offset channels)
    T rt, at, qt, dt, q2t, w2, ang;  // the angle channels, its pre, the angle
    float2 u;
    int f, in;
    vec2_t<T> er, eap, eq;      // edge pixel
    T ert, eat, eqt, ew2, eang;
    float2 eu;
    int ef, ein;
};
template <typename T>
struct RRow {
    T px, py, pt, c, s;
    float ux, uy;
    int act, fit;
    T rx, ry, rt;      // r_i (for r.W Ap)
    T w0, w2;          // PCGStep2's weights of the Offset / angle channels
    T epx, epy;        // edge pixel, as PRow
    float eux, euy;
    int eact;
    T ejx, ejy;
};
// byte offsets of pixel i's Offset pair, angle channel (tb = 2 N sizeof(T)) and scalar
template <typename T>
struct POff {
    unsigned xy, t, s;
    __device__ __forceinline__ POff(unsigned i, unsigned tb) : xy(i * 2u * (unsigned)sizeof(T)),
        t(tb + i * (unsigned)sizeof(T)), s(i * (unsigned)sizeof(T)) {}
};
// own: a row of this wave (the halo rows y0-1 and y1 feed the stencil only: no delta terms)
// P0 (lIterations >= 3): p_0 = pre r_0 is not stored by PCGInit1; pass 1 (E = 0) forms its
// p_{i-1} from the r_0 it reads anyway, and pass 2 (E = 1) reads r_0 through pin2 (the r
// buffer it is about to overwrite with r_2, own pixel only) for the deferred alpha_0 p_0
template <typename T, int DM, bool NT, int E, bool P0 = false>
__device__ __forceinline__ RRaw<T> raw_rrow(const Args<T>& a, const WaveGeom& g, int y, unsigned tb,
                                            const T* pin, const T* rin, const T* Apin, const T* pre,
                                            const T* delta, const T* pin2, bool own) {
    RRaw<T> q;
    q.in = present(a.dom, g.x, y);
    const unsigned i = q.in ? (unsigned)a.dom.off(g.x, y) : 0u;
    const POff<T> o(i, tb);
    q.f = ldb<false, uint8_t>(a.flags, i);
    q.u = ldb<false, float2>(a.U, 8u * i);
    q.ang = ldb<false, T>(a.A, o.s);
    q.r = ldb<NT, vec2_t<T>>(rin, o.xy); q.rt = ldb<NT, T>(rin, o.t);
    q.ap = ldb<NT, vec2_t<T>>(Apin, o.xy); q.at = ldb<NT, T>(Apin, o.t);
    q.w2 = ldb<NT, T>(pre, o.s);
    if (!(P0 && !E)) { q.q = ldb<NT, vec2_t<T>>(pin, o.xy); q.qt = ldb<NT, T>(pin, o.t); }
    if (DM == 2 && own) { q.d = ldb<NT, vec2_t<T>>(delta, o.xy); q.dt = ldb<NT, T>(delta, o.t); }
    if (E && own) { q.q2 = ldb<NT, vec2_t<T>>(pin2, o.xy); q.q2t = ldb<NT, T>(pin2, o.t); }
    q.ein = 0;
    if (g.edge_lane) {
        q.ein = present(a.dom, g.ex, y);
        const unsigned e = q.ein ? (unsigned)a.dom.off(g.ex, y) : 0u;
        const POff<T> oe(e, tb);
        q.ef = ldb<false, uint8_t>(a.flags, e);
        q.eu = ldb<false, float2>(a.U, 8u * e);
        q.eang = ldb<false, T>(a.A, oe.s);
        q.er = ldb<false, vec2_t<T>>(rin, oe.xy); q.ert = ldb<false, T>(rin, oe.t);
        q.eap = ldb<false, vec2_t<T>>(Apin, oe.xy); q.eat = ldb<false, T>(Apin, oe.t);
        q.ew2 = ldb<false, T>(pre, oe.s);
        if (!(P0 && !E)) { q.eq = ldb<false, vec2_t<T>>(pin, oe.xy); q.eqt = ldb<false, T>(pin, oe.t); }
    }
    return q;
}
// r_i from r_{i-1}, Ap_{i-1} (iw_residual's expression), then z_i and p_i (make_p<2>)
template <typename T>
__device__ __forceinline__ void make_rp(const Args<T>& a, int f, T alpha, T beta, T r0, T r1, T r2, T a0, T a1,
                                        T a2, T w2, T q0, T q1, T q2, T& rx, T& ry, T& rt, T& px, T& py,
                                        T& pt) {
    rx = r0 - alpha * a0; ry = r1 - alpha * a1; rt = r2 - alpha * a2;
    make_p<T, 2>(a, f, beta, rx, ry, rt, w2, q0, q1, q2, px, py, pt);
}
// Finish a raw row: r_i, p_i, the edge pixel's p and residual; an owned row (own) also
// stores r_i (unless rout is null) and the updated delta right here and adds its r_i.W r_i.
template <typename T, int DM, bool NT, int E, bool P0 = false>
__device__ __forceinline__ RRow<T> finish_rrow(const Args<T>& a, const RRaw<T>& qin, T beta, T alpha, T alpha2, bool own,
                                               const WaveGeom& g, int y, unsigned tb, T* rout, T* delta,
                                               acc_t& rzd) {
    RRow<T> o;
    RRaw<T> q = qin;
    const int f = q.in ? q.f : 0;
    if constexpr (P0) {   // p_0 = pre r_0 (PCGInit1's p, iw_jtf_apply's cpx / cpy / cpt: the same T products)
        const T w0 = pre_offset(a, f);
        if (E == 0) { q.q.x = opaque(w0 * q.r.x); q.q.y = opaque(w0 * q.r.y); q.qt = opaque(q.w2 * q.rt); }
        else { q.q2.x = opaque(w0 * q.q2.x); q.q2.y = opaque(w0 * q.q2.y); q.q2t = opaque(q.w2 * q.q2t); }   // pin2 held r_0
    }
    o.act = f & 1;
    o.fit = (f >> 1) & 1;
    o.ux = q.in ? q.u.x : 0.f;
    o.uy = q.in ? q.u.y : 0.f;
    sc_of(q.in ? q.ang : (T)0, &o.c, &o.s);
    make_rp(a, f, alpha, beta, q.r.x, q.r.y, q.rt, q.ap.x, q.ap.y, q.at, q.w2, q.q.x, q.q.y, q.qt, o.rx, o.ry, o.rt,
            o.px, o.py, o.pt);
    o.w0 = a.use_pre ? pre_offset(a, f) : (T)1;
    o.w2 = a.use_pre ? q.w2 : (T)1;
    if (own && g.out_lane) {
        const POff<T> off((unsigned)a.dom.off(g.x, y), tb);
        if (DM != 0) {
            // delta (+)= [alpha_{i-2} p_{i-2} (E)] + alpha_{i-1} p_{i-1}, term by term
            vec2_t<T> d;
            T dt;
            if (E) {
                if (DM == 1) { d.x = alpha2 * q.q2.x; d.y = alpha2 * q.q2.y; dt = alpha2 * q.q2t; }
                else { d.x = fmad(alpha2, q.q2.x, q.d.x); d.y = fmad(alpha2, q.q2.y, q.d.y); dt = fmad(alpha2, q.q2t, q.dt); }
                d.x = fmad(alpha, q.q.x, d.x); d.y = fmad(alpha, q.q.y, d.y); dt = fmad(alpha, q.qt, dt);
            } else if (DM == 1) {
                d.x = alpha * q.q.x; d.y = alpha * q.q.y; dt = alpha * q.qt;
            } else {
                d.x = fmad(alpha, q.q.x, q.d.x); d.y = fmad(alpha, q.q.y, q.d.y); dt = fmad(alpha, q.qt, q.dt);
            }
            if (!o.act) { d.x = 0; d.y = 0; dt = 0; }
            stb<NT>(delta, off.xy, d); stb<NT>(delta, off.t, dt);
        }
        if (rout) {
            vec2_t<T> r; r.x = o.rx; r.y = o.ry;
            stb<NT>(rout, off.xy, r); stb<NT>(rout, off.t, o.rt);
        }
        rzd += wdot3(o.w0, o.rx, o.rx, o.w0, o.ry, o.ry, o.w2, o.rt, o.rt);
    }
    if (!o.act) { o.px = 0; o.py = 0; o.pt = 0; }
    const int ef = q.ein ? q.ef : 0;
    if constexpr (P0 && E == 0) {
        const T we = pre_offset(a, ef);
        q.eq.x = opaque(we * q.er.x); q.eq.y = opaque(we * q.er.y); q.eqt = opaque(q.ew2 * q.ert);
    }
    o.eact = ef & 1;
    o.eux = q.ein ? q.eu.x : 0.f;
    o.euy = q.ein ? q.eu.y : 0.f;
    T ec, es, ept, erx, ery, ert, ax, ay;
    sc_of(q.ein ? q.eang : (T)0, &ec, &es);
    make_rp(a, ef, alpha, beta, q.er.x, q.er.y, q.ert, q.eap.x, q.eap.y, q.eat, q.ew2, q.eq.x, q.eq.y, q.eqt, erx,
            ery, ert, o.epx, o.epy, ept);
    if (!o.eact) { o.epx = 0; o.epy = 0; ept = 0; }
    jedge(o.epx, o.epy, ept, ec, es, o.eux, o.euy, o.px, o.py, o.ux, o.uy, o.eact && o.act, a.wr,
          o.ejx, o.ejy, ax, ay);
    return o;
}
// P0: see raw_rrow; pass 2 then reads r_0 through pin2 from the buffer it writes r_2 to
// (rout), own pixel before own pixel: those two are not __restrict__
template <typename T, int DM, int NT = 2, int E = 0, bool P0 = false>
__global__ __launch_bounds__(kBlock) void iw_apply_res(Args<T> a, const T* __restrict__ pin,
                                                       const T* __restrict__ rin, const T* __restrict__ Apin,
                                                       const T* __restrict__ pre, T* __restrict__ pout,
                                                       T* rout, T* __restrict__ Apout,
                                                       T* __restrict__ delta, double* __restrict__ sc,
                                                       int prev, double base_scale, ReduceSlot rs,
                                                       const T* pin2 = nullptr) {
    constexpr bool LNT = (NT & 1) != 0, SNT = (NT & 2) != 0;
    IW_PRE_TABLE(a);
    // 64-column strips with the 2-lane edge record (iw_apply's geometry): every store is a
    // whole aligned 256-B run per wave. (62-column strips without the edge record — 116
    // instead of 154 VGPRs, 4 waves per SIMD — took 423-502 us against 406-441: their
    // stores split cache lines between waves.)
    const WaveGeom g = geom(a);
    // iteration i-1's scalars: alpha_{i-1} = rz / pAp; beta_i from the identity over rz
    const double rzp = sc[prev], papp = sc[prev + 1];
    // the identity takes alpha as the pixels apply it (rounded to T): with the cancellation
    // in it (rz_i << rz_{i-1}) the fp64 alpha would be off by ~1e-7 x rz_{i-1} / rz_i
    const T alpha = pcg_alpha<T>(rzp, papp);
    const double alpha_d = (double)alpha;
    const double rz_id = base_scale * rzp - 2.0 * alpha_d * sc[prev + 2] + alpha_d * alpha_d * sc[prev + 3];
    // The identity subtracts fp64 sums of size rz_{i-1}: its absolute error is ~1e-14 rz_{i-1},
    // i.e. ~1e-14 in beta whatever rz_i / rz_{i-1} is, negligible in p_i. It cancels to <= 0
    // only where the true beta is itself below that error: beta_i = 0 there (the direct
    // r_i.z_i of this pass is >= 0 by construction, so a negative beta is never right).
    const T beta = rz_id > 0.0 && rzp > 0.0 ? (T)(rz_id / rzp) : (T)0;
    // E: p_{i-2}'s delta term was deferred by the previous pass; alpha_{i-2} from its slots
    const T alpha2 = E ? pcg_alpha<T>(sc[prev - kSlots], sc[prev - kSlots + 1]) : (T)0;
    if (blockIdx.x == 0 && threadIdx.x == 0) sc[prev + kSlots + 4] = rz_id;
    const T wr = a.wr, wf2 = a.wf * a.wf;
    const unsigned tb = (unsigned)(2 * a.dom.npix_mem() * (long long)sizeof(T));
    acc_t rzd = 0, papd = 0, rapd = 0, apapd = 0;
    if (g.y0 < g.y1) {
        auto raw = [&](int y) {
            return raw_rrow<T, DM, LNT, E, P0>(a, g, y, tb, pin, rin, Apin, pre, delta, pin2, y >= g.y0 && y < g.y1);
        };
        auto fin = [&](const RRaw<T>& q, int y) {
            return finish_rrow<T, DM, SNT, E, P0>(a, q, beta, alpha, alpha2, y >= g.y0 && y < g.y1, g, y, tb, rout,
                                                  delta, rzd);
        };
        const RRow<T> up = fin(raw(g.y0 - 1), g.y0 - 1);
        RRow<T> A = fin(raw(g.y0), g.y0);
        RRow<T> B = fin(raw(g.y0 + 1), g.y0 + 1);
        T in_up_x, in_up_y, my_x, my_y, thm, ax, ay;
        jedge(up.px, up.py, up.pt, up.c, up.s, up.ux, up.uy, A.px, A.py, A.ux, A.uy,
              up.act && A.act, wr, in_up_x, in_up_y, ax, ay);
        jedge(A.px, A.py, A.pt, A.c, A.s, A.ux, A.uy, up.px, up.py, up.ux, up.uy,
              up.act && A.act, wr, my_x, my_y, ax, ay);
        thm = -wr * (ax * my_x + ay * my_y);
        // Ap of row y from (cur, dn) and the carries from the row above; rolls the carries
        auto apply_row = [&](const RRow<T>& cur, const RRow<T>& dn, int y) {
            const T lpx = from_left(cur.px, cur.epx), lpy = from_left(cur.py, cur.epy);
            const T rpx = from_right(cur.px, cur.epx), rpy = from_right(cur.py, cur.epy);
            const float lux = from_left(cur.ux, cur.eux), luy = from_left(cur.uy, cur.euy);
            const float rux = from_right(cur.ux, cur.eux), ruy = from_right(cur.uy, cur.euy);
            const int lact = from_left_i(cur.act, cur.eact), ract = from_right_i(cur.act, cur.eact);
            T jpx_x, jpx_y, apx_x, apx_y, jmx_x, jmx_y, amx_x, amx_y;
            T jpy_x, jpy_y, apy_x, apy_y, jdn_x, jdn_y, adn_x, adn_y;
            jedge(cur.px, cur.py, cur.pt, cur.c, cur.s, cur.ux, cur.uy, rpx, rpy, rux, ruy,
                  cur.act && ract, wr, jpx_x, jpx_y, apx_x, apx_y);
            jedge(cur.px, cur.py, cur.pt, cur.c, cur.s, cur.ux, cur.uy, lpx, lpy, lux, luy,
                  cur.act && lact, wr, jmx_x, jmx_y, amx_x, amx_y);
            jedge(cur.px, cur.py, cur.pt, cur.c, cur.s, cur.ux, cur.uy, dn.px, dn.py, dn.ux, dn.uy,
                  cur.act && dn.act, wr, jpy_x, jpy_y, apy_x, apy_y);
            jedge(dn.px, dn.py, dn.pt, dn.c, dn.s, dn.ux, dn.uy, cur.px, cur.py, cur.ux, cur.uy,
                  cur.act && dn.act, wr, jdn_x, jdn_y, adn_x, adn_y);
            const T inpx_x = from_right(jmx_x, cur.ejx), inpx_y = from_right(jmx_y, cur.ejy);
            const T inmx_x = from_left(jpx_x, cur.ejx), inmx_y = from_left(jpx_y, cur.ejy);
            T aox = wr * ((jpx_x + jmx_x + jpy_x + my_x) - (inpx_x + inmx_x + jdn_x + in_up_x));
            T aoy = wr * ((jpx_y + jmx_y + jpy_y + my_y) - (inpx_y + inmx_y + jdn_y + in_up_y));
            if (cur.fit) { aox += wf2 * cur.px; aoy += wf2 * cur.py; }
            T aot = thm - wr * ((apx_x * jpx_x + apx_y * jpx_y) + (amx_x * jmx_x + amx_y * jmx_y) +
                                (apy_x * jpy_x + apy_y * jpy_y));
            if (!cur.act) { aox = 0; aoy = 0; aot = 0; }
            if (g.out_lane) {
                const POff<T> off((unsigned)a.dom.off(g.x, y), tb);
                if (Apout) {
                    vec2_t<T> v; v.x = aox; v.y = aoy;
                    stb<SNT>(Apout, off.xy, v); stb<SNT>(Apout, off.t, aot);
                }
                vec2_t<T> pv; pv.x = cur.px; pv.y = cur.py;
                stb<SNT>(pout, off.xy, pv); stb<SNT>(pout, off.t, cur.pt);
                papd += dot3(cur.px, aox, cur.py, aoy, cur.pt, aot);
                rapd += wdot3(cur.w0, cur.rx, aox, cur.w0, cur.ry, aoy, cur.w2, cur.rt, aot);
                apapd += wdot3(cur.w0, aox, aox, cur.w0, aoy, aoy, cur.w2, aot, aot);
            }
            in_up_x = jpy_x; in_up_y = jpy_y;
            my_x = jdn_x; my_y = jdn_y;
            thm = -wr * (adn_x * jdn_x + adn_y * jdn_y);
        };
        // two rows per trip, the two row records swapping roles (no register copies). Rows
        // past the halo row y1 are never needed: the last trip's prefetch re-reads row y1
        // (an L2 hit) instead of fetching row y1 + 1 from HBM
        for (int y = g.y0; y < g.y1; y += 2) {
            const RRaw<T> n1 = raw(min(y + 2, g.y1));
            apply_row(A, B, y);
            A = fin(n1, y + 2);
            if (y + 1 >= g.y1) break;
            const RRaw<T> n2 = raw(min(y + 3, g.y1));
            apply_row(B, A, y + 1);
            B = fin(n2, y + 3);
        }
    }
    double v[4] = {(double)rzd, (double)papd, (double)rapd, (double)apapd};
    block_reduce_publish<4>(v, rs, g.tile);
}

// ------------------------------------------- PCG iteration without a stored Ap
// iw_pcg: iw_apply_res's iteration i >= 1 (PCGStep2 + PCGStep3 of iteration i-1, PCGStep1
// of iteration i; :665-731, :814-845, :607-632) with Ap_{i-1} RECOMPUTED from p_{i-1}
// instead of read back: the pass reads r_{i-1} and p_{i-1} (+ the per-pixel angle, UrShape,
// flags and angle pre) and writes r_i and p_i; Ap is never stored (-24 B/px per pass:
// the Ap_{i-1} read and the Ap_i write). Ap_{i-1} is the same expression over the same
// stored p_{i-1} as the previous pass's Ap_{i-1} (apply_ap2 is the one body every pass and
// iw_jtf_apply use), so the identity's sums and r_i agree.
// Geometry: iw_jtf_apply's 60-column strips (x = 60 strip - 2 + lane, no edge record): per
// row, stage A recomputes Ap_{i-1} at every lane from the p_{i-1} window (valid at lanes
// 1..62), forms r_i and p_i there; stage B applies J^T J to p_i one row behind (lanes
// 2..61 are the outputs). A wave reads the unknown rows y0-2 .. y1+1 (p_{i-1} at radius 2).
// The (x, y) pairs are two-lane vectors: the Offset channels, the residuals' two
// components and the rotation derivative become v_pk_{fma,mul,add}_f32 (two fp32 operations
// per instruction), which the pass needs: with twice iw_apply_res's stencil work per
// pixel its VALU issue, not HBM, set its time (round 5, profiles/r05_pcg_pmc.json).
template <typename T>
__device__ __forceinline__ vec2_t<T> shl2(vec2_t<T> v) {   // lane l gets lane l-1's (0 at lane 0)
    vec2_t<T> o;
    o.x = from_left0(v.x); o.y = from_left0(v.y);
    return o;
}
template <typename T>
__device__ __forceinline__ vec2_t<T> shr2(vec2_t<T> v) {   // lane l gets lane l+1's (0 at lane 63)
    vec2_t<T> o;
    o.x = from_right0(v.x); o.y = from_right0(v.y);
    return o;
}
// jedge in pairs: the residual pair J(j -> t) applied to p, and a = dR(t_j)/dt (U_j - U_t)
template <typename T>
__device__ __forceinline__ void jedge2(vec2_t<T> pj, T pjt, T cj, T sj, vec2_t<float> uj, vec2_t<T> pt,
                                       vec2_t<float> ut, bool v, T wr, vec2_t<T>& J, vec2_t<T>& ad) {
    const vec2_t<float> du = uj - ut;   // float subtractions, as the reference's Image reads
    const T dx = (T)du.x, dy = (T)du.y;
    vec2_t<T> ms, cs;
    ms.x = -sj; ms.y = cj;
    cs.x = cj; cs.y = sj;
    ad = ms * dx - cs * dy;
    const vec2_t<T> j = wr * ((pj - pt) - ad * pjt);
    J = v ? j : (vec2_t<T>)0;
}
// Carries of the apply's row recursion: J(up->cur), J(cur->up) and its angle term
template <typename T>
struct ACarry {
    vec2_t<T> in_up, my;
    T thm;
};
template <typename T>
__device__ __forceinline__ ACarry<T> acarry_init(vec2_t<T> up, T upt, T uc, T us, vec2_t<float> uu, bool uact,
                                                 vec2_t<T> cp, T cpt, T cc, T cs, vec2_t<float> cu, bool cact, T wr) {
    ACarry<T> k;
    vec2_t<T> ad;
    jedge2(up, upt, uc, us, uu, cp, cu, uact && cact, wr, k.in_up, ad);
    jedge2(cp, cpt, cc, cs, cu, up, uu, uact && cact, wr, k.my, ad);
    const vec2_t<T> th = ad * k.my;
    k.thm = -wr * (th.x + th.y);
    return k;
}
// Ap = J^T J p of row cur from (cur, dn) and the carry; no edge operand (lanes 0 / 63 are
// never used). Leaves the carry of row dn.
template <typename T>
__device__ __forceinline__ void apply_ap2(vec2_t<T> cp, T cpt, T cc, T cs, vec2_t<float> cu, bool cact, bool cfit,
                                          vec2_t<T> dp, T dpt, T dc, T ds, vec2_t<float> du, bool dact, T wr, T wf2,
                                          ACarry<T>& k, vec2_t<T>& ao, T& aot) {
    const vec2_t<T> lp = shl2(cp), rp = shr2(cp);
    const vec2_t<float> lu = shl2(cu), ru = shr2(cu);
    const int lact = from_left0_i((int)cact), ract = from_right0_i((int)cact);
    vec2_t<T> jpx, apx, jmx, amx, jpy, apy, jdn, adn;
    jedge2(cp, cpt, cc, cs, cu, rp, ru, cact && ract, wr, jpx, apx);
    jedge2(cp, cpt, cc, cs, cu, lp, lu, cact && lact, wr, jmx, amx);
    jedge2(cp, cpt, cc, cs, cu, dp, du, cact && dact, wr, jpy, apy);
    jedge2(dp, dpt, dc, ds, du, cp, cu, cact && dact, wr, jdn, adn);
    const vec2_t<T> inpx = shr2(jmx), inmx = shl2(jpx);
    ao = wr * ((jpx + jmx + jpy + k.my) - (inpx + inmx + jdn + k.in_up));
    if (cfit) ao += wf2 * cp;
    const vec2_t<T> tt = apx * jpx + amx * jmx + apy * jpy;
    aot = k.thm - wr * (tt.x + tt.y);
    if (!cact) { ao = (vec2_t<T>)0; aot = 0; }
    k.in_up = jpy;
    k.my = jdn;
    const vec2_t<T> th = adn * jdn;
    k.thm = -wr * (th.x + th.y);
}
// Raw buffer access (gfx9 V#, dword3 0x00020000): an access at an offset >= num_records is
// dropped (a store) or returns 0 (a load) by the hardware, without touching memory. iw_pcg
// issues every conditional store and own-row load this way, at an out-of-range offset where
// it does not apply, so every row issues the same vector-memory instructions with no branch
// around them. With exec-masked stores the compiler cannot know how many stores follow the
// next row's loads and waits for vmcnt(0) — this row's stores included — before it may use
// them; with a fixed count it waits only for the loads (vmcnt(#stores issued after them)).
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bres(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, p ? (int)bytes : 0, 0x00020000);
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, unsigned off, vec2_t<float> v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, unsigned off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, unsigned off, vec2_t<double> v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}
template <typename V> __device__ __forceinline__ V bld(__amdgpu_buffer_rsrc_t r, unsigned off);
template <> __device__ __forceinline__ float bld<float>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
template <> __device__ __forceinline__ vec2_t<float> bld<vec2_t<float>>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(vec2_t<float>, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
template <> __device__ __forceinline__ double bld<double>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
template <> __device__ __forceinline__ vec2_t<double> bld<vec2_t<double>>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(vec2_t<double>, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <typename T>
struct GRow {          // a finished row of p_{i-1} with the pixel's static data
    vec2_t<T> p;       // p_{i-1} (0 on inactive pixels)
    T pt;
    T c, s;            // cos / sin of the angle
    vec2_t<float> u;
    int f;             // flag byte
    vec2_t<T> r;       // r_{i-1}
    T rt, w2;          // its angle channel, the angle pre
    vec2_t<T> d, q2;   // own rows: delta, p_{i-2} (E)
    T dt, q2t;
    __device__ __forceinline__ bool act() const { return f & 1; }
    __device__ __forceinline__ bool fit() const { return (f >> 1) & 1; }
};
template <typename T>
struct GRaw {
    vec2_t<T> p, r, d, q2;
    T pt, rt, w2, ang, dt, q2t;
    vec2_t<float> u;
    int f, in;
};
// REC: flags, S and the record of iteration i-1 (pin == rin); p_{i-2} (E) from its record,
// r_0's part when P0 (pass 2 forms p_0 from it). oob: an offset past every buffer.
template <typename T, int DM, int E, bool P0, bool REC, bool PRC = false>
__device__ __forceinline__ GRaw<T> raw_grow(const Args<T>& a, const WaveGeom& g, int y, unsigned tb, const T* pin,
                                            const T* rin, const T* pre, __amdgpu_buffer_rsrc_t rdl,
                                            __amdgpu_buffer_rsrc_t rq2, unsigned oob, bool own) {
    GRaw<T> q;
    q.in = present(a.dom, g.x, y);
    const unsigned i = q.in ? (unsigned)a.dom.off(g.x, y) : 0u;
    const POff<T> o(i, tb);
    q.f = ldb<false, uint8_t>(a.flags, i);
    own = own && g.out_lane;
    const unsigned oxy = own ? o.xy : oob, ot = own ? o.t : oob;
    if constexpr (REC) {
        const ROff<T> ro(i);
        ld_srec(a.S, ro.s, q.u, q.ang, q.w2);
        q.r = ldb<false, vec2_t<T>>(rin, ro.r);
        const vec2_t<T> tt = ldb<false, vec2_t<T>>(rin, ro.t);
        q.rt = tt.x; q.pt = tt.y;
        if (!(P0 && !E)) q.p = ldb<false, vec2_t<T>>(rin, ro.p);
        if (DM == 2) { q.d = bld<vec2_t<T>>(rdl, oxy); q.dt = bld<T>(rdl, ot); }
        if (E) {
            q.q2 = bld<vec2_t<T>>(rq2, own ? (P0 ? ro.r : ro.p) : oob);
            const vec2_t<T> t2 = bld<vec2_t<T>>(rq2, own ? ro.t : oob);
            q.q2t = P0 ? t2.x : t2.y;
        }
        return q;
    }
    q.u = ldb<false, vec2_t<float>>(a.U, 8u * i);
    q.ang = ldb<false, T>(a.A, o.s);
    q.r = ldb<false, vec2_t<T>>(rin, o.xy); q.rt = ldb<false, T>(rin, o.t);
    if constexpr (!PRC) q.w2 = ldb<false, T>(pre, o.s);
    else q.w2 = 0;
    if (!(P0 && !E)) { q.p = ldb<false, vec2_t<T>>(pin, o.xy); q.pt = ldb<false, T>(pin, o.t); }
    if (DM == 2) { q.d = bld<vec2_t<T>>(rdl, oxy); q.dt = bld<T>(rdl, ot); }
    if (E) { q.q2 = bld<vec2_t<T>>(rq2, oxy); q.q2t = bld<T>(rq2, ot); }
    return q;
}
template <typename T, int E, bool P0>
__device__ __forceinline__ GRow<T> finish_grow(const Args<T>& a, const GRaw<T>& q) {
    GRow<T> o;
    o.f = q.in ? q.f : 0;
    o.u = q.in ? q.u : (vec2_t<float>)0.f;
    sc_of(q.in ? q.ang : (T)0, &o.c, &o.s);
    o.r = q.r; o.rt = q.rt; o.w2 = q.w2;
    o.d = q.d; o.dt = q.dt;
    o.q2 = q.q2; o.q2t = q.q2t;
    if constexpr (P0) {   // p_0 = pre r_0 (iw_jtf_apply's FRow::p: the same rounded T products)
        const T w0 = pre_offset(a, o.f);
        if (E == 0) { o.p = opaque(w0 * q.r); o.pt = opaque(q.w2 * q.rt); }
        else { o.q2 = opaque(w0 * q.q2); o.q2t = opaque(q.w2 * q.q2t); o.p = q.p; o.pt = q.pt; }
    } else {
        o.p = q.p; o.pt = q.pt;
    }
    if (!o.act()) { o.p = (vec2_t<T>)0; o.pt = 0; }
    return o;
}
// Stage B's view of a row: p_i, r_i, the weights and the static data
template <typename T>
struct HRow {
    vec2_t<T> p;
    T pt, c, s;
    vec2_t<float> u;
    bool act, fit;
    vec2_t<T> r;
    T rt, w0, w2;
};
// SNT: streaming stores. The 60-column strips store 240-byte row segments that straddle
// cache lines shared with the neighbouring strips; plain stores let the L2 merge them.
// U2: two rows per loop trip with the row records swapping roles (no register copies, but
// more VGPRs live: 138-168 against 120-142, 3 waves per SIMD instead of 4 on the odd passes)
// PF2 (with U2): two raw rows in flight per wave instead of one.
// REC: the REC layout (Args::S): pin == rin is the record of iteration i-1, pout == rout
// that of iteration i, both halves stored by stage A; pin2 the record of iteration i-2.
// PRC (passes without P0): the angle preconditioner recomputed from the stencil's geometry
// (diag_a2 over the four edges, in iw_jtf's order, pre_angle) instead of read: bitwise the
// stored value, 4 B/px less per pass.
template <typename T, int DM, int E, bool P0, bool SNT, bool U2, bool PF2, bool REC, bool PRC = false>
__device__ __forceinline__ void iw_pcg_body(const Args<T>& a, const T* __restrict__ pin, const T* __restrict__ rin,
                                            const T* __restrict__ pre, T* __restrict__ pout, T* rout,
                                            T* __restrict__ delta, double* __restrict__ sc, int prev,
                                            double base_scale, ReduceSlot rs, const T* pin2) {
    IW_PRE_TABLE(a);
    const WaveGeom g = geom_fused(a);
    // the scalars exactly as iw_apply_res forms them
    const double rzp = sc[prev], papp = sc[prev + 1];
    const T alpha = pcg_alpha<T>(rzp, papp);
    const double alpha_d = (double)alpha;
    const double rz_id = base_scale * rzp - 2.0 * alpha_d * sc[prev + 2] + alpha_d * alpha_d * sc[prev + 3];
    const T beta = rz_id > 0.0 && rzp > 0.0 ? (T)(rz_id / rzp) : (T)0;
    const T alpha2 = E ? pcg_alpha<T>(sc[prev - kSlots], sc[prev - kSlots + 1]) : (T)0;
    if (blockIdx.x == 0 && threadIdx.x == 0) sc[prev + kSlots + 4] = rz_id;
    const T wr = a.wr, wf2 = a.wf * a.wf;
    const long long nplane = a.dom.npix_mem();
    const unsigned tb = (unsigned)(2 * nplane * (long long)sizeof(T));
    // the unknown-layout vectors' byte size (REC: the records'): the buffers' range and the
    // drop offset
    const unsigned vb = (unsigned)(3 * nplane * (long long)sizeof(T));
    const unsigned oob = REC ? 2u * vb : vb;
    const __amdgpu_buffer_rsrc_t r_out = bres(rout, oob), r_p = bres(pout, oob), r_d = bres(delta, vb),
                                 r_q2 = bres(pin2, oob);
    acc_t rzd = 0, papd = 0, rapd = 0, apapd = 0;
    if (g.y0 < g.y1) {
        auto raw = [&](int y) {
            return raw_grow<T, DM, E, P0, REC, PRC>(a, g, y, tb, pin, rin, pre, r_d, r_q2, oob, y >= g.y0 && y < g.y1);
        };
        auto fin = [&](const GRaw<T>& q) { return finish_grow<T, E, P0>(a, q); };
        // stage A at row y (cur = row y, dn = row y+1, carry from row y-1): Ap_{i-1}, then
        // r_i and p_i (stores r_i and delta on an owned row)
        ACarry<T> ka;
        const T wr2 = a.wr * a.wr;
        T dthm_a = 0;   // PRC: the angle diag term of the edge to the previous row (iw_jtf's k.dthm)
        auto stage_a = [&](const GRow<T>& cur, const GRow<T>& dn, int y) {
            vec2_t<T> ap;
            T at;
            apply_ap2(cur.p, cur.pt, cur.c, cur.s, cur.u, cur.act(), cur.fit(), dn.p, dn.pt, dn.c, dn.s, dn.u,
                      dn.act(), wr, wf2, ka, ap, at);
            HRow<T> h;
            h.c = cur.c; h.s = cur.s; h.u = cur.u; h.act = cur.act(); h.fit = cur.fit();
            // r_i = r_{i-1} - alpha Ap_{i-1}, z_i = pre r_i, p_i = z_i + beta p_{i-1}
            const T w0 = pre_offset(a, cur.f);
            h.r = cur.r - alpha * ap;
            h.rt = cur.rt - alpha * at;
            // (z = 1 r = r exactly without a preconditioner: one select per weight, not per channel)
            h.w0 = a.use_pre ? w0 : (T)1;
            if constexpr (PRC) {   // iw_jtf's dt: previous row's edge, +x, -x, next row's edge
                const vec2_t<float> lu = shl2(cur.u), ru = shr2(cur.u);
                const bool ca = cur.act(), da = dn.act();
                const bool lact = from_left0_i((int)ca) != 0, ract = from_right0_i((int)ca) != 0;
                const T dt = dthm_a + (ca && ract ? diag_a2(cur.c, cur.s, cur.u.x, cur.u.y, ru.x, ru.y, wr2) : (T)0) +
                             (ca && lact ? diag_a2(cur.c, cur.s, cur.u.x, cur.u.y, lu.x, lu.y, wr2) : (T)0) +
                             (ca && da ? diag_a2(cur.c, cur.s, cur.u.x, cur.u.y, dn.u.x, dn.u.y, wr2) : (T)0);
                dthm_a = ca && da ? diag_a2(dn.c, dn.s, dn.u.x, dn.u.y, cur.u.x, cur.u.y, wr2) : (T)0;
                h.w2 = a.use_pre ? (ca ? pre_angle(dt) : (T)0) : (T)1;
            } else {
                h.w2 = a.use_pre ? cur.w2 : (T)1;
            }
            const vec2_t<T> z = h.w0 * h.r;
            const T zt = h.w2 * h.rt;
            h.p = z + beta * cur.p;
            h.pt = zt + beta * cur.pt;
            const bool mine = y >= g.y0 && y < g.y1 && g.out_lane;
            {
                const unsigned iy = mine ? (unsigned)a.dom.off(g.x, y) : 0u;
                const POff<T> off(iy, tb);
                const unsigned oxy = mine ? off.xy : oob, ot = mine ? off.t : oob;
                if (DM != 0) {   // iw_apply_res's deferred delta terms, term by term (explicit fmas)
                    vec2_t<T> d;
                    T dt;
                    if (E) {
                        if (DM == 1) { d = alpha2 * cur.q2; dt = alpha2 * cur.q2t; }
                        else { d = __builtin_elementwise_fma((vec2_t<T>)alpha2, cur.q2, cur.d); dt = fmad(alpha2, cur.q2t, cur.dt); }
                        d = __builtin_elementwise_fma((vec2_t<T>)alpha, cur.p, d); dt = fmad(alpha, cur.pt, dt);
                    } else if (DM == 1) {
                        d = alpha * cur.p; dt = alpha * cur.pt;
                    } else {
                        d = __builtin_elementwise_fma((vec2_t<T>)alpha, cur.p, cur.d); dt = fmad(alpha, cur.pt, cur.dt);
                    }
                    if (!h.act) { d = (vec2_t<T>)0; dt = 0; }
                    bst(r_d, oxy, d); bst(r_d, ot, dt);
                }
                if constexpr (REC) {   // the whole record (p_i zero on inactive pixels, as stage B's)
                    const ROff<T> ro(iy);
                    const vec2_t<T> pm = h.act ? h.p : (vec2_t<T>)0;
                    vec2_t<T> tt;
                    tt.x = h.rt; tt.y = h.act ? h.pt : (T)0;
                    bst(r_out, mine ? ro.r : oob, h.r); bst(r_out, mine ? ro.p : oob, pm);
                    bst(r_out, mine ? ro.t : oob, tt);
                } else {
                    bst(r_out, oxy, h.r); bst(r_out, ot, h.rt);   // rout null (last pass): dropped
                }
                const acc_t rz = wdot3(h.w0, h.r.x, h.r.x, h.w0, h.r.y, h.r.y, h.w2, h.rt, h.rt);
                rzd += mine ? rz : 0.0;
            }
            if (!h.act) { h.p = (vec2_t<T>)0; h.pt = 0; }
            return h;
        };
        // the walk: row Y(k), k = 0 .. n - 1 (halo rows Y(-2), Y(-1), Y(n), Y(n + 1)); top to
        // bottom, or with Args::alt on odd row chunks bottom to top — the same chain with
        // "the next row" the one above (apply_ap2's carries then come from below: the same
        // residual values, summed in the mirrored order)
        const int n = g.y1 - g.y0;
        const bool up = a.alt && (((g.y0 - a.dom.y_lo) / a.rows) & 1);
        auto Y = [&](int k) { return up ? g.y1 - 1 - k : g.y0 + k; };
        const GRow<T> g0 = fin(raw(Y(-2)));
        GRow<T> qc = fin(raw(Y(-1)));
        GRow<T> qd = fin(raw(Y(0)));
        ka = acarry_init(g0.p, g0.pt, g0.c, g0.s, g0.u, g0.act(), qc.p, qc.pt, qc.c, qc.s, qc.u, qc.act(), wr);
        if constexpr (PRC)
            dthm_a = g0.act() && qc.act() ? diag_a2(qc.c, qc.s, qc.u.x, qc.u.y, g0.u.x, g0.u.y, wr2) : (T)0;
        HRow<T> hup = stage_a(qc, qd, Y(-1));
        qc = qd;
        qd = fin(raw(Y(1)));
        HRow<T> hc = stage_a(qc, qd, Y(0));
        qc = qd;
        qd = fin(raw(Y(2)));
        ACarry<T> kb = acarry_init(hup.p, hup.pt, hup.c, hup.s, hup.u, hup.act, hc.p, hc.pt, hc.c, hc.s, hc.u, hc.act, wr);
        // stage B at row y: Ap_i from (cur = row y, dn = row y+1), stores p_i, the three sums
        auto stage_b = [&](const HRow<T>& cur, const HRow<T>& dn, int y) {
            vec2_t<T> ao;
            T aot;
            apply_ap2(cur.p, cur.pt, cur.c, cur.s, cur.u, cur.act, cur.fit, dn.p, dn.pt, dn.c, dn.s, dn.u, dn.act, wr,
                      wf2, kb, ao, aot);
            {
                if constexpr (!REC) {
                    const unsigned iy = g.out_lane ? (unsigned)a.dom.off(g.x, y) : 0u;
                    const POff<T> off(iy, tb);
                    bst(r_p, g.out_lane ? off.xy : oob, cur.p); bst(r_p, g.out_lane ? off.t : oob, cur.pt);
                }
                const acc_t s1 = dot3(cur.p.x, ao.x, cur.p.y, ao.y, cur.pt, aot);
                const acc_t s2 = wdot3(cur.w0, cur.r.x, ao.x, cur.w0, cur.r.y, ao.y, cur.w2, cur.rt, aot);
                const acc_t s3 = wdot3(cur.w0, ao.x, ao.x, cur.w0, ao.y, ao.y, cur.w2, aot, aot);
                papd += g.out_lane ? s1 : 0.0;
                rapd += g.out_lane ? s2 : 0.0;
                apapd += g.out_lane ? s3 : 0.0;
            }
        };
        // two rows per trip, the row records swapping roles (no register copies): entering a
        // trip at row y, q0 / q1 hold rows y+1 / y+2 and h0 row y
        if constexpr (!U2) {
            for (int k = 0; k < n; ++k) {
                const GRaw<T> nx = raw(Y(min(k + 3, n + 1)));
                const HRow<T> hd = stage_a(qc, qd, Y(k + 1));
                stage_b(hc, hd, Y(k));
                hc = hd;
                qc = qd;
                qd = fin(nx);
            }
        } else if constexpr (PF2) {
            GRow<T> q0 = qc, q1 = qd;
            HRow<T> h0 = hc, h1;
            GRaw<T> na = raw(Y(min(3, n + 1))), nb = raw(Y(min(4, n + 1)));
            for (int k = 0; k < n; k += 2) {
                h1 = stage_a(q0, q1, Y(k + 1));
                stage_b(h0, h1, Y(k));
                q0 = fin(na);
                if (k + 1 >= n) break;
                na = raw(Y(min(k + 5, n + 1)));
                h0 = stage_a(q1, q0, Y(k + 2));
                stage_b(h1, h0, Y(k + 1));
                q1 = fin(nb);
                nb = raw(Y(min(k + 6, n + 1)));
            }
        } else {
        GRow<T> q0 = qc, q1 = qd;
        HRow<T> h0 = hc, h1;
        for (int k = 0; k < n; k += 2) {
            // stage A needs rows up to Y(n + 1); the last trip re-reads that row (an L2 hit)
            const GRaw<T> n1 = raw(Y(min(k + 3, n + 1)));
            h1 = stage_a(q0, q1, Y(k + 1));
            stage_b(h0, h1, Y(k));
            q0 = fin(n1);
            if (k + 1 >= n) break;
            const GRaw<T> n2 = raw(Y(min(k + 4, n + 1)));
            h0 = stage_a(q1, q0, Y(k + 2));
            stage_b(h1, h0, Y(k + 1));
            q1 = fin(n2);
        }
        }
    }
    double v[4] = {(double)rzd, (double)papd, (double)rapd, (double)apapd};
    block_reduce_publish<4>(v, rs, g.tile);
}
template <typename T, int DM, int E = 0, bool P0 = false, bool SNT = false, bool U2 = false, bool PF2 = false,
          bool REC = false, bool PRC = false>
#ifndef IW_PCG_WAVES
#define IW_PCG_WAVES 1   // A/B builds (tools/ab_build.sh): the minimum waves per SIMD iw_pcg is held to
#endif
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(IW_PCG_WAVES))) void iw_pcg(Args<T> a, const T* __restrict__ pin, const T* __restrict__ rin,
                                                 const T* __restrict__ pre, T* __restrict__ pout, T* rout,
                                                 T* __restrict__ delta, double* __restrict__ sc, int prev,
                                                 double base_scale, ReduceSlot rs, const T* pin2 = nullptr) {
    iw_pcg_body<T, DM, E, P0, SNT, U2, PF2, REC, PRC>(a, pin, rin, pre, pout, rout, delta, sc, prev, base_scale, rs,
                                                      pin2);
}

// ------------------------------------------------------------- value rows
template <typename T>
struct VRaw {
    Vec2<T> o;
    T t;
    float2 u, c;
    float m;
    int in;
    Vec2<T> eo;        // edge pixel
    T et;
    float2 eu;
    float em;
    int ein;
};
template <typename T>
struct VRow {
    T ox, oy, t, c, s;
    float ux, uy, cx, cy;
    int act, fit;
    T eox, eoy;        // edge pixel seen by this lane
    float eux, euy;
    int eact;
    T ec, es;          // its cos / sin (only the J^T F kernel needs them)
};
// EDGE: the strip's two outside columns ride along (lanes 0 / 63); EDGE_ANGLE: with
// their angle (only J^T F needs it)
template <typename T, bool EDGE_ANGLE, bool EDGE = true>
__device__ __forceinline__ VRaw<T> raw_vrow(const Args<T>& a, const WaveGeom& g, int y) {
    VRaw<T> q;
    q.in = present(a.dom, g.x, y);
    if (!EDGE) {   // iw_jtf_apply: 32-bit byte offsets from uniform bases (offsets_fit_32)
        const unsigned i = q.in ? (unsigned)a.dom.off(g.x, y) : 0u;
        const vec2_t<T> o = ldb<false, vec2_t<T>>(a.O, i * 2u * (unsigned)sizeof(T));
        q.o = Vec2<T>{o.x, o.y};
        q.t = ldb<false, T>(a.A, i * (unsigned)sizeof(T));
        q.u = ldb<false, float2>(a.U, 8u * i);
        q.c = ldb<false, float2>(a.C, 8u * i);
        q.m = ldb<false, float>(a.M, 4u * i);
        q.ein = 0;
        return q;
    }
    const long long i = q.in ? a.dom.off(g.x, y) : 0;
    q.o = reinterpret_cast<const Vec2<T>*>(a.O)[i];
    q.t = a.A[i];
    q.u = reinterpret_cast<const float2*>(a.U)[i];
    q.c = reinterpret_cast<const float2*>(a.C)[i];
    q.m = a.M[i];
    q.ein = 0;
    if (EDGE && g.edge_lane) {
        q.ein = present(a.dom, g.ex, y);
        const long long e = q.ein ? a.dom.off(g.ex, y) : 0;
        q.eo = reinterpret_cast<const Vec2<T>*>(a.O)[e];
        if (EDGE_ANGLE) q.et = a.A[e];
        q.eu = reinterpret_cast<const float2*>(a.U)[e];
        q.em = a.M[e];
    }
    return q;
}
template <typename T, bool EDGE_ANGLE, bool EDGE = true>
__device__ __forceinline__ VRow<T> finish_vrow(const VRaw<T>& r) {
    VRow<T> q;
    q.ox = r.in ? r.o.x : (T)0;
    q.oy = r.in ? r.o.y : (T)0;
    q.t = r.in ? r.t : (T)0;
    q.ux = r.in ? r.u.x : 0.f; q.uy = r.in ? r.u.y : 0.f;
    q.cx = r.in ? r.c.x : -1.f; q.cy = r.in ? r.c.y : -1.f;
    q.act = r.in && (r.m == 0.f);
    q.fit = (q.cx >= 0.f) && (q.cy >= 0.f);
    sc_of(q.t, &q.c, &q.s);
    if (!EDGE) {
        q.eox = 0; q.eoy = 0; q.eux = 0.f; q.euy = 0.f; q.eact = 0; q.ec = 0; q.es = 0;
        return q;
    }
    q.eox = r.ein ? r.eo.x : (T)0;
    q.eoy = r.ein ? r.eo.y : (T)0;
    q.eux = r.ein ? r.eu.x : 0.f; q.euy = r.ein ? r.eu.y : 0.f;
    q.eact = r.ein && (r.em == 0.f);
    if (EDGE_ANGLE) sc_of(r.ein ? r.et : (T)0, &q.ec, &q.es);
    return q;
}

// ------------------------------------------------------------- J^T F rows
// What a J^T F row evaluation carries from the row above: the residual of the pixel
// above pointing down at this pixel (inup), this pixel's residual pointing up (my) with
// its angle-gradient term (thm) and angle-diagonal term (dthm), and whether it is valid.
template <typename T>
struct JCarry {
    T inup_x, inup_y, my_x, my_y, thm, dthm;
    int vmy;
};
template <typename T>
__device__ __forceinline__ JCarry<T> jcarry_init(const VRow<T>& up, const VRow<T>& cur, T wr) {
    JCarry<T> k;
    T ax, ay;
    const bool vup = up.act && cur.act;
    eedge(up.ox, up.oy, up.c, up.s, up.ux, up.uy, cur.ox, cur.oy, cur.ux, cur.uy, vup, wr,
          k.inup_x, k.inup_y, ax, ay);
    eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, up.ox, up.oy, up.ux, up.uy, vup, wr,
          k.my_x, k.my_y, ax, ay);
    k.thm = -wr * (ax * k.my_x + ay * k.my_y);
    k.dthm = vup ? diag_a2(cur.c, cur.s, cur.ux, cur.uy, up.ux, up.uy, wr * wr) : (T)0;
    k.vmy = vup;
    return k;
}
// One row of evalJTF (o.t:2870-2913) at the unknowns: the gradient F = J^T e per
// channel (fx, fy, ft), the angle channel's diag(J^T J) (dt), the number of valid
// rigidity residuals (nv). Consumes the carry of row cur and leaves the carry of row dn.
template <typename T>
struct JRow {
    T fx, fy, ft, dt;
    int nv;
};
// EDGE = false (iw_jtf_apply): no outside columns; the values at lanes 0 / 63 are
// meaningless and unused.
template <typename T, bool EDGE = true>
__device__ __forceinline__ JRow<T> jtf_row(const Args<T>& a, const VRow<T>& cur, const VRow<T>& dn,
                                           JCarry<T>& k) {
    const T wr = a.wr, wf = a.wf, wr2 = a.wr * a.wr;
    JRow<T> o;
    T ax, ay;
    // (EDGE = false: zero-fill shifts, the end lanes' values are unused)
    const T lox = EDGE ? from_left(cur.ox, cur.eox) : from_left0(cur.ox);
    const T loy = EDGE ? from_left(cur.oy, cur.eoy) : from_left0(cur.oy);
    const T rox = EDGE ? from_right(cur.ox, cur.eox) : from_right0(cur.ox);
    const T roy = EDGE ? from_right(cur.oy, cur.eoy) : from_right0(cur.oy);
    const float lux = EDGE ? from_left(cur.ux, cur.eux) : from_left0(cur.ux);
    const float luy = EDGE ? from_left(cur.uy, cur.euy) : from_left0(cur.uy);
    const float rux = EDGE ? from_right(cur.ux, cur.eux) : from_right0(cur.ux);
    const float ruy = EDGE ? from_right(cur.uy, cur.euy) : from_right0(cur.uy);
    const int lact = EDGE ? from_left_i(cur.act, cur.eact) : from_left0_i(cur.act);
    const int ract = EDGE ? from_right_i(cur.act, cur.eact) : from_right0_i(cur.act);
    const bool vpx = cur.act && ract, vmx = cur.act && lact, vpy = cur.act && dn.act;
    T epx_x, epx_y, apx_x, apx_y, emx_x, emx_y, amx_x, amx_y;
    T epy_x, epy_y, apy_x, apy_y, edn_x, edn_y, adn_x, adn_y, ee_x, ee_y;
    eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, rox, roy, rux, ruy, vpx, wr, epx_x,
          epx_y, apx_x, apx_y);
    eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, lox, loy, lux, luy, vmx, wr, emx_x,
          emx_y, amx_x, amx_y);
    eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, dn.ox, dn.oy, dn.ux, dn.uy, vpy, wr,
          epy_x, epy_y, apy_x, apy_y);
    eedge(dn.ox, dn.oy, dn.c, dn.s, dn.ux, dn.uy, cur.ox, cur.oy, cur.ux, cur.uy, vpy, wr,
          edn_x, edn_y, adn_x, adn_y);
    // the strip's outside neighbour's residual pointing at lane 0 / 63
    if (EDGE) {
        eedge(cur.eox, cur.eoy, cur.ec, cur.es, cur.eux, cur.euy, cur.ox, cur.oy, cur.ux, cur.uy,
              cur.eact && cur.act, wr, ee_x, ee_y, ax, ay);
    } else {
        ee_x = 0; ee_y = 0;
    }
    const T inpx_x = EDGE ? from_right(emx_x, ee_x) : from_right0(emx_x);
    const T inpx_y = EDGE ? from_right(emx_y, ee_y) : from_right0(emx_y);
    const T inmx_x = EDGE ? from_left(epx_x, ee_x) : from_left0(epx_x);
    const T inmx_y = EDGE ? from_left(epx_y, ee_y) : from_left0(epx_y);
    o.fx = wr * ((epx_x + emx_x + epy_x + k.my_x) - (inpx_x + inmx_x + edn_x + k.inup_x));
    o.fy = wr * ((epx_y + emx_y + epy_y + k.my_y) - (inpx_y + inmx_y + edn_y + k.inup_y));
    o.ft = k.thm - wr * ((apx_x * epx_x + apx_y * epx_y) + (amx_x * emx_x + amx_y * emx_y) +
                         (apy_x * epy_x + apy_y * epy_y));
    o.nv = (int)vpx + (int)vmx + (int)vpy + k.vmy;
    o.dt = k.dthm + (vpx ? diag_a2(cur.c, cur.s, cur.ux, cur.uy, rux, ruy, wr2) : (T)0) +
           (vmx ? diag_a2(cur.c, cur.s, cur.ux, cur.uy, lux, luy, wr2) : (T)0) +
           (vpy ? diag_a2(cur.c, cur.s, cur.ux, cur.uy, dn.ux, dn.uy, wr2) : (T)0);
    if (cur.fit) {
        o.fx += wf * wf * (cur.ox - (T)cur.cx);
        o.fy += wf * wf * (cur.oy - (T)cur.cy);
    }
    k.inup_x = epy_x; k.inup_y = epy_y;
    k.my_x = edn_x; k.my_y = edn_y;
    k.thm = -wr * (adn_x * edn_x + adn_y * edn_y);
    k.dthm = vpy ? diag_a2(dn.c, dn.s, dn.ux, dn.uy, cur.ux, cur.uy, wr2) : (T)0;
    k.vmy = vpy;
    return o;
}
// The solver's per-pixel outputs of a J^T F row: r = -F, the flag byte, the Offset and
// angle preconditioners (guardedInvert, :478-507; 1/(1+1)^2 when UsePreconditioner(false),
// PCGInit1 :543-550) — every value zero on an inactive pixel.
template <typename T>
struct JOut {
    T rx, ry, rt, wo, wt;
    int f;
};
template <typename T>
__device__ __forceinline__ JOut<T> jtf_out(const Args<T>& a, const VRow<T>& cur, const JRow<T>& j) {
    JOut<T> o;
    o.f = cur.act | (cur.fit << 1) | (j.nv << 2);
    o.rx = 0; o.ry = 0; o.rt = 0; o.wo = 0; o.wt = 0;
    if (cur.act) {
        o.rx = -j.fx; o.ry = -j.fy; o.rt = -j.ft;
        o.wo = pre_offset(a, o.f);   // 1/(1+sqrt(2 wr^2 nv + wf^2 [fit]))^2
        if (a.use_pre) {
            o.wt = pre_angle(j.dt);
        } else {
            o.wt = (T)0.25;
        }
    }
    return o;
}

// ------------------------------------------------------------- J^T F kernel
// r = -J^T F, pre = 1/(1+sqrt(diag J^T J))^2 (1/(1+1)^2 when UsePreconditioner(false)),
// flags, and sc[rs.out] = sum r.(pre r) over active pixels (alpha numerator).
// OUT 0: only the angle channel of pre (the solver's compressed layout, Args::preO);
// OUT 1: all three preconditioner channels (OptAMD_EvalJTF layout);
// OUT 2: diag(J^T J) in all three channels instead of pre, no reduction (the generic
//        GN/LM driver, which forms pre / the LM diagonal itself).
// ACC: rz[0] summed as iw_jtf_apply sums it (fp64 products and sums, wdot3), the base of
// iw_apply_res's identity on row slabs (an fp32 sum is off by ~1e-7 of rz[0], which the
// identity's cancellation would amplify)
template <typename T, int OUT, bool ACC = false>
__global__ __launch_bounds__(kBlock) void iw_jtf(Args<T> a, T* __restrict__ r, T* __restrict__ pre,
                                                 ReduceSlot rs) {
    IW_PRE_TABLE(a);
    const WaveGeom g = geom(a);
    const T wf = a.wf, wr2 = a.wr * a.wr;
    const long long N = a.dom.npix_mem();
    T dot = 0;
    acc_t dotd = 0;
    if (g.y0 < g.y1) {
        const VRow<T> up = finish_vrow<T, true>(raw_vrow<T, true>(a, g, g.y0 - 1));
        VRow<T> cur = finish_vrow<T, true>(raw_vrow<T, true>(a, g, g.y0)),
                dn = finish_vrow<T, true>(raw_vrow<T, true>(a, g, g.y0 + 1));
        JCarry<T> k = jcarry_init(up, cur, a.wr);
        for (int y = g.y0; y < g.y1; ++y) {
            const VRaw<T> nx = raw_vrow<T, true>(a, g, min(y + 2, g.y1));
            const JRow<T> j = jtf_row(a, cur, dn, k);
            if (g.out_lane) {
                const long long i = a.dom.off(g.x, y);
                const JOut<T> o = jtf_out(a, cur, j);
                a.flags[i] = (uint8_t)o.f;
                if (ACC) {
                    if (cur.act) dotd += wdot3(o.wo, o.rx, o.rx, o.wo, o.ry, o.ry, o.wt, o.rt, o.rt);
                } else if (cur.act) {
                    dot += o.rx * (o.wo * o.rx) + o.ry * (o.wo * o.ry) + o.rt * (o.wt * o.rt);
                }
                r[2 * i] = o.rx; r[2 * i + 1] = o.ry; r[2 * N + i] = o.rt;
                if (OUT == 2) {
                    // the reference sums (d e/d O)^2 = wr^2 once per valid residual, then wf^2
                    T dox = 0, dt = j.dt;
                    for (int q = 0; q < 2 * j.nv; ++q) dox += wr2;
                    if (cur.fit) dox += wf * wf;
                    if (!cur.act) { dox = 0; dt = 0; }
                    pre[2 * i] = dox; pre[2 * i + 1] = dox; pre[2 * N + i] = dt;
                } else if (OUT == 1) {
                    pre[2 * i] = o.wo; pre[2 * i + 1] = o.wo; pre[2 * N + i] = o.wt;
                } else {
                    pre[i] = o.wt;
                }
            }
            cur = dn;
            dn = finish_vrow<T, true>(nx);
        }
    }
    if (OUT == 2) return;
    double v[1] = {ACC ? (double)dotd : (double)dot};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// ---------------------------------------- fused PCGInit1 + first PCGStep1
// The first PCG iteration's p = pre r depends on nothing global, so PCGInit1 (J^T F,
// preconditioner, flags, rz[0] = r.(pre r)) and the first apply (Ap = J^T J p,
// pAp[0] = p.Ap) run as ONE strip pass from the arrays bound at this Step: the same
// r / pre / flags as iw_jtf<0> (bitwise) and the same J^T J p as iw_apply<1,0> up to the
// summation order of the pairs (apply_ap2, round 5), without writing r / pre / flags and
// reading them back. Geometry: a wavefront owns 60 output columns, x = 60*strip - 2 + lane;
// J^T F is evaluated at all 64 lanes (valid at lanes 1..62), so the apply at lanes 2..61
// finds every horizontal neighbour's p in a lane neighbour (DPP) and needs no edge
// record. Rows: J^T F runs one row ahead of the apply (rows y0-1 .. y1,
// the outer two for the apply's vertical neighbours only; unknown rows y0-2 .. y1+1).
// One reduction of four scalars (fp64 per lane): sc[rs.out + 0..3] = {rz[0], pAp[0],
// r_0.W Ap_0, Ap_0.W Ap_0} — the last two for iw_apply_res's identity for rz[1] (W r_0
// is summed from r_0, not taken as p_0: p_0 is rounded to T, and the identity cancels
// rz[0] down to rz[1], 2e4 x smaller on the test problems).
template <typename T>
struct FRow {          // a finished row of the fused kernel's apply window
    T rx, ry, rt;      // r_0 (0 on inactive pixels)
    T wo, wt;          // the preconditioner of the Offset / angle channels
    T c, s;
    float ux, uy;
    bool act, fit;
    // p_0 = pre r_0, formed where it is used (iw_apply<1>'s make_p: zero on inactive pixels,
    // where r_0 = pre = 0): three multiplies instead of three more VGPRs per held row
    __device__ __forceinline__ T px() const { return opaque(wo * rx); }
    __device__ __forceinline__ T py() const { return opaque(wo * ry); }
    __device__ __forceinline__ T pt() const { return opaque(wt * rt); }
    __device__ __forceinline__ vec2_t<T> p() const {
        vec2_t<T> r;
        r.x = rx; r.y = ry;
        return opaque(wo * r);
    }
    __device__ __forceinline__ vec2_t<float> u() const {
        vec2_t<float> v;
        v.x = ux; v.y = uy;
        return v;
    }
};
// REC: r_0 (and p_0 unless pout is null) go to the record r, UrShape / the angle / pre_t
// to the S record (Args::S); pre is not written
template <typename T, int NT = 2, bool REC = false>
__device__ __forceinline__ void iw_jtf_apply_body(const Args<T>& a, T* __restrict__ r, T* __restrict__ pre,
                                                  T* __restrict__ pout, T* __restrict__ Ap, ReduceSlot rs) {
    IW_PRE_TABLE(a);
    const WaveGeom g = geom_fused(a);
    const T wr = a.wr, wf2 = a.wf * a.wf;
    const unsigned tb = (unsigned)(2 * a.dom.npix_mem() * (long long)sizeof(T));
    acc_t rzdot = 0, papdot = 0, rapd = 0, apapd = 0;
    // J^T F of row y from the window (cur = row y, dn = row y+1): stores r / pre / flags
    // when the row is this wave's, returns the apply's view of the row (p = pre r)
    auto jrow = [&](const VRow<T>& cur, const VRow<T>& dn, JCarry<T>& k, int y, bool own) {
        const JRow<T> j = jtf_row<T, false>(a, cur, dn, k);
        const JOut<T> o = jtf_out(a, cur, j);
        if (own && g.out_lane) {
            // 32-bit byte offsets from uniform bases (the plan takes this kernel only when
            // they fit, offsets_fit_32), the Offset pair as one 8/16-byte store
            const unsigned i = (unsigned)a.dom.off(g.x, y);
            vec2_t<T> rv; rv.x = o.rx; rv.y = o.ry;
            stb<false>(a.flags, i, (uint8_t)o.f);
            if constexpr (REC) {   // p_0 = pre r_0 as FRow::p / pt form it (whole records: a
                // record left partly unwritten costs a partial-line write per line)
                const ROff<T> ro(i);
                stb<(NT & 2) != 0>(r, ro.r, rv);
                vec2_t<T> tt;
                tt.x = o.rt; tt.y = opaque(o.wt * o.rt);
                stb<(NT & 2) != 0>(r, ro.t, tt);
                stb<(NT & 2) != 0>(r, ro.p, opaque(o.wo * rv));
                st_srec<(NT & 2) != 0>(a.S, ro.s, cur.ux, cur.uy, cur.t, o.wt);
            } else {
                const POff<T> off(i, tb);
                stb<(NT & 2) != 0>(r, off.xy, rv); stb<(NT & 2) != 0>(r, off.t, o.rt);
                stb<(NT & 2) != 0>(pre, off.s, o.wt);
            }
            if (cur.act) rzdot += wdot3(o.wo, o.rx, o.rx, o.wo, o.ry, o.ry, o.wt, o.rt, o.rt);
        }
        FRow<T> p;
        p.rx = o.rx; p.ry = o.ry; p.rt = o.rt; p.wo = o.wo; p.wt = o.wt;
        p.c = cur.c; p.s = cur.s; p.ux = cur.ux; p.uy = cur.uy; p.act = cur.act; p.fit = cur.fit;
        return p;
    };
    if (g.y0 < g.y1) {
        const VRow<T> vm2 = finish_vrow<T, false, false>(raw_vrow<T, false, false>(a, g, g.y0 - 2));
        VRow<T> vcur = finish_vrow<T, false, false>(raw_vrow<T, false, false>(a, g, g.y0 - 1));
        VRow<T> vdn = finish_vrow<T, false, false>(raw_vrow<T, false, false>(a, g, g.y0));
        JCarry<T> k = jcarry_init(vm2, vcur, wr);
        FRow<T> up = jrow(vcur, vdn, k, g.y0 - 1, false);
        vcur = vdn;
        vdn = finish_vrow<T, false, false>(raw_vrow<T, false, false>(a, g, g.y0 + 1));
        FRow<T> cur = jrow(vcur, vdn, k, g.y0, true);
        vcur = vdn;
        vdn = finish_vrow<T, false, false>(raw_vrow<T, false, false>(a, g, g.y0 + 2));
        // apply carries from the row above (apply_ap2's recursion, the body iw_pcg recomputes
        // Ap_0 with: both act on the same rounded p_0 and agree bitwise)
        ACarry<T> k2 = acarry_init(up.p(), up.pt(), up.c, up.s, up.u(), up.act, cur.p(), cur.pt(), cur.c, cur.s,
                                   cur.u(), cur.act, wr);
        for (int y = g.y0; y < g.y1; ++y) {
            // J^T F needs rows up to y1 + 1; the last trip re-reads that row (an L2 hit)
            // instead of fetching row y1 + 2
            const VRaw<T> nx = raw_vrow<T, false, false>(a, g, min(y + 3, g.y1 + 1));
            const FRow<T> dn = jrow(vcur, vdn, k, y + 1, y + 1 < g.y1);
            const vec2_t<T> cp = cur.p();
            const T cpt = cur.pt();
            vec2_t<T> ao;
            T aot;
            apply_ap2(cp, cpt, cur.c, cur.s, cur.u(), cur.act, cur.fit, dn.p(), dn.pt(), dn.c, dn.s, dn.u(), dn.act,
                      wr, wf2, k2, ao, aot);
            if (g.out_lane) {
                const unsigned iy = (unsigned)a.dom.off(g.x, y);
                const POff<T> off(iy, tb);
                if (Ap) {   // null when lIterations == 1 or when iw_pcg recomputes Ap_0 (always with REC)
                    stb<(NT & 2) != 0>(Ap, off.xy, ao); stb<(NT & 2) != 0>(Ap, off.t, aot);
                }
                if (!REC && pout) {   // null when the loop forms p_0 from r_0 itself (lIterations >= 3)
                    stb<(NT & 2) != 0>(pout, off.xy, cp); stb<(NT & 2) != 0>(pout, off.t, cpt);
                }
                papdot += dot3(cp.x, ao.x, cp.y, ao.y, cpt, aot);
                // PCGStep2's weights: pre, or 1 without a preconditioner
                const T w0 = a.use_pre ? cur.wo : (T)1, w2 = a.use_pre ? cur.wt : (T)1;
                rapd += wdot3(w0, cur.rx, ao.x, w0, cur.ry, ao.y, w2, cur.rt, aot);
                apapd += wdot3(w0, ao.x, ao.x, w0, ao.y, ao.y, w2, aot, aot);
            }
            cur = dn;
            vcur = vdn;
            vdn = finish_vrow<T, false, false>(nx);
        }
    }
    double v[4] = {(double)rzdot, (double)papdot, (double)rapd, (double)apapd};
    block_reduce_publish<4>(v, rs, g.tile);
}
// (the compiler's 112-114 VGPRs give 4 waves per SIMD; forcing 5 spills: 504 vs 373 us)
template <typename T, int NT = 2, bool REC = false>
__global__ __launch_bounds__(kBlock) void iw_jtf_apply(Args<T> a, T* __restrict__ r, T* __restrict__ pre,
                                                       T* __restrict__ pout, T* __restrict__ Ap, ReduceSlot rs) {
    iw_jtf_apply_body<T, NT, REC>(a, r, pre, pout, Ap, rs);
}

// ----------------------------------------------------------------- cost kernel
// sc[rs.out] = sum over active pixels of 1/2 (sum_s |e_reg(k,s)|^2 + |e_fit(k)|^2).
template <typename T>
__global__ __launch_bounds__(kBlock) void iw_cost(Args<T> a, ReduceSlot rs) {
    const WaveGeom g = geom(a);
    const T wr = a.wr, wf = a.wf;
    T acc = 0;
    if (g.y0 < g.y1) {
        VRow<T> up = finish_vrow<T, false>(raw_vrow<T, false>(a, g, g.y0 - 1)),
                cur = finish_vrow<T, false>(raw_vrow<T, false>(a, g, g.y0)),
                dn = finish_vrow<T, false>(raw_vrow<T, false>(a, g, g.y0 + 1));
        for (int y = g.y0; y < g.y1; ++y) {
            const VRaw<T> nx = raw_vrow<T, false>(a, g, min(y + 2, g.y1));
            const T lox = from_left(cur.ox, cur.eox), loy = from_left(cur.oy, cur.eoy);
            const T rox = from_right(cur.ox, cur.eox), roy = from_right(cur.oy, cur.eoy);
            const float lux = from_left(cur.ux, cur.eux), luy = from_left(cur.uy, cur.euy);
            const float rux = from_right(cur.ux, cur.eux), ruy = from_right(cur.uy, cur.euy);
            const int lact = from_left_i(cur.act, cur.eact), ract = from_right_i(cur.act, cur.eact);
            T ex, ey, ax, ay, sum = 0;
            eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, rox, roy, rux, ruy,
                  cur.act && ract, wr, ex, ey, ax, ay);
            sum += ex * ex + ey * ey;
            eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, lox, loy, lux, luy,
                  cur.act && lact, wr, ex, ey, ax, ay);
            sum += ex * ex + ey * ey;
            eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, dn.ox, dn.oy, dn.ux, dn.uy,
                  cur.act && dn.act, wr, ex, ey, ax, ay);
            sum += ex * ex + ey * ey;
            eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, up.ox, up.oy, up.ux, up.uy,
                  cur.act && up.act, wr, ex, ey, ax, ay);
            sum += ex * ex + ey * ey;
            if (cur.fit) {
                const T fx = wf * (cur.ox - (T)cur.cx), fy = wf * (cur.oy - (T)cur.cy);
                sum += fx * fx + fy * fy;
            }
            if (g.out_lane && cur.act) acc += (T)0.5 * sum;
            up = cur; cur = dn;
            dn = finish_vrow<T, false>(nx);
        }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// The same cost on iw_jtf_apply's 60-column strips (geom_fused, x = 60 strip - 2 + lane):
// every horizontal neighbour of an output lane (2..61) is a lane neighbour, so there is no
// edge record — round 4's 64-column form above fetched the strip's two outside columns per
// row with separate 2-lane loads (141 us at 4096^2, 0.48 of 8 TB/s). Per pixel the same
// eedge calls in the same order; the sums group by 60-column strips instead.
// FL (round 6, the cost at the end of a Step): the flag byte this Step's iw_jtf_apply wrote
// (bit 0 inside and Mask == 0, bit 1 Constraints >= 0 — the same tests on the same arrays
// bound at this Step) stands in for Mask, and Constraints are read only where bit 1 says the
// fit term exists (a raw buffer load at an out-of-range offset elsewhere touches no memory):
// 32 -> 21 B/px plus the few constraint pixels, bitwise the same cost.
template <typename T>
struct CRaw {
    vec2_t<T> o;
    T t;
    vec2_t<float> u;
    int f, in;
    unsigned i;
};
template <typename T, bool FL = false>
__global__ __launch_bounds__(kBlock) void iw_cost60(Args<T> a, ReduceSlot rs) {
    const WaveGeom g = geom_fused(a);
    const T wr = a.wr, wf = a.wf;
    T acc = 0;
    const unsigned cb = (unsigned)(8 * a.dom.npix_mem());   // Constraints' bytes: the drop offset
    const __amdgpu_buffer_rsrc_t r_c = bres(a.C, cb);
    if (g.y0 < g.y1) {
        auto raw = [&](int y) {
            if constexpr (FL) {
                CRaw<T> q;
                q.in = present(a.dom, g.x, y);
                q.i = q.in ? (unsigned)a.dom.off(g.x, y) : 0u;
                q.o = ldb<false, vec2_t<T>>(a.O, q.i * 2u * (unsigned)sizeof(T));
                q.t = ldb<false, T>(a.A, q.i * (unsigned)sizeof(T));
                q.u = ldb<false, vec2_t<float>>(a.U, 8u * q.i);
                q.f = ldb<false, uint8_t>(a.flags, q.i);
                return q;
            } else {
                return raw_vrow<T, false, false>(a, g, y);
            }
        };
        auto row = [&](const auto& q) {
            if constexpr (FL) {
                VRow<T> v;
                v.ox = q.in ? q.o.x : (T)0;
                v.oy = q.in ? q.o.y : (T)0;
                v.t = q.in ? q.t : (T)0;
                v.ux = q.in ? q.u.x : 0.f; v.uy = q.in ? q.u.y : 0.f;
                v.act = q.in && (q.f & 1);
                v.fit = q.in && ((q.f >> 1) & 1);
                // the row's Constraints, only where the fit term exists (used two rows later)
                const vec2_t<float> c = bld<vec2_t<float>>(r_c, v.fit ? 8u * q.i : cb);
                v.cx = c.x; v.cy = c.y;
                sc_of(v.t, &v.c, &v.s);
                v.eox = 0; v.eoy = 0; v.eux = 0.f; v.euy = 0.f; v.eact = 0; v.ec = 0; v.es = 0;
                return v;
            } else {
                return finish_vrow<T, false, false>(q);
            }
        };
        VRow<T> up = row(raw(g.y0 - 1)), cur = row(raw(g.y0)), dn = row(raw(g.y0 + 1));
        // two raw rows in flight (the walk waits on memory, not on issue: SQ_WAIT_ANY 0.49)
        auto n1 = raw(min(g.y0 + 2, g.y1));
        for (int y = g.y0; y < g.y1; ++y) {
            const auto nx = n1;
            n1 = raw(min(y + 3, g.y1));
            const T lox = from_left0(cur.ox), loy = from_left0(cur.oy);
            const T rox = from_right0(cur.ox), roy = from_right0(cur.oy);
            const float lux = from_left0(cur.ux), luy = from_left0(cur.uy);
            const float rux = from_right0(cur.ux), ruy = from_right0(cur.uy);
            const int lact = from_left0_i(cur.act), ract = from_right0_i(cur.act);
            T ex, ey, ax, ay, sum = 0;
            eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, rox, roy, rux, ruy,
                  cur.act && ract, wr, ex, ey, ax, ay);
            sum += ex * ex + ey * ey;
            eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, lox, loy, lux, luy,
                  cur.act && lact, wr, ex, ey, ax, ay);
            sum += ex * ex + ey * ey;
            eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, dn.ox, dn.oy, dn.ux, dn.uy,
                  cur.act && dn.act, wr, ex, ey, ax, ay);
            sum += ex * ex + ey * ey;
            eedge(cur.ox, cur.oy, cur.c, cur.s, cur.ux, cur.uy, up.ox, up.oy, up.ux, up.uy,
                  cur.act && up.act, wr, ex, ey, ax, ay);
            sum += ex * ex + ey * ey;
            if (cur.fit) {
                const T fx = wf * (cur.ox - (T)cur.cx), fy = wf * (cur.oy - (T)cur.cy);
                sum += fx * fx + fy * fy;
            }
            if (g.out_lane && cur.act) acc += (T)0.5 * sum;
            up = cur; cur = dn;
            dn = row(nx);
        }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, g.tile);
}

// ----------------------------------------------------------- model cost kernel
// LM only, once per step: sc[rs.out] = sum over active pixels of
// 1/2 (sum_s |e_reg(k,s) + J_reg(k,s) delta|^2 + |e_fit(k) + wf delta_O(k)|^2)
// (createmodelcost, o.t:2915-2943). Strip geometry (same grid, hence the same
// reduction slot, as the other stencil kernels); neighbours are direct loads (L2 hits).
template <typename T>
__global__ __launch_bounds__(kBlock) void iw_model_cost(Args<T> a, const T* __restrict__ delta, ReduceSlot rs) {
    const WaveGeom g = geom(a);
    const long long N = a.dom.npix_mem();
    const int x = g.x;
    T acc = 0;
    for (int y = g.y0; y < g.y1 && g.out_lane; ++y) {
        const long long k = a.dom.off(x, y);
        if (a.M[k] != 0.f) continue;
        const T ox = a.O[2 * k], oy = a.O[2 * k + 1];
        T c, s;
        sc_of(a.A[k], &c, &s);
        const float ux = a.U[2 * k], uy = a.U[2 * k + 1];
        const T dkx = delta[2 * k], dky = delta[2 * k + 1], dkt = delta[2 * N + k];
        constexpr int DX[4] = {1, -1, 0, 0}, DY[4] = {0, 0, 1, -1};
        T sum = 0;
        for (int d = 0; d < 4; ++d) {
            const int tx = x + DX[d], ty = y + DY[d];
            if (!present(a.dom, tx, ty)) continue;
            const long long t = a.dom.off(tx, ty);
            if (a.M[t] != 0.f) continue;
            T ex, ey, ax, ay, jx, jy;
            eedge(ox, oy, c, s, ux, uy, a.O[2 * t], a.O[2 * t + 1], a.U[2 * t], a.U[2 * t + 1], true, a.wr,
                  ex, ey, ax, ay);
            jedge(dkx, dky, dkt, c, s, ux, uy, delta[2 * t], delta[2 * t + 1], a.U[2 * t], a.U[2 * t + 1], true,
                  a.wr, jx, jy, ax, ay);
            ex += jx; ey += jy;
            sum += ex * ex + ey * ey;
        }
        const float cx = a.C[2 * k], cy = a.C[2 * k + 1];
        if (cx >= 0.f && cy >= 0.f) {
            const T fx = a.wf * (ox - (T)cx) + a.wf * dkx, fy = a.wf * (oy - (T)cy) + a.wf * dky;
            sum += fx * fx + fy * fy;
        }
        acc += (T)0.5 * sum;
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// ------------------------------------------------------------ residual kernel
// PCGStep2's residual half for this layout (pcg_kernels.h has the generic flat form):
//   r -= alpha Ap;  rz[i+1] = sum r.(pre r)  (pre = r's preconditioner; 1 when
//   UsePreconditioner(false), :705-708). Two pixels per lane: Offset parts as one
//   16-B access, angle parts and the angle preconditioner as 8-B, flags as 2 bytes.
//   Walking each XCD's eighth backwards (so the first reads fall on the Ap lines the
//   apply wrote last, in the 256 MB infinity cache) was measured: 4.41 -> 4.43 ms per
//   GN step with streaming loads, 4.57 -> 4.47 without (gpurun_out sweep, tools/sweep_env.py)
//   — the streaming form stays, in grid-stride order.
template <typename T, bool NT = false>
__global__ __launch_bounds__(kBlock) void iw_residual(Args<T> a, const T* __restrict__ Ap,
                                                      const T* __restrict__ pre, T* __restrict__ r,
                                                      const double* __restrict__ sc, int i_num, int i_den,
                                                      ReduceSlot rs) {
    IW_PRE_TABLE(a);
    const long long N = a.dom.npix_mem();
    const T alpha = (T)(sc[i_num] / sc[i_den]);
    const long long b0 = a.dom.off(0, a.dom.y_lo), e = a.dom.off(0, a.dom.y_hi);
    const long long b = b0 + (b0 & 1);   // 16-B aligned pairs (slabs may start on an odd pixel)
    const long long npairs = (e - b) / 2;
    T acc = 0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < npairs; q += stride) {
        const long long i = b + 2 * q;
        V4<T> ro, ao;
        Vec2<T> rt, at, wt;
        if constexpr (NT) {   // streaming forms: every element is touched once
            ro = ld4nt(r + 2 * i); ao = ld4nt(Ap + 2 * i);
            rt = {ld_v<true>(r + 2 * N + i), ld_v<true>(r + 2 * N + i + 1)};
            at = {ld_v<true>(Ap + 2 * N + i), ld_v<true>(Ap + 2 * N + i + 1)};
            wt = {ld_v<true>(pre + i), ld_v<true>(pre + i + 1)};
        } else {
            ro = *reinterpret_cast<const V4<T>*>(r + 2 * i);
            ao = *reinterpret_cast<const V4<T>*>(Ap + 2 * i);
            rt = *reinterpret_cast<const Vec2<T>*>(r + 2 * N + i);
            at = *reinterpret_cast<const Vec2<T>*>(Ap + 2 * N + i);
            wt = *reinterpret_cast<const Vec2<T>*>(pre + i);
        }
        const unsigned short ff = *reinterpret_cast<const unsigned short*>(a.flags + i);
        const int f0 = ff & 0xff, f1 = ff >> 8;
        ro.a -= alpha * ao.a; ro.b -= alpha * ao.b; ro.c -= alpha * ao.c; ro.d -= alpha * ao.d;
        rt.x -= alpha * at.x; rt.y -= alpha * at.y;
        if constexpr (NT) {
            st4nt(r + 2 * i, ro);
            st_v<true>(r + 2 * N + i, rt.x); st_v<true>(r + 2 * N + i + 1, rt.y);
        } else {
            *reinterpret_cast<V4<T>*>(r + 2 * i) = ro;
            *reinterpret_cast<Vec2<T>*>(r + 2 * N + i) = rt;
        }
        if (a.use_pre) {
            const T w0 = pre_offset(a, f0), w1 = pre_offset(a, f1);
            acc += w0 * ro.a * ro.a + w0 * ro.b * ro.b + w1 * ro.c * ro.c + w1 * ro.d * ro.d +
                   wt.x * rt.x * rt.x + wt.y * rt.y * rt.y;
        } else {
            acc += ro.a * ro.a + ro.b * ro.b + ro.c * ro.c + ro.d * ro.d + rt.x * rt.x + rt.y * rt.y;
        }
    }
    // unpaired pixels (odd start, odd count): block 0 threads 0 / 1
    const long long single = (threadIdx.x == 0) ? ((b0 & 1) ? b0 : -1) : (((e - b) & 1) ? e - 1 : -1);
    if (blockIdx.x == 0 && threadIdx.x < 2 && single >= 0) {
        const long long i = single;
        const int f = a.flags[i];
        T r0 = r[2 * i] - alpha * Ap[2 * i], r1 = r[2 * i + 1] - alpha * Ap[2 * i + 1];
        T r2 = r[2 * N + i] - alpha * Ap[2 * N + i];
        r[2 * i] = r0; r[2 * i + 1] = r1; r[2 * N + i] = r2;
        if (a.use_pre) {
            const T w0 = pre_offset(a, f);
            acc += w0 * r0 * r0 + w0 * r1 * r1 + pre[i] * r2 * r2;
        } else {
            acc += r0 * r0 + r1 * r1 + r2 * r2;
        }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// --------------------------------------------------------------- flag kernel
// Only for the standalone apply entry point: flags without a J^T F evaluation.
template <typename T>
__global__ __launch_bounds__(kBlock) void iw_flags(Args<T> a) {
    const long long n = (long long)a.dom.W * a.dom.mem_rows;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const float2 c = reinterpret_cast<const float2*>(a.C)[i];
        const int act = a.M[i] == 0.f, fit = (c.x >= 0.f) && (c.y >= 0.f);
        a.flags[i] = (uint8_t)(act | (fit << 1));
    }
}

// --------------------------------------------------------------- update kernel
// delta_L of one element: (the deferred alpha_{L-2} p_{L-2} term first, E2), then
// alpha_{L-1} p_{L-1}; every term an explicit fma onto the pending delta, as
// iw_apply_res forms the terms it folds, so the deferred delta is bitwise the
// per-iteration one
template <typename T, bool HAS_DELTA, bool E2>
__device__ __forceinline__ T upd_delta(T alpha, T q, T alpha2, T q2, T d) {
    if (E2) d = HAS_DELTA ? fmad(alpha2, q2, d) : alpha2 * q2;
    return (HAS_DELTA || E2) ? fmad(alpha, q, d) : alpha * q;
}
// X += delta_L on active pixels of the owned rows (PCGLinearUpdate, :854-859), where
// delta_L = delta_{L-1} + alpha_{L-1} p_{L-1} is the last PCG iteration's delta update
// (HAS_DELTA = false when lIterations == 1: delta_0 = 0). REC: p and p2 are records.
template <typename T, bool HAS_DELTA, bool E2 = false, bool REC = false>
__global__ __launch_bounds__(kBlock) void iw_update(Args<T> a, T* __restrict__ O, T* __restrict__ A,
                                                    const T* __restrict__ delta, const T* __restrict__ p,
                                                    const double* __restrict__ sc, int ia_num, int ia_den,
                                                    const T* __restrict__ p2 = nullptr, int ia2_num = 0,
                                                    int ia2_den = 0) {
    const long long N = a.dom.npix_mem();
    const T alpha = pcg_alpha<T>(sc[ia_num], sc[ia_den]);
    const T alpha2 = E2 ? pcg_alpha<T>(sc[ia2_num], sc[ia2_den]) : (T)0;
    const long long b = a.dom.off(0, a.dom.y_lo), e = a.dom.off(0, a.dom.y_hi);
    for (long long i = b + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < e;
         i += (long long)gridDim.x * blockDim.x) {
        const int f = a.flags[i];
        const Vec2<T> o = reinterpret_cast<const Vec2<T>*>(O)[i];
        const T t = A[i];
        // p.xy and p.t of a vector / record (REC: [r.xy | p.xy | r.t p.t])
        auto pget = [&](const T* v, Vec2<T>& xy, T& pt) {
            if constexpr (REC) {
                xy = reinterpret_cast<const Vec2<T>*>(v)[3 * i + 1];
                pt = reinterpret_cast<const Vec2<T>*>(v)[3 * i + 2].y;
            } else {
                xy = reinterpret_cast<const Vec2<T>*>(v)[i];
                pt = v[2 * N + i];
            }
        };
        Vec2<T> pp, d{}, q2{};
        T pt, dt = 0, q2t = 0;
        pget(p, pp, pt);
        if (HAS_DELTA) {
            d = reinterpret_cast<const Vec2<T>*>(delta)[i];
            dt = delta[2 * N + i];
        }
        if (E2) pget(p2, q2, q2t);
        d.x = upd_delta<T, HAS_DELTA, E2>(alpha, pp.x, alpha2, q2.x, d.x);
        d.y = upd_delta<T, HAS_DELTA, E2>(alpha, pp.y, alpha2, q2.y, d.y);
        dt = upd_delta<T, HAS_DELTA, E2>(alpha, pt, alpha2, q2t, dt);
        if (f & 1) {
            reinterpret_cast<Vec2<T>*>(O)[i] = Vec2<T>{o.x + d.x, o.y + d.y};
            A[i] = t + dt;
        }
    }
}

// PCGLinearUpdate with every p_i kept (ALLP, lIterations <= kAllPMax): the passes carry no
// delta terms at all, and this kernel forms delta_L = sum_i alpha_i p_i per pixel in
// PCGStep2's order — alpha_0 p_0, then one fma per iteration — so it is bitwise the
// per-iteration (and the deferred) update. p_i = pall + i * pstride.
constexpr int kAllPMax = 16;
// (L a template parameter: the loop unrolls with every load of a pixel issued back to back)
// P0R: p_0 = pre r_0 formed here from r0 / pre (FRow::p's rounded products), not read
template <typename T, int L, bool P0R, bool NT = false>
__global__ __launch_bounds__(kBlock) void iw_update_all(Args<T> a, T* __restrict__ O, T* __restrict__ A,
                                                        const T* __restrict__ pall, long long pstride,
                                                        const double* __restrict__ sc, int sc0,
                                                        const T* __restrict__ r0, const T* __restrict__ pre) {
    IW_PRE_TABLE(a);
    const long long N = a.dom.npix_mem();
    T al[L];
#pragma unroll
    for (int i = 0; i < L; ++i) al[i] = pcg_alpha<T>(sc[sc0 + kSlots * i], sc[sc0 + kSlots * i + 1]);
    const long long b = a.dom.off(0, a.dom.y_lo), e = a.dom.off(0, a.dom.y_hi);
    for (long long kf = b + (long long)blockIdx.x * blockDim.x + threadIdx.x; kf < e;
         kf += (long long)gridDim.x * blockDim.x) {
        const long long k = a.rev ? e - 1 - (kf - b) : kf;   // Args::rev: last pixel first
        const int f = a.flags[k];
        Vec2<T> q[L];
        T qt[L];
#pragma unroll
        for (int i = P0R ? 1 : 0; i < L; ++i) {
            if constexpr (NT) {   // streaming: every p element is read once
                const T* pi = pall + i * pstride;
                q[i] = Vec2<T>{ld_v<true>(pi + 2 * k), ld_v<true>(pi + 2 * k + 1)};
                qt[i] = ld_v<true>(pi + 2 * N + k);
            } else {
                q[i] = reinterpret_cast<const Vec2<T>*>(pall + i * pstride)[k];
                qt[i] = pall[i * pstride + 2 * N + k];
            }
        }
        if constexpr (P0R) {
            const T w0 = pre_offset(a, f);
            const Vec2<T> r = reinterpret_cast<const Vec2<T>*>(r0)[k];
            vec2_t<T> rv;
            rv.x = r.x; rv.y = r.y;
            const vec2_t<T> pv = opaque(w0 * rv);
            q[0] = Vec2<T>{pv.x, pv.y};
            qt[0] = opaque(pre[k] * r0[2 * N + k]);
        }
        T dx = al[0] * q[0].x, dy = al[0] * q[0].y, dt = al[0] * qt[0];
#pragma unroll
        for (int i = 1; i < L; ++i) {
            dx = fmad(al[i], q[i].x, dx);
            dy = fmad(al[i], q[i].y, dy);
            dt = fmad(al[i], qt[i], dt);
        }
        if (f & 1) {
            const Vec2<T> o = reinterpret_cast<const Vec2<T>*>(O)[k];
            reinterpret_cast<Vec2<T>*>(O)[k] = Vec2<T>{o.x + dx, o.y + dy};
            A[k] = A[k] + dt;
        }
    }
}

// iw_update_all over pixel PAIRS (round 6): each thread loads two pixels'
// Offset pairs of every p_i as one 16-B vector (8-B for the angle channel), so the pass
// issues half the load instructions, each twice as wide. Every value is formed by the same
// expressions in the same order as iw_update_all: bitwise the same update. The plan takes it
// when the pairs are aligned (N % 4 == 0, even row starts, 16-B aligned arrays).
template <typename T>
using vec4_t = T __attribute__((ext_vector_type(4)));
#ifndef IW_UPD_WAVES
#define IW_UPD_WAVES 1   // A/B builds (tools/ab_build.sh): the minimum waves per SIMD iw_update_all2 is held to
#endif
template <typename T, int L, bool P0R, bool NT = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(IW_UPD_WAVES))) void iw_update_all2(Args<T> a, T* __restrict__ O, T* __restrict__ A,
                                                         const T* __restrict__ pall, long long pstride,
                                                         const double* __restrict__ sc, int sc0,
                                                         const T* __restrict__ r0, const T* __restrict__ pre) {
    IW_PRE_TABLE(a);
    const long long N = a.dom.npix_mem();
    T al[L];
#pragma unroll
    for (int i = 0; i < L; ++i) al[i] = pcg_alpha<T>(sc[sc0 + kSlots * i], sc[sc0 + kSlots * i + 1]);
    const long long b = a.dom.off(0, a.dom.y_lo), np = (a.dom.off(0, a.dom.y_hi) - b) >> 1;
    for (long long jf = (long long)blockIdx.x * blockDim.x + threadIdx.x; jf < np; jf += (long long)gridDim.x * blockDim.x) {
        const long long j = a.rev ? np - 1 - jf : jf;   // Args::rev: last pair first
        const long long k = b + 2 * j;
        const unsigned short ff = *reinterpret_cast<const unsigned short*>(a.flags + k);
        const int f0 = ff & 255, f1 = ff >> 8;
        vec4_t<T> q[L];
        vec2_t<T> qt[L];
#pragma unroll
        for (int i = P0R ? 1 : 0; i < L; ++i) {
            const T* pi = pall + i * pstride;
            q[i] = ld_v<NT>(reinterpret_cast<const vec4_t<T>*>(pi + 2 * k));
            qt[i] = ld_v<NT>(reinterpret_cast<const vec2_t<T>*>(pi + 2 * N + k));
        }
        if constexpr (P0R) {   // iw_update_all's p_0 per pixel: the same rounded products
            const vec4_t<T> r = *reinterpret_cast<const vec4_t<T>*>(r0 + 2 * k);
            const vec2_t<T> rt = *reinterpret_cast<const vec2_t<T>*>(r0 + 2 * N + k);
            const vec2_t<T> w2 = *reinterpret_cast<const vec2_t<T>*>(pre + k);
            vec2_t<T> ra, rb;
            ra.x = r.x; ra.y = r.y; rb.x = r.z; rb.y = r.w;
            const vec2_t<T> pa = opaque(pre_offset(a, f0) * ra), pb = opaque(pre_offset(a, f1) * rb);
            q[0].x = pa.x; q[0].y = pa.y; q[0].z = pb.x; q[0].w = pb.y;
            qt[0].x = opaque(w2.x * rt.x);
            qt[0].y = opaque(w2.y * rt.y);
        }
        vec4_t<T> d = al[0] * q[0];
        vec2_t<T> dt = al[0] * qt[0];
#pragma unroll
        for (int i = 1; i < L; ++i) {
            d = __builtin_elementwise_fma((vec4_t<T>)al[i], q[i], d);
            dt = __builtin_elementwise_fma((vec2_t<T>)al[i], qt[i], dt);
        }
        const bool a0 = f0 & 1, a1 = f1 & 1;
        if (a0 && a1) {
            vec4_t<T>* op = reinterpret_cast<vec4_t<T>*>(O + 2 * k);
            vec2_t<T>* ap = reinterpret_cast<vec2_t<T>*>(A + k);
            *op = *op + d;
            *ap = *ap + dt;
        } else if (a0 || a1) {
            const long long kk = a0 ? k : k + 1;
            Vec2<T>* op = reinterpret_cast<Vec2<T>*>(O) + kk;
            const Vec2<T> o = *op;
            *op = a0 ? Vec2<T>{o.x + d.x, o.y + d.y} : Vec2<T>{o.x + d.z, o.y + d.w};
            A[kk] = A[kk] + (a0 ? dt.x : dt.y);
        }
    }
}

// ---------------------------------------------------- materialized Jacobian
// saveJToCRS (solverGPUGaussNewton.t:1004-1022) with generateDumpJ (:385-442): every
// pixel (excluded ones included, as the reference) writes its 10 residual rows — for s
// in (+x,-x,+y,-y): channel x, channel y; then the two fit channels — with
// 3 + ... + 3 + 1 + 1 = 26 nonzeros at rowPtr = 26 k + offset. Columns are the unknown
// indices image_offset + channels * tooffset(neighbour) + channel, wrapped into
// [0, nUnknowns) as the reference's wrap() (:365-381), and sorted inside each row
// (sortCol). Values are the partials of Select(valid, wr (...), 0) and wf Select(has, ...).
template <typename T>
__device__ __forceinline__ void sort3(int* c, T* v) {
    auto sw = [&](int i, int j) {
        if (c[j] < c[i]) {
            const int tc = c[i]; c[i] = c[j]; c[j] = tc;
            const T tv = v[i]; v[i] = v[j]; v[j] = tv;
        }
    };
    sw(0, 1); sw(1, 2); sw(0, 1);
}
// A block stages the rows of 256 consecutive pixels in LDS and stores them as one
// contiguous run (6656 nonzeros, 2560 row pointers): every global store is coalesced.
template <typename T>
__global__ __launch_bounds__(kBlock) void iw_dump_j(Args<T> a, int* __restrict__ rowPtr, int* __restrict__ colInd,
                                                    T* __restrict__ val) {
    __shared__ int s_col[kBlock * 26];
    __shared__ T s_val[kBlock * 26];
    __shared__ int s_row[kBlock * 10];
    const int W = a.dom.W, H = a.dom.H;
    const long long N = (long long)W * H, n = 3 * N;
    constexpr int SXd[4] = {1, -1, 0, 0}, SYd[4] = {0, 0, 1, -1};
    auto wrap = [n](long long c) -> int { return (int)(c < 0 ? c + n : (c >= n ? c - n : c)); };
    const int t = threadIdx.x;
    for (long long k0 = (long long)blockIdx.x * kBlock; k0 < N; k0 += (long long)gridDim.x * kBlock) {
        const long long k = k0 + t;
        if (k < N) {
            const int x = (int)(k % W), y = (int)(k / W);
            const bool mk = a.M[k] == 0.f;
            T ck, sk;
            sc_of(a.A[k], &ck, &sk);
            const float ukx = a.U[2 * k], uky = a.U[2 * k + 1];
            int* sc = s_col + 26 * t;
            T* sv = s_val + 26 * t;
            for (int s = 0; s < 4; ++s) {
                const int tx = x + SXd[s], ty = y + SYd[s];
                const bool in = tx >= 0 && tx < W && ty >= 0 && ty < H;
                const long long tp = in ? (long long)ty * W + tx : 0;
                const bool v = in && mk && a.M[tp] == 0.f;
                const T dx = in ? (T)(ukx - a.U[2 * tp]) : (T)0, dy = in ? (T)(uky - a.U[2 * tp + 1]) : (T)0;
                const T drot[2] = {-sk * dx - ck * dy, ck * dx - sk * dy};
                const long long tn = k + SXd[s] + (long long)SYd[s] * W;   // tooffset of the (maybe outside) neighbour
                for (int c = 0; c < 2; ++c) {
                    const int row = 2 * s + c;
                    s_row[10 * t + row] = (int)(26 * k + 3 * row);
                    int cc[3] = {(int)(2 * k + c), wrap(2 * tn + c), (int)(2 * N + k)};
                    T vv[3] = {v ? a.wr : (T)0, v ? -a.wr : (T)0, v ? -a.wr * drot[c] : (T)0};
                    sort3(cc, vv);
                    for (int q = 0; q < 3; ++q) {
                        sc[3 * row + q] = cc[q];
                        sv[3 * row + q] = vv[q];
                    }
                }
            }
            const bool has = a.C[2 * k] >= 0.f && a.C[2 * k + 1] >= 0.f;
            for (int c = 0; c < 2; ++c) {
                s_row[10 * t + 8 + c] = (int)(26 * k + 24 + c);
                sc[24 + c] = (int)(2 * k + c);
                sv[24 + c] = has ? a.wf : (T)0;
            }
        }
        __syncthreads();
        const int np = (int)min((long long)kBlock, N - k0);
        for (int e = t; e < 26 * np; e += kBlock) {
            colInd[26 * k0 + e] = s_col[e];
            val[26 * k0 + e] = s_val[e];
        }
        for (int e = t; e < 10 * np; e += kBlock) rowPtr[10 * k0 + e] = s_row[e];
        __syncthreads();
    }
    if (blockIdx.x == 0 && t == 0) rowPtr[10 * N] = (int)(26 * N);
}

}  // namespace iw

// ====================================================================== plan

template <typename T>
class ImageWarpingPlan final : public Plan {
public:
    ImageWarpingPlan(const ProblemSpec& spec, const StateOptions& opts, unsigned W, unsigned H)
        : Plan(spec, opts) {
        dom_ = Domain{(int)W, (int)H, 0, (int)H, 0, (int)H};
        // roles by declared index order (image_warping.t:12-27)
        idx_O_ = spec.unknown(0)->index;
        idx_A_ = spec.unknown(1)->index;
        idx_U_ = spec.array(0)->index;
        idx_C_ = spec.array(1)->index;
        idx_M_ = spec.array(2)->index;
        std::vector<DeclParam> ps = spec.params;
        std::sort(ps.begin(), ps.end(), [](auto& x, auto& y) { return x.index < y.index; });
        idx_wf_ = ps[0].index;
        idx_wr_ = ps[1].index;
        // by declared index: the routing matched this file's structural signature, in which
        // each parameter is identified by its problemparams index (generic.hip: generic_signature),
        // against the canonical energy's (fit weight declared first), so names play no part
        read_knobs();
        timer_.apply_name = apply_kernel_name();
        timer_.aux_names = {"iw_jtf_apply", "iw_apply_res", "iw_pcg", "iw_update", "iw_cost"};
        allocate();
    }
    ~ImageWarpingPlan() override {
        OPT_HIP_CHECK(hipStreamSynchronize(stream_));
        release();
    }

    // rows of neighbour data a slab holds: 2, the reach of iw_jtf_apply (J^T F one row
    // ahead of the apply) and of iw_pcg (Ap_{i-1} recomputed around p_i's stencil); the
    // 4-neighbour stencil itself reaches 1
    int halo() const override { return 2; }

    std::string set_decomposition(Comm* comm, int y_lo, int y_hi) override {
        if (opts_.host_buffers) return "row-slab decomposition needs backend_cuda (device arrays)";
        if (y_lo < 0 || y_hi > dom_.H || y_hi - y_lo < halo()) return "invalid slab rows";
        comm_ = comm;
        OPT_HIP_CHECK(hipStreamSynchronize(stream_));
        release();
        dom_.y_lo = y_lo;
        dom_.y_hi = y_hi;
        dom_.y_mem0 = std::max(0, y_lo - halo());
        dom_.mem_rows = std::min(dom_.H, y_hi + halo()) - dom_.y_mem0;
        allocate();
        initialised_ = false;
        return "";
    }

    long long unknown_count() const override { return nvec_; }
    std::string family() const override { return "image_warping"; }
    std::string apply_kernel_name() const override { return "iw_apply"; }

    void init(void** params) override {
        begin_call();
        bind(params, true);
        exchange_unknowns();
        tbegin("iw_cost"); launch_cost(kScCost); tend();
        allreduce(kScCost);
        prev_cost_ = read_scalar(kScCost);
        n_iter_ = 0;
        initialised_ = true;
        end_call();
        if (opts_.verbosity > 0) fprintf(stderr, "[opt_amd] init cost %.9g\n", prev_cost_);
    }

    int step(void** params) override {
        if (!initialised_) init(params);
        if (n_iter_ >= sp_.nIterations) {
            cleanup_log();
            return 0;
        }
        begin_call();
        bind(params, false);
        exchange_unknowns();
        const int L = std::max(0, sp_.lIterations);
        red_.ensure(std::max({stencil_blocks(), fused_blocks(), side_blocks(), fused_side_blocks(), cost_side_blocks(), 2048}), 4,
                    kScBase + iw::kSlots * (L + 2));
        if (print_addr_) {   // OPT_AMD_PRINT_ADDR=1: placement of every stream (HBM channel study)
            print_addr_ = false;
            fprintf(stderr, "[opt_amd] addr r=%p r1=%p p0=%p p1=%p Ap=%p Ap1=%p delta=%p pre=%p flags=%p "
                    "O=%p A=%p U=%p C=%p M=%p\n", (void*)r_, (void*)r1_, (void*)p0_, (void*)p1_, (void*)Ap_,
                    (void*)Ap1_, (void*)delta_, (void*)pre_, (void*)flags_, (void*)cur_O_, (void*)cur_A_,
                    (void*)cur_U_, (void*)cur_C_, (void*)cur_M_);
        }
        T* pcur = p0_;
        T* pprev = p1_;
        // PCGInit1 (r, pre, flags, rz[0]) from the arrays bound at THIS Step, as the
        // reference does on every Step (:2001, :2028): problem parameters may be updated
        // in place between Steps (Opt.h:64-65). On one domain it is fused with the first
        // PCG iteration's apply (iw_jtf_apply: the first p = pre r needs no global scalar).
        const bool fused = fused_init_ && offsets32_ && L >= 1;
        // iterations 1.. as iw_apply_res (the residual update folded into the next apply;
        // needs the sums r_0.W Ap_0, Ap_0.W Ap_0 of iteration 0), on one domain and on row
        // slabs: ONE all-reduce of four scalars per PCG iteration instead of two
        // (its 32-bit byte offsets must fit: above ~358 M pixels in fp32 / ~179 M in fp64 the
        // separate passes, which index with 64 bits, run instead)
        const bool res = fused_res_ && offsets32_ && L >= 1;
        // res with defer_: p_i in pb[i % 3]; the delta terms of odd iterations are folded
        // in pairs by the next even iteration (or the update), which reads p_{i-2} again
        // every p_i kept (OPT_AMD_IW_ALLP, lIterations <= kAllPMax): no pass carries a delta
        // term, iw_update_all forms delta once at the end
        const bool allp = allp_ && fused_init_ && offsets32_ && res && apfree_ && !recl_ && L >= 2 &&
                          L <= iw::kAllPMax && ensure_pall(L);
        const bool defer = res && defer_ && !allp;
        T* pb[3] = {p0_, p1_, p2_};
        // allp with P0: r_0 stays in r_ for the update (the passes ping-pong r over r1_ and the
        // unused Ap_), which forms p_0 = pre r_0 itself, so PCGInit1 does not store it
        const bool keep0 = allp && res && L >= 3;
        if (allp) pcur = pall_;
        // lIterations >= 3 with the fused loop: nothing but passes 1 and 2 reads p_0, and both
        // form it from r_0 (iw_apply_res P0), so PCGInit1 does not store it
        const bool p0 = res && L >= 3;
        // iterations 1.. as iw_pcg: Ap_{i-1} recomputed from p_{i-1}, never stored
        const bool apfree = res && apfree_;
        // the PCG vectors as records (Args::S): iw_jtf_apply, iw_pcg, iw_update
        const bool rec = recl_ && fused && apfree;
        if (rec) { pcur = rec_[0]; pb[0] = rec_[0]; pb[1] = rec_[1]; pb[2] = rec_[2]; }
        if (fused) {
            launch_jtf_apply(p0 ? nullptr : pcur, L == 1 || apfree, rec);
            allreduce(rz(0), 4);   // rz_0, p.Ap_0, r_0.W Ap_0, Ap_0.W Ap_0
            if (distributed()) {   // the next pass reads r_0 (and forms p_0) in the halo rows
                std::vector<HaloPlane> pl;
                if (rec) {   // r_0 / p_0's record, S, flags
                    pl.push_back({(void*)rec_[0], 6 * sizeof(T) * dom_.W});
                    pl.push_back({(void*)srec_, 4 * sizeof(T) * dom_.W});
                } else {
                    add_vec_planes(pl, r_);
                    pl.push_back({(void*)pre_, sizeof(T) * dom_.W});
                    if (!p0) add_vec_planes(pl, pcur);
                    if (!apfree) add_vec_planes(pl, Ap_);
                }
                pl.push_back({(void*)flags_, (size_t)dom_.W});
                exchange(pl);
            }
        } else {
            tbegin("iw_jtf"); launch_jtf(r_, pre_, rz(0), false, res); tend();
            allreduce(rz(0));
            if (distributed()) {
                std::vector<HaloPlane> pl;
                add_vec_planes(pl, r_);
                pl.push_back({(void*)pre_, sizeof(T) * dom_.W});
                pl.push_back({(void*)flags_, (size_t)dom_.W});
                exchange(pl);
            }
        }
        // (a hipGraph of this loop was measured: 4.38-4.41 ms/step against 4.38 with
        // plain launches — the 4-6 us gaps at the apply/residual boundaries are not
        // launch overhead, so the loop stays as plain stream launches)
        // row slabs with >= 3 row blocks: the halo refresh of r and p_{i-1} runs beside the
        // interior row blocks of the next apply (halo_mark / halo_begin / halo_join)
        // (the last row block / chunk must hold >= 2 rows: only the first and last read halo rows)
        const bool split = distributed() && overlap_ && comm_->concurrent_halo() &&
                           (pcg_side_ && apfree ? side_chunks() >= 3 && (dom_.y_hi - dom_.y_lo) - (side_chunks() - 1) * rows_ >= 2
                                                : nrowblocks_ >= 3 && (dom_.y_hi - dom_.y_lo) - (nrowblocks_ - 1) * 4 * rows_ >= 2);
        if (res) {
            // p_i in pb[i % 3] (deferred delta) or pb[i % 2]
            auto pbuf = [&](int i) { return allp ? pall_ + (size_t)i * 3 * dom_.npix_mem() : pb[defer ? i % 3 : i % 2]; };
            if (!fused) {   // iteration 0 with the two extra sums (PCGInit1 ran as iw_jtf)
                launch_apply<1, 0>(nullptr, pbuf(0), pap(0), 0, 0, 0, 0, nullptr, L == 1, 0, true);
                allreduce(pap(0), 3);
            }
            for (int i = 1; i < L; ++i) {
                const bool last = i + 1 == L;
                T* rb[2] = {r_, r1_};
                T* ab[2] = {Ap_, Ap1_};
                // pass 2 with P0: p_0 is formed from r_0, still in the r buffer pass 2 writes r_2 to
                const T* pin2 = (defer && i >= 2) ? ((p0 && i == 2 && !rec) ? rb[0] : pbuf(i - 2)) : nullptr;
                // part 0: every row block; 1: the interior ones; 2: the first and last
                auto pass = [&](int part) {
                    if (apfree) launch_pcg(i, pbuf(i - 1), pbuf(i), last, pin2, p0, part, rec, allp, keep0);
                    else launch_apply_res(i, pbuf(i - 1), pbuf(i), last, pin2, part, p0);
                };
                if (distributed()) {   // the pass reads r and p (and Ap) of iteration i-1 in the halo rows
                    std::vector<HaloPlane> pl;
                    if (rec) {
                        pl.push_back({(void*)pbuf(i - 1), 6 * sizeof(T) * dom_.W});
                    } else {
                        add_vec_planes(pl, rvec(i - 1, keep0));
                        if (!apfree) add_vec_planes(pl, ab[(i - 1) & 1]);
                        if (!(p0 && i == 1)) add_vec_planes(pl, pbuf(i - 1));   // P0: pass 1 forms p_0 from r_0
                    }
                    if (fused && i == 1) {   // iw_jtf_apply's exchange carried r_0 (and p_0, Ap_0)
                        pass(0);
                    } else if (split) {   // beside the interior row blocks
                        halo_mark();
                        pass(1);
                        halo_begin(comm_, pl, dom_, halo());
                        halo_join();
                        pass(2);
                    } else {
                        exchange(pl);
                        pass(0);
                    }
                } else if (apfree) {
                    launch_pcg(i, pbuf(i - 1), pbuf(i), last, pin2, p0, 0, rec, allp, keep0);
                } else {
                    launch_apply_res(i, pbuf(i - 1), pbuf(i), last, pin2, 0, p0);
                }
                allreduce(rz(i), 4);   // rz, pAp, r.W Ap, Ap.W Ap of iteration i
            }
            pcur = pbuf(L - 1);
        }
        for (int i = 0; i < L && !res; ++i) {
            if (i > 0 || !fused) std::swap(pcur, pprev);   // pcur <- new p, pprev <- old p
            const bool last = i + 1 == L;   // timed by events on the launch (launch_apply)
            if (i == 0 && fused) {   // iw_jtf_apply above
            }
            else if (i == 0) launch_apply<1, 0>(nullptr, pcur, pap(i), 0, 0, 0, 0, nullptr, last);
            else if (split) {
                halo_mark();
                if (i == 1) launch_apply<2, 1>(pprev, pcur, pap(i), rz(i), rz(i - 1), rz(i - 1), pap(i - 1), nullptr, last, 1);
                else launch_apply<2, 2>(pprev, pcur, pap(i), rz(i), rz(i - 1), rz(i - 1), pap(i - 1), nullptr, last, 1);
                std::vector<HaloPlane> pl;
                add_vec_planes(pl, r_);
                add_vec_planes(pl, pprev);
                halo_begin(comm_, pl, dom_, 1);
                halo_join();
                if (i == 1) launch_apply<2, 1>(pprev, pcur, pap(i), rz(i), rz(i - 1), rz(i - 1), pap(i - 1), nullptr, last, 2);
                else launch_apply<2, 2>(pprev, pcur, pap(i), rz(i), rz(i - 1), rz(i - 1), pap(i - 1), nullptr, last, 2);
            }
            else if (i == 1) launch_apply<2, 1>(pprev, pcur, pap(i), rz(i), rz(i - 1), rz(i - 1), pap(i - 1), nullptr, last);
            else launch_apply<2, 2>(pprev, pcur, pap(i), rz(i), rz(i - 1), rz(i - 1), pap(i - 1), nullptr, last);
            allreduce(pap(i));
            // the last iteration's residual update only feeds a beta nobody reads
            // (the update below takes alpha from rz[L-1] / pAp[L-1])
            if (i + 1 == L) break;
            tbegin("iw_residual");
            launch_residual(rz(i), pap(i), rz(i + 1));
            tend();
            allreduce(rz(i + 1));
            if (distributed() && !split && i + 1 < L) {   // the next apply reads r and p_i in the halo rows
                std::vector<HaloPlane> pl;
                add_vec_planes(pl, r_);
                add_vec_planes(pl, pcur);
                exchange(pl);
            }
        }
        // PCGLinearUpdate (with the last delta += alpha p) + cost
        if (allp) {
            tbegin("iw_update");
            launch_update_all(L, keep0);
            tend();
            exchange_unknowns();
        } else if (L > 0 && defer) {
            // pending: p_{L-1}, and p_{L-2} too when L-1 is odd (the even iterations fold pairs)
            const int ub = flat_grid(dom_.npix_mem(), 1);
            const T* pl = pb[(L - 1) % 3];
            const T* pl2 = L >= 2 ? pb[(L - 2) % 3] : nullptr;
            const bool e2 = L % 2 == 0, has = L >= 3;
            tbegin("iw_update");
            if (e2 && has)
                hipLaunchKernelGGL((rec ? iw::iw_update<T, true, true, true> : iw::iw_update<T, true, true>), dim3(ub), dim3(kBlock), 0, stream_, args(), cur_O_,
                                   cur_A_, (const T*)delta_, pl, red_.scalars, rz(L - 1), pap(L - 1), pl2, rz(L - 2),
                                   pap(L - 2));
            else if (e2)
                hipLaunchKernelGGL((rec ? iw::iw_update<T, false, true, true> : iw::iw_update<T, false, true>), dim3(ub), dim3(kBlock), 0, stream_, args(), cur_O_,
                                   cur_A_, (const T*)delta_, pl, red_.scalars, rz(L - 1), pap(L - 1), pl2, rz(L - 2),
                                   pap(L - 2));
            else if (has)
                hipLaunchKernelGGL((rec ? iw::iw_update<T, true, false, true> : iw::iw_update<T, true>), dim3(ub), dim3(kBlock), 0, stream_, args(), cur_O_,
                                   cur_A_, (const T*)delta_, pl, red_.scalars, rz(L - 1), pap(L - 1),
                                   (const T*)nullptr, 0, 0);
            else
                hipLaunchKernelGGL((rec ? iw::iw_update<T, false, false, true> : iw::iw_update<T, false>), dim3(ub), dim3(kBlock), 0, stream_, args(), cur_O_,
                                   cur_A_, (const T*)delta_, pl, red_.scalars, rz(L - 1), pap(L - 1),
                                   (const T*)nullptr, 0, 0);
            OPT_HIP_CHECK(hipGetLastError());
            tend();
            exchange_unknowns();
        } else if (L > 0) {
            const int ub = flat_grid(dom_.npix_mem(), 1);
            tbegin("iw_update");
            if (L >= 2)
                hipLaunchKernelGGL((rec ? iw::iw_update<T, true, false, true> : iw::iw_update<T, true>), dim3(ub), dim3(kBlock), 0, stream_, args(), cur_O_,
                                   cur_A_, (const T*)delta_, (const T*)pcur, red_.scalars, rz(L - 1), pap(L - 1),
                                   (const T*)nullptr, 0, 0);
            else
                hipLaunchKernelGGL((rec ? iw::iw_update<T, false, false, true> : iw::iw_update<T, false>), dim3(ub), dim3(kBlock), 0, stream_, args(), cur_O_,
                                   cur_A_, (const T*)delta_, (const T*)pcur, red_.scalars, rz(L - 1), pap(L - 1),
                                   (const T*)nullptr, 0, 0);
            OPT_HIP_CHECK(hipGetLastError());
            tend();
            exchange_unknowns();
        }
        // computeCost at the updated unknowns (:2245); the flags of this Step's J^T F pass
        // (Args::rev: backward after a forward update, so the next Step's forward J^T F pass
        // starts where it ends)
        tbegin("iw_cost"); launch_cost(kScCost, true, mall_rev_ && (allp ? ((L - 1) & 1) != 0 : true)); tend();
        allreduce(kScCost);
        const double c = read_scalar(kScCost);
        unbind_after_step();
        end_call();
        prev_cost_ = c;
        ++n_iter_;
        if (opts_.verbosity > 0) fprintf(stderr, "[opt_amd] GN iter %d cost %.9g\n", n_iter_, c);
        return 1;
    }

    int eval_jtf(void** params, void* r, void* pre, double* rzv) override {
        begin_call();
        bind(params, false);
        exchange_unknowns();
        launch_jtf((T*)r, (T*)pre, kScTmp, true);
        allreduce(kScTmp);
        *rzv = read_scalar(kScTmp);
        end_call();
        return 0;
    }
    int apply_jtj(void** params, const void* p, void* Ap, double* pAp) override {
        begin_call();
        bind(params, false);
        exchange_unknowns();
        if (distributed()) {
            std::vector<HaloPlane> pl;
            add_vec_planes(pl, (const T*)p);
            exchange(pl);
        }
        launch_flags();
        launch_apply<0, 0>((const T*)p, nullptr, kScTmp, 0, 0, 0, 0, (T*)Ap);
        allreduce(kScTmp);
        *pAp = read_scalar(kScTmp);
        end_call();
        return 0;
    }
    double eval_cost(void** params) override {
        begin_call();
        bind(params, false);
        exchange_unknowns();
        launch_cost(kScTmp);
        allreduce(kScTmp);
        double c = read_scalar(kScTmp);
        end_call();
        return c;
    }
    double time_apply(void** params, const void* p, void* Ap, int reps) override {
        begin_call();
        bind(params, false);
        launch_flags();
        hipEvent_t e0, e1;
        OPT_HIP_CHECK(hipEventCreate(&e0));
        OPT_HIP_CHECK(hipEventCreate(&e1));
        launch_apply<0, 0>((const T*)p, nullptr, kScTmp, 0, 0, 0, 0, (T*)Ap);   // warm
        OPT_HIP_CHECK(hipEventRecord(e0, stream_));
        for (int i = 0; i < reps; ++i) launch_apply<0, 0>((const T*)p, nullptr, kScTmp, 0, 0, 0, 0, (T*)Ap);
        OPT_HIP_CHECK(hipEventRecord(e1, stream_));
        OPT_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        OPT_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        end_call();
        return 1000.0 * ms / std::max(1, reps);
    }

private:
    // Measurement / A-B knobs, read once when the plan is created (never inside a Step):
    // OPT_AMD_ROWS rows per wave (0: iw::rows_for), OPT_AMD_STAGGER the vectors' placement,
    // and the separate-pass forms the tests compare bitwise with the fused loop
    // (OPT_AMD_IW_FUSED_INIT / _FUSED_RES / _DEFER = 0).
    void read_knobs() {
        const int rw = env_int("OPT_AMD_ROWS", 0);
        if (rw > 0) { rows_ = rw; rows_auto_ = false; }
        stagger_ = env_int("OPT_AMD_STAGGER", kStagger) & ~255LL;
        print_addr_ = env_int("OPT_AMD_PRINT_ADDR", 0) != 0;
        fused_init_ = env_int("OPT_AMD_IW_FUSED_INIT", 1) != 0;
        fused_res_ = env_int("OPT_AMD_IW_FUSED_RES", 1) != 0;
        defer_ = env_int("OPT_AMD_IW_DEFER", 1) != 0;
        side_ = env_int("OPT_AMD_IW_SIDE", 0) != 0;
        apfree_ = env_int("OPT_AMD_IW_APFREE", 1) != 0;
        rec_on_ = env_int("OPT_AMD_IW_REC", 0) != 0;
        cost60_ = env_int("OPT_AMD_IW_COST60", 1) != 0;
        cost_rows_ = (int)env_int("OPT_AMD_IW_COST_ROWS", 0);
        allp_ = env_int("OPT_AMD_IW_ALLP", 1) != 0;
        upd_nt_ = env_int("OPT_AMD_IW_UPD_NT", 1) != 0;
        upd_blocks_ = std::max(1, env_int("OPT_AMD_IW_UPD_BLOCKS", 2048));
        pcg_nt_ = env_int("OPT_AMD_IW_PCG_NT", 0) != 0;
        pcg_u2_ = env_int("OPT_AMD_IW_PCG_U2", 1);
        slab_rows_ = env_int("OPT_AMD_IW_SLAB_ROWS", 1) != 0;
        // iw_jtf_apply's 60-column strips store 240-B row segments that share cache lines
        // with the neighbouring strips: plain stores (merged in the L2) measured 217-220 us
        // against 233-245 with streaming ones (round 5, same box, interleaved)
        jtf_nt_ = env_int("OPT_AMD_IW_JTF_NT", 0) != 0;
        pall_limit_mb_ = env_int("OPT_AMD_IW_ALLP_LIMIT_MB", -1);
        pcg_side_ = env_int("OPT_AMD_IW_PCG_SIDE", 1) != 0;
        jtf_side_ = env_int("OPT_AMD_IW_JTF_SIDE", 0) != 0;
        cost_side_ = env_int("OPT_AMD_IW_COST_SIDE", 0) != 0;
        upd_pairs_ = env_int("OPT_AMD_IW_UPD_PAIRS", 1) != 0;
        pcg_alt_ = env_int("OPT_AMD_IW_PCG_ALT", 0) != 0;
        pcg_prc_ = env_int("OPT_AMD_IW_PCG_PRC", 1) != 0;
        cost_flags_ = env_int("OPT_AMD_IW_COST_FLAGS", 1) != 0;
        mall_rev_ = env_int("OPT_AMD_IW_MALL_REV", 1) != 0;
    }
    // A zeroed plan vector with kSlack spare bytes: place() may move each vector's base
    // within them between Steps (every vector is rewritten before it is read in a Step).
    static constexpr size_t kSlack = 1 << 20;
    // default stagger: 9 pages. On one plan (same physical pages) staggers of 0 .. 128 KiB
    // moved the 4096^2 GN step by 1-2.5 %, 0 the slowest and 36 KiB among the fastest on
    // three plans (tools/ab_knobs.py)
    static constexpr long long kStagger = 36864;
    void* vec_alloc(size_t bytes) {
        char* p = (char*)dmalloc(bytes + kSlack);
        raw_.push_back(p);
        OPT_HIP_CHECK(hipMemset(p, 0, bytes + kSlack));
        return p;
    }
    // OPT_AMD_STAGGER=S: vector k starts (k S) mod kSlack bytes into its allocation (HBM
    // placement study: the step time moves by up to ~8% with where the streams land)
    void place() {
        T** vs[] = {&r_, &p0_, &p1_, &Ap_, &delta_, &r1_, &Ap1_, &pre_, &p2_};
        if (raw_.size() < 10) return;
        for (int k = 0; k < 8; ++k) *vs[k] = (T*)(raw_[k] + ((size_t)stagger_ * k) % kSlack);
        flags_ = (uint8_t*)(raw_[8] + ((size_t)stagger_ * 8) % kSlack);
        p2_ = (T*)(raw_[9] + ((size_t)stagger_ * 9) % kSlack);
        if (recl_ && raw_.size() >= 14) {
            for (int k = 0; k < 3; ++k) rec_[k] = (T*)(raw_[10 + k] + ((size_t)stagger_ * (10 + k)) % kSlack);
            srec_ = (T*)(raw_[13] + ((size_t)stagger_ * 13) % kSlack);
        }
    }
    void allocate() {
        const long long N = dom_.npix_mem();
        nvec_ = 3 * N;
        offsets32_ = iw::offsets_fit_32<T>(N);
        for (T** v : {&r_, &p0_, &p1_, &Ap_, &delta_, &r1_, &Ap1_})
            *v = (T*)vec_alloc(sizeof(T) * 3 * N);
        pre_ = (T*)vec_alloc(sizeof(T) * N);   // angle channel only (Args::preO)
        flags_ = (uint8_t*)vec_alloc(N);
        p2_ = (T*)vec_alloc(sizeof(T) * 3 * N);   // third p buffer (deferred delta)
        // the REC layout (Args::S) for the fused loop
        recl_ = rec_on_ && fused_init_ && fused_res_ && apfree_ && iw::offsets_fit_rec<T>(N);
        if (recl_) {
            for (T*& v : rec_) v = (T*)vec_alloc(sizeof(T) * 6 * N);
            srec_ = (T*)vec_alloc(sizeof(T) * 4 * N);
        }
        place();
        nstrips_ = (dom_.W + iw::kStrip - 1) / iw::kStrip;
        if (rows_ <= 0 || rows_auto_) {
            rows_auto_ = true;
            rows_ = iw::rows_for(nstrips_, dom_.y_hi - dom_.y_lo);
            // a proper row slab (set_decomposition over part of the image; a one-rank
            // "split" of the whole image keeps the single-domain tiling, bitwise that path)
            if (rows_ <= 16 && comm_ && slab_rows_ && (dom_.y_lo > 0 || dom_.y_hi < dom_.H)) {
                int dev = 0, cu = 0;
                OPT_HIP_CHECK(hipGetDevice(&dev));
                OPT_HIP_CHECK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev));
                const int ng = (fused_strips() + kBlock / kWave - 1) / (kBlock / kWave);
                rows_ = iw::rows_one_round(ng, dom_.y_hi - dom_.y_lo, std::max(1, cu));
            }
        }
        nrowblocks_ = (dom_.y_hi - dom_.y_lo + rows_ * 4 - 1) / (rows_ * 4);
        red_.ensure(std::max({stencil_blocks(), fused_blocks(), cost_blocks(), cost_side_blocks(), fused_side_blocks(), 2048}),
                    1, 64);
        if (opts_.host_buffers) {
            dO_ = (T*)dmalloc(sizeof(T) * 2 * N);
            dA_ = (T*)dmalloc(sizeof(T) * N);
            dU_ = (float*)dmalloc(sizeof(float) * 2 * N);
            dC_ = (float*)dmalloc(sizeof(float) * 2 * N);
            dM_ = (float*)dmalloc(sizeof(float) * N);
        }
    }
    template <int K>
    void launch_update_all_k(int L, bool p0r) {
        if constexpr (K <= iw::kAllPMax) {
            if (L != K) { launch_update_all_k<K + 1>(L, p0r); return; }
            auto k = upd_nt_ ? (p0r ? iw::iw_update_all<T, K, true, true> : iw::iw_update_all<T, K, false, true>)
                             : (p0r ? iw::iw_update_all<T, K, true> : iw::iw_update_all<T, K, false>);
            // pixel pairs when every pair is aligned (iw_update_all2)
            const long long Np = dom_.npix_mem(), b = dom_.off(0, dom_.y_lo), e = dom_.off(0, dom_.y_hi);
            auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
            const bool pairs = upd_pairs_ && Np % 4 == 0 && b % 2 == 0 && (e - b) % 2 == 0 && al16(pall_) &&
                               al16(cur_O_) && ((uintptr_t)cur_A_ & (2 * sizeof(T) - 1)) == 0 && al16(r_) && al16(pre_);
            // Args::rev: the update starts where the last pass ended (pass L-1 runs backward when
            // L-1 is odd, launch_pcg)
            iw::Args<T> ua = args();
            ua.rev = mall_rev_ && !((L - 1) & 1) ? 1 : 0;
            if (pairs) {
                auto k2 = upd_nt_ ? (p0r ? iw::iw_update_all2<T, K, true, true> : iw::iw_update_all2<T, K, false, true>)
                                  : (p0r ? iw::iw_update_all2<T, K, true> : iw::iw_update_all2<T, K, false>);
                const long long need = ((e - b) / 2 + kBlock - 1) / kBlock;
                const int grid = (int)std::max(1LL, std::min<long long>(need, upd_blocks_));
                hipLaunchKernelGGL(k2, dim3(grid), dim3(kBlock), 0, stream_, ua, cur_O_, cur_A_,
                                   (const T*)pall_, 3 * Np, (const double*)red_.scalars, rz(0), (const T*)r_,
                                   (const T*)pre_);
                OPT_HIP_CHECK(hipGetLastError());
                return;
            }
            const long long need = (dom_.npix_mem() + kBlock - 1) / kBlock;
            const int grid = (int)std::max(1LL, std::min<long long>(need, upd_blocks_));
            hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, stream_, ua, cur_O_, cur_A_,
                               (const T*)pall_, 3 * dom_.npix_mem(), (const double*)red_.scalars, rz(0),
                               (const T*)r_, (const T*)pre_);
            OPT_HIP_CHECK(hipGetLastError());
        } else {
            throw std::logic_error("iw_update_all: lIterations above kAllPMax");
        }
    }
    // p0r: p_0 formed from r_0 (r_, pre_) as iw_jtf_apply forms it, instead of read
    void launch_update_all(int L, bool p0r) { launch_update_all_k<2>(L, p0r); }
    // r_i of the fused loop: r_ / r1_ alternating, or with keep0 (r_0 kept for
    // iw_update_all) r_0 in r_ and r_1, r_2, ... alternating over r1_ and Ap_ (Ap-free passes
    // never use Ap_)
    T* rvec(int i, bool keep0) const {
        if (!keep0) return (i & 1) ? r1_ : r_;
        return i == 0 ? r_ : (i & 1) ? r1_ : Ap_;
    }
    // allp's p vectors, grown to L (lIterations may rise between Steps). False when the L
    // vectors (3 N L values: 2 GB at 4096^2 fp32, L = 10) do not fit in the free HBM: the
    // Step then runs the deferred-delta loop, which needs no extra vectors
    bool ensure_pall(int L) {
        if (L <= pall_cap_) return true;
        OPT_HIP_CHECK(hipStreamSynchronize(stream_));
        dfree(pall_);
        pall_ = nullptr;
        pall_cap_ = 0;
        const size_t bytes = sizeof(T) * 3 * (size_t)dom_.npix_mem() * L;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || bytes + (64u << 20) > free_b ||
            (pall_limit_mb_ >= 0 && bytes > ((size_t)pall_limit_mb_ << 20)) ||
            hipMalloc((void**)&pall_, bytes) != hipSuccess) {
            (void)hipGetLastError();
            pall_ = nullptr;
            if (!pall_warned_) {
                fprintf(stderr, "[opt_amd] image_warping: %zu MiB for the kept p vectors do not fit (%zu MiB free): "
                        "deferred-delta loop\n", bytes >> 20, free_b >> 20);
                pall_warned_ = true;
            }
            return false;
        }
        // (ordered on the plan's stream: a null-stream memset is not ordered against it)
        OPT_HIP_CHECK(hipMemsetAsync(pall_, 0, bytes, stream_));
        pall_cap_ = L;
        return true;
    }
    void release() {
        for (char* p : raw_) dfree(p);
        raw_.clear();
        dfree(pall_);
        pall_ = nullptr;
        pall_cap_ = 0;
        for (T** v : {&r_, &pre_, &p0_, &p1_, &Ap_, &delta_, &r1_, &Ap1_, &p2_}) *v = nullptr;
        flags_ = nullptr;
        for (T*& v : rec_) v = nullptr;
        srec_ = nullptr;
        for (T** v : {&dO_, &dA_}) { dfree(*v); *v = nullptr; }
        for (float** v : {&dU_, &dC_, &dM_}) { dfree(*v); *v = nullptr; }
    }

    bool distributed() const { return comm_ && comm_->size() > 1; }
    // sum a scalar slot over ranks (no-op on one rank)
    void allreduce(int idx, int n = 1) {
        if (distributed()) comm_->allreduce_sum(red_.scalars + idx, n, stream_);
    }
    // halo planes of an unknown-layout vector [Offset.xy | Angle]
    void add_vec_planes(std::vector<HaloPlane>& v, const T* x) const {
        const long long plane = dom_.npix_mem();
        v.push_back({(void*)x, sizeof(T) * 2 * dom_.W});
        v.push_back({(void*)(x + 2 * plane), sizeof(T) * dom_.W});
    }
    void exchange(const std::vector<HaloPlane>& planes) {
        if (!distributed()) return;
        tbegin("halo_exchange");
        comm_->halo_exchange(planes, dom_, halo(), stream_);
        tend();
    }
    void exchange_unknowns() {
        exchange({{(void*)cur_O_, sizeof(T) * 2 * dom_.W}, {(void*)cur_A_, sizeof(T) * dom_.W}});
    }

    // scalar slots in red_.scalars: iteration i owns kSlots adjacent slots from rz(i):
    // rz, pAp, r.W Ap, Ap.W Ap, rz by the identity (iw_jtf_apply / iw_apply_res reduce the
    // first four at once)
    static constexpr int kScCost = 0, kScTmp = 1, kScBase = 2;
    int rz(int i) const { return kScBase + iw::kSlots * i; }
    int pap(int i) const { return rz(i) + 1; }

    int stencil_blocks() const { return nstrips_ * nrowblocks_; }
    // tiles of the side-by-side geometry (Args::side): groups of 4 strips x row chunks
    int side_blocks() const {
        return (nstrips_ + kBlock / kWave - 1) / (kBlock / kWave) * ((dom_.y_hi - dom_.y_lo + rows_ - 1) / rows_);
    }
    // tiles of iw_jtf_apply: 60-column strips
    int fused_strips() const { return (dom_.W + iw::kFStrip - 1) / iw::kFStrip; }
    // the same with side-by-side waves (Args::side): groups of 4 strips x row chunks of rows_
    int side_chunks() const { return (dom_.y_hi - dom_.y_lo + rows_ - 1) / rows_; }
    int fused_side_blocks() const {
        return (fused_strips() + kBlock / kWave - 1) / (kBlock / kWave) * side_chunks();
    }
    int fused_blocks() const { return fused_strips() * nrowblocks_; }
    // iw_cost60's rows per wave (OPT_AMD_IW_COST_ROWS; 0: the plan's rows, 32 at 4096^2 —
    // 16 / 24 / 48 / 64 ran 138-146 us against 132-135, tools/r05_cost_rows_ab.sh; held to
    // 64 VGPRs for 8 waves per SIMD instead of 6 it spilled and ran 141-142)
    int cost_rows() const { return cost_rows_ > 0 ? cost_rows_ : rows_; }
    int cost_side_blocks() const {
        return (fused_strips() + kBlock / kWave - 1) / (kBlock / kWave) *
               ((dom_.y_hi - dom_.y_lo + cost_rows() - 1) / cost_rows());
    }
    int cost_blocks() const {
        return fused_strips() * ((dom_.y_hi - dom_.y_lo + cost_rows() * 4 - 1) / (cost_rows() * 4));
    }

    iw::Args<T> args() const {
        iw::Args<T> a;
        a.dom = dom_;
        a.O = cur_O_; a.A = cur_A_; a.U = cur_U_; a.C = cur_C_; a.M = cur_M_;
        a.flags = flags_;
        a.wf = (T)wf_; a.wr = (T)wr_;
        a.use_pre = spec_.use_preconditioner ? 1 : 0;
        a.nstrips = nstrips_; a.nrowblocks = nrowblocks_; a.rows = rows_;
        a.tb0 = 0; a.tn0 = nstrips_ * nrowblocks_; a.tb1 = 0;
        a.side = 0;
        a.alt = 0;
        a.rev = 0;
        a.S = srec_;
        // same float expression the reference's evalJTF + guardedInvert evaluate
        const T wr2 = (T)wr_ * (T)wr_, wf2 = (T)wf_ * (T)wf_;
        for (int fit = 0; fit < 2; ++fit)
            for (int nv = 0; nv < 5; ++nv) {
                T d = wr2 * (T)(2 * nv);
                if (fit) d += wf2;
                const T s1 = (T)1 + std::sqrt(d);
                a.preO[fit][nv] = spec_.use_preconditioner ? (T)1 / (s1 * s1) : (T)0.25;
            }
        return a;
    }

    // Re-read the problemparams pointers (setGPUptr on every step, :2001) and the
    // scalar parameters; stage host arrays for the CPU-backend ABI modes.
    void bind(void** params, bool /*is_init*/) {
        wf_ = *(const float*)params[idx_wf_];
        wr_ = *(const float*)params[idx_wr_];
        user_O_ = (T*)params[idx_O_];
        user_A_ = (T*)params[idx_A_];
        if (!opts_.host_buffers) {
            cur_O_ = user_O_; cur_A_ = user_A_;
            cur_U_ = (const float*)params[idx_U_];
            cur_C_ = (const float*)params[idx_C_];
            cur_M_ = (const float*)params[idx_M_];
        } else {
            const long long N = dom_.npix_mem();
            OPT_HIP_CHECK(hipMemcpyAsync(dO_, user_O_, sizeof(T) * 2 * N, hipMemcpyHostToDevice, stream_));
            OPT_HIP_CHECK(hipMemcpyAsync(dA_, user_A_, sizeof(T) * N, hipMemcpyHostToDevice, stream_));
            OPT_HIP_CHECK(hipMemcpyAsync(dU_, params[idx_U_], sizeof(float) * 2 * N, hipMemcpyHostToDevice, stream_));
            OPT_HIP_CHECK(hipMemcpyAsync(dC_, params[idx_C_], sizeof(float) * 2 * N, hipMemcpyHostToDevice, stream_));
            OPT_HIP_CHECK(hipMemcpyAsync(dM_, params[idx_M_], sizeof(float) * N, hipMemcpyHostToDevice, stream_));
            cur_O_ = dO_; cur_A_ = dA_; cur_U_ = dU_; cur_C_ = dC_; cur_M_ = dM_;
        }
    }
    void unbind_after_step() {
        if (!opts_.host_buffers) return;
        const long long N = dom_.npix_mem();
        OPT_HIP_CHECK(hipMemcpyAsync(user_O_, dO_, sizeof(T) * 2 * N, hipMemcpyDeviceToHost, stream_));
        OPT_HIP_CHECK(hipMemcpyAsync(user_A_, dA_, sizeof(T) * N, hipMemcpyDeviceToHost, stream_));
    }

    double read_scalar(int idx) {
        return read_device_scalar(red_.scalars + idx);
    }

    void launch_jtf(T* r, T* pre, int sc_out, bool full_pre = false, bool acc = false) {
        const int nb = stencil_blocks();
        if (acc)
            hipLaunchKernelGGL((iw::iw_jtf<T, 0, true>), dim3(nb), dim3(kBlock), 0, stream_, args(), r, pre,
                               red_.slot(nb, sc_out));
        else if (full_pre)
            hipLaunchKernelGGL((iw::iw_jtf<T, 1>), dim3(nb), dim3(kBlock), 0, stream_, args(), r, pre,
                               red_.slot(nb, sc_out));
        else
            hipLaunchKernelGGL((iw::iw_jtf<T, 0>), dim3(nb), dim3(kBlock), 0, stream_, args(), r, pre,
                               red_.slot(nb, sc_out));
        OPT_HIP_CHECK(hipGetLastError());
    }
    // A launch with HIP events attached to it when the plan's timer asks for `name`.
    template <typename X> struct same { typedef X type; };
    template <typename... KA>
    void launch_timed(const char* name, void (*k)(KA...), int grid, typename same<KA>::type... args) {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        const bool ev = timer_.ext_pair(name, &e0, &e1);
        if (ev) hipExtLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, stream_, e0, e1, 0, args...);
        else hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, stream_, args...);
        OPT_HIP_CHECK(hipGetLastError());
        if (ev) timer_.ext_record(name, e0, e1);
    }
    // PCGInit1 + the first apply: r, pre, flags, p_0 = pre r (into pout), Ap_0 (unless
    // lIterations == 1: nothing reads that Ap), the four sums from sc[rz(0)].
    // REC: r_0 (and p_0 when pout, the same record rec_[0]) and the S record; no Ap
    void launch_jtf_apply(T* pout, bool no_ap, bool rec = false) {
        iw::Args<T> a = args();
        a.nstrips = fused_strips();
        a.side = jtf_side_ ? 1 : 0;
        const int nb = jtf_side_ ? fused_side_blocks() : fused_blocks();
        a.tb0 = 0; a.tn0 = nb; a.tb1 = 0;   // every tile (geom_fused)
        if (rec) {
            if (!no_ap || (pout && pout != rec_[0])) throw std::logic_error("iw_jtf_apply<REC>: record 0 only, no Ap");
            launch_timed("iw_jtf_apply", jtf_nt_ ? iw::iw_jtf_apply<T, 2, true> : iw::iw_jtf_apply<T, 0, true>, nb, a,
                         rec_[0], (T*)nullptr, pout, (T*)nullptr, red_.slot(nb, rz(0)));
            return;
        }
        launch_timed("iw_jtf_apply", jtf_nt_ ? iw::iw_jtf_apply<T, 2> : iw::iw_jtf_apply<T, 0>, nb, a, r_, pre_, pout,
                     no_ap ? nullptr : Ap_, red_.slot(nb, rz(0)));
    }
    // PCG iteration i >= 1 without a stored Ap (iw_pcg): reads r_{i-1} and p_{i-1}, writes
    // r_i (unless last) and p_i; the deferred delta and P0 exactly as launch_apply_res
    // part 0: every row block; 1: the interior row blocks [1, nrb - 1); 2: the first and last
    // (the only ones that read halo rows: a wave reads rows y0 - 2 .. y1 + 1)
    // REC: pin / pout / pin2 are the records of iterations i-1, i, i-2 (r and p together)
    // nodelta (allp): no delta term in any pass (iw_update_all forms delta)
    void launch_pcg(int i, const T* pin, T* pout, bool last, const T* pin2, bool p0, int part = 0, bool rec = false,
                    bool nodelta = false, bool keep0 = false) {
        const T* rin = rec ? pin : rvec(i - 1, keep0);
        T* rout = rec ? pout : (last ? nullptr : rvec(i, keep0));
        const double base_scale = (i == 1 && !spec_.use_preconditioner) ? 4.0 : 1.0;
        iw::Args<T> a = args();
        const int fs = fused_strips();
        a.nstrips = fs;
        const int nb = fused_blocks();   // the reduction slot spans every tile
        a.tb0 = 0; a.tn0 = nb; a.tb1 = 0;
        int grid = nb;
        int nbr = nb;
        a.alt = pcg_alt_ ? 1 : 0;
        a.rev = mall_rev_ && (i & 1) ? 1 : 0;   // pass i after a forward iw_jtf_apply: odd passes backward
        // the angle preconditioner recomputed (iw_pcg PRC): the mirrored walk sums its four
        // edge terms in another order, so not with alt
        const bool prc = pcg_prc_ && !pcg_alt_ && !rec;
        if (pcg_side_) {   // side-by-side waves (Args::side): tile = row chunk x group of 4 strips
            const int ng = (fs + kBlock / kWave - 1) / (kBlock / kWave), nch = side_chunks();
            a.side = 1;
            nbr = grid = a.tn0 = ng * nch;
            if (part == 1) {
                a.tb0 = ng; a.tn0 = ng * (nch - 2);
                grid = a.tn0;
            } else if (part == 2) {
                a.tb0 = 0; a.tn0 = ng; a.tb1 = ng * (nch - 1);
                grid = 2 * ng;
            }
        } else if (part == 1) {
            a.tb0 = fs; a.tn0 = fs * (nrowblocks_ - 2);
            grid = a.tn0;
        } else if (part == 2) {
            a.tb0 = 0; a.tn0 = fs; a.tb1 = fs * (nrowblocks_ - 1);
            grid = 2 * fs;
        }
        const ReduceSlot rs = red_.slot(nbr, rz(i));
        auto go = [&](auto kern) {
            launch_timed("iw_pcg", kern, grid, a, pin, rin, (const T*)pre_, pout, rout, delta_, red_.scalars,
                         rz(i - 1), base_scale, rs, pin2);
        };
        auto pick = [&](auto nt, auto u2, auto pf2, auto dp) {
            constexpr bool SNT = decltype(nt)::value, U2 = decltype(u2)::value, PF2 = decltype(pf2)::value,
                           DP = decltype(dp)::value;
            if (nodelta) {
                if constexpr (!DP && !PF2 && !SNT) {
                    if (prc && !(i == 1 && p0)) {
                        go(iw::iw_pcg<T, 0, 0, false, SNT, U2, PF2, DP, true>);
                        return;
                    }
                }
                if (i == 1 && p0) go(iw::iw_pcg<T, 0, 0, true, SNT, U2, PF2, DP>);
                else go(iw::iw_pcg<T, 0, 0, false, SNT, U2, PF2, DP>);
            } else if (pin2 || (defer_ && i == 1)) {
                if (i == 1 && p0) go(iw::iw_pcg<T, 0, 0, true, SNT, U2, PF2, DP>);
                else if (i % 2 == 1) go(iw::iw_pcg<T, 0, 0, false, SNT, U2, PF2, DP>);
                else if (i == 2 && p0) go(iw::iw_pcg<T, 1, 1, true, SNT, U2, PF2, DP>);
                else if (i == 2) go(iw::iw_pcg<T, 1, 1, false, SNT, U2, PF2, DP>);
                else go(iw::iw_pcg<T, 2, 1, false, SNT, U2, PF2, DP>);
            } else if (i == 1 && p0) go(iw::iw_pcg<T, 1, 0, true, SNT, U2, PF2, DP>);
            else if (i == 1) go(iw::iw_pcg<T, 1, 0, false, SNT, U2, PF2, DP>);
            else go(iw::iw_pcg<T, 2, 0, false, SNT, U2, PF2, DP>);
        };
        using F = std::false_type;
        using Tt = std::true_type;
        // row pairs only on waves of >= 16 rows: the 8-row waves of a row slab spend the
        // pair loop's prologue on too few rows (8 slabs of 4096 x 512 on one GPU, GN step
        // 7.2-7.6 ms with pairs against 6.5-7.0 without)
        const int u2 = rows_ >= 16 ? pcg_u2_ : 0;
        if (rec) {
            if (u2 == 2) pick(F{}, Tt{}, Tt{}, Tt{});
            else pick(F{}, F{}, F{}, Tt{});
        } else if (u2 == 2) pick(F{}, Tt{}, Tt{}, F{});
        else if (u2) pick(F{}, Tt{}, F{}, F{});
        else if (pcg_nt_) pick(Tt{}, F{}, F{}, F{});
        else pick(F{}, F{}, F{}, F{});
    }
    // part 0: every row block; 1: the interior row blocks [1, nrb - 1); 2: the first and
    // last row blocks (the only ones whose stencil reads halo rows)
    template <int MODE, int DM>
    void launch_apply(const T* pin, T* pout, int sc_out, int ib_num, int ib_den, int ia_num, int ia_den,
                      T* Ap = nullptr, bool no_ap = false, int part = 0, bool sums = false) {
        const int nb = stencil_blocks();
        Ap = no_ap ? nullptr : (Ap ? Ap : Ap_);
        iw::Args<T> a = args();
        int grid = nb;
        if (part == 1) {
            a.tb0 = nstrips_; a.tn0 = nstrips_ * (nrowblocks_ - 2);
            grid = a.tn0;
        } else if (part == 2) {
            a.tb0 = 0; a.tn0 = nstrips_; a.tb1 = nstrips_ * (nrowblocks_ - 1);
            grid = 2 * nstrips_;
        }
        if constexpr (MODE == 1) {
            if (sums) {   // iteration 0 of the fused loop (iw_apply_res's identity needs its sums)
                launch_timed("iw_apply", iw::iw_apply<T, 1, 0, false, 2, true>, grid, a, pin, (const T*)r_,
                             (const T*)pre_, pout, Ap, delta_, (const double*)red_.scalars, ib_num, ib_den, ia_num,
                             ia_den, red_.slot(nb, sc_out), (const T*)nullptr, (const int*)nullptr);
                return;
            }
        }
        launch_apply_grid<MODE, DM>(a, grid, pin, pout, sc_out, ib_num, ib_den, ia_num, ia_den, Ap);
    }
    template <int MODE, int DM>
    void launch_apply_grid(const iw::Args<T>& a, int grid, const T* pin, T* pout, int sc_out, int ib_num,
                           int ib_den, int ia_num, int ia_den, T* Ap) {
        const int nb = stencil_blocks();   // the reduction slot spans every tile
        // streaming (nontemporal) stores of the PCG vectors (NT = 2); streaming loads as
        // well, or plain stores, measured +1-5 % (round 3)
        launch_timed("iw_apply", iw::iw_apply<T, MODE, DM, false, 2>, grid, a, pin, (const T*)r_, (const T*)pre_,
                     pout, Ap, delta_, (const double*)red_.scalars, ib_num, ib_den, ia_num, ia_den,
                     red_.slot(nb, sc_out), (const T*)nullptr, (const int*)nullptr);
    }
    // PCG iteration i >= 1 of the fused loop: r_{i-1} / Ap_{i-1} in buffer (i-1) & 1 (r_ / Ap_
    // for even), r_i / Ap_i into the other one (none in the last iteration)
    // part: 0 every row block, 1 the interior ones, 2 the first and last (launch_apply)
    void launch_apply_res(int i, const T* pin, T* pout, bool last, const T* pin2 = nullptr, int part = 0,
                          bool p0 = false) {
        T* rb[2] = {r_, r1_};
        T* ab[2] = {Ap_, Ap1_};
        const T* rin = rb[(i - 1) & 1];
        const T* Apin = ab[(i - 1) & 1];
        T* rout = last ? nullptr : rb[i & 1];
        T* Apout = last ? nullptr : ab[i & 1];
        const double base_scale = (i == 1 && !spec_.use_preconditioner) ? 4.0 : 1.0;
        iw::Args<T> a = args();
        const bool side = side_ && part == 0;
        const int nb = side ? side_blocks() : stencil_blocks();   // the reduction slot spans every tile
        int grid = nb;
        if (side) { a.side = 1; a.tn0 = nb; }
        if (part == 1) {
            a.tb0 = nstrips_; a.tn0 = nstrips_ * (nrowblocks_ - 2);
            grid = a.tn0;
        } else if (part == 2) {
            a.tb0 = 0; a.tn0 = nstrips_; a.tb1 = nstrips_ * (nrowblocks_ - 1);
            grid = 2 * nstrips_;
        }
        const ReduceSlot rs = red_.slot(nb, rz(i));
        auto go = [&](auto kern) {
            launch_timed("iw_apply_res", kern, grid, a, pin, rin, Apin, (const T*)pre_, pout, rout, Apout, delta_,
                         red_.scalars, rz(i - 1), base_scale, rs, pin2);
        };
        // streaming stores of the PCG vectors (NT = 2; streaming loads too, or plain
        // stores, measured +1-5 %, round 3); P0: passes 1 and 2 form p_0 from r_0
        if (pin2 || (defer_ && i == 1)) {   // deferred delta: odd i none, i = 2 starts it, even i > 2 folds a pair
            if (i == 1 && p0) go(iw::iw_apply_res<T, 0, 2, 0, true>);
            else if (i % 2 == 1) go(iw::iw_apply_res<T, 0, 2, 0>);
            else if (i == 2 && p0) go(iw::iw_apply_res<T, 1, 2, 1, true>);
            else if (i == 2) go(iw::iw_apply_res<T, 1, 2, 1>);
            else go(iw::iw_apply_res<T, 2, 2, 1>);
        } else if (i == 1 && p0) go(iw::iw_apply_res<T, 1, 2, 0, true>);
        else if (i == 1) go(iw::iw_apply_res<T, 1, 2>);
        else go(iw::iw_apply_res<T, 2, 2>);
    }
    void launch_residual(int i_num, int i_den, int sc_out) {
        const int nb = flat_grid(dom_.npix_mem(), 2);
        hipLaunchKernelGGL((iw::iw_residual<T, true>), dim3(nb), dim3(kBlock), 0, stream_, args(), (const T*)Ap_,
                           (const T*)pre_, r_, red_.scalars, i_num, i_den, red_.slot(nb, sc_out));
        OPT_HIP_CHECK(hipGetLastError());
    }
    // iw_cost60 on the fused strips when its 32-bit offsets fit (offsets32_), else iw_cost
    // fl: the flag byte of this Step's iw_jtf_apply / iw_jtf is valid for the bound arrays
    // (the cost at the end of a Step; not Init's or OptAMD_EvalCost's)
    void launch_cost(int sc_out, bool fl = false, bool rev = false) {
        if (offsets32_ && cost60_) {
            iw::Args<T> a = args();
            a.nstrips = fused_strips();
            a.rows = cost_rows();
            a.nrowblocks = (dom_.y_hi - dom_.y_lo + a.rows * 4 - 1) / (a.rows * 4);
            int nb = a.nstrips * a.nrowblocks;
            if (cost_side_) {   // side-by-side waves (Args::side)
                a.side = 1;
                nb = cost_side_blocks();
            }
            a.tb0 = 0; a.tn0 = nb; a.tb1 = 0;
            a.rev = rev ? 1 : 0;
            if (fl && cost_flags_)
                hipLaunchKernelGGL((iw::iw_cost60<T, true>), dim3(nb), dim3(kBlock), 0, stream_, a, red_.slot(nb, sc_out));
            else
                hipLaunchKernelGGL(iw::iw_cost60<T>, dim3(nb), dim3(kBlock), 0, stream_, a, red_.slot(nb, sc_out));
        } else {
            const int nb = stencil_blocks();
            hipLaunchKernelGGL(iw::iw_cost<T>, dim3(nb), dim3(kBlock), 0, stream_, args(), red_.slot(nb, sc_out));
        }
        OPT_HIP_CHECK(hipGetLastError());
    }
    void launch_flags() {
        hipLaunchKernelGGL(iw::iw_flags<T>, dim3(flat_grid(dom_.npix_mem(), 1)), dim3(kBlock), 0, stream_,
                           args());
        OPT_HIP_CHECK(hipGetLastError());
    }

    Domain dom_;
    int idx_O_, idx_A_, idx_U_, idx_C_, idx_M_, idx_wf_, idx_wr_;
    long long nvec_ = 0;
    T *r_ = nullptr, *pre_ = nullptr, *p0_ = nullptr, *p1_ = nullptr, *Ap_ = nullptr, *delta_ = nullptr;
    T *r1_ = nullptr, *Ap1_ = nullptr;   // iw_apply_res ping-pongs r and Ap (neighbours read the old ones)
    T* p2_ = nullptr;                    // p_i in {p0_, p1_, p2_}[i % 3] with the deferred delta
    std::vector<char*> raw_;             // the plan vectors' allocations (vec_alloc)
    long long stagger_ = kStagger;
    bool print_addr_ = false;
    uint8_t* flags_ = nullptr;
    bool fused_init_ = true;            // OPT_AMD_IW_FUSED_INIT=0: iw_jtf, then iw_apply<1,0>
    bool fused_res_ = true;             // OPT_AMD_IW_FUSED_RES=0: iw_apply<2> + iw_residual per iteration
    bool defer_ = true;                 // OPT_AMD_IW_DEFER=0: iw_apply_res updates delta in every iteration
    bool side_ = false;                 // OPT_AMD_IW_SIDE=1: iw_apply_res with side-by-side waves (Args::side)
    bool apfree_ = true;                // OPT_AMD_IW_APFREE=0: iw_apply_res (stored Ap) instead of iw_pcg
    // OPT_AMD_IW_REC=1: the fused loop's vectors as records (Args::S). Measured slower (round 5,
    // interleaved A/B, 4096^2 fp32 GN step 3.99 against 3.75 ms: iw_jtf_apply writes 41 B/px
    // instead of 17, 318 against 218 us; iw_pcg 354 against 347 us — the pass is bound by its
    // VALU work and latency, not by the strip edges' partial lines)
    bool rec_on_ = false;
    // OPT_AMD_IW_COST60=0: the cost on 64-column strips with edge loads (iw_cost; 147 against
    // 141 us at 4096^2 fp32). A flat one-pixel-per-thread form with direct neighbour loads
    // measured 297 us, a bitwise copy of sincosf's small-argument path no change (the device
    // library already branches around its large-argument reduction): the strip kernels are
    // bound by their VALU work and load latency, not by the sine
    bool cost60_ = true;
    // OPT_AMD_IW_ALLP=0: the deferred delta (pairs folded by the even passes) instead of every
    // p_i kept for iw_update_all
    bool allp_ = true;
    // OPT_AMD_IW_UPD_NT=0: iw_update_all with plain loads of the p vectors (streaming: update
    // 510-518 -> 474 us, the following cost 116 -> 135 us, GN step 3.39-3.40 -> 3.34-3.37 ms)
    bool upd_nt_ = true;
    int upd_blocks_ = 2048;             // OPT_AMD_IW_UPD_BLOCKS: iw_update_all's grid cap (grid-stride beyond)
    T* pall_ = nullptr;                 // allp: lIterations p vectors of 3 N, p_i = pall_ + 3 N i
    int pall_cap_ = 0;
    bool pall_warned_ = false;
    bool mall_rev_ = true;              // OPT_AMD_IW_MALL_REV=0: every kernel of the Step walks forward (Args::rev)
    bool cost_flags_ = true;            // OPT_AMD_IW_COST_FLAGS=0: the Step's cost reads Mask and every Constraint
    bool pcg_prc_ = true;               // OPT_AMD_IW_PCG_PRC=0: iw_pcg reads the stored angle preconditioner
    bool pcg_alt_ = false;              // OPT_AMD_IW_PCG_ALT=1: iw_pcg's odd row chunks walk upward (Args::alt)
    bool upd_pairs_ = true;             // OPT_AMD_IW_UPD_PAIRS=0: iw_update_all one pixel per thread
    // OPT_AMD_IW_PCG_SIDE (default 1): iw_pcg with side-by-side waves (Args::side) — the block's
    // four waves walk the same rows of four adjacent 60-column strips (round 6: 270 -> 257 us
    // per pass at 4096^2, same box interleaved); 0 the four waves stacked over one strip
    bool pcg_side_ = true;
    bool jtf_side_ = false;             // OPT_AMD_IW_JTF_SIDE=1: iw_jtf_apply side by side
    bool cost_side_ = false;            // OPT_AMD_IW_COST_SIDE=1: iw_cost60 side by side
    long long pall_limit_mb_ = -1;      // OPT_AMD_IW_ALLP_LIMIT_MB: cap on the kept p vectors (tests the fallback)
    bool recl_ = false;                 // the plan holds the REC layout (rec_on_ and the fused loop's knobs)
    T* rec_[3] = {nullptr, nullptr, nullptr};   // REC: iteration i's record in rec_[i % 3] (i % 2 undeferred)
    T* srec_ = nullptr;                 // REC: the S record [u.x u.y angle pre_t], written by iw_jtf_apply
    bool pcg_nt_ = false;               // OPT_AMD_IW_PCG_NT=1: iw_pcg with streaming stores
    // OPT_AMD_IW_PCG_U2: 0 one row per loop trip, 1 (default since the kept-p loop: 275 ->
    // 270 us per pass, GN step 3.35 -> 3.30 ms) two rows with the records swapping roles,
    // 2 the same with two raw rows in flight
    int pcg_u2_ = 1;
    bool slab_rows_ = true;   // OPT_AMD_IW_SLAB_ROWS=0: row slabs keep rows_for's 16-row floor (iw::rows_one_round)
    int cost_rows_ = 0;
    bool jtf_nt_ = false;               // OPT_AMD_IW_JTF_NT=1: iw_jtf_apply with streaming stores
    bool offsets32_ = true;             // iw_apply_res's 32-bit byte offsets cover every plan vector
    int rows_ = 0, nstrips_ = 0, nrowblocks_ = 0;
    bool rows_auto_ = true;
    Comm* comm_ = nullptr;
    const bool overlap_ = env_int("OPT_AMD_HALO_OVERLAP", 1) != 0;   // 0: blocking halo before each apply
    float wf_ = 0, wr_ = 0;
    T *user_O_ = nullptr, *user_A_ = nullptr;
    T *cur_O_ = nullptr, *cur_A_ = nullptr;
    const float *cur_U_ = nullptr, *cur_C_ = nullptr, *cur_M_ = nullptr;
    // host-buffer staging (backend_cpu*)
    T *dO_ = nullptr, *dA_ = nullptr;
    float *dU_ = nullptr, *dC_ = nullptr, *dM_ = nullptr;
};

// ====================================================== operator for LM
// image_warping under the generic GN/LM driver (stencil_plan.h): used for LMGPU, where
// the trust-region diagonal, the residual resets and the device-side zeta exit live in
// the driver and the family supplies J^T F + diag, J^T J p (+ CtC p), cost and model
// cost. Same strip kernels as the GN plan above.
template <typename TT>
class ImageWarpingOp {
public:
    using T = TT;
    static constexpr const char* kName = "image_warping";
    static constexpr const char* kApplyName = "iw_apply";
    static constexpr bool kSlabs = true;
    ImageWarpingOp(const ProblemSpec& spec, const StateOptions& opts, Domain dom) : dom_(dom), opts_(opts) {
        idx_O_ = spec.unknown(0)->index;
        idx_A_ = spec.unknown(1)->index;
        idx_U_ = spec.array(0)->index;
        idx_C_ = spec.array(1)->index;
        idx_M_ = spec.array(2)->index;
        std::vector<DeclParam> ps = spec.params;
        std::sort(ps.begin(), ps.end(), [](auto& x, auto& y) { return x.index < y.index; });
        idx_wf_ = ps[0].index;
        idx_wr_ = ps[1].index;
        // by declared index: the routing matched this file's structural signature, in which
        // each parameter is identified by its problemparams index (generic.hip: generic_signature),
        // against the canonical energy's (fit weight declared first), so names play no part
        use_pre_ = spec.use_preconditioner;
        rows_ = env_int("OPT_AMD_ROWS", 0);   // 0: iw::rows_for (per domain)
        nstrips_ = (dom_.W + iw::kStrip - 1) / iw::kStrip;
        if (rows_ <= 0 || rows_auto_) { rows_auto_ = true; rows_ = iw::rows_for(nstrips_, dom_.y_hi - dom_.y_lo); }
        nrowblocks_ = (dom_.y_hi - dom_.y_lo + rows_ * 4 - 1) / (rows_ * 4);
        const long long N = dom_.npix_mem();
        if (opts.host_buffers) {
            dO_ = (T*)dmalloc(sizeof(T) * 2 * N);
            dA_ = (T*)dmalloc(sizeof(T) * N);
            dU_ = (float*)dmalloc(sizeof(float) * 2 * N);
            dC_ = (float*)dmalloc(sizeof(float) * 2 * N);
            dM_ = (float*)dmalloc(sizeof(float) * N);
        }
    }
    ~ImageWarpingOp() {
        dfree(dO_); dfree(dA_);
        for (float* v : {dU_, dC_, dM_}) dfree(v);
    }
    VecLayout layout() const {
        VecLayout L{};
        const long long N = dom_.npix_mem();
        L.nimg = 2;
        L.ch[0] = 2; L.ch[1] = 1;
        L.off[0] = 0; L.off[1] = 2 * N; L.off[2] = 3 * N;
        L.N = N;
        return L;
    }
    int halo() const { return 1; }
    int stencil_blocks() const { return nstrips_ * nrowblocks_; }
    void bind(void** params, hipStream_t s) {
        a_.wf = (T)*(const float*)params[idx_wf_];
        a_.wr = (T)*(const float*)params[idx_wr_];
        user_O_ = (T*)params[idx_O_];
        user_A_ = (T*)params[idx_A_];
        if (!opts_.host_buffers) {
            a_.O = user_O_; a_.A = user_A_;
            a_.U = (const float*)params[idx_U_];
            a_.C = (const float*)params[idx_C_];
            a_.M = (const float*)params[idx_M_];
        } else {
            const long long N = dom_.npix_mem();
            OPT_HIP_CHECK(hipMemcpyAsync(dO_, user_O_, sizeof(T) * 2 * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dA_, user_A_, sizeof(T) * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dU_, params[idx_U_], sizeof(float) * 2 * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dC_, params[idx_C_], sizeof(float) * 2 * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dM_, params[idx_M_], sizeof(float) * N, hipMemcpyHostToDevice, s));
            a_.O = dO_; a_.A = dA_; a_.U = dU_; a_.C = dC_; a_.M = dM_;
        }
        a_.dom = dom_;
        a_.use_pre = use_pre_ ? 1 : 0;
        a_.nstrips = nstrips_; a_.nrowblocks = nrowblocks_; a_.rows = rows_;
        a_.tb0 = 0; a_.tn0 = nstrips_ * nrowblocks_; a_.tb1 = 0;
        a_.side = 0;
        a_.rev = 0;
        for (int f = 0; f < 2; ++f)
            for (int v = 0; v < 5; ++v) a_.preO[f][v] = 0;   // MODE 0 never reads them
    }
    void unbind(hipStream_t s) {
        if (!opts_.host_buffers) return;
        const long long N = dom_.npix_mem();
        OPT_HIP_CHECK(hipMemcpyAsync(user_O_, dO_, sizeof(T) * 2 * N, hipMemcpyDeviceToHost, s));
        OPT_HIP_CHECK(hipMemcpyAsync(user_A_, dA_, sizeof(T) * N, hipMemcpyDeviceToHost, s));
    }
    T* unknown(int k) { return k == 0 ? (T*)a_.O : (T*)a_.A; }
    void precompute(hipStream_t) {}   // no ComputedArrays in this energy
    void computed_planes(std::vector<HaloPlane>&) const {}
    void jtf(T* r, T* diag, uint8_t* flags, hipStream_t s) {
        a_.flags = flags;
        hipLaunchKernelGGL((iw::iw_jtf<T, 2>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, r, diag, ReduceSlot{});
        OPT_HIP_CHECK(hipGetLastError());
    }
    void apply(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL((iw::iw_apply<T, 0, 0, true>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, p,
                           (const T*)nullptr, (const T*)nullptr, (T*)nullptr, Ap, (T*)nullptr,
                           (const double*)nullptr, 0, 0, 0, 0, rs, dadd, stop);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void cost(ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL(iw::iw_cost<T>, dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void model_cost(const T* delta, ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL(iw::iw_model_cost<T>, dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, delta, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }

    // materialized Jacobian (csr.h): 10 residual rows / 26 nonzeros per pixel
    long long jacobian_rows() const { return 10LL * dom_.W * dom_.H; }
    long long jacobian_nnz() const { return 26LL * dom_.W * dom_.H; }
    void dump_j(int* rowPtr, int* colInd, T* val, hipStream_t s) {
        hipLaunchKernelGGL(iw::iw_dump_j<T>, dim3(flat_grid((long long)dom_.W * dom_.H, 1)), dim3(kBlock), 0, s, a_,
                           rowPtr, colInd, val);
        OPT_HIP_CHECK(hipGetLastError());
    }

private:
    Domain dom_;
    StateOptions opts_;
    int idx_O_, idx_A_, idx_U_, idx_C_, idx_M_, idx_wf_, idx_wr_;
    bool use_pre_ = true;
    int rows_ = 32, nstrips_ = 0, nrowblocks_ = 0;
    bool rows_auto_ = false;
    iw::Args<T> a_{};
    T *user_O_ = nullptr, *user_A_ = nullptr, *dO_ = nullptr, *dA_ = nullptr;
    float *dU_ = nullptr, *dC_ = nullptr, *dM_ = nullptr;
};

std::unique_ptr<Plan> make_image_warping_plan(const ProblemSpec& spec, const StateOptions& opts,
                                              const unsigned* dims, std::string* err) {
    // Dim("W",0), Dim("H",1)
    unsigned W = 0, H = 0;
    for (auto& d : spec.dims) {
        if (d.name == spec.unknown(0)->dims[0]) W = dims[d.index];
        if (d.name == spec.unknown(0)->dims[1]) H = dims[d.index];
    }
    if (W == 0 || H == 0) { *err = "image_warping: zero-sized domain"; return nullptr; }
    if (spec.lm() || opts.materialized) {   // generic driver (LM; materialized J^T J)
        Domain dom{(int)W, (int)H, 0, (int)H, 0, (int)H};
        if (opts.double_precision) return make_stencil_plan<ImageWarpingOp<double>>(spec, opts, dom, err);
        return make_stencil_plan<ImageWarpingOp<float>>(spec, opts, dom, err);
    }
    if (opts.double_precision)
        return std::unique_ptr<Plan>(new ImageWarpingPlan<double>(spec, opts, W, H));
    return std::unique_ptr<Plan>(new ImageWarpingPlan<float>(spec, opts, W, H));
}

}  // namespace optamd
