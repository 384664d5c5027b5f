// arap.hip — kernels for the arap_mesh_deformation energy (graph domain)
// (reference examples/arap_mesh_deformation/arap_mesh_deformation.t):
//
//   unknowns Offset O, Angle A (3 per vertex); knowns UrShape U, Constraints C (float3)
//   graph G: edges v0 -> v1 (int32); UsePreconditioner(true)
//   e_fit(v) = C(v).x >= -999999.9 ? w_fit (O(v) - C(v)) : 0          (centred, per vertex)
//   e_reg(e) = w_reg ((O(v0) - O(v1)) - R(A(v0)) (U(v0) - U(v1)))     (per edge, 3 comps)
//
// The reference scatters every graph term with float atomics (createjtjgraph /
// createjtfgraph, o.t:2833-2867, 2969-2994; PCGStep1_Graph, solverGPUGaussNewton.t:
// 1216-1233). Here the graph is turned into two CSR adjacency lists once per bind
// (out-edges grouped by v0, in-edges grouped by v1; stable radix sorts, so the per-vertex
// order is the edge order) and every kernel is a deterministic per-vertex gather:
//   J_e p = w (p_O(v0) - p_O(v1) - K_v0 d_e),  K_v = sum_j p_A,j(v) dR/dA_j(v),  d_e = U(v0) - U(v1)
//   (J^T J p)_O(v) = w sum_out J_e p - w sum_in J_e p (+ w_fit^2 p_O(v))
//   (J^T J p)_A,j(v) = -w sum_out (dR_j(v) d_e) . J_e p
// K is computed once per vertex per apply by a first pass (arap_kdir, 36 B/vertex) so
// the in-edge terms read the neighbour's K instead of rebuilding its rotation derivatives.
// The apply reads its adjacency as sliced ELL (64-vertex slices, one slot row per wave
// load) built from the CSR lists once per bind.
//
// The apply walks one merged neighbour list (arap_apply_merged): on a mesh whose edges go
// both ways every neighbour's p and UrShape are gathered once for its out- and its
// in-edge term (kdir + apply 61 -> 53 us at 1 M vertices; OPT_AMD_ARAP_MERGED=0 keeps
// the two lists).
// Measured at 1 M vertices with the two lists (profiles/r02_arap_*): kdir + apply ~60 us. Counters (r02q):
// HBM traffic = the compulsory 176 B/vertex of the apply (132 B/vertex algorithmic + the
// K gather 36 + CSR offsets 8) and 60 B/vertex of kdir; the apply is bound by the
// texture/load path (TA busy 59 %, TD 67 % averaged over the dispatch incl. ramp and
// tail; ~650 B/vertex requested through it by the 12 neighbour gathers) with 54 % of wave
// time parked on loads. Variants measured within +-5 % or slower: edge batches 2-6 out x
// 2-6 in, waves/EU forced to 5, branch-free tails, sin/cos stored per step (slower:
// 6 loads beat 3 sincos), K recomputed per in-edge from the neighbour's angles (no kdir:
// 63 us), an edge-parallel apply (100-143 us).
// K as AoS rows (12-float stride, three 16-byte loads per neighbour) instead of 9 SoA
// planes: 53 -> 63 us, so K stays SoA.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cmath>
#include "plan.h"
#include "graph_util.h"
#include "stencil_plan.h"

namespace optamd {
namespace arap {

template <typename T>
struct Args {
    int N;
    T* O;
    T* A;
    const float* U;
    const float* C;
    const int* out_off;
    const int* out_nbr;
    const int* in_off;
    const int* in_nbr;
    // the same lists as sliced ELL for the apply: slice s = vertices [64 s, 64 s + 64),
    // its slot b of lane l at ell[eoff[s] + 64 b + l] (-1 past the vertex's degree), slot
    // count ew[s] (a multiple of the apply's batch size)
    const int *out_ell, *out_eoff, *out_ew;
    const int *in_ell, *in_eoff, *in_ew;
    // merged neighbour list (sliced ELL as above): every out-neighbour in out-list order,
    // flagged when the same neighbour also sends an edge here (its in-edge is then taken
    // in the same slot), then the unmatched in-neighbours; slot = u | kind << 28
    // (kind 1 out, 2 in, 3 both), -1 padding
    const int *nb_ell, *nb_eoff, *nb_ew;
    uint8_t* flags;
    T wf, wr;
};

template <typename T> struct V3 { T x, y, z; };
template <typename T, typename S>
__device__ __forceinline__ V3<T> ld3(const S* a, long long v) {
    return V3<T>{(T)a[3 * v], (T)a[3 * v + 1], (T)a[3 * v + 2]};
}
// Gathers address a neighbour as uniform base + 32-bit byte offset (the global_load
// saddr form: one full-rate multiply per address instead of a 64-bit multiply-add;
// make_arap_plan bounds N so 24 N and 72 N fit in 32 bits)
template <typename T, typename S>
__device__ __forceinline__ V3<T> gld3(const S* a, int u) {
    const S* q = (const S*)((const char*)a + (unsigned)u * (unsigned)(3 * sizeof(S)));
    return V3<T>{(T)q[0], (T)q[1], (T)q[2]};
}
template <typename S>
__device__ __forceinline__ S gld(const S* a, int u) {
    return *(const S*)((const char*)a + (unsigned)u * (unsigned)sizeof(S));
}
// Element u of plane q of an N-strided SoA array: one uniform base for every plane and a
// 32-bit offset (q N + u) sizeof(S) (make_arap_plan bounds 9 N sizeof(S) below 2^32), so
// the nine K gathers of a neighbour use the saddr form instead of nine 64-bit per-lane
// addresses (27 VGPR pairs at three neighbours per batch)
template <typename S>
__device__ __forceinline__ S gldq(const S* a, unsigned qN, int u) {
    return *(const S*)((const char*)a + (qN + (unsigned)u) * (unsigned)sizeof(S));
}
template <typename T>
__device__ __forceinline__ V3<T> mv(const T* M, const V3<T>& v) {
    return {M[0] * v.x + M[1] * v.y + M[2] * v.z, M[3] * v.x + M[4] * v.y + M[5] * v.z,
            M[6] * v.x + M[7] * v.y + M[8] * v.z};
}
__device__ __forceinline__ void sc(float t, float* s, float* c) { sincosf(t, s, c); }
__device__ __forceinline__ void sc(double t, double* s, double* c) { sincos(t, s, c); }

// Rotate3D (API/src/lib.t:84-98) and its partials w.r.t. the three angles
template <typename T>
__device__ __forceinline__ void rotation(const V3<T>& a, T* R, T dR[3][9]) {
    T sa, ca, sb, cb, sg, cg;
    sc(a.x, &sa, &ca); sc(a.y, &sb, &cb); sc(a.z, &sg, &cg);
    R[0] = cg * cb;  R[1] = -sg * ca + cg * sb * sa; R[2] = sg * sa + cg * sb * ca;
    R[3] = sg * cb;  R[4] = cg * ca + sg * sb * sa;  R[5] = -cg * sa + sg * sb * ca;
    R[6] = -sb;      R[7] = cb * sa;                 R[8] = cb * ca;
    if (!dR) return;
    dR[0][0] = 0; dR[0][1] = sg * sa + cg * sb * ca; dR[0][2] = sg * ca - cg * sb * sa;
    dR[0][3] = 0; dR[0][4] = -cg * sa + sg * sb * ca; dR[0][5] = -cg * ca - sg * sb * sa;
    dR[0][6] = 0; dR[0][7] = cb * ca; dR[0][8] = -cb * sa;
    dR[1][0] = -cg * sb; dR[1][1] = cg * cb * sa; dR[1][2] = cg * cb * ca;
    dR[1][3] = -sg * sb; dR[1][4] = sg * cb * sa; dR[1][5] = sg * cb * ca;
    dR[1][6] = -cb;      dR[1][7] = -sb * sa;     dR[1][8] = -sb * ca;
    dR[2][0] = -sg * cb; dR[2][1] = -cg * ca - sg * sb * sa; dR[2][2] = cg * sa - sg * sb * ca;
    dR[2][3] = cg * cb;  dR[2][4] = -sg * ca + cg * sb * sa; dR[2][5] = sg * sa + cg * sb * ca;
    dR[2][6] = 0;        dR[2][7] = 0;                       dR[2][8] = 0;
}
// K = sum_j q_j dR_j
template <typename T>
__device__ __forceinline__ void directional(T dR[3][9], const V3<T>& q, T* K) {
#pragma unroll
    for (int i = 0; i < 9; ++i) K[i] = q.x * dR[0][i] + q.y * dR[1][i] + q.z * dR[2][i];
}
template <typename T>
__device__ __forceinline__ bool fit_valid(const Args<T>& a, int v) { return a.C[3 * v] >= -999999.9f; }

// ------------------------------------------------------------------ J^T F
template <typename T>
__global__ __launch_bounds__(kBlock) void arap_jtf(Args<T> a, T* __restrict__ r, T* __restrict__ diag) {
    const int v = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;   // contiguous vertex ranges per XCD
    if (v >= a.N) return;
    const long long N = a.N;
    const T wr = a.wr, wf = a.wf;
    const V3<T> Ov = ld3<T>(a.O, v), Av = ld3<T>(a.A, v);
    const V3<float> Uv = ld3<float>(a.U, v);
    T R[9], dR[3][9];
    rotation(Av, R, dR);
    V3<T> rO = {0, 0, 0}, dO = {0, 0, 0}, rA = {0, 0, 0}, dA = {0, 0, 0};
    if (fit_valid(a, v)) {
        const V3<float> Cv = ld3<float>(a.C, v);
        rO = {-(wf * (wf * (Ov.x - (T)Cv.x))), -(wf * (wf * (Ov.y - (T)Cv.y))), -(wf * (wf * (Ov.z - (T)Cv.z)))};
        dO = {wf * wf, wf * wf, wf * wf};
    }
    for (int i = a.out_off[v]; i < a.out_off[v + 1]; ++i) {   // residuals centred here
        const int u = a.out_nbr[i];
        const V3<T> Ou = ld3<T>(a.O, u);
        const V3<float> Uu = ld3<float>(a.U, u);
        const V3<T> d = {(T)(Uv.x - Uu.x), (T)(Uv.y - Uu.y), (T)(Uv.z - Uu.z)};
        const V3<T> Rd = mv(R, d);
        const V3<T> e = {wr * ((Ov.x - Ou.x) - Rd.x), wr * ((Ov.y - Ou.y) - Rd.y), wr * ((Ov.z - Ou.z) - Rd.z)};
        rO.x -= wr * e.x; rO.y -= wr * e.y; rO.z -= wr * e.z;
        dO.x += wr * wr; dO.y += wr * wr; dO.z += wr * wr;
        T* rAj[3] = {&rA.x, &rA.y, &rA.z};
        T* dAj[3] = {&dA.x, &dA.y, &dA.z};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const V3<T> col = mv(dR[j], d);
            const T px = -wr * col.x, py = -wr * col.y, pz = -wr * col.z;
            *rAj[j] -= px * e.x + py * e.y + pz * e.z;
            *dAj[j] += px * px + py * py + pz * pz;
        }
    }
    for (int i = a.in_off[v]; i < a.in_off[v + 1]; ++i) {     // residuals whose tail is v
        const int u = a.in_nbr[i];
        const V3<T> Ou = ld3<T>(a.O, u), Au = ld3<T>(a.A, u);
        const V3<float> Uu = ld3<float>(a.U, u);
        T Ru[9];
        rotation<T>(Au, Ru, nullptr);
        const V3<T> d = {(T)(Uu.x - Uv.x), (T)(Uu.y - Uv.y), (T)(Uu.z - Uv.z)};
        const V3<T> Rd = mv(Ru, d);
        const V3<T> e = {wr * ((Ou.x - Ov.x) - Rd.x), wr * ((Ou.y - Ov.y) - Rd.y), wr * ((Ou.z - Ov.z) - Rd.z)};
        rO.x += wr * e.x; rO.y += wr * e.y; rO.z += wr * e.z;
        dO.x += wr * wr; dO.y += wr * wr; dO.z += wr * wr;
    }
    r[3 * v] = rO.x; r[3 * v + 1] = rO.y; r[3 * v + 2] = rO.z;
    r[3 * N + 3 * v] = rA.x; r[3 * N + 3 * v + 1] = rA.y; r[3 * N + 3 * v + 2] = rA.z;
    diag[3 * v] = dO.x; diag[3 * v + 1] = dO.y; diag[3 * v + 2] = dO.z;
    diag[3 * N + 3 * v] = dA.x; diag[3 * N + 3 * v + 1] = dA.y; diag[3 * N + 3 * v + 2] = dA.z;
    a.flags[v] = 1;
}

// ------------------------------------------------------------------ J^T J p
// First pass of the apply: K_v = sum_j p_A,j(v) dR/dA_j(v) for every vertex (9 values,
// stored structure-of-arrays),
// so the in-edge terms of the gather read a neighbour's K instead of rebuilding its
// rotation derivatives (three sincos and ~80 FMA per in-edge).
// STEP3: PCGStep3 of the generic driver folded in (stencil_plan.h HasFusedStep3): the
// vertex's six p entries become z + beta p first (step3_kernel's expression), then K is
// formed from the new angle part.
template <typename T, bool STEP3 = false>
__global__ __launch_bounds__(kBlock) void arap_kdir(Args<T> a, const T* __restrict__ pin, T* __restrict__ Kout,
                                                    const int* stop, const T* __restrict__ pre = nullptr,
                                                    const T* __restrict__ r = nullptr, const double* sc = nullptr,
                                                    int i_num = 0, int i_den = 0, int use_pre = 0) {
    if (stop && *stop) return;
    const int v = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;   // contiguous vertex ranges per XCD
    if (v >= a.N) return;
    const long long N = a.N;
    T* p = const_cast<T*>(pin);
    V3<T> pA;
    if constexpr (STEP3) {
        const T beta = (T)(sc[i_num] / sc[i_den]);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const long long e = 3 * N * h + 3 * v + c;
                const T z = use_pre ? pre[e] * r[e] : r[e];
                p[e] = z + beta * p[e];
                if (h == 1) (c == 0 ? pA.x : c == 1 ? pA.y : pA.z) = p[e];
            }
    } else {
        pA = ld3<T>(p + 3 * N, v);
    }
    T R[9], dR[3][9], K[9];
    rotation(ld3<T>(a.A, v), R, dR);
    directional(dR, pA, K);
#pragma unroll
    for (int i = 0; i < 9; ++i) Kout[i * N + v] = K[i];   // SoA: a wave's gathers of K_u hit 2 lines per entry
}

constexpr int kEBO = 6, kEBI = 3;   // apply edge batches (out, in); ELL widths are padded to them
template <typename T, int EBO = kEBO, int EBI = kEBI>
__global__ __launch_bounds__(kBlock) void arap_apply(Args<T> a, const T* __restrict__ p, T* __restrict__ Ap,
                                                     const T* __restrict__ Kall, const T* __restrict__ dadd,
                                                     const int* stop, ReduceSlot rs) {
    if (stop && *stop) return;
    const int v = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;   // contiguous vertex ranges per XCD
    T dot = 0;
    if (v < a.N) {
        const long long N = a.N;
        const T wr = a.wr, wf = a.wf;
        const V3<T> pO = ld3<T>(p, v), pA = ld3<T>(p + 3 * N, v);
        const V3<T> Av = ld3<T>(a.A, v);
        const V3<float> Uv = ld3<float>(a.U, v);
        T K[9];
        {
            T R[9], dR[3][9];
            rotation(Av, R, dR);
            directional(dR, pA, K);
        }
        // Angle rows: sum_e (dR_j d_e) . Jp_e = <dR_j, M>, M = sum_e Jp_e d_e^T, so the 27
        // rotation derivatives are rebuilt once after the out-edges instead of held live
        // through the gathers (register pressure: more waves in flight)
        T M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        V3<T> aO = {0, 0, 0}, aA = {0, 0, 0};
        if (fit_valid(a, v)) aO = {wf * (wf * pO.x), wf * (wf * pO.y), wf * (wf * pO.z)};
        // Edges in batches of EBO / EBI from the sliced-ELL lists: a wave's indices for one
        // slot are 256 contiguous bytes, and a batch's indices, then all of its neighbour
        // data, are loaded before any is used (memory-level parallelism for the dependent
        // gathers). Padding slots (-1) gather the vertex itself and contribute exact zeros
        // through a select; slots run in the CSR's (edge) order.
        const int lane = v & 63;
        const int* oel = a.out_ell + a.out_eoff[v >> 6] + lane;
        const int ow = a.out_ew[v >> 6];
        for (int i0 = 0; i0 < ow; i0 += EBO) {
            int u[EBO];
            bool okb[EBO];
#pragma unroll
            for (int b = 0; b < EBO; ++b) {
                const int x = oel[64 * (i0 + b)];
                okb[b] = x >= 0;
                u[b] = okb[b] ? x : v;
            }
            V3<T> pu[EBO];
            V3<float> Uu[EBO];
#pragma unroll
            for (int b = 0; b < EBO; ++b) { pu[b] = gld3<T>(p, u[b]); Uu[b] = gld3<float>(a.U, u[b]); }
#pragma unroll
            for (int b = 0; b < EBO; ++b) {
                const bool ok = okb[b];
        const V3<T> d = {(T)(Uv.x - Uu[b].x), (T)(Uv.y - Uu[b].y), (T)(Uv.z - Uu[b].z)};
                const V3<T> Kd = mv(K, d);
                const V3<T> jp = {ok ? wr * (pO.x - pu[b].x - Kd.x) : (T)0, ok ? wr * (pO.y - pu[b].y - Kd.y) : (T)0,
                                  ok ? wr * (pO.z - pu[b].z - Kd.z) : (T)0};
                const V3<T> dd = {ok ? d.x : (T)0, ok ? d.y : (T)0, ok ? d.z : (T)0};
                aO.x += wr * jp.x; aO.y += wr * jp.y; aO.z += wr * jp.z;
                M[0] += jp.x * dd.x; M[1] += jp.x * dd.y; M[2] += jp.x * dd.z;
                M[3] += jp.y * dd.x; M[4] += jp.y * dd.y; M[5] += jp.y * dd.z;
                M[6] += jp.z * dd.x; M[7] += jp.z * dd.y; M[8] += jp.z * dd.z;
            }
        }
        {
            T R[9], dR[3][9];
            rotation(Av, R, dR);
            T s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
            for (int q = 0; q < 9; ++q) { s0 += dR[0][q] * M[q]; s1 += dR[1][q] * M[q]; s2 += dR[2][q] * M[q]; }
            aA = {-wr * s0, -wr * s1, -wr * s2};
        }
        const int* iel = a.in_ell + a.in_eoff[v >> 6] + lane;
        const int iw = a.in_ew[v >> 6];
        for (int i0 = 0; i0 < iw; i0 += EBI) {
            int u[EBI];
            bool okb[EBI];
#pragma unroll
            for (int b = 0; b < EBI; ++b) {
                const int x = iel[64 * (i0 + b)];
                okb[b] = x >= 0;
                u[b] = okb[b] ? x : v;
            }
            V3<T> pu[EBI];
            V3<float> Uu[EBI];
            T Ku[EBI][9];
#pragma unroll
            for (int b = 0; b < EBI; ++b) {
                pu[b] = gld3<T>(p, u[b]);
                Uu[b] = gld3<float>(a.U, u[b]);
#pragma unroll
                for (int q = 0; q < 9; ++q) Ku[b][q] = gldq(Kall, (unsigned)q * (unsigned)N, u[b]);
            }
#pragma unroll
            for (int b = 0; b < EBI; ++b) {
                const bool ok = okb[b];
                const V3<T> d = {(T)(Uu[b].x - Uv.x), (T)(Uu[b].y - Uv.y), (T)(Uu[b].z - Uv.z)};
                const V3<T> Kd = mv(Ku[b], d);
                const V3<T> jp = {ok ? wr * (pu[b].x - pO.x - Kd.x) : (T)0, ok ? wr * (pu[b].y - pO.y - Kd.y) : (T)0,
                                  ok ? wr * (pu[b].z - pO.z - Kd.z) : (T)0};
                aO.x -= wr * jp.x; aO.y -= wr * jp.y; aO.z -= wr * jp.z;
            }
        }
        if (dadd) {
            aO.x += dadd[3 * v] * pO.x; aO.y += dadd[3 * v + 1] * pO.y; aO.z += dadd[3 * v + 2] * pO.z;
            aA.x += dadd[3 * N + 3 * v] * pA.x; aA.y += dadd[3 * N + 3 * v + 1] * pA.y;
            aA.z += dadd[3 * N + 3 * v + 2] * pA.z;
        }
        Ap[3 * v] = aO.x; Ap[3 * v + 1] = aO.y; Ap[3 * v + 2] = aO.z;
        Ap[3 * N + 3 * v] = aA.x; Ap[3 * N + 3 * v + 1] = aA.y; Ap[3 * N + 3 * v + 2] = aA.z;
        dot = pO.x * aO.x + pO.y * aO.y + pO.z * aO.z + pA.x * aA.x + pA.y * aA.y + pA.z * aA.z;
    }
    double vv[1] = {(double)dot};
    block_reduce_publish<1>(vv, rs, blockIdx.x);
}

// The same J^T J p over the merged neighbour list: a neighbour that is both an out- and
// an in-neighbour (every neighbour of a mesh whose edges go both ways) has its p and
// UrShape gathered once for both terms. The in-terms are summed in merged-list order
// (the out-terms, and so the angle rows, keep the out-list order).
// merged slots per batch; widths are padded to it. Round 3: 2 slots (89 VGPRs, 5 waves
// per SIMD) 50.6-50.9 us against 3 slots (110 VGPRs, 4 waves) 52.4-52.5 us for kdir +
// apply at 1 M vertices (profiles/r03_arap_eb.txt); OPT_AMD_ARAP_EB=3 restores 3
constexpr int kEBM = 2;
template <typename T, int EB = kEBM>
__global__ __launch_bounds__(kBlock) void arap_apply_merged(Args<T> a, const T* __restrict__ p, T* __restrict__ Ap,
                                                            const T* __restrict__ Kall, const T* __restrict__ dadd,
                                                            const int* stop, ReduceSlot rs) {
    if (stop && *stop) return;
    const int v = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;   // contiguous vertex ranges per XCD
    T dot = 0;
    if (v < a.N) {
        const long long N = a.N;
        const T wr = a.wr, wf = a.wf;
        const V3<T> pO = ld3<T>(p, v), pA = ld3<T>(p + 3 * N, v);
        const V3<T> Av = ld3<T>(a.A, v);
        const V3<float> Uv = ld3<float>(a.U, v);
        T K[9];
        {
            T R[9], dR[3][9];
            rotation(Av, R, dR);
            directional(dR, pA, K);
        }
        T M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        V3<T> aO = {0, 0, 0}, aA = {0, 0, 0};
        if (fit_valid(a, v)) aO = {wf * (wf * pO.x), wf * (wf * pO.y), wf * (wf * pO.z)};
        const int lane = v & 63;
        const int* nel = a.nb_ell + a.nb_eoff[v >> 6] + lane;
        const int nw = a.nb_ew[v >> 6];
        // one merged slot: the neighbour's p_O, UrShape and K (kind 0: padding, the vertex
        // itself, contributing exact zeros through the selects below)
        struct Slot { int kind; V3<T> pu; V3<float> Uu; T Ku[9]; };
        auto gather = [&](int x, Slot& sl) {
            sl.kind = x < 0 ? 0 : (x >> 28);
            const int u = x < 0 ? v : (x & 0x0FFFFFFF);
            sl.pu = gld3<T>(p, u);
            sl.Uu = gld3<float>(a.U, u);
#pragma unroll
            for (int q = 0; q < 9; ++q) sl.Ku[q] = gldq(Kall, (unsigned)q * (unsigned)N, u);
        };
        auto use = [&](const Slot& sl) {
            const bool out = sl.kind & 1, in = sl.kind & 2;
            const V3<T> d = {(T)(Uv.x - sl.Uu.x), (T)(Uv.y - sl.Uu.y), (T)(Uv.z - sl.Uu.z)};
            {   // out-edge v -> u
                const V3<T> Kd = mv(K, d);
                const V3<T> jp = {out ? wr * (pO.x - sl.pu.x - Kd.x) : (T)0, out ? wr * (pO.y - sl.pu.y - Kd.y) : (T)0,
                                  out ? wr * (pO.z - sl.pu.z - Kd.z) : (T)0};
                const V3<T> dd = {out ? d.x : (T)0, out ? d.y : (T)0, out ? d.z : (T)0};
                aO.x += wr * jp.x; aO.y += wr * jp.y; aO.z += wr * jp.z;
                M[0] += jp.x * dd.x; M[1] += jp.x * dd.y; M[2] += jp.x * dd.z;
                M[3] += jp.y * dd.x; M[4] += jp.y * dd.y; M[5] += jp.y * dd.z;
                M[6] += jp.z * dd.x; M[7] += jp.z * dd.y; M[8] += jp.z * dd.z;
            }
            {   // in-edge u -> v
                const V3<T> di = {(T)(sl.Uu.x - Uv.x), (T)(sl.Uu.y - Uv.y), (T)(sl.Uu.z - Uv.z)};
                const V3<T> Kd = mv(sl.Ku, di);
                const V3<T> jp = {in ? wr * (sl.pu.x - pO.x - Kd.x) : (T)0, in ? wr * (sl.pu.y - pO.y - Kd.y) : (T)0,
                                  in ? wr * (sl.pu.z - pO.z - Kd.z) : (T)0};
                aO.x -= wr * jp.x; aO.y -= wr * jp.y; aO.z -= wr * jp.z;
            }
        };
        // the next batch's slot ids are loaded while this batch gathers (one dependent load
        // latency per batch instead of two)
        int xn[EB];
#pragma unroll
        for (int b = 0; b < EB; ++b) xn[b] = nw > 0 ? nel[64 * b] : -1;
        for (int i0 = 0; i0 < nw; i0 += EB) {
            Slot sl[EB];
#pragma unroll
            for (int b = 0; b < EB; ++b) gather(xn[b], sl[b]);
            if (i0 + EB < nw) {
#pragma unroll
                for (int b = 0; b < EB; ++b) xn[b] = nel[64 * (i0 + EB + b)];
            }
#pragma unroll
            for (int b = 0; b < EB; ++b) use(sl[b]);
        }
        {
            T R[9], dR[3][9];
            rotation(Av, R, dR);
            T s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
            for (int q = 0; q < 9; ++q) { s0 += dR[0][q] * M[q]; s1 += dR[1][q] * M[q]; s2 += dR[2][q] * M[q]; }
            aA = {-wr * s0, -wr * s1, -wr * s2};
        }
        if (dadd) {
            aO.x += dadd[3 * v] * pO.x; aO.y += dadd[3 * v + 1] * pO.y; aO.z += dadd[3 * v + 2] * pO.z;
            aA.x += dadd[3 * N + 3 * v] * pA.x; aA.y += dadd[3 * N + 3 * v + 1] * pA.y;
            aA.z += dadd[3 * N + 3 * v + 2] * pA.z;
        }
        Ap[3 * v] = aO.x; Ap[3 * v + 1] = aO.y; Ap[3 * v + 2] = aO.z;
        Ap[3 * N + 3 * v] = aA.x; Ap[3 * N + 3 * v + 1] = aA.y; Ap[3 * N + 3 * v + 2] = aA.z;
        dot = pO.x * aO.x + pO.y * aO.y + pO.z * aO.z + pA.x * aA.x + pA.y * aA.y + pA.z * aA.z;
    }
    double vv[1] = {(double)dot};
    block_reduce_publish<1>(vv, rs, blockIdx.x);
}

// Merged list of one vertex (one thread per vertex): count (fill = false) or write
// (fill = true) the entries as described at Args::nb_ell.
__device__ __forceinline__ int merge_vertex(const int* oo, const int* on, const int* io, const int* in_, int v,
                                            int* out, int stride) {
    const int ob = oo[v], oe = oo[v + 1], ib = io[v], ie = io[v + 1];
    unsigned long long used = 0;   // in-entries matched so far (a vertex with > 64 in-edges: see below)
    int k = 0;
    for (int i = ob; i < oe; ++i) {
        const int u = on[i];
        int kind = 1;
        for (int j = ib; j < ie && j - ib < 64; ++j)
            if (!(used >> (j - ib) & 1ull) && in_[j] == u) {
                used |= 1ull << (j - ib);
                kind = 3;
                break;
            }
        if (out) out[(long long)k * stride] = u | (kind << 28);
        ++k;
    }
    for (int j = ib; j < ie; ++j)
        if (j - ib >= 64 || !(used >> (j - ib) & 1ull)) {
            if (out) out[(long long)k * stride] = in_[j] | (2 << 28);
            ++k;
        }
    return k;
}
__global__ void merged_width(const int* oo, const int* on, const int* io, const int* in_, int N, int nslices,
                             int pad, int* ew) {
    const int s = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, l = threadIdx.x & 63;
    if (s >= nslices) return;
    const int v = 64 * s + l;
    int d = v < N ? merge_vertex(oo, on, io, in_, v, nullptr, 0) : 0;
    for (int m = 32; m >= 1; m >>= 1) d = max(d, __shfl_xor(d, m));
    if (l == 0) ew[s] = (d + pad - 1) / pad * pad;
}
__global__ void merged_fill(const int* oo, const int* on, const int* io, const int* in_, int N, const int* eoff,
                            const int* ew, int* ell) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x, s = v >> 6;
    if (64 * s >= N) return;
    int* e = ell + eoff[s] + (v & 63);
    const int k = v < N ? merge_vertex(oo, on, io, in_, v, e, 64) : 0;
    for (int b = k; b < ew[s]; ++b) e[64 * b] = -1;
}

// ------------------------------------------------------- cost / model cost
// Each edge residual is summed by its head vertex (the edge's out-list owner).
template <typename T>
__global__ __launch_bounds__(kBlock) void arap_cost(Args<T> a, const T* __restrict__ delta, ReduceSlot rs) {
    const int v = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;   // contiguous vertex ranges per XCD
    T acc = 0;
    if (v < a.N) {
        const long long N = a.N;
        const T wr = a.wr, wf = a.wf;
        const V3<T> Ov = ld3<T>(a.O, v), Av = ld3<T>(a.A, v);
        const V3<float> Uv = ld3<float>(a.U, v);
        V3<T> dO = {0, 0, 0}, dAv = {0, 0, 0};
        if (delta) { dO = ld3<T>(delta, v); dAv = ld3<T>(delta + 3 * N, v); }
        T R[9], dR[3][9], K[9];
        rotation(Av, R, delta ? dR : nullptr);
        if (delta) directional(dR, dAv, K);
        T fit = 0;
        if (fit_valid(a, v)) {
            const V3<float> Cv = ld3<float>(a.C, v);
            T ex = wf * (Ov.x - (T)Cv.x), ey = wf * (Ov.y - (T)Cv.y), ez = wf * (Ov.z - (T)Cv.z);
            if (delta) { ex += wf * dO.x; ey += wf * dO.y; ez += wf * dO.z; }
            fit = (T)0.5 * (ex * ex + ey * ey + ez * ez);
        }
        T reg = 0;
        for (int i = a.out_off[v]; i < a.out_off[v + 1]; ++i) {
            const int u = a.out_nbr[i];
            const V3<T> Ou = ld3<T>(a.O, u);
            const V3<float> Uu = ld3<float>(a.U, u);
            const V3<T> d = {(T)(Uv.x - Uu.x), (T)(Uv.y - Uu.y), (T)(Uv.z - Uu.z)};
            const V3<T> Rd = mv(R, d);
            V3<T> e = {wr * ((Ov.x - Ou.x) - Rd.x), wr * ((Ov.y - Ou.y) - Rd.y), wr * ((Ov.z - Ou.z) - Rd.z)};
            if (delta) {
                const V3<T> du = ld3<T>(delta, u);
                const V3<T> Kd = mv(K, d);
                e.x += wr * (dO.x - du.x - Kd.x);
                e.y += wr * (dO.y - du.y - Kd.y);
                e.z += wr * (dO.z - du.z - Kd.z);
            }
            reg += (T)0.5 * (e.x * e.x + e.y * e.y + e.z * e.z);
        }
        acc = fit + reg;
    }
    double vv[1] = {(double)acc};
    block_reduce_publish<1>(vv, rs, blockIdx.x);
}

// Sliced ELL of a CSR (one wave per 64-vertex slice): slot counts, then the slots.
__global__ void ell_width(const int* off, int N, int nslices, int pad, int* ew) {
    const int s = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, l = threadIdx.x & 63;
    if (s >= nslices) return;
    const int v = 64 * s + l;
    int d = v < N ? off[v + 1] - off[v] : 0;
    for (int m = 32; m >= 1; m >>= 1) d = max(d, __shfl_xor(d, m));
    if (l == 0) ew[s] = (d + pad - 1) / pad * pad;
}
__global__ void ell_fill(const int* off, const int* nbr, int N, const int* eoff, const int* ew, int* ell) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x, s = v >> 6;
    if (64 * s >= N) return;
    const int b0 = v < N ? off[v] : 0, d = v < N ? off[v + 1] - b0 : 0;
    int* e = ell + eoff[s] + (v & 63);
    for (int b = 0; b < ew[s]; ++b) e[64 * b] = b < d ? nbr[b0 + b] : -1;
}

// vertex indices of the graph must lie in [0, N): checked once per CSR build
__global__ void check_indices(const int* v0, const int* v1, int E, int N, int* bad) {
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < E; e += gridDim.x * blockDim.x)
        if (v0[e] < 0 || v0[e] >= N || v1[e] < 0 || v1[e] >= N) atomicOr(bad, 1);
}
__global__ void count_heads(const int* keys, int E, int* counts) {
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < E; e += gridDim.x * blockDim.x)
        atomicAdd(&counts[keys[e]], 1);
}


// ---------------------------------------------------- materialized Jacobian
// saveJToCRS / saveJToCRS_Graph (solverGPUGaussNewton.t:1004-1022, 1287-1305) with
// generateDumpJ (:385-442). Rows: the fit residuals first (centred, vertex v owns rows
// 3v + c, one nonzero {O_c(v): wf [has target]}), then the graph residuals (edge e owns
// rows 3N + 3e + c, nonzeros {O_c(v0): wr, O_c(v1): -wr, A_j(v0): -wr (dR_j d_e)_c} for
// the angles row c of Rotate3D reads — all three for x and y, alpha and beta for z
// (lib.t:84-97: row z is -sin b, cos b sin a, cos b cos a), so 5 + 5 + 4 per edge as the
// template's unknown accesses), columns = unknown indices ([Offset 3N | Angle 3N]) sorted
// inside each row.
template <typename T>
__global__ __launch_bounds__(kBlock) void arap_dump_fit(Args<T> a, int E, int* __restrict__ rowPtr,
                                                        int* __restrict__ colInd, T* __restrict__ val) {
    if (E == 0 && blockIdx.x == 0 && threadIdx.x == 0) rowPtr[3LL * a.N] = 3 * a.N;
    for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < a.N; v += gridDim.x * blockDim.x) {
        const T w = fit_valid(a, v) ? a.wf : (T)0;
        for (int c = 0; c < 3; ++c) {
            rowPtr[3 * v + c] = 3 * v + c;
            colInd[3 * v + c] = 3 * v + c;
            val[3 * v + c] = w;
        }
    }
}
template <typename T>
__global__ __launch_bounds__(kBlock) void arap_dump_edges(Args<T> a, const int* __restrict__ v0s,
                                                          const int* __restrict__ v1s, int E, int* __restrict__ rowPtr,
                                                          int* __restrict__ colInd, T* __restrict__ val) {
    const long long N = a.N;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < E; e += gridDim.x * blockDim.x) {
        const int v0 = v0s[e], v1 = v1s[e];
        T R[9], dR[3][9];
        rotation(ld3<T>(a.A, v0), R, dR);
        const V3<float> U0 = ld3<float>(a.U, v0), U1 = ld3<float>(a.U, v1);
        const V3<T> dd = {(T)(U0.x - U1.x), (T)(U0.y - U1.y), (T)(U0.z - U1.z)};
        V3<T> col[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) col[j] = mv(dR[j], dd);
        for (int c = 0; c < 3; ++c) {
            const long long row = 3 * N + 3LL * e + c, nz = 3 * N + 14LL * e + 5 * c;
            const int K = c == 2 ? 4 : 5;   // row z has no gamma access
            rowPtr[row] = (int)nz;
            int cc[5] = {(int)(3 * v0 + c), (int)(3 * v1 + c), (int)(3 * N + 3 * v0), (int)(3 * N + 3 * v0 + 1),
                         (int)(3 * N + 3 * v0 + 2)};
            T vv[5] = {a.wr, -a.wr, -a.wr * (c == 0 ? col[0].x : c == 1 ? col[0].y : col[0].z),
                       -a.wr * (c == 0 ? col[1].x : c == 1 ? col[1].y : col[1].z),
                       -a.wr * (c == 0 ? col[2].x : c == 1 ? col[2].y : col[2].z)};
            for (int i = 1; i < K; ++i)   // sortCol
                for (int j = i; j > 0 && cc[j] < cc[j - 1]; --j) {
                    const int tc = cc[j]; cc[j] = cc[j - 1]; cc[j - 1] = tc;
                    const T tv = vv[j]; vv[j] = vv[j - 1]; vv[j - 1] = tv;
                }
            for (int q = 0; q < K; ++q) {
                colInd[nz + q] = cc[q];
                val[nz + q] = vv[q];
            }
        }
        if (e == E - 1) rowPtr[3 * N + 3LL * E] = (int)(3 * N + 14LL * E);
    }
}

}  // namespace arap

// Deterministic CSR of a directed edge list grouped by `keys` (stable: edge order kept).
struct GraphCSR {
    int* off = nullptr;   // N + 1
    int* nbr = nullptr;   // E
    int* ell = nullptr;   // sliced ELL of the same lists (arap::Args)
    int* eoff = nullptr;  // per slice: first slot entry (nslices + 1, exclusive scan of 64 ew)
    int* ew = nullptr;    // per slice: slot count
    void release() {
        for (int** q : {&off, &nbr, &ell, &eoff, &ew}) { dfree(*q); *q = nullptr; }
    }
};

template <typename TT>
class ArapOp {
public:
    using T = TT;
    static constexpr const char* kName = "arap_mesh_deformation";
    static constexpr const char* kApplyName = "arap_apply";
    static constexpr bool kSlabs = false;   // graph domain: single GPU (replicas only)
    ArapOp(const ProblemSpec& spec, const StateOptions& opts, Domain dom) : opts_(opts) {
        N_ = dom.W;
        E_ = dom.edges;
        idx_O_ = spec.unknown(0)->index;
        idx_A_ = spec.unknown(1)->index;
        idx_U_ = spec.array(0)->index;
        idx_C_ = spec.array(1)->index;
        idx_v0_ = spec.graphs[0].vertices[0].second;
        idx_v1_ = spec.graphs[0].vertices[1].second;
        std::vector<DeclParam> ps = spec.params;
        std::sort(ps.begin(), ps.end(), [](auto& x, auto& y) { return x.index < y.index; });
        idx_wf_ = ps[0].index;
        idx_wr_ = ps[1].index;
        // by declared index: the routing matched this file's structural signature, in which
        // each parameter is identified by its problemparams index (generic.hip: generic_signature),
        // against the canonical energy's (fit weight declared first), so names play no part
        K_ = (T*)dmalloc(sizeof(T) * 9 * std::max(N_, 1));
        if (opts.host_buffers) {
            dO_ = (T*)dmalloc(sizeof(T) * 3 * N_);
            dA_ = (T*)dmalloc(sizeof(T) * 3 * N_);
            dU_ = (float*)dmalloc(sizeof(float) * 3 * N_);
            dC_ = (float*)dmalloc(sizeof(float) * 3 * N_);
            dv0_ = (int*)dmalloc(sizeof(int) * std::max(E_, 1));
            dv1_ = (int*)dmalloc(sizeof(int) * std::max(E_, 1));
        }
    }
    ~ArapOp() {
        out_.release(); in_.release(); nb_.release();
        dfree(dO_); dfree(dA_); dfree(dU_); dfree(dC_); dfree(dv0_); dfree(dv1_);
        dfree(scratch_); dfree(keys_tmp_); dfree(K_); dfree(fp_scratch_);
    }
    VecLayout layout() const {
        VecLayout L{};
        L.nimg = 2;
        L.ch[0] = 3; L.ch[1] = 3;
        L.off[0] = 0; L.off[1] = 3LL * N_; L.off[2] = 6LL * N_;
        L.N = N_;
        return L;
    }
    int halo() const { return 0; }
    int stencil_blocks() const { return (N_ + kBlock - 1) / kBlock; }
    void bind(void** params, hipStream_t s) {
        a_.wf = (T)*(const float*)params[idx_wf_];
        a_.wr = (T)*(const float*)params[idx_wr_];
        userO_ = (T*)params[idx_O_];
        userA_ = (T*)params[idx_A_];
        const int* v0;
        const int* v1;
        if (!opts_.host_buffers) {
            a_.O = userO_; a_.A = userA_;
            a_.U = (const float*)params[idx_U_];
            a_.C = (const float*)params[idx_C_];
            v0 = (const int*)params[idx_v0_];
            v1 = (const int*)params[idx_v1_];
        } else {
            OPT_HIP_CHECK(hipMemcpyAsync(dO_, userO_, sizeof(T) * 3 * N_, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dA_, userA_, sizeof(T) * 3 * N_, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dU_, params[idx_U_], sizeof(float) * 3 * N_, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dC_, params[idx_C_], sizeof(float) * 3 * N_, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dv0_, params[idx_v0_], sizeof(int) * E_, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dv1_, params[idx_v1_], sizeof(int) * E_, hipMemcpyHostToDevice, s));
            a_.O = dO_; a_.A = dA_; a_.U = dU_; a_.C = dC_;
            v0 = dv0_;
            v1 = dv1_;
        }
        // rebuild the adjacency when the edges change (content, not address: graph_util.h)
        const int* vs[2] = {v0, v1};
        const unsigned long long h = graph_fingerprint(vs, 2, E_, s, fp_scratch_);
        if (v0 != graph_v0_ || v1 != graph_v1_ || h != fingerprint_) {
            build_csr(v0, v1, s);
            fingerprint_ = h;
        }
        a_.N = N_;
        a_.out_off = out_.off; a_.out_nbr = out_.nbr;
        a_.in_off = in_.off; a_.in_nbr = in_.nbr;
        a_.out_ell = out_.ell; a_.out_eoff = out_.eoff; a_.out_ew = out_.ew;
        a_.in_ell = in_.ell; a_.in_eoff = in_.eoff; a_.in_ew = in_.ew;
        a_.nb_ell = nb_.ell; a_.nb_eoff = nb_.eoff; a_.nb_ew = nb_.ew;
    }
    void unbind(hipStream_t s) {
        if (!opts_.host_buffers) return;
        OPT_HIP_CHECK(hipMemcpyAsync(userO_, dO_, sizeof(T) * 3 * N_, hipMemcpyDeviceToHost, s));
        OPT_HIP_CHECK(hipMemcpyAsync(userA_, dA_, sizeof(T) * 3 * N_, hipMemcpyDeviceToHost, s));
    }
    T* unknown(int k) { return k == 0 ? a_.O : a_.A; }
    void precompute(hipStream_t) {}
    void computed_planes(std::vector<HaloPlane>&) const {}
    void jtf(T* r, T* diag, uint8_t* flags, hipStream_t s) {
        a_.flags = flags;
        hipLaunchKernelGGL((arap::arap_jtf<T>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, r, diag);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void apply(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL((arap::arap_kdir<T>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, p, K_, stop,
                           (const T*)nullptr, (const T*)nullptr, (const double*)nullptr, 0, 0, 0);
        apply_prepared(p, Ap, dadd, stop, rs, s);
    }
    // PCGStep3 + the apply's K pass in one kernel; the next apply is apply_prepared
    void step3_fused(const T* pre, const T* r, T* p, const double* sc, int i_num, int i_den, int use_pre,
                     const int* stop, hipStream_t s) {
        hipLaunchKernelGGL((arap::arap_kdir<T, true>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, (const T*)p,
                           K_, stop, pre, r, sc, i_num, i_den, use_pre);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void apply_prepared(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s) {
        if (merged_on_ && eb_ == 3)
            hipLaunchKernelGGL((arap::arap_apply_merged<T, 3>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, p, Ap,
                               (const T*)K_, dadd, stop, rs);
        else if (merged_on_)
            hipLaunchKernelGGL((arap::arap_apply_merged<T, 2>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, p, Ap,
                               (const T*)K_, dadd, stop, rs);
        else
            hipLaunchKernelGGL((arap::arap_apply<T>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, p, Ap,
                               (const T*)K_, dadd, stop, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void cost(ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL((arap::arap_cost<T>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, (const T*)nullptr, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void model_cost(const T* delta, ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL((arap::arap_cost<T>), dim3(stencil_blocks()), dim3(kBlock), 0, s, a_, delta, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    // materialized Jacobian (csr.h): 3 fit rows per vertex (1 nonzero each), then 3 rows
    // per directed edge (5 + 5 + 4 nonzeros)
    long long jacobian_rows() const { return 3LL * N_ + 3LL * E_; }
    long long jacobian_nnz() const { return 3LL * N_ + 14LL * E_; }
    void dump_j(int* rowPtr, int* colInd, T* val, hipStream_t s) {
        hipLaunchKernelGGL((arap::arap_dump_fit<T>), dim3(std::max(1, std::min((N_ + 255) / 256, 4096))), dim3(kBlock),
                           0, s, a_, E_, rowPtr, colInd, val);
        if (E_ > 0)
            hipLaunchKernelGGL((arap::arap_dump_edges<T>), dim3(std::min((E_ + 255) / 256, 4096)), dim3(kBlock), 0, s,
                               a_, graph_v0_, graph_v1_, E_, rowPtr, colInd, val);
        OPT_HIP_CHECK(hipGetLastError());
    }

private:
    // CSR of the edges grouped by `keys` with `vals` as the neighbour: stable radix sort
    // of (key, neighbour) pairs + histogram / exclusive scan of the head counts.
    void csr(const int* keys, const int* vals, GraphCSR& g, hipStream_t s) {
        g.release();
        g.off = (int*)dmalloc(sizeof(int) * (N_ + 1));
        g.nbr = (int*)dmalloc(sizeof(int) * std::max(E_, 1));
        OPT_HIP_CHECK(hipMemsetAsync(g.off, 0, sizeof(int) * (N_ + 1), s));
        if (E_ == 0) return;
        int bits = 1;
        while ((1LL << bits) < N_) ++bits;
        size_t need = 0, need2 = 0;
        OPT_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, keys, keys_tmp_, vals, g.nbr, E_, 0, bits, s));
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need2, g.off, g.off, N_ + 1, s));
        need = std::max(need, need2);
        if (need > scratch_bytes_) {
            dfree(scratch_);
            scratch_ = dmalloc(need);
            scratch_bytes_ = need;
        }
        OPT_HIP_CHECK(
            hipcub::DeviceRadixSort::SortPairs(scratch_, need, keys, keys_tmp_, vals, g.nbr, E_, 0, bits, s));
        hipLaunchKernelGGL(arap::count_heads, dim3(std::min((E_ + 255) / 256, 4096)), dim3(256), 0, s, keys, E_,
                           g.off);
        size_t n2 = scratch_bytes_;
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scratch_, n2, g.off, g.off, N_ + 1, s));
    }
    // sliced ELL of g's lists, slot counts padded to multiples of `pad`
    void ell(GraphCSR& g, int pad, hipStream_t s) {
        const int ns = (N_ + 63) / 64;
        g.ew = (int*)dmalloc(sizeof(int) * (ns + 1));
        g.eoff = (int*)dmalloc(sizeof(int) * (ns + 1));
        OPT_HIP_CHECK(hipMemsetAsync(g.ew, 0, sizeof(int) * (ns + 1), s));
        hipLaunchKernelGGL(arap::ell_width, dim3((ns + 3) / 4), dim3(256), 0, s, g.off, N_, ns, pad, g.ew);
        // eoff = 64 x exclusive scan of ew: scan the widths, then scale on the host copy
        size_t need = 0;
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, g.ew, g.eoff, ns + 1, s));
        if (need > scratch_bytes_) {
            dfree(scratch_);
            scratch_ = dmalloc(need);
            scratch_bytes_ = need;
        }
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scratch_, need, g.ew, g.eoff, ns + 1, s));
        std::vector<int> h(ns + 1);
        OPT_HIP_CHECK(hipMemcpyAsync(h.data(), g.eoff, sizeof(int) * (ns + 1), hipMemcpyDeviceToHost, s));
        OPT_HIP_CHECK(hipStreamSynchronize(s));
        const long long total = 64LL * h[ns];
        if (total >= (1LL << 31)) {
            throw PlanError("arap_mesh_deformation: adjacency too large (" + std::to_string(total) +
                            " ELL slots, the limit is 2^31)");
        }
        for (auto& x : h) x *= 64;
        OPT_HIP_CHECK(hipMemcpyAsync(g.eoff, h.data(), sizeof(int) * (ns + 1), hipMemcpyHostToDevice, s));
        g.ell = (int*)dmalloc(sizeof(int) * std::max(total, 1LL));
        hipLaunchKernelGGL(arap::ell_fill, dim3((64LL * ns + 255) / 256), dim3(256), 0, s, g.off, g.nbr, N_, g.eoff,
                           g.ew, g.ell);
        OPT_HIP_CHECK(hipGetLastError());
        OPT_HIP_CHECK(hipStreamSynchronize(s));   // h is a host temporary
    }
    // the merged neighbour list (arap::Args nb_*) from the two CSRs, as sliced ELL
    void merged_ell(hipStream_t s) {
        nb_.release();
        const int ns = (N_ + 63) / 64;
        nb_.ew = (int*)dmalloc(sizeof(int) * (ns + 1));
        nb_.eoff = (int*)dmalloc(sizeof(int) * (ns + 1));
        OPT_HIP_CHECK(hipMemsetAsync(nb_.ew, 0, sizeof(int) * (ns + 1), s));
        hipLaunchKernelGGL(arap::merged_width, dim3((ns + 3) / 4), dim3(256), 0, s, (const int*)out_.off,
                           (const int*)out_.nbr, (const int*)in_.off, (const int*)in_.nbr, N_, ns, eb_, nb_.ew);
        size_t need = 0;
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need, nb_.ew, nb_.eoff, ns + 1, s));
        if (need > scratch_bytes_) {
            dfree(scratch_);
            scratch_ = dmalloc(need);
            scratch_bytes_ = need;
        }
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scratch_, need, nb_.ew, nb_.eoff, ns + 1, s));
        std::vector<int> h(ns + 1);
        OPT_HIP_CHECK(hipMemcpyAsync(h.data(), nb_.eoff, sizeof(int) * (ns + 1), hipMemcpyDeviceToHost, s));
        OPT_HIP_CHECK(hipStreamSynchronize(s));
        const long long total = 64LL * h[ns];
        if (total >= (1LL << 31)) {
            throw PlanError("arap_mesh_deformation: adjacency too large (" + std::to_string(total) +
                            " merged slots, the limit is 2^31)");
        }
        for (auto& x : h) x *= 64;
        OPT_HIP_CHECK(hipMemcpyAsync(nb_.eoff, h.data(), sizeof(int) * (ns + 1), hipMemcpyHostToDevice, s));
        nb_.ell = (int*)dmalloc(sizeof(int) * std::max(total, 1LL));
        hipLaunchKernelGGL(arap::merged_fill, dim3((64LL * ns + 255) / 256), dim3(256), 0, s, (const int*)out_.off,
                           (const int*)out_.nbr, (const int*)in_.off, (const int*)in_.nbr, N_, (const int*)nb_.eoff,
                           (const int*)nb_.ew, nb_.ell);
        OPT_HIP_CHECK(hipGetLastError());
        OPT_HIP_CHECK(hipStreamSynchronize(s));   // h is a host temporary
    }
    void build_csr(const int* v0, const int* v1, hipStream_t s) {
        if (E_ > 0) {
            int* bad = (int*)dmalloc(sizeof(int));
            OPT_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int), s));
            hipLaunchKernelGGL(arap::check_indices, dim3(std::min((E_ + 255) / 256, 4096)), dim3(256), 0, s, v0, v1,
                               E_, N_, bad);
            int hbad = 0;
            OPT_HIP_CHECK(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, s));
            OPT_HIP_CHECK(hipStreamSynchronize(s));
            dfree(bad);
            if (hbad) {
                fprintf(stderr, "[opt_amd] arap_mesh_deformation: graph vertex index outside [0, %d)\n", N_);
                exit(1);   // fail-stop, as the reference does on invalid input (backend_cuda.t:26-40)
            }
            dfree(keys_tmp_);
            keys_tmp_ = (int*)dmalloc(sizeof(int) * E_);
        }
        csr(v0, v1, out_, s);
        csr(v1, v0, in_, s);
        ell(out_, arap::kEBO, s);
        ell(in_, arap::kEBI, s);
        merged_ell(s);
        graph_v0_ = v0;
        graph_v1_ = v1;
    }

    StateOptions opts_;
    int N_ = 0, E_ = 0;
    int idx_O_, idx_A_, idx_U_, idx_C_, idx_v0_, idx_v1_, idx_wf_, idx_wr_;
    arap::Args<T> a_{};
    GraphCSR out_, in_, nb_;   // nb_: the merged list (ell / eoff / ew only)
    const int* graph_v0_ = nullptr;
    const int* graph_v1_ = nullptr;
    unsigned long long fingerprint_ = 0;
    unsigned long long* fp_scratch_ = (unsigned long long*)dmalloc(sizeof(unsigned long long) * (1 + kFingerprintGrid));
    void* scratch_ = nullptr;
    size_t scratch_bytes_ = 0;
    int* keys_tmp_ = nullptr;
    T* K_ = nullptr;   // per-vertex directional rotation derivative of the current p
    const bool merged_on_ = env_int("OPT_AMD_ARAP_MERGED", 1) != 0;   // 0: separate out / in lists
    // merged slots per batch of arap_apply_merged (the merged ELL widths are padded to it)
    const int eb_ = env_int("OPT_AMD_ARAP_EB", arap::kEBM) == 3 ? 3 : 2;
    T *userO_ = nullptr, *userA_ = nullptr, *dO_ = nullptr, *dA_ = nullptr;
    float *dU_ = nullptr, *dC_ = nullptr;
    int *dv0_ = nullptr, *dv1_ = nullptr;
};

std::unique_ptr<Plan> make_arap_plan(const ProblemSpec& spec, const StateOptions& opts, const unsigned* dims,
                                     std::string* err) {
    if (spec.graphs.size() != 1 || spec.graphs[0].vertices.size() != 2 || spec.graphs[0].dims.empty()) {
        *err = "arap_mesh_deformation: expects one graph with two vertex slots";
        return nullptr;
    }
    unsigned N = 0, E = 0;
    for (auto& d : spec.dims) {
        if (d.name == spec.unknown(0)->dims[0]) N = dims[d.index];
        if (d.name == spec.graphs[0].dims[0]) E = dims[d.index];
    }
    if (N == 0) { *err = "arap_mesh_deformation: zero vertices"; return nullptr; }
    // 3 N sizeof(T) bytes (arap::gld3 of p / delta; UrShape and Constraints are float) and
    // 9 N sizeof(T) bytes (arap::gldq, the K planes) must fit the gathers' 32-bit offsets:
    // at most ~119 M vertices in fp32, ~59.6 M in fp64
    const unsigned long long kbytes = 9ULL * N * (opts.double_precision ? sizeof(double) : sizeof(float));
    if (kbytes >= (1ULL << 32) || E > (1u << 30)) { *err = "arap_mesh_deformation: graph too large"; return nullptr; }
    Domain dom{(int)N, 1, 0, 1, 0, 1};
    dom.edges = (int)E;
    if (opts.double_precision) return make_stencil_plan<ArapOp<double>>(spec, opts, dom, err);
    return make_stencil_plan<ArapOp<float>>(spec, opts, dom, err);
}

}  // namespace optamd
