// stencil_driver.h — the GN / LM + PCG solver for image-domain energies whose kernels
// are supplied by a family operator (`Op`). This is the reference's solver skeleton
// (API/src/solverGPUGaussNewton.t: init :1766-1897, step :1913-2349) with its kernels
// PCGInit1 / PCGFinalizeDiagonal / PCGStep2 / PCGStep3 / the residual-reset halves /
// PCGLinearUpdate / savePreviousUnknowns / revertUpdate as flat HBM streams over the
// unknown vector, and the family's stencil kernels (J^T F + diag, J^T J p, cost,
// model cost) from Op. The LM q/zeta early exit is decided on the device: the PCG
// iterations are all enqueued, and once zeta < q_tolerance every later kernel of the
// step returns at entry (the reference blocks on a D2H copy of q each iteration,
// :2211-2220).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#include "pcg_kernels.h"
#include "plan.h"

namespace optamd {

struct LMScalars {      // trust-region parameters the diagonal kernels need
    float radius, min_diag, max_diag;
};

__device__ __forceinline__ bool stopped(const int* stop) { return stop && *stop; }

template <typename T>
__device__ __forceinline__ T guarded_invert(T d) {   // CERES form, :480-487
    const T s = (T)1 + sqrt(d);
    return (T)1 / (s * s);
}

// PCGInit1's preconditioner and direction (after the family's evalJTF):
// pre = guardedInvert(diag) (guardedInvert(1) = 1/4 for UsePreconditioner(false)),
// p = pre r, rz[0] = sum r.p. Excluded unknowns get pre = p = 0; so do the halo rows of
// a decomposed slab (pixels outside [pix_lo, pix_hi)), whose r is zeroed too.
// The per-element init / update kernels find each element's pixel flag first (a load that
// the element's own loads wait on); each thread keeps kIlp elements of its grid-stride
// sequence in flight (their loads issued together, then the arithmetic in element order),
// as one element per iteration left too few loads outstanding to stream at HBM speed.
constexpr int kIlp = 4;

template <typename T>
__global__ __launch_bounds__(kBlock) void gn_init_kernel(VecLayout L, const uint8_t* __restrict__ flags,
                                                         T* __restrict__ r, const T* __restrict__ diag,
                                                         T* __restrict__ pre, T* __restrict__ p, int use_pre,
                                                         long long pix_lo, long long pix_hi, ReduceSlot rs) {
    const long long n = L.off[L.nimg];
    const long long stride = (long long)gridDim.x * blockDim.x;
    T acc = 0;
    for (long long e0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; e0 < n; e0 += kIlp * stride) {
        bool in[kIlp], own[kIlp];
        uint8_t f[kIlp];
        T dv[kIlp], rv[kIlp];
#pragma unroll
        for (int u = 0; u < kIlp; ++u) {
            const long long e = e0 + u * stride;
            in[u] = e < n;
            const long long px = in[u] ? L.pix(e) : 0;
            own[u] = in[u] && px >= pix_lo && px < pix_hi;
            f[u] = flags[px];
            rv[u] = r[in[u] ? e : 0];
            dv[u] = use_pre ? diag[in[u] ? e : 0] : (T)1;
        }
#pragma unroll
        for (int u = 0; u < kIlp; ++u) {
            if (!in[u]) continue;
            const long long e = e0 + u * stride;
            const bool act = own[u] && (f[u] & 1);
            const T w = act ? guarded_invert(use_pre ? dv[u] : (T)1) : (T)0;
            const T re = own[u] ? rv[u] : (T)0;
            const T pp = w * re;
            if (!own[u]) r[e] = 0;
            pre[e] = w;
            p[e] = pp;
            acc += re * pp;
        }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// LM: PCGSaveSSq (first step), PCGComputeCtC (diag / radius, o.t:2996-3030) and
// PCGFinalizeDiagonal (:1061-1103): CtC = clamp(diag/radius, min_lm/(SSq radius),
// max_lm/(SSq radius)); pre = 1/(CtC + radius diag/radius); b = r; p = pre r;
// rz[0] = sum r.p (q = 0 since delta = 0).
template <typename T, bool FIRST>
__global__ __launch_bounds__(kBlock) void lm_init_kernel(VecLayout L, const uint8_t* __restrict__ flags,
                                                         T* __restrict__ r, const T* __restrict__ diag,
                                                         T* __restrict__ SSq, T* __restrict__ CtC,
                                                         T* __restrict__ pre, T* __restrict__ b, T* __restrict__ p,
                                                         int use_pre, LMScalars lm, long long pix_lo,
                                                         long long pix_hi, ReduceSlot rs) {
    const long long n = L.off[L.nimg];
    const long long stride = (long long)gridDim.x * blockDim.x;
    const T radius = (T)lm.radius;
    const T inv_radius = (T)1 / radius;
    T acc = 0;
    for (long long e0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; e0 < n; e0 += kIlp * stride) {
        bool in[kIlp], own[kIlp];
        uint8_t f[kIlp];
        T dv[kIlp], rv[kIlp], sv[kIlp];
#pragma unroll
        for (int u = 0; u < kIlp; ++u) {
            const long long e = e0 + u * stride;
            in[u] = e < n;
            const long long ec = in[u] ? e : 0;
            const long long px = in[u] ? L.pix(e) : 0;
            own[u] = in[u] && px >= pix_lo && px < pix_hi;
            f[u] = flags[px];
            rv[u] = r[ec];
            dv[u] = diag[ec];
            if (!FIRST) sv[u] = SSq[ec];
        }
#pragma unroll
        for (int u = 0; u < kIlp; ++u) {
            if (!in[u]) continue;
            const long long e = e0 + u * stride;
            if (!own[u] || !(f[u] & 1)) {
                if (FIRST) SSq[e] = 0;
                CtC[e] = 0; pre[e] = 0; b[e] = 0; p[e] = 0;
                if (!own[u]) r[e] = 0;
                continue;
            }
            T ssq;
            if (FIRST) { ssq = guarded_invert(use_pre ? dv[u] : (T)1); SSq[e] = ssq; }
            else ssq = sv[u];
            const T unclamped = dv[u] * inv_radius;
            const T clampm = ((T)1 / ssq) / radius;
            const T lo = (T)lm.min_diag * clampm, hi = (T)lm.max_diag * clampm;
            const T c = std::min(std::max(unclamped, lo), hi);
            const T w = (T)1 / (c + radius * unclamped);
            const T re = rv[u];
            CtC[e] = c;
            pre[e] = w;
            b[e] = re;
            p[e] = w * re;
            acc += re * (w * re);
        }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// LM inner-loop exit test (:2211-2220) folded into the kernel that reduces q (one GPU:
// the local q is the global one): zeta = (lIter+1) (Q1 - Q0) / Q1 in opt_float
// arithmetic; stop if zeta < q_tolerance, else Q0 = Q1. on = 0: the driver launches
// zeta_kernel after the all-reduce instead (row slabs).
struct ZetaArgs {
    double* q0;
    int* stop;
    int liter;
    float q_tol;
    int on;
};
template <typename T>
__device__ __forceinline__ void zeta_test(const ZetaArgs& z, double q1) {
    const T Q1 = (T)q1, Q0 = (T)*z.q0;
    const T zeta = (T)(z.liter + 1) * (Q1 - Q0) / Q1;
    if (zeta < (T)z.q_tol) *z.stop = 1;
    else *z.q0 = (double)Q1;
}

// PCGStep2 (:665-731): alpha = sc[i_num]/sc[i_den]; delta (+)= alpha p; r -= alpha Ap;
// z = pre r (r when UsePreconditioner(false)); out[0] = sum z.r; LM: out[1] = q =
// sum 1/2 delta.(r + b).
// (16-byte vector accesses per thread were measured: shape_from_shading LM 3.46 -> 3.41 ms,
// optical_flow fp64 LM 5.02 -> 5.05, generated image_warping GN 7.98 -> 8.27 — kept scalar.)
// DELTA false (GN): the delta update is left to step3_kernel, which reads p_old anyway.
template <typename T, bool FIRST, bool LM, bool DELTA = true>
__global__ __launch_bounds__(kBlock) void step2_kernel(long long n, const T* __restrict__ p,
                                                       const T* __restrict__ Ap, const T* __restrict__ pre,
                                                       const T* __restrict__ b, T* __restrict__ r,
                                                       T* __restrict__ delta, const double* __restrict__ sc,
                                                       int i_num, int i_den, int use_pre, const int* stop,
                                                       ReduceSlot rs, ZetaArgs z = {}) {
    if (stopped(stop)) return;
    const T alpha = (T)(sc[i_num] / sc[i_den]);
    T acc = 0, accq = 0;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        const T rr = r[e] - alpha * Ap[e];
        T d = 0;
        if (DELTA) {
            d = FIRST ? alpha * p[e] : delta[e] + alpha * p[e];
            delta[e] = d;
        }
        r[e] = rr;
        const T z = use_pre ? pre[e] * rr : rr;
        acc += z * rr;
        if (LM) accq += (T)0.5 * (d * (rr + b[e]));
    }
    double v[2] = {(double)acc, (double)accq};
    if (LM) {
        double tot[2];
        if (block_reduce_publish<2>(v, rs, blockIdx.x, tot) && z.on) zeta_test<T>(z, tot[1]);
    } else {
        double v1[1] = {v[0]};
        block_reduce_publish<1>(v1, rs, blockIdx.x);
    }
}

// PCGStep3 (:814-845): beta = sc[i_num]/sc[i_den]; p = z + beta p.
// DM (GN, PCGStep2's delta update moved here, where p_old is read anyway; same
// expression): 1 delta = alpha p_old, 2 delta += alpha p_old, alpha = sc[ia_num]/sc[ia_den].
// GUARD (the fused loop's residual-reset iterations): beta = 0 unless both rz
// are positive, as step23_kernel — bitwise the plain division wherever that is finite and
// positive; the classic loop keeps the reference's unguarded division (:842).
template <typename T, int DM = 0, bool GUARD = false>
__global__ __launch_bounds__(kBlock) void step3_kernel(long long n, const T* __restrict__ pre,
                                                       const T* __restrict__ r, T* __restrict__ p,
                                                       const double* __restrict__ sc, int i_num, int i_den,
                                                       int use_pre, const int* stop, T* __restrict__ delta = nullptr,
                                                       int ia_num = 0, int ia_den = 0) {
    if (stopped(stop)) return;
    const T beta = (!GUARD || (sc[i_num] > 0.0 && sc[i_den] > 0.0)) ? (T)(sc[i_num] / sc[i_den]) : (T)0;
    const T alpha = DM ? (T)(sc[ia_num] / sc[ia_den]) : (T)0;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        const T z = use_pre ? pre[e] * r[e] : r[e];
        const T po = p[e];
        if (DM == 1) delta[e] = alpha * po;
        if (DM == 2) delta[e] = delta[e] + alpha * po;
        p[e] = z + beta * po;
    }
}

// PCGStep2 + PCGStep3 of iteration i in ONE pass: the family's apply also reduced
// p.Ap_i, r_i.W Ap_i, Ap_i.W Ap_i and r_i.W r_i in fp64 (Op::apply_sums), so PCGStep3's
// beta numerator comes from the exact identity
//   r_{i+1}.W r_{i+1} = r_i.W r_i - 2 alpha r_i.W Ap_i + alpha^2 Ap_i.W Ap_i
// (alpha = rz_i / pAp_i as the elements apply it, W = pre with UsePreconditioner, else 1:
// PCGStep2's weighting, :705-708), and p_{i+1} = z_{i+1} + beta p_i is formed in the same
// pass as r_{i+1}, z_{i+1} and delta += alpha p_i (PCGStep2's expressions; GN's delta too).
// The denominator is rz_i as the classic step has it (PCGInit1's r.(pre r) at i = 0). The
// direct rz_{i+1} (fp64 products w r r) is still reduced, for alpha_{i+1}, with LM's q
// beside it (and the device-side zeta test on one GPU); the identity's value goes to
// sc[id_out] for the tests. Slots: i_rz = rz_i, i_rz + 2 .. + 5 = the apply's four sums.
template <typename T, bool FIRST, bool LM>
__global__ __launch_bounds__(kBlock) void step23_kernel(long long n, T* __restrict__ p, const T* __restrict__ Ap,
                                                        const T* __restrict__ pre, const T* __restrict__ b,
                                                        T* __restrict__ r, T* __restrict__ delta,
                                                        double* __restrict__ sc, int i_rz, int id_out, int use_pre,
                                                        const int* stop, ReduceSlot rs, ZetaArgs z = {}) {
    if (stopped(stop)) return;
    const double rz = sc[i_rz];
    // a zero step where p.Ap is not positive (far past convergence, once p and Ap
    // underflow; the reference's unguarded division gives NaN there: iw_apply_res)
    const T alpha = sc[i_rz + 2] > 0.0 ? (T)(rz / sc[i_rz + 2]) : (T)0;
    const double ad = (double)alpha;
    const double rz_id = sc[i_rz + 5] - 2.0 * ad * sc[i_rz + 3] + ad * ad * sc[i_rz + 4];
    // non-positive only where the true beta is below the identity's ~1e-14 absolute error
    // (iw_apply_res): beta = 0 there
    const T beta = rz_id > 0.0 && rz > 0.0 ? (T)(rz_id / rz) : (T)0;
    if (blockIdx.x == 0 && threadIdx.x == 0) sc[id_out] = rz_id;
    double acc = 0;
    T accq = 0;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        const T po = p[e];
        const T rr = r[e] - alpha * Ap[e];
        const T d = FIRST ? alpha * po : delta[e] + alpha * po;
        delta[e] = d;
        r[e] = rr;
        const T w = use_pre ? pre[e] : (T)1;
        const T zz = use_pre ? w * rr : rr;
        acc += (double)w * (double)rr * (double)rr;
        if (LM) accq += (T)0.5 * (d * (rr + b[e]));
        p[e] = zz + beta * po;
    }
    double v[2] = {acc, (double)accq};
    double tot[2];
    if (block_reduce_publish<2>(v, rs, blockIdx.x, tot) && LM && z.on) zeta_test<T>(z, tot[1]);
}

// Residual reset, LM only (:738-801): first half delta += alpha p ...
// GUARD: alpha = 0 unless p.Ap is positive (step23_kernel's zero step far past convergence)
template <typename T, bool GUARD = false>
__global__ __launch_bounds__(kBlock) void half1_kernel(long long n, const T* __restrict__ p,
                                                       T* __restrict__ delta, const double* __restrict__ sc,
                                                       int i_num, int i_den, const int* stop) {
    if (stopped(stop)) return;
    const T alpha = (!GUARD || sc[i_den] > 0.0) ? (T)(sc[i_num] / sc[i_den]) : (T)0;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x)
        delta[e] = delta[e] + alpha * p[e];
}
// ... second half, after Adelta = (J^T J + CtC) delta: r = b - Adelta, rz, q.
template <typename T>
__global__ __launch_bounds__(kBlock) void half2_kernel(long long n, const T* __restrict__ Adelta,
                                                       const T* __restrict__ b, const T* __restrict__ pre,
                                                       const T* __restrict__ delta, T* __restrict__ r,
                                                       int use_pre, const int* stop, ReduceSlot rs,
                                                       ZetaArgs z = {}) {
    if (stopped(stop)) return;
    T acc = 0, accq = 0;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        const T rr = b[e] - Adelta[e];
        r[e] = rr;
        const T z = use_pre ? pre[e] * rr : rr;
        acc += z * rr;
        accq += (T)0.5 * (delta[e] * (rr + b[e]));
    }
    double v[2] = {(double)acc, (double)accq};
    double tot[2];
    if (block_reduce_publish<2>(v, rs, blockIdx.x, tot) && z.on) zeta_test<T>(z, tot[1]);
}

// LM inner-loop exit test (:2211-2220), in opt_float arithmetic:
// zeta = (lIter+1) (Q1 - Q0) / Q1; stop if zeta < q_tolerance, else Q0 = Q1.
template <typename T>
__global__ void zeta_kernel(const double* __restrict__ sc, int i_q1, double* __restrict__ q0, int liter,
                            float q_tol, int* stop) {
    if (*stop) return;
    const T Q1 = (T)sc[i_q1], Q0 = (T)*q0;
    const T zeta = (T)(liter + 1) * (Q1 - Q0) / Q1;
    if (zeta < (T)q_tol) *stop = 1;
    else *q0 = (double)Q1;
}

}  // namespace optamd
