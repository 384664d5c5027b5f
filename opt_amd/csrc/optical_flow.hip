// optical_flow.hip — kernels for the optical_flow energy
// (reference examples/optical_flow/optical_flow.t):
//
//   unknown X (2 per pixel: the flow), knowns I, I_hat, I_hat_dx, I_hat_dy (float)
//   UsePreconditioner(false); no Exclude
//   e_fit(k)   = wf (I_k - S(I_hat; i + X0, j + X1))
//   e_reg(k,s) = InBounds(k+s) ? wr (X_k - X_{k+s}) : 0,   s in 4-neighbours
//
// S is Image:sample (o.t:863-876): floor / ceil taps, lerp (1-t) v0 + t v1, zero
// outside the image. The fit term's Jacobian is -wf (S(I_hat_dx), S(I_hat_dy)) at the
// same point (SampledImage partials, o.t:3270-3280).
//
// MI355X layout of the work: the data-dependent bilinear gathers (12 taps over three
// images) happen once per GN/LM step, in of_jtf, which caches the sampled gradient
// G_k = (S(I_hat_dx), S(I_hat_dy)) in unknown precision. Within PCG the fit block is
// the rank-1 2x2 wf^2 G G^T, so the J^T J p apply is a pure 5-point stencil stream
// over p plus one G read — no gathers and no X / I_hat traffic in the hot loop
// (the reference re-samples I_hat_dx / I_hat_dy in every apply).
// One thread per pixel, 64 x 4 pixel blocks, 2-wide vector accesses.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include "plan.h"
#include "stencil_plan.h"

namespace optamd {
namespace of {

template <typename T> struct alignas(2 * sizeof(T)) V2 { T x, y; };

template <typename T>
struct Args {
    Domain dom;
    T* X;              // flow, 2 per pixel
    const float* I;
    const float* Ih;   // I_hat
    const float* Ihx;  // I_hat_dx
    const float* Ihy;  // I_hat_dy
    T* G;              // cached sampled gradient (2 per pixel)
    T* Ef;             // cached fit residual wf (I - S(I_hat)) at the step's X (the model cost)
    uint8_t* flags;
    T wf, wr;
};

__device__ __forceinline__ PixGeom pix(const Domain& d) {
    PixGeom g;
    g.x = blockIdx.x * 64 + (threadIdx.x & 63);
    g.y = d.y_lo + blockIdx.y * 4 + (threadIdx.x >> 6);
    g.ok = g.x < d.W && g.y < d.y_hi;
    g.i = g.ok ? d.off(g.x, g.y) : 0;
    return g;
}
__device__ __forceinline__ bool inside(const Domain& d, int x, int y) {
    return x >= 0 && x < d.W && y >= 0 && y < d.H;
}
template <typename T>
__device__ __forceinline__ V2<T> ld2(const T* a, long long i) {
    return reinterpret_cast<const V2<T>*>(a)[i];
}
template <typename T>
__device__ __forceinline__ void st2(T* a, long long i, T x, T y) {
    reinterpret_cast<V2<T>*>(a)[i] = V2<T>{x, y};
}

// Image:get + Image:sample in opt_float arithmetic
template <typename T>
__device__ __forceinline__ T tap(const float* im, const Domain& d, int x, int y) {
    return (x >= 0 && x < d.W && y >= 0 && y < d.H) ? (T)im[(long long)y * d.W + x] : (T)0;
}
template <typename T>
__device__ __forceinline__ T lerp(T v0, T v1, T t) { return ((T)1 - t) * v0 + t * v1; }

struct Taps { int x0, x1, y0, y1; };
template <typename T>
__device__ __forceinline__ Taps taps_of(T x, T y, T& xn, T& yn) {
    Taps t;
    t.x0 = (int)floor(x); t.x1 = (int)ceil(x);
    t.y0 = (int)floor(y); t.y1 = (int)ceil(y);
    xn = x - (T)t.x0;
    yn = y - (T)t.y0;
    return t;
}
template <typename T>
__device__ __forceinline__ T sample(const float* im, const Domain& d, const Taps& t, T xn, T yn) {
    const T u = lerp(tap<T>(im, d, t.x0, t.y0), tap<T>(im, d, t.x1, t.y0), xn);
    const T b = lerp(tap<T>(im, d, t.x0, t.y1), tap<T>(im, d, t.x1, t.y1), xn);
    return lerp(u, b, yn);
}

constexpr int DX[4] = {1, -1, 0, 0};
constexpr int DY[4] = {0, 0, 1, -1};

// r = -J^T F, diag = sum (dr/dx)^2 (evalJTF, o.t:2870-2913), flags (all active), and
// the cached gradient G for the applies of this step.
template <typename T>
__global__ __launch_bounds__(kBlock) void of_jtf(Args<T> a, T* __restrict__ r, T* __restrict__ diag) {
    const PixGeom g = pix(a.dom);
    if (!g.ok) return;
    const V2<T> xk = ld2(a.X, g.i);
    T xn, yn;
    const Taps t = taps_of((T)g.x + xk.x, (T)g.y + xk.y, xn, yn);
    const T s = sample<T>(a.Ih, a.dom, t, xn, yn);
    const T gx = sample<T>(a.Ihx, a.dom, t, xn, yn);
    const T gy = sample<T>(a.Ihy, a.dom, t, xn, yn);
    const T ef = a.wf * ((T)a.I[g.i] - s);
    const T wr = a.wr;
    const T dfx = -a.wf * gx, dfy = -a.wf * gy;
    T Fx = dfx * ef, Fy = dfy * ef, Dx = dfx * dfx, Dy = dfy * dfy;
    for (int d = 0; d < 4; ++d) {
        const int tx = g.x + DX[d], ty = g.y + DY[d];
        if (inside(a.dom, tx, ty)) {   // instance centred at k
            const V2<T> xt = ld2(a.X, a.dom.off(tx, ty));
            Fx += wr * (wr * (xk.x - xt.x));
            Fy += wr * (wr * (xk.y - xt.y));
            Dx += wr * wr; Dy += wr * wr;
        }
        const int jx = g.x - DX[d], jy = g.y - DY[d];
        if (inside(a.dom, jx, jy)) {   // instance centred at k - s (k is its neighbour)
            const V2<T> xj = ld2(a.X, a.dom.off(jx, jy));
            Fx += -wr * (wr * (xj.x - xk.x));
            Fy += -wr * (wr * (xj.y - xk.y));
            Dx += (-wr) * (-wr); Dy += (-wr) * (-wr);
        }
    }
    st2(r, g.i, -Fx, -Fy);
    st2(diag, g.i, Dx, Dy);
    st2(a.G, g.i, gx, gy);
    a.Ef[g.i] = ef;
    a.flags[g.i] = 1;
}

// Ap = J^T J p (+ dadd p for LM), sum p.Ap; returns at entry once *stop is set.
// J^T J p = wf^2 G (G.p) + 2 wr^2 sum_{in-bounds t} (p_k - p_t), evaluated in the
// reference's gather order (fit, then per direction: own instance, neighbour's).
// Persistent: a capped grid walks 64 x 4 pixel tiles (common.h tile_range / tile_pix).

template <typename T>
__global__ __launch_bounds__(kBlock) void of_apply(Args<T> a, const T* __restrict__ p, T* __restrict__ Ap,
                                                   const T* __restrict__ dadd, const int* stop, ReduceSlot rs) {
    if (stop && *stop) return;
    const TileRange tr = tile_range(pix_tiles(a.dom));
    T dot = 0;
    for (int tile = tr.first; tile < tr.end; tile += tr.step) {
    const PixGeom g = tile_pix(a.dom, tile);
    if (g.ok) {
        const V2<T> pk = ld2(p, g.i);
        const V2<T> gk = ld2((const T*)a.G, g.i);
        const T wr = a.wr;
        const T jx = -a.wf * gk.x, jy = -a.wf * gk.y;
        const T jp = jx * pk.x + jy * pk.y;
        T ax = jx * jp, ay = jy * jp;
        for (int d = 0; d < 4; ++d) {
            const int tx = g.x + DX[d], ty = g.y + DY[d];
            if (inside(a.dom, tx, ty)) {
                const V2<T> pt = ld2(p, a.dom.off(tx, ty));
                ax += wr * (wr * (pk.x - pt.x));
                ay += wr * (wr * (pk.y - pt.y));
            }
            const int qx = g.x - DX[d], qy = g.y - DY[d];
            if (inside(a.dom, qx, qy)) {
                const V2<T> pj = ld2(p, a.dom.off(qx, qy));
                ax += -wr * (wr * (pj.x - pk.x));
                ay += -wr * (wr * (pj.y - pk.y));
            }
        }
        if (dadd) {
            const V2<T> c = ld2(dadd, g.i);
            ax += c.x * pk.x;
            ay += c.y * pk.y;
        }
        st2(Ap, g.i, ax, ay);
        dot += pk.x * ax + pk.y * ay;
    }
    }
    double v[1] = {(double)dot};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// The same apply as a register strip (round 6): a wave owns 62 output columns
// (x = 62 strip - 1 + lane, outputs at lanes 1..62) and walks `rows` rows keeping p of rows
// y-1, y, y+1 in registers (row y+2, G and dadd of row y+1 in flight), the horizontal
// neighbours are DPP lane shifts; a block's four waves are side by side over four adjacent
// strips (as iw_pcg). Each p element is loaded once per wave instead of five times per
// pixel by the flat kernel's gathers. Same terms in the same order per pixel (fit, then per
// direction the own instance and the neighbour's, then dadd); p.Ap sums in lane / row order.
constexpr int kOfOut = 62;
template <typename T>
__device__ __forceinline__ V2<T> of_lane_left(V2<T> v) { return V2<T>{from_left0(v.x), from_left0(v.y)}; }
template <typename T>
__device__ __forceinline__ V2<T> of_lane_right(V2<T> v) { return V2<T>{from_right0(v.x), from_right0(v.y)}; }
template <typename T>
__global__ __launch_bounds__(kBlock) void of_apply_strip(Args<T> a, const T* __restrict__ p, T* __restrict__ Ap,
                                                         const T* __restrict__ dadd, const int* stop, ReduceSlot rs,
                                                         int nstrips, int rows) {
    if (stop && *stop) return;
    const Domain& d = a.dom;
    const int lane = threadIdx.x & (kWave - 1);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int ng = (nstrips + kBlock / kWave - 1) / (kBlock / kWave);
    const int strip = (lb % ng) * (kBlock / kWave) + w;
    const int y0 = d.y_lo + (lb / ng) * rows, y1 = strip < nstrips ? min(y0 + rows, d.y_hi) : y0;
    const int x = strip * kOfOut - 1 + lane;
    const bool xin = x >= 0 && x < d.W;
    const bool out = xin && lane >= 1 && lane <= kOfOut;
    T dot = 0;
    if (y0 < y1) {
        // masked loads without a branch: element 0 when outside, the value selected after
        auto ld = [&](const T* b, int y) -> V2<T> {
            const bool ok = xin && y >= 0 && y < d.H;
            const V2<T> v = ld2(b, ok ? d.off(x, y) : 0);
            return ok ? v : V2<T>{0, 0};
        };
        V2<T> pm = ld(p, y0 - 1), pc = ld(p, y0), pn = ld(p, y0 + 1);
        V2<T> gc = ld((const T*)a.G, y0), cc = dadd ? ld(dadd, y0) : V2<T>{0, 0};
        const T wr = a.wr;
        for (int y = y0; y < y1; ++y) {
            const V2<T> pnn = ld(p, y + 2), gn = ld((const T*)a.G, y + 1);
            const V2<T> cn = dadd ? ld(dadd, y + 1) : V2<T>{0, 0};
            const V2<T> pk = pc;
            const V2<T> pr = of_lane_right(pc), pl = of_lane_left(pc);
            const T jx = -a.wf * gc.x, jy = -a.wf * gc.y;
            const T jp = jx * pk.x + jy * pk.y;
            T ax = jx * jp, ay = jy * jp;
            const bool in_r = x + 1 < d.W, in_l = x - 1 >= 0, in_d = y + 1 < d.H, in_u = y - 1 >= 0;
            // DX / DY order: (+1, 0), (-1, 0), (0, +1), (0, -1); per direction the instance
            // centred here (t = k + s), then the neighbour's (q = k - s)
            const V2<T> nt[4] = {pr, pl, pn, pm}, nq[4] = {pl, pr, pm, pn};
            const bool it[4] = {in_r, in_l, in_d, in_u}, iq[4] = {in_l, in_r, in_u, in_d};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (it[k]) {
                    ax += wr * (wr * (pk.x - nt[k].x));
                    ay += wr * (wr * (pk.y - nt[k].y));
                }
                if (iq[k]) {
                    ax += -wr * (wr * (nq[k].x - pk.x));
                    ay += -wr * (wr * (nq[k].y - pk.y));
                }
            }
            if (dadd) {
                ax += cc.x * pk.x;
                ay += cc.y * pk.y;
            }
            if (out) {
                st2(Ap, d.off(x, y), ax, ay);
                dot += pk.x * ax + pk.y * ay;
            }
            pm = pc; pc = pn; pn = pnn; gc = gn; cc = cn;
        }
    }
    double v[1] = {(double)dot};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}

// cost 1/2 sum r^2 (delta == nullptr) or the LM model cost 1/2 sum (r + J delta)^2
// (o.t:3119-3129, 2915-2943)
template <typename T>
__global__ __launch_bounds__(kBlock) void of_cost(Args<T> a, const T* __restrict__ delta, ReduceSlot rs) {
    const TileRange tr = tile_range(pix_tiles(a.dom));
    T acc = 0;
    for (int tile = tr.first; tile < tr.end; tile += tr.step) {
    const PixGeom g = tile_pix(a.dom, tile);
    if (g.ok) {
        const V2<T> xk = ld2((const T*)a.X, g.i);
        T ef;
        V2<T> dk = {0, 0};
        if (delta) {
            // the model cost is taken at the step's X, where of_jtf sampled the fit residual
            // and its gradient with these same expressions: no gathers
            dk = ld2(delta, g.i);
            const V2<T> gk = ld2((const T*)a.G, g.i);
            ef = a.Ef[g.i] + ((-a.wf * gk.x) * dk.x + (-a.wf * gk.y) * dk.y);
        } else {
            T xn, yn;
            const Taps t = taps_of((T)g.x + xk.x, (T)g.y + xk.y, xn, yn);
            ef = a.wf * ((T)a.I[g.i] - sample<T>(a.Ih, a.dom, t, xn, yn));
        }
        T s2 = ef * ef;
        for (int d = 0; d < 4; ++d) {
            const int tx = g.x + DX[d], ty = g.y + DY[d];
            if (!inside(a.dom, tx, ty)) continue;
            const long long j = a.dom.off(tx, ty);
            const V2<T> xt = ld2((const T*)a.X, j);
            T ex = a.wr * (xk.x - xt.x), ey = a.wr * (xk.y - xt.y);
            if (delta) {
                const V2<T> dt = ld2(delta, j);
                ex = ex + (a.wr * dk.x + (-a.wr) * dt.x);
                ey = ey + (a.wr * dk.y + (-a.wr) * dt.y);
            }
            s2 += ex * ex + ey * ey;
        }
        acc += (T)0.5 * s2;
    }
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.x);
}


// saveJToCRS / generateDumpJ (solverGPUGaussNewton.t:385-442, 1004-1022): pixel k owns
// rows 9k.. 9k+8 — the fit residual {X0(k): -wf G.x, X1(k): -wf G.y} (the SampledImage
// partials at the current flow, cached by of_jtf), then for s in (+x,-x,+y,-y) and each
// channel {X_c(k): b wr, X_c(k+s): -b wr}, b = InBounds(k+s) — 18 nonzeros at 18 k,
// columns wrapped (wrap(), :365-381) and sorted.
template <typename T>
__global__ __launch_bounds__(kBlock) void of_dump_j(Args<T> a, int* __restrict__ rowPtr, int* __restrict__ colInd,
                                                    T* __restrict__ val) {
    const Domain& d = a.dom;
    const long long N = (long long)d.W * d.H, n = 2 * N;
    constexpr int SX[4] = {1, -1, 0, 0}, SY[4] = {0, 0, 1, -1};
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < N; k += (long long)gridDim.x * blockDim.x) {
        const int x = (int)(k % d.W), y = (int)(k / d.W);
        const V2<T> g = ld2(a.G, k);
        const long long rb = 9 * k, nb = 18 * k;
        rowPtr[rb] = (int)nb;
        colInd[nb] = (int)(2 * k); val[nb] = -a.wf * g.x;
        colInd[nb + 1] = (int)(2 * k + 1); val[nb + 1] = -a.wf * g.y;
        for (int s = 0; s < 4; ++s) {
            const bool in = inside(d, x + SX[s], y + SY[s]);
            const long long tn = k + SX[s] + (long long)SY[s] * d.W;
            for (int c = 0; c < 2; ++c) {
                const long long row = rb + 1 + 2 * s + c, nz = nb + 2 + 4 * s + 2 * c;
                rowPtr[row] = (int)nz;
                long long c0 = 2 * k + c, c1 = 2 * tn + c;
                c1 = c1 < 0 ? c1 + n : (c1 >= n ? c1 - n : c1);
                T v0 = in ? a.wr : (T)0, v1 = in ? -a.wr : (T)0;
                if (c1 < c0) {
                    const long long tc = c0; c0 = c1; c1 = tc;
                    const T tv = v0; v0 = v1; v1 = tv;
                }
                colInd[nz] = (int)c0; val[nz] = v0;
                colInd[nz + 1] = (int)c1; val[nz + 1] = v1;
            }
        }
        if (k == N - 1) rowPtr[9 * N] = (int)(18 * N);
    }
}

}  // namespace of

template <typename TT>
class OpticalFlowOp {
public:
    using T = TT;
    static constexpr const char* kName = "optical_flow";
    static constexpr const char* kApplyName = "of_apply";
    static constexpr bool kSlabs = false;   // sampled reads land anywhere in the image
    OpticalFlowOp(const ProblemSpec& spec, const StateOptions& opts, Domain dom) : dom_(dom), opts_(opts) {
        idx_X_ = spec.unknown(0)->index;
        idx_I_ = spec.array(0)->index;
        idx_Ih_ = spec.array(1)->index;
        idx_Ihx_ = spec.array(2)->index;
        idx_Ihy_ = spec.array(3)->index;
        std::vector<DeclParam> ps = spec.params;
        std::sort(ps.begin(), ps.end(), [](auto& x, auto& y) { return x.index < y.index; });
        idx_wf_ = ps[0].index;
        idx_wr_ = ps[1].index;
        const long long N = dom_.npix_mem();
        G_ = (T*)dmalloc(sizeof(T) * 2 * N);
        Ef_ = (T*)dmalloc(sizeof(T) * N);
        OPT_HIP_CHECK(hipMemset(G_, 0, sizeof(T) * 2 * N));
        if (opts.host_buffers) {
            dX_ = (T*)dmalloc(sizeof(T) * 2 * N);
            for (float** v : {&dI_, &dIh_, &dIhx_, &dIhy_}) *v = (float*)dmalloc(sizeof(float) * N);
        }
    }
    ~OpticalFlowOp() {
        dfree(G_);
        dfree(Ef_);
        dfree(dX_);
        for (float* v : {dI_, dIh_, dIhx_, dIhy_}) dfree(v);
    }
    VecLayout layout() const {
        VecLayout L{};
        L.nimg = 1;
        L.ch[0] = 2;
        L.off[0] = 0;
        L.off[1] = 2 * dom_.npix_mem();
        L.N = dom_.npix_mem();
        return L;
    }
    int halo() const { return 1; }
    int stencil_blocks() const { return std::max<int>(std::max<int>(grid().x * grid().y, tgrid()), strip_blocks()); }
    void bind(void** params, hipStream_t s) {
        a_.wf = (T)*(const float*)params[idx_wf_];
        a_.wr = (T)*(const float*)params[idx_wr_];
        userX_ = (T*)params[idx_X_];
        const long long N = dom_.npix_mem();
        if (!opts_.host_buffers) {
            a_.X = userX_;
            a_.I = (const float*)params[idx_I_];
            a_.Ih = (const float*)params[idx_Ih_];
            a_.Ihx = (const float*)params[idx_Ihx_];
            a_.Ihy = (const float*)params[idx_Ihy_];
        } else {
            OPT_HIP_CHECK(hipMemcpyAsync(dX_, userX_, sizeof(T) * 2 * N, hipMemcpyHostToDevice, s));
            const int idx[4] = {idx_I_, idx_Ih_, idx_Ihx_, idx_Ihy_};
            float* dst[4] = {dI_, dIh_, dIhx_, dIhy_};
            for (int k = 0; k < 4; ++k)
                OPT_HIP_CHECK(hipMemcpyAsync(dst[k], params[idx[k]], sizeof(float) * N, hipMemcpyHostToDevice, s));
            a_.X = dX_; a_.I = dI_; a_.Ih = dIh_; a_.Ihx = dIhx_; a_.Ihy = dIhy_;
        }
        a_.G = G_;
        a_.Ef = Ef_;
        a_.dom = dom_;
    }
    void unbind(hipStream_t s) {
        if (opts_.host_buffers)
            OPT_HIP_CHECK(hipMemcpyAsync(userX_, dX_, sizeof(T) * 2 * dom_.npix_mem(), hipMemcpyDeviceToHost, s));
    }
    T* unknown(int k) { return k == 0 ? a_.X : nullptr; }
    void precompute(hipStream_t) {}   // no ComputedArrays in this energy
    void computed_planes(std::vector<HaloPlane>&) const {}
    void jtf(T* r, T* diag, uint8_t* flags, hipStream_t s) {
        a_.flags = flags;
        hipLaunchKernelGGL((of::of_jtf<T>), grid(), dim3(kBlock), 0, s, a_, r, diag);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void apply(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s) {
        if (strip_) {   // OPT_AMD_OF_STRIP (default 1): of_apply_strip
            const int ns = (dom_.W + of::kOfOut - 1) / of::kOfOut;
            rs.nblocks = strip_blocks();
            hipLaunchKernelGGL((of::of_apply_strip<T>), dim3(rs.nblocks), dim3(kBlock), 0, s, a_, p, Ap, dadd, stop, rs,
                               ns, strip_rows_);
        } else {
            rs.nblocks = tgrid();
            hipLaunchKernelGGL((of::of_apply<T>), dim3(tgrid()), dim3(kBlock), 0, s, a_, p, Ap, dadd, stop, rs);
        }
        OPT_HIP_CHECK(hipGetLastError());
    }
    void cost(ReduceSlot rs, hipStream_t s) {
        rs.nblocks = tgrid();
        hipLaunchKernelGGL((of::of_cost<T>), dim3(tgrid()), dim3(kBlock), 0, s, a_, (const T*)nullptr, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void model_cost(const T* delta, ReduceSlot rs, hipStream_t s) {
        rs.nblocks = tgrid();
        hipLaunchKernelGGL((of::of_cost<T>), dim3(tgrid()), dim3(kBlock), 0, s, a_, delta, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    // materialized Jacobian (csr.h): 9 residual rows / 18 nonzeros per pixel; the fit
    // partials come from the gradient of_jtf cached (jtf runs first in every step)
    long long jacobian_rows() const { return 9LL * dom_.W * dom_.H; }
    long long jacobian_nnz() const { return 18LL * dom_.W * dom_.H; }
    void dump_j(int* rowPtr, int* colInd, T* val, hipStream_t s) {
        hipLaunchKernelGGL(of::of_dump_j<T>, dim3(flat_grid((long long)dom_.W * dom_.H, 1)), dim3(kBlock), 0, s, a_,
                           rowPtr, colInd, val);
        OPT_HIP_CHECK(hipGetLastError());
    }

private:
    dim3 grid() const { return dim3((dom_.W + 63) / 64, (dom_.y_hi - dom_.y_lo + 3) / 4); }
    int tgrid() const { return tile_blocks(pix_tiles(dom_)); }
    // the strip apply's grid: groups of four 62-column strips x row chunks of strip_rows_
    int strip_blocks() const {
        const int ns = (dom_.W + of::kOfOut - 1) / of::kOfOut;
        return (ns + kBlock / kWave - 1) / (kBlock / kWave) * ((dom_.y_hi - dom_.y_lo + strip_rows_ - 1) / strip_rows_);
    }
    const bool strip_ = env_int("OPT_AMD_OF_STRIP", 1) != 0;
    const int strip_rows_ = std::max(1, env_int("OPT_AMD_OF_ROWS", 8));   // 8 / 16 / 32: 81.5 / 88.2 / 89.1 us at 3840x2160 fp64
    Domain dom_;
    StateOptions opts_;
    int idx_X_, idx_I_, idx_Ih_, idx_Ihx_, idx_Ihy_, idx_wf_, idx_wr_;
    of::Args<T> a_{};
    T* G_ = nullptr;
    T* Ef_ = nullptr;   // fit residual at the step's X (of_jtf -> model cost)
    T* userX_ = nullptr;
    T* dX_ = nullptr;
    float *dI_ = nullptr, *dIh_ = nullptr, *dIhx_ = nullptr, *dIhy_ = nullptr;
};

std::unique_ptr<Plan> make_optical_flow_plan(const ProblemSpec& spec, const StateOptions& opts,
                                             const unsigned* dims, std::string* err) {
    unsigned W = 0, H = 0;
    for (auto& d : spec.dims) {
        if (d.name == spec.unknown(0)->dims[0]) W = dims[d.index];
        if (d.name == spec.unknown(0)->dims[1]) H = dims[d.index];
    }
    if (W == 0 || H == 0) { *err = "optical_flow: zero-sized domain"; return nullptr; }
    if (spec.unknown(0)->channels != 2) { *err = "optical_flow: expects a 2-channel unknown"; return nullptr; }
    Domain dom{(int)W, (int)H, 0, (int)H, 0, (int)H};
    if (opts.double_precision) return make_stencil_plan<OpticalFlowOp<double>>(spec, opts, dom, err);
    return make_stencil_plan<OpticalFlowOp<float>>(spec, opts, dom, err);
}

}  // namespace optamd
