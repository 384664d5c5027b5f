// poisson.hip — kernels for the poisson_image_editing energy
// (reference examples/poisson_image_editing/poisson_image_editing.t):
//
//   unknown X (float4 per pixel), knowns T (float4, the inserted image), M (mask)
//   Exclude(M != 0); UsePreconditioner(false)
//   for s in {(1,0),(-1,0),(0,1),(0,-1)}:  e(k,s) = InBounds(k+s) ? (X_k - X_{k+s}) - (T_k - T_{k+s}) : 0
//
// The residual does not test the mask: excluded pixels are fixed Dirichlet values that
// still enter every residual, and the gathers of an active pixel include the residuals
// centred at excluded neighbours (residualsincludingX00, o.t:2723-2733), while
// computeCost skips excluded centres (solverGPUGaussNewton.t:971-997).
// Per channel, with b(k,s) = InBounds(k+s):
//   J^T F(k)  = sum_s b(k,s) e(k,s) - b(k,-s) e(k-s,s)          (o.t:2870-2913)
//   diag(k)   = sum_s b(k,s) + b(k,-s)
//   J^T J p(k)= sum_s b(k,s)(p_k - p_{k+s}) - b(k,-s)(p_{k-s} - p_k)   (p = 0 off the solve)
// One thread per pixel, 16-byte float4 accesses; the neighbours' rows are L2 hits.
#include <hip/hip_runtime.h>
#include <algorithm>
#include "plan.h"
#include "stencil_plan.h"

namespace optamd {
namespace pie {

template <typename T> struct V4t { T x, y, z, w; };

template <typename T>
struct Args {
    Domain dom;
    const T* X;
    const float* Tg;     // target image T (float4)
    const float* M;
    uint8_t* flags;      // bit0 active (Mask == 0)
};

__device__ __forceinline__ bool inside(const Domain& d, int x, int y) {
    return x >= 0 && x < d.W && y >= 0 && y < d.H;
}
template <typename T>
__device__ __forceinline__ V4t<T> ld(const T* a, long long i) {
    return reinterpret_cast<const V4t<T>*>(a)[i];
}
__device__ __forceinline__ V4t<float> ldf(const float* a, long long i) {
    return reinterpret_cast<const V4t<float>*>(a)[i];
}
template <typename T>
__device__ __forceinline__ V4t<T> resid(const V4t<T>& xk, const V4t<T>& xj, const V4t<float>& tk,
                                        const V4t<float>& tj) {
    return {(xk.x - xj.x) - (T)(tk.x - tj.x), (xk.y - xj.y) - (T)(tk.y - tj.y),
            (xk.z - xj.z) - (T)(tk.z - tj.z), (xk.w - xj.w) - (T)(tk.w - tj.w)};
}

constexpr int DX[4] = {1, -1, 0, 0};
constexpr int DY[4] = {0, 0, 1, -1};

__device__ __forceinline__ PixGeom pix(const Domain& d) {
    PixGeom g;
    g.x = blockIdx.x * 64 + (threadIdx.x & 63);
    g.y = d.y_lo + blockIdx.y * 4 + (threadIdx.x >> 6);
    g.ok = g.x < d.W && g.y < d.y_hi;
    g.i = g.ok ? d.off(g.x, g.y) : 0;
    return g;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void pie_jtf(Args<T> a, T* __restrict__ r, T* __restrict__ diag) {
    const PixGeom g = pix(a.dom);
    if (!g.ok) return;
    const bool act = a.M[g.i] == 0.f;
    a.flags[g.i] = act;
    V4t<T> F = {0, 0, 0, 0};
    T D = 0;
    if (act) {
        const V4t<T> xk = ld(a.X, g.i);
        const V4t<float> tk = ldf(a.Tg, g.i);
        for (int s = 0; s < 4; ++s) {
            const int tx = g.x + DX[s], ty = g.y + DY[s];
            if (inside(a.dom, tx, ty)) {   // instance centred at k
                const long long j = a.dom.off(tx, ty);
                const V4t<T> e = resid(xk, ld(a.X, j), tk, ldf(a.Tg, j));
                F.x += e.x; F.y += e.y; F.z += e.z; F.w += e.w;
                D += (T)1;
            }
            const int jx = g.x - DX[s], jy = g.y - DY[s];
            if (inside(a.dom, jx, jy)) {   // instance centred at k - s (its neighbour is k)
                const long long j = a.dom.off(jx, jy);
                const V4t<T> e = resid(ld(a.X, j), xk, ldf(a.Tg, j), tk);
                F.x -= e.x; F.y -= e.y; F.z -= e.z; F.w -= e.w;
                D += (T)1;
            }
        }
    }
    reinterpret_cast<V4t<T>*>(r)[g.i] = {-F.x, -F.y, -F.z, -F.w};
    reinterpret_cast<V4t<T>*>(diag)[g.i] = {D, D, D, D};
}

template <typename T>
__global__ __launch_bounds__(kBlock) void pie_apply(Args<T> a, const T* __restrict__ p, T* __restrict__ Ap,
                                                    const T* __restrict__ dadd, const int* stop, ReduceSlot rs) {
    if (stop && *stop) return;
    const PixGeom g = pix(a.dom);
    T dot = 0;
    if (g.ok) {
        const bool act = a.flags[g.i] & 1;
        V4t<T> o = {0, 0, 0, 0};
        if (act) {
            const V4t<T> pk = ld(p, g.i);
            auto pv = [&](long long j) -> V4t<T> {   // p is 0 on excluded unknowns
                return (a.flags[j] & 1) ? ld(p, j) : V4t<T>{0, 0, 0, 0};
            };
            for (int s = 0; s < 4; ++s) {
                const int tx = g.x + DX[s], ty = g.y + DY[s];
                if (inside(a.dom, tx, ty)) {
                    const V4t<T> pj = pv(a.dom.off(tx, ty));
                    o.x += pk.x - pj.x; o.y += pk.y - pj.y; o.z += pk.z - pj.z; o.w += pk.w - pj.w;
                }
                const int jx = g.x - DX[s], jy = g.y - DY[s];
                if (inside(a.dom, jx, jy)) {
                    const V4t<T> pj = pv(a.dom.off(jx, jy));
                    o.x -= pj.x - pk.x; o.y -= pj.y - pk.y; o.z -= pj.z - pk.z; o.w -= pj.w - pk.w;
                }
            }
            if (dadd) {
                const V4t<T> c = ld(dadd, g.i);
                o.x += c.x * pk.x; o.y += c.y * pk.y; o.z += c.z * pk.z; o.w += c.w * pk.w;
            }
            dot = pk.x * o.x + pk.y * o.y + pk.z * o.z + pk.w * o.w;
        }
        reinterpret_cast<V4t<T>*>(Ap)[g.i] = o;
    }
    double v[1] = {(double)dot};
    block_reduce_publish<1>(v, rs, blockIdx.y * gridDim.x + blockIdx.x);
}

// cost (delta == nullptr) or LM model cost 1/2 sum (e + J delta)^2 (o.t:2915-2943)
template <typename T>
__global__ __launch_bounds__(kBlock) void pie_cost(Args<T> a, const T* __restrict__ delta, ReduceSlot rs) {
    const PixGeom g = pix(a.dom);
    T acc = 0;
    if (g.ok && a.M[g.i] == 0.f) {
        const V4t<T> xk = ld(a.X, g.i);
        const V4t<float> tk = ldf(a.Tg, g.i);
        V4t<T> dk = {0, 0, 0, 0};
        if (delta) dk = ld(delta, g.i);
        for (int s = 0; s < 4; ++s) {
            const int tx = g.x + DX[s], ty = g.y + DY[s];
            if (!inside(a.dom, tx, ty)) continue;
            const long long j = a.dom.off(tx, ty);
            V4t<T> e = resid(xk, ld(a.X, j), tk, ldf(a.Tg, j));
            if (delta) {
                const V4t<T> dj = (a.M[j] == 0.f) ? ld(delta, j) : V4t<T>{0, 0, 0, 0};
                e.x += dk.x - dj.x; e.y += dk.y - dj.y; e.z += dk.z - dj.z; e.w += dk.w - dj.w;
            }
            acc += e.x * e.x + e.y * e.y + e.z * e.z + e.w * e.w;
        }
        acc = (T)0.5 * acc;
    }
    double v[1] = {(double)acc};
    block_reduce_publish<1>(v, rs, blockIdx.y * gridDim.x + blockIdx.x);
}


// saveJToCRS / generateDumpJ (solverGPUGaussNewton.t:385-442, 1004-1022): every pixel
// writes 16 rows (s-major, channel-minor), each {X_c(k): b, X_c(k+s): -b} with
// b = InBounds(k+s), columns wrapped (wrap(), :365-381) and sorted.
// Rows of 128 consecutive pixels staged in LDS (4096 nonzeros, 2048 row pointers) and
// stored contiguously; two threads per pixel (channels 0-1 / 2-3).
template <typename T>
__global__ __launch_bounds__(kBlock) void pie_dump_j(Domain d, int* __restrict__ rowPtr, int* __restrict__ colInd,
                                                     T* __restrict__ val) {
    constexpr int P = kBlock / 2;
    __shared__ int s_col[P * 32];
    __shared__ T s_val[P * 32];
    __shared__ int s_row[P * 16];
    const long long N = (long long)d.W * d.H, n = 4 * N;
    const int t = threadIdx.x, tp = t >> 1, half = t & 1;
    for (long long k0 = (long long)blockIdx.x * P; k0 < N; k0 += (long long)gridDim.x * P) {
        const long long k = k0 + tp;
        if (k < N) {
            const int x = (int)(k % d.W), y = (int)(k / d.W);
            for (int s = 0; s < 4; ++s) {
                const bool in = inside(d, x + DX[s], y + DY[s]);
                const long long tn = k + DX[s] + (long long)DY[s] * d.W;
                for (int cc = 0; cc < 2; ++cc) {
                    const int c = 2 * half + cc;
                    const int row = 4 * s + c, nz = 2 * row;
                    s_row[16 * tp + row] = (int)(32 * k + nz);
                    long long c0 = 4 * k + c, c1 = 4 * tn + c;
                    c1 = c1 < 0 ? c1 + n : (c1 >= n ? c1 - n : c1);
                    T v0 = in ? (T)1 : (T)0, v1 = in ? (T)-1 : (T)0;
                    if (c1 < c0) {
                        const long long tc = c0; c0 = c1; c1 = tc;
                        const T tv = v0; v0 = v1; v1 = tv;
                    }
                    s_col[32 * tp + nz] = (int)c0; s_val[32 * tp + nz] = v0;
                    s_col[32 * tp + nz + 1] = (int)c1; s_val[32 * tp + nz + 1] = v1;
                }
            }
        }
        __syncthreads();
        const int np = (int)min((long long)P, N - k0);
        for (int e = t; e < 32 * np; e += kBlock) {
            colInd[32 * k0 + e] = s_col[e];
            val[32 * k0 + e] = s_val[e];
        }
        for (int e = t; e < 16 * np; e += kBlock) rowPtr[16 * k0 + e] = s_row[e];
        __syncthreads();
    }
    if (blockIdx.x == 0 && t == 0) rowPtr[16 * N] = (int)(32 * N);
}

}  // namespace pie

template <typename TT>
class PoissonOp {
public:
    using T = TT;
    static constexpr const char* kName = "poisson_image_editing";
    static constexpr const char* kApplyName = "pie_apply";
    static constexpr bool kSlabs = true;
    PoissonOp(const ProblemSpec& spec, const StateOptions& opts, Domain dom) : dom_(dom), opts_(opts) {
        idx_X_ = spec.unknown(0)->index;
        idx_T_ = spec.array(0)->index;
        idx_M_ = spec.array(1)->index;
        const long long N = dom_.npix_mem();
        if (opts.host_buffers) {
            dX_ = (T*)dmalloc(sizeof(T) * 4 * N);
            dT_ = (float*)dmalloc(sizeof(float) * 4 * N);
            dM_ = (float*)dmalloc(sizeof(float) * N);
        }
    }
    ~PoissonOp() { dfree(dX_); dfree(dT_); dfree(dM_); }
    VecLayout layout() const {
        VecLayout L{};
        L.nimg = 1;
        L.ch[0] = 4;
        L.off[0] = 0;
        L.off[1] = 4 * dom_.npix_mem();
        L.N = dom_.npix_mem();
        return L;
    }
    int halo() const { return 1; }
    int stencil_blocks() const { return grid().x * grid().y; }
    void bind(void** params, hipStream_t s) {
        userX_ = (T*)params[idx_X_];
        const long long N = dom_.npix_mem();
        if (!opts_.host_buffers) {
            a_.X = userX_;
            a_.Tg = (const float*)params[idx_T_];
            a_.M = (const float*)params[idx_M_];
        } else {
            OPT_HIP_CHECK(hipMemcpyAsync(dX_, userX_, sizeof(T) * 4 * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dT_, params[idx_T_], sizeof(float) * 4 * N, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipMemcpyAsync(dM_, params[idx_M_], sizeof(float) * N, hipMemcpyHostToDevice, s));
            a_.X = dX_; a_.Tg = dT_; a_.M = dM_;
        }
        a_.dom = dom_;
    }
    void unbind(hipStream_t s) {
        if (opts_.host_buffers)
            OPT_HIP_CHECK(hipMemcpyAsync(userX_, dX_, sizeof(T) * 4 * dom_.npix_mem(), hipMemcpyDeviceToHost, s));
    }
    T* unknown(int k) { return k == 0 ? (T*)a_.X : nullptr; }
    void precompute(hipStream_t) {}   // no ComputedArrays in this energy
    void computed_planes(std::vector<HaloPlane>&) const {}
    void jtf(T* r, T* diag, uint8_t* flags, hipStream_t s) {
        a_.flags = flags;
        hipLaunchKernelGGL((pie::pie_jtf<T>), grid(), dim3(kBlock), 0, s, a_, r, diag);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void apply(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL((pie::pie_apply<T>), grid(), dim3(kBlock), 0, s, a_, p, Ap, dadd, stop, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void cost(ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL((pie::pie_cost<T>), grid(), dim3(kBlock), 0, s, a_, (const T*)nullptr, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    void model_cost(const T* delta, ReduceSlot rs, hipStream_t s) {
        hipLaunchKernelGGL((pie::pie_cost<T>), grid(), dim3(kBlock), 0, s, a_, delta, rs);
        OPT_HIP_CHECK(hipGetLastError());
    }
    // materialized Jacobian (csr.h): 16 residual rows / 32 nonzeros per pixel
    long long jacobian_rows() const { return 16LL * dom_.W * dom_.H; }
    long long jacobian_nnz() const { return 32LL * dom_.W * dom_.H; }
    void dump_j(int* rowPtr, int* colInd, T* val, hipStream_t s) {
        hipLaunchKernelGGL(pie::pie_dump_j<T>, dim3(flat_grid((long long)dom_.W * dom_.H * 2, 1)), dim3(kBlock), 0,
                           s, dom_, rowPtr, colInd, val);
        OPT_HIP_CHECK(hipGetLastError());
    }

private:
    dim3 grid() const {
        return dim3((dom_.W + 63) / 64, (dom_.y_hi - dom_.y_lo + 3) / 4);
    }
    Domain dom_;
    StateOptions opts_;
    int idx_X_, idx_T_, idx_M_;
    pie::Args<T> a_{};
    T* userX_ = nullptr;
    T* dX_ = nullptr;
    float *dT_ = nullptr, *dM_ = nullptr;
};

std::unique_ptr<Plan> make_poisson_plan(const ProblemSpec& spec, const StateOptions& opts, const unsigned* dims,
                                        std::string* err) {
    unsigned W = 0, H = 0;
    for (auto& d : spec.dims) {
        if (d.name == spec.unknown(0)->dims[0]) W = dims[d.index];
        if (d.name == spec.unknown(0)->dims[1]) H = dims[d.index];
    }
    if (W == 0 || H == 0) { *err = "poisson_image_editing: zero-sized domain"; return nullptr; }
    if (spec.unknown(0)->channels != 4) { *err = "poisson_image_editing: expects a 4-channel unknown"; return nullptr; }
    Domain dom{(int)W, (int)H, 0, (int)H, 0, (int)H};
    if (opts.double_precision) return make_stencil_plan<PoissonOp<double>>(spec, opts, dom, err);
    return make_stencil_plan<PoissonOp<float>>(spec, opts, dom, err);
}

}  // namespace optamd
