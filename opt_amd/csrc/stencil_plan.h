// stencil_plan.h — host side of the generic image-domain GN / LM solver
// (stencil_driver.h kernels + a family operator). Control flow follows the
// reference's init / step exactly (API/src/solverGPUGaussNewton.t:1766-2349),
// including the LM trust-region update and its early exits.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>
#include "csr.h"
#include "stencil_driver.h"

namespace optamd {

// Device pointers of the unknown images (VecLayout order).
template <typename T>
struct UnknownPtrs {
    T* x[4];
};

// X += delta on the active pixels (PCGLinearUpdate, :854-859); LM also keeps the
// previous unknowns (savePreviousUnknowns :882-887) for revertUpdate (:864-869).
template <typename T, bool SAVE>
__global__ __launch_bounds__(kBlock) void update_images_kernel(VecLayout L, const uint8_t* __restrict__ flags,
                                                               UnknownPtrs<T> X, const T* __restrict__ delta,
                                                               T* __restrict__ prev, long long pix_lo,
                                                               long long pix_hi) {
    const long long n = L.off[L.nimg];
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long e0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; e0 < n; e0 += kIlp * stride) {
        bool on[kIlp];
        T* xp[kIlp];
        T xv[kIlp], dv[kIlp];
#pragma unroll
        for (int u = 0; u < kIlp; ++u) {   // kIlp elements' loads in flight together
            const long long e = e0 + u * stride;
            const bool in = e < n;
            int k = 0;
            long long local = 0;
            const long long px = in ? L.locate(e, &k, &local) : 0;
            on[u] = in && px >= pix_lo && px < pix_hi && (flags[px] & 1);
            xp[u] = X.x[k] + local;
            xv[u] = *xp[u];
            dv[u] = delta[in ? e : 0];
        }
#pragma unroll
        for (int u = 0; u < kIlp; ++u) {
            if (!on[u]) continue;
            if (SAVE) prev[e0 + u * stride] = xv[u];
            *xp[u] = xv[u] + dv[u];
        }
    }
}
template <typename T>
__global__ __launch_bounds__(kBlock) void revert_images_kernel(VecLayout L, const uint8_t* __restrict__ flags,
                                                               UnknownPtrs<T> X, const T* __restrict__ prev,
                                                               long long pix_lo, long long pix_hi) {
    const long long n = L.off[L.nimg];
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        int k;
        long long local;
        const long long px = L.locate(e, &k, &local);
        if (px < pix_lo || px >= pix_hi || !(flags[px] & 1)) continue;
        X.x[k][local] = prev[e];
    }
}

// Op contract (see poisson.hip):
//   using T; static constexpr const char* kName, kApplyName;
//   static constexpr bool kSlabs                          — row-slab decomposition allowed
//   Op(const ProblemSpec&, const StateOptions&, Domain)   — roles from declarations
//   VecLayout layout() const; int halo() const;
//   void bind(void** params, hipStream_t)                 — pointers + scalar params
//   T* unknown(int k)                                     — device unknown image k
//   void precompute(hipStream_t)                           — materialise ComputedArrays
//                     (init, after each update and after a revert: :1876, 2242, 2284)
//   void computed_planes(std::vector<HaloPlane>&)          — what precompute writes
//   void jtf(T* r, T* diag, uint8_t* flags, hipStream_t)  — r = -J^T F, diag(J^T J), flags
//   void apply(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot, hipStream_t)
//                     — Ap = J^T J p (+ dadd p), sum p.Ap; returns early if *stop
//   void cost(ReduceSlot, hipStream_t); void model_cost(const T* delta, ReduceSlot, hipStream_t)
//   void unbind(hipStream_t)                               — copy unknowns back (host mode)
//   optional, for the materialized path (useMaterializedJTJ, csr.h):
//   long long jacobian_rows() const, jacobian_nnz() const;
//   void dump_j(int* rowPtr, int* colInd, T* val, hipStream_t)  — J in CSR (saveJToCRS)
// All stencil kernels cover the owned rows [y_lo, y_hi) of the Domain and read up to
// halo() rows beyond them.
//
// Row-slab decomposition: each rank owns rows [y_lo, y_hi) and holds
// halo() rows of each neighbour. The flat PCG kernels run over the whole memory slab:
// the init kernels zero pre / p / r / b / CtC outside the owned rows (and the stencil
// kernels write Ap only there), so every flat reduction sums owned elements only. The
// exchanges are: unknowns after bind / update / revert, computed arrays after each
// precompute, flags after J^T F, p before each apply (delta before an apply of delta
// and before the model cost); every scalar is all-reduced right after its kernel.
template <class Op, class = void>
struct HasDumpJ : std::false_type {};
template <class Op>
struct HasDumpJ<Op, std::void_t<decltype(std::declval<Op&>().dump_j((int*)nullptr, (int*)nullptr,
                                                                     (typename Op::T*)nullptr, hipStream_t{}))>>
    : std::true_type {};

// Ops whose apply can run as interior + boundary launches (row slabs: the halo refresh
// of p overlaps the interior part): bool can_split() const; void apply_split(int part,
// ... apply's arguments) with part 1 = no halo reads, 2 = the rest, 0 = everything.
template <class Op, class = void>
struct HasApplySplit : std::false_type {};
template <class Op>
struct HasApplySplit<Op, std::void_t<decltype(std::declval<const Op&>().can_split())>> : std::true_type {};

// Ops whose apply can also reduce the fused PCG step's sums (shape_from_shading):
// apply_sums(part, p, Ap, dadd, stop, rs, r, w, stream, e0, e1) reduces {p.Ap, r.W Ap,
// Ap.W Ap, r.W r} (fp64) into rs; the driver then runs PCGStep2 + PCGStep3 as ONE pass
// (step23_kernel, beta's numerator from the identity over those sums) and, on row slabs,
// one all-reduce per PCG iteration.
template <class Op, class = void>
struct HasApplySums : std::false_type {};
template <class Op>
struct HasApplySums<Op, std::void_t<decltype(std::declval<Op&>().apply_sums(
                            0, (const typename Op::T*)nullptr, (typename Op::T*)nullptr, (const typename Op::T*)nullptr,
                            (const int*)nullptr, ReduceSlot{}, (const typename Op::T*)nullptr,
                            (const typename Op::T*)nullptr, hipStream_t{}, hipEvent_t{}, hipEvent_t{}))>>
    : std::true_type {};

// Ops that fold PCGStep3 into the first pass of their next apply (ARAP: p = z + beta p
// per vertex, then K of the new p): step3_fused(pre, r, p, sc, i_num, i_den, use_pre,
// stop, s) replaces step3_kernel; apply_prepared(...apply's arguments) is the apply
// without that first pass.
template <class Op, class = void>
struct HasFusedStep3 : std::false_type {};
template <class Op>
struct HasFusedStep3<Op, std::void_t<decltype(std::declval<Op&>().step3_fused(
                             (const typename Op::T*)nullptr, (const typename Op::T*)nullptr, (typename Op::T*)nullptr,
                             (const double*)nullptr, 0, 0, 0, (const int*)nullptr, hipStream_t{}))>> : std::true_type {};

// Optional Op::apply_ext(p, Ap, dadd, stop, rs, stream, e0, e1): the apply with HIP
// events attached to its launch (hipExtLaunchKernelGGL), so the per-kernel timer measures
// the kernel itself instead of event records around the launch.
template <class Op, class = void>
struct HasApplyExt : std::false_type {};
template <class Op>
struct HasApplyExt<Op, std::void_t<decltype(std::declval<Op&>().apply_ext(
                           (const typename Op::T*)nullptr, (typename Op::T*)nullptr, (const typename Op::T*)nullptr,
                           (const int*)nullptr, ReduceSlot{}, hipStream_t{}, hipEvent_t{}, hipEvent_t{}))>> : std::true_type {};

template <class Op, class = void>
struct HasSlabRefusal : std::false_type {};
template <class Op>
struct HasSlabRefusal<Op, std::void_t<decltype(std::declval<const Op&>().slab_refusal())>> : std::true_type {};

// Ops that keep private per-step caches of values derived from the bound arrays
// (GenericOp: transcendentals of centred and graph-slot reads): refresh_caches(stream)
// recomputes them from the arrays as bound at THIS Step. The reference evaluates those
// values inline from the arrays at every Step (setGPUptr, solverGPUGaussNewton.t:2001), so
// a caller may rewrite or rebind arrays between Steps (Opt.h:64-65); ComputedArrays
// themselves keep the reference's schedule (init, after update, after revert).
template <class Op, class = void>
struct HasRefreshCaches : std::false_type {};
template <class Op>
struct HasRefreshCaches<Op, std::void_t<decltype(std::declval<Op&>().refresh_caches(hipStream_t{}))>>
    : std::true_type {};

// Ops that describe their own hipGraph capture gate and key (GenericOp: the kernel
// argument block the generated launches receive) instead of the declaration parser's.
template <class Op, class = void>
struct HasCaptureKey : std::false_type {};
template <class Op>
struct HasCaptureKey<Op, std::void_t<decltype(std::declval<const Op&>().capture_key(
                             (std::vector<unsigned long long>*)nullptr))>> : std::true_type {};

template <class Op>
class StencilPlan final : public Plan {
public:
    using T = typename Op::T;
    StencilPlan(const ProblemSpec& spec, const StateOptions& opts, Domain dom) : Plan(spec, opts), dom_(dom) {
        lm_ = spec.lm();
        stop_ = (int*)dmalloc(64);
        OPT_HIP_CHECK(hipMemset(stop_, 0, 64));
        timer_.apply_name = Op::kApplyName;
        allocate();
    }
    ~StencilPlan() override {
        OPT_HIP_CHECK(hipStreamSynchronize(stream_));
        release();
        dfree(stop_);
    }

    long long unknown_count() const override { return n_; }
    std::string family() const override { return Op::kName; }
    std::string apply_kernel_name() const override { return mat_ ? mat_->apply_name() : Op::kApplyName; }
    int halo() const override { return op_->halo(); }

    std::string set_decomposition(Comm* comm, int y_lo, int y_hi) override {
        if (!Op::kSlabs) return std::string(Op::kName) + ": no row-slab decomposition (data-dependent reads)";
        if constexpr (HasSlabRefusal<Op>::value) {
            const std::string why = op_->slab_refusal();
            if (!why.empty()) return why;
        }
        if (opts_.host_buffers) return "row-slab decomposition needs backend_cuda (device arrays)";
        if (opts_.materialized) return "row-slab decomposition of the materialized Jacobian path is not supported";
        const int h = op_->halo();
        if (y_lo < 0 || y_hi > dom_.H || y_hi - y_lo < h) return "invalid slab rows";
        comm_ = comm;
        OPT_HIP_CHECK(hipStreamSynchronize(stream_));
        release();
        dom_.y_lo = y_lo;
        dom_.y_hi = y_hi;
        dom_.y_mem0 = std::max(0, y_lo - h);
        dom_.mem_rows = std::min(dom_.H, y_hi + h) - dom_.y_mem0;
        allocate();
        initialised_ = false;
        return "";
    }

    void init(void** params) override {
        begin_call();
        op_->bind(params, stream_);
        exchange_unknowns();
        // reference init: LM parameters copied into the plan (:1863-1872), precompute,
        // prevCost = cost; PCGInit1 is redone by every step
        radius_ = sp_.trust_region_radius;
        decrease_ = sp_.radius_decrease_factor;
        precompute();
        tbegin("cost"); op_->cost(red_.slot(nb(), kScCost), stream_); tend();
        allreduce(kScCost, 1);
        prev_cost_ = read(kScCost);
        n_iter_ = 0;
        initialised_ = true;
        end_call();
    }

    int step(void** params) override {
        if (!initialised_) init(params);
        if (n_iter_ >= sp_.nIterations) {
            cleanup_log();
            return 0;
        }
        begin_call();
        op_->bind(params, stream_);
        exchange_unknowns();
        if constexpr (HasRefreshCaches<Op>::value) {
            if (op_->refresh_caches(stream_)) exchange_computed();
        }
        const int Lit = std::max(0, sp_.lIterations);
        red_.ensure(std::max(op_->stencil_blocks(), 4096), 4, kScBase + kSlots * (Lit + 2));
        OPT_HIP_CHECK(hipMemsetAsync(stop_, 0, 64, stream_));
        OPT_HIP_CHECK(hipMemsetAsync(delta_, 0, sizeof(T) * n_, stream_));   // PCGInit1: delta = 0
        const int use_pre = spec_.use_preconditioner ? 1 : 0;
        const long long lo = pix_lo(), hi = pix_hi();
        // PCGInit1 (+ LM diagonal)
        tbegin("jtf"); op_->jtf(r_, diag_, flags_, stream_); tend();
        exchange({{(void*)flags_, (size_t)dom_.W}});
        if (!lm_) {
            tbegin("gn_init");
            hipLaunchKernelGGL((gn_init_kernel<T>), dim3(fg()), dim3(kBlock), 0, stream_, L_, (const uint8_t*)flags_,
                               r_, (const T*)diag_, pre_, p_, use_pre, lo, hi, red_.slot(fg(), rz(0)));
            tend();
        } else {
            LMScalars lm{radius_, sp_.min_lm_diagonal, sp_.max_lm_diagonal};
            tbegin("lm_init");
            if (n_iter_ == 0)
                hipLaunchKernelGGL((lm_init_kernel<T, true>), dim3(fg()), dim3(kBlock), 0, stream_, L_,
                                   (const uint8_t*)flags_, r_, (const T*)diag_, SSq_, CtC_, pre_, b_, p_,
                                   use_pre, lm, lo, hi, red_.slot(fg(), rz(0)));
            else
                hipLaunchKernelGGL((lm_init_kernel<T, false>), dim3(fg()), dim3(kBlock), 0, stream_, L_,
                                   (const uint8_t*)flags_, r_, (const T*)diag_, SSq_, CtC_, pre_, b_, p_,
                                   use_pre, lm, lo, hi, red_.slot(fg(), rz(0)));
            tend();
            OPT_HIP_CHECK(hipMemsetAsync(red_.scalars + kScQ0, 0, sizeof(double), stream_));
        }
        OPT_HIP_CHECK(hipGetLastError());
        allreduce(rz(0), 1);
        const int* stop = lm_ ? stop_ : nullptr;
        if (mat_) materialize();   // cusparseOuter (:2068): J, J^T (, J^T J) at the current X
        if (pcg_graph_begin(params, Lit)) {
            pcg_loop(Lit, use_pre, stop);
            pcg_graph_end();
        }
        if (!lm_) {
            if (Lit > 0) update(false);
            precompute();
            tbegin("cost"); op_->cost(red_.slot(nb(), kScCost), stream_); tend();
            allreduce(kScCost, 1);
            const double c = read(kScCost);
            op_->unbind(stream_);
            end_call();
            prev_cost_ = c;
            ++n_iter_;
            return 1;
        }
        return lm_finish_step();
    }

    // PCG inner loop (PCGStep1-3, :607-845) of one step; launches only, no host sync.
    void pcg_loop(int Lit, int use_pre, const int* stop) {
        if constexpr (HasApplySums<Op>::value)
            if (!mat_ && (fuse23_ == 1 || (fuse23_ == 2 && distributed()))) {
                pcg_loop_fused(Lit, use_pre, stop);
                return;
            }
        const bool fuse3 = !distributed() && !mat_ && fuse3_on_;
        // GN with step3_kernel: the delta update rides in PCGStep3 (reads p_old anyway)
        bool d3 = !lm_ && delta3_on_;
        if constexpr (HasFusedStep3<Op>::value) d3 = d3 && !fuse3;
        for (int i = 0; i < Lit; ++i) {
            // the zeta test rides in the kernel that reduces q (one GPU), else its own launch
            const ZetaArgs z{red_.scalars + kScQ0, stop_, i, sp_.q_tolerance, (lm_ && !distributed()) ? 1 : 0};
            bool split = false;
            if constexpr (HasApplySplit<Op>::value)
                split = distributed() && overlap_ && comm_->concurrent_halo() && !mat_ && op_->can_split();
            if (!split) exchange_vec(p_);
            if (split) {
                if constexpr (HasApplySplit<Op>::value) {
                    // halo refresh of p beside the interior blocks (Plan::halo_mark/begin/join)
                    tbegin(Op::kApplyName);
                    halo_mark();
                    const ReduceSlot rs = red_.slot(nb(), pap(i));
                    op_->apply_split(1, p_, Ap_, lm_ ? CtC_ : nullptr, stop, rs, stream_);
                    halo_begin(comm_, vec_planes(p_), dom_, op_->halo());
                    halo_join();
                    op_->apply_split(2, p_, Ap_, lm_ ? CtC_ : nullptr, stop, rs, stream_);
                    tend();
                }
            } else if (mat_) {
                // cusparseInner + PCGStep1_Finish (:2101-2118): the SpMV replaces PCGStep1;
                // as in the reference, the LM CtC term is not part of this product
                mat_apply(p_, Ap_, stop, pap(i));
            } else {
                bool done = false;
                if constexpr (HasFusedStep3<Op>::value)
                    if (i > 0 && fuse3) {   // step3 of i-1 already ran the apply's first pass
                        tbegin(Op::kApplyName);
                        op_->apply_prepared(p_, Ap_, lm_ ? CtC_ : nullptr, stop, red_.slot(nb(), pap(i)), stream_);
                        tend();
                        done = true;
                    }
                if constexpr (HasApplyExt<Op>::value) {
                    hipEvent_t e0 = nullptr, e1 = nullptr;
                    if (!done && timer_.mode && timer_.ext_pair(Op::kApplyName, &e0, &e1)) {
                        op_->apply_ext(p_, Ap_, lm_ ? CtC_ : nullptr, stop, red_.slot(nb(), pap(i)), stream_, e0, e1);
                        timer_.ext_record(Op::kApplyName, e0, e1);
                        done = true;
                    }
                }
                if (!done) {
                    tbegin(Op::kApplyName);
                    op_->apply(p_, Ap_, lm_ ? CtC_ : nullptr, stop, red_.slot(nb(), pap(i)), stream_);
                    tend();
                }
            }
            allreduce(pap(i), 1);
            const bool reset = lm_ && ((i + 1) % std::max(1, sp_.residual_reset_period)) == 0;
            if (reset) {   // the classic halves, the reference's unguarded division (:742)
                hipLaunchKernelGGL((half1_kernel<T>), dim3(fg()), dim3(kBlock), 0, stream_, n_, (const T*)p_,
                                   delta_, red_.scalars, rz(i), pap(i), stop);
                exchange_vec(delta_);
                op_->apply(delta_, Adelta_, CtC_, stop, red_.slot(nb(), kScTmp), stream_);
                hipLaunchKernelGGL((half2_kernel<T>), dim3(fg()), dim3(kBlock), 0, stream_, n_, (const T*)Adelta_,
                                   (const T*)b_, (const T*)pre_, (const T*)delta_, r_, use_pre, stop,
                                   red_.slot(fg(), rz(i + 1)), z);
            } else {
                tbegin("step2");
                launch_step2(i == 0, rz(i), pap(i), rz(i + 1), stop, z, !d3);
                tend();
            }
            allreduce(rz(i + 1), lm_ ? 2 : 1);   // rz and q sit side by side
            tbegin("step3");
            bool fused = false;
            if constexpr (HasFusedStep3<Op>::value)
                if (fuse3) {
                    op_->step3_fused(pre_, r_, p_, red_.scalars, rz(i + 1), rz(i), use_pre, stop, stream_);
                    fused = true;
                }
            if (!fused && d3 && i == 0)
                hipLaunchKernelGGL((step3_kernel<T, 1>), dim3(fg()), dim3(kBlock), 0, stream_, n_, (const T*)pre_,
                                   (const T*)r_, p_, red_.scalars, rz(i + 1), rz(i), use_pre, stop, delta_, rz(i), pap(i));
            else if (!fused && d3)
                hipLaunchKernelGGL((step3_kernel<T, 2>), dim3(fg()), dim3(kBlock), 0, stream_, n_, (const T*)pre_,
                                   (const T*)r_, p_, red_.scalars, rz(i + 1), rz(i), use_pre, stop, delta_, rz(i), pap(i));
            else if (!fused)
                hipLaunchKernelGGL((step3_kernel<T>), dim3(fg()), dim3(kBlock), 0, stream_, n_, (const T*)pre_,
                                   (const T*)r_, p_, red_.scalars, rz(i + 1), rz(i), use_pre, stop);
            tend();
            if (lm_ && !z.on)
                hipLaunchKernelGGL((zeta_kernel<T>), dim3(1), dim3(1), 0, stream_, red_.scalars, q(i + 1),
                                   red_.scalars + kScQ0, i, sp_.q_tolerance, stop_);
            OPT_HIP_CHECK(hipGetLastError());
        }
    }

    // The PCG loop with PCGStep2 + PCGStep3 as one pass (HasApplySums, UsePreconditioner):
    // per iteration the apply (+ its four sums) and step23_kernel; on row slabs ONE
    // all-reduce per iteration — step23's rz / q ride in the next apply's call — and LM's
    // zeta test on the all-reduced q before the next step23 (the apply in between is
    // wasted when it stops: the reference would have left the loop before it). Residual-reset
    // iterations (LM) run the classic sequence.
    void pcg_loop_fused(int Lit, int use_pre, const int* stop) {
        const T* w = use_pre ? pre_ : nullptr;   // PCGStep2's weighting W (1 without a preconditioner)
        bool pending = false;   // rz(i) / q(i) of the previous step23 not all-reduced yet
        for (int i = 0; i < Lit; ++i) {
            const ZetaArgs z{red_.scalars + kScQ0, stop_, i, sp_.q_tolerance, (lm_ && !distributed()) ? 1 : 0};
            bool split = false;
            if constexpr (HasApplySplit<Op>::value)
                split = distributed() && overlap_ && comm_->concurrent_halo() && op_->can_split();
            const ReduceSlot rs = red_.slot(nb(), pap(i));
            auto launch = [&](int part) {
                hipEvent_t e0 = nullptr, e1 = nullptr;
                const bool ev = part == 0 && timer_.mode && timer_.ext_pair(Op::kApplyName, &e0, &e1);
                if (!ev) tbegin(Op::kApplyName);
                op_->apply_sums(part, p_, Ap_, lm_ ? CtC_ : nullptr, stop, rs, r_, w, stream_, e0, e1);
                if (ev) timer_.ext_record(Op::kApplyName, e0, e1);
                else tend();
            };
            if (split) {
                halo_mark();
                launch(1);
                halo_begin(comm_, vec_planes(p_), dom_, op_->halo());
                halo_join();
                launch(2);
            } else {
                exchange_vec(p_);
                launch(0);
            }
            if (distributed()) {
                allreduce(pending ? rz(i) : pap(i), pending ? 6 : 4);
                if (pending && lm_)   // the previous iteration's exit test on the global q
                    hipLaunchKernelGGL((zeta_kernel<T>), dim3(1), dim3(1), 0, stream_, red_.scalars, q(i),
                                       red_.scalars + kScQ0, i - 1, sp_.q_tolerance, stop_);
                pending = false;
            }
            const bool reset = lm_ && ((i + 1) % std::max(1, sp_.residual_reset_period)) == 0;
            if (reset) {   // the classic halves with step23's guards (a zero step / beta = 0)
                hipLaunchKernelGGL((half1_kernel<T, true>), dim3(fg()), dim3(kBlock), 0, stream_, n_, (const T*)p_, delta_,
                                   red_.scalars, rz(i), pap(i), stop);
                exchange_vec(delta_);
                op_->apply(delta_, Adelta_, CtC_, stop, red_.slot(nb(), kScTmp), stream_);
                hipLaunchKernelGGL((half2_kernel<T>), dim3(fg()), dim3(kBlock), 0, stream_, n_, (const T*)Adelta_,
                                   (const T*)b_, (const T*)pre_, (const T*)delta_, r_, use_pre, stop,
                                   red_.slot(fg(), rz(i + 1)), z);
                allreduce(rz(i + 1), 2);
                tbegin("step3");
                hipLaunchKernelGGL((step3_kernel<T, 0, true>), dim3(fg()), dim3(kBlock), 0, stream_, n_,
                                   (const T*)pre_, (const T*)r_, p_, red_.scalars, rz(i + 1), rz(i), use_pre, stop);
                tend();
                if (!z.on)
                    hipLaunchKernelGGL((zeta_kernel<T>), dim3(1), dim3(1), 0, stream_, red_.scalars, q(i + 1),
                                       red_.scalars + kScQ0, i, sp_.q_tolerance, stop_);
                OPT_HIP_CHECK(hipGetLastError());
                continue;
            }
            tbegin("step23");
            const ReduceSlot rs2 = red_.slot(fg(), rz(i + 1));
#define S23(F, L)                                                                                              \
    hipLaunchKernelGGL((step23_kernel<T, F, L>), dim3(fg()), dim3(kBlock), 0, stream_, n_, p_, (const T*)Ap_,      \
                       (const T*)pre_, (const T*)b_, r_, delta_, red_.scalars, rz(i), rz(i + 1) + 6, use_pre, stop, rs2, \
                       z)
            if (i == 0 && lm_) S23(true, true);
            else if (lm_) S23(false, true);
            else if (i == 0) S23(true, false);
            else S23(false, false);
#undef S23
            OPT_HIP_CHECK(hipGetLastError());
            tend();
            if (distributed()) pending = true;
        }
    }

    // The PCG loop of a launch-bound (small) problem costs more in launches than in
    // kernel time (poisson 512^2: ~30 launches of a few us each per step), so on one GPU
    // it is captured once as a hipGraph and replayed. The graph is keyed on everything
    // its launches bake in: the bound arrays and scalar parameter values, the plan's
    // buffers and lIterations; for generated kernels, the whole argument block they
    // receive (Op::capture_key, built from the lowered model, not the declaration
    // parser). Not used with timers (per-kernel events), row slabs (RCCL calls between
    // launches), the materialized path, or graph-domain energies (their adjacency may be
    // rebuilt on bind). OPT_AMD_NO_GRAPH=1 turns it off.
    // Returns true when the caller must issue the launches (eagerly or under capture).
    bool pcg_graph_begin(void** params, int Lit) {
        bool graphs = !spec_.graphs.empty();
        std::vector<unsigned long long> op_key;
        if constexpr (HasCaptureKey<Op>::value) graphs = !op_->capture_key(&op_key);
        if (distributed() || mat_ || timer_.mode || graphs || Lit <= 0 || graph_off_) {
            drop_graph();
            return true;
        }
        std::vector<unsigned long long> key{(unsigned long long)Lit, (unsigned long long)(uintptr_t)red_.scalars,
                                            (unsigned long long)(uintptr_t)red_.partials,
                                            (unsigned long long)(uintptr_t)red_.ticket,
                                            (unsigned long long)(uintptr_t)op_.get(),
                                            (unsigned long long)(uintptr_t)p_};
        key.insert(key.end(), op_key.begin(), op_key.end());
        if constexpr (!HasCaptureKey<Op>::value) {
            for (const DeclImage& im : spec_.images)   // arrays by address, scalars by value (below)
                if (im.index >= 0 && im.index < spec_.n_params_total)
                    key.push_back((unsigned long long)(uintptr_t)params[im.index]);
            for (const DeclParam& d : spec_.params) {
                unsigned long long v = 0;
                if (d.index >= 0 && d.index < spec_.n_params_total && params[d.index])
                    memcpy(&v, params[d.index], d.type == "double" ? 8 : 4);
                key.push_back(v);
            }
        }
        {   // solver parameters the loop bakes in (Opt_SetSolverParameter may change them)
            unsigned long long qt = 0;
            memcpy(&qt, &sp_.q_tolerance, sizeof(sp_.q_tolerance) <= 8 ? sizeof(sp_.q_tolerance) : 8);
            key.push_back(qt);
            key.push_back((unsigned long long)sp_.residual_reset_period);
        }
        if (graph_exec_ && key == graph_key_) {
            OPT_HIP_CHECK(hipGraphLaunch(graph_exec_, stream_));
            return false;
        }
        drop_graph();
        graph_key_ = key;
        OPT_HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeRelaxed));
        capturing_ = true;
        return true;
    }
    void pcg_graph_end() {
        if (!capturing_) return;
        capturing_ = false;
        hipGraph_t g = nullptr;
        OPT_HIP_CHECK(hipStreamEndCapture(stream_, &g));
        OPT_HIP_CHECK(hipGraphInstantiate(&graph_exec_, g, nullptr, nullptr, 0));
        OPT_HIP_CHECK(hipGraphDestroy(g));
        OPT_HIP_CHECK(hipGraphLaunch(graph_exec_, stream_));
    }
    void drop_graph() {
        if (graph_exec_) OPT_HIP_CHECK(hipGraphExecDestroy(graph_exec_));
        graph_exec_ = nullptr;
        graph_key_.clear();
    }

    // ---- LM: model cost, speculative update, accept / reject (:2229-2292)
    int lm_finish_step() {
        const int Lit = std::max(0, sp_.lIterations);
        exchange_vec(delta_);
        tbegin("model_cost"); op_->model_cost(delta_, red_.slot(nb(), kScModel), stream_); tend();
        if (Lit > 0) update(true);
        precompute();
        tbegin("cost"); op_->cost(red_.slot(nb(), kScCost), stream_); tend();
        allreduce(kScModel, 2);   // model cost and cost
        double h[2];
        OPT_HIP_CHECK(hipMemcpyAsync(h, red_.scalars + kScModel, sizeof(h), hipMemcpyDeviceToHost, stream_));
        OPT_HIP_CHECK(hipStreamSynchronize(stream_));
        const T model_cost = (T)h[0], new_cost = (T)h[1];
        const T prev = (T)prev_cost_;
        const T model_change = prev - model_cost;
        log_solver(" cost=%f \n", (double)prev);   // computeModelCostChange (:1505-1513)
        log_solver(" model_cost=%f \n", (double)model_cost);
        log_solver(" model_cost_change=%f \n", (double)model_change);
        const T cost_change = prev - new_cost;
        const T rel = cost_change / model_change;
        int ret = 1;
        if (cost_change >= (T)0 && rel > (T)sp_.min_relative_decrease) {
            const T abs_tol = prev * (T)sp_.function_tolerance;
            if (cost_change <= abs_tol) {
                ret = 0;   // function tolerance reached (prevCost is left as it was, :2254-2258)
                log_solver("\nFunction tolerance reached, exiting\n");
            } else {
                const T qv = rel;
                const T min_factor = (T)(1.0 / 3.0);
                const T tmp = (T)1 - (T)std::pow((double)((T)2 * qv - (T)1), 3.0);
                float rad = (float)((T)radius_ / std::max(min_factor, tmp));
                radius_ = std::min(rad, sp_.max_trust_region_radius);
                decrease_ = 2.0f;
                prev_cost_ = (double)new_cost;
            }
        } else {
            if (Lit > 0) revert();
            precompute();
            radius_ = radius_ / decrease_;
            log_solver(" trust_region_radius=%f \n", (double)radius_);
            decrease_ = 2.0f * decrease_;
            if (radius_ <= sp_.min_trust_region_radius) {
                ret = 0;
                log_solver("\nTrust_region_radius is less than the min, exiting\n");
            } else {
                log_solver("REVERT\n");
            }
        }
        op_->unbind(stream_);
        end_call();
        if (ret) ++n_iter_;
        else cleanup_log();
        return ret;
    }

    int eval_jtf(void** params, void* r, void* pre, double* rzv) override {
        begin_call();
        prepare(params);
        op_->jtf((T*)r, diag_, flags_, stream_);
        hipLaunchKernelGGL((gn_init_kernel<T>), dim3(fg()), dim3(kBlock), 0, stream_, L_, (const uint8_t*)flags_,
                           (T*)r, (const T*)diag_, (T*)pre, p_, spec_.use_preconditioner ? 1 : 0, pix_lo(),
                           pix_hi(), red_.slot(fg(), kScTmp));
        allreduce(kScTmp, 1);
        *rzv = read(kScTmp);
        end_call();
        return 0;
    }
    int apply_jtj(void** params, const void* p, void* Ap, double* pAp) override {
        begin_call();
        prepare(params);
        op_->jtf(r_, diag_, flags_, stream_);   // flags for the exclusion mask
        exchange({{(void*)flags_, (size_t)dom_.W}});
        exchange_vec((T*)p);
        if (mat_) {
            materialize();
            mat_apply((const T*)p, (T*)Ap, nullptr, kScTmp);
        } else {
            tbegin(Op::kApplyName);   // the same timer entry as the PCG loop's applies
            op_->apply((const T*)p, (T*)Ap, nullptr, nullptr, red_.slot(nb(), kScTmp), stream_);
            tend();
        }
        allreduce(kScTmp, 1);
        *pAp = read(kScTmp);
        end_call();
        return 0;
    }
    double eval_cost(void** params) override {
        begin_call();
        prepare(params);
        op_->cost(red_.slot(nb(), kScTmp), stream_);
        allreduce(kScTmp, 1);
        const double c = read(kScTmp);
        end_call();
        return c;
    }
    double time_apply(void** params, const void* p, void* Ap, int reps) override {
        begin_call();
        prepare(params);
        op_->jtf(r_, diag_, flags_, stream_);
        if (mat_) materialize();
        auto run = [&]() {
            if (mat_) mat_apply((const T*)p, (T*)Ap, nullptr, kScTmp);
            else op_->apply((const T*)p, (T*)Ap, nullptr, nullptr, red_.slot(nb(), kScTmp), stream_);
        };
        hipEvent_t e0, e1;
        OPT_HIP_CHECK(hipEventCreate(&e0));
        OPT_HIP_CHECK(hipEventCreate(&e1));
        run();
        OPT_HIP_CHECK(hipEventRecord(e0, stream_));
        for (int i = 0; i < reps; ++i) run();
        OPT_HIP_CHECK(hipEventRecord(e1, stream_));
        OPT_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        OPT_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        end_call();
        return 1000.0 * ms / std::max(1, reps);
    }

    long long jacobian_shape(long long* rows) const override {
        if constexpr (HasDumpJ<Op>::value) {
            if (rows) *rows = op_->jacobian_rows();
            return op_->jacobian_nnz();
        }
        return Plan::jacobian_shape(rows);
    }
    bool materialized_nonzeros(long long* nnzJ, long long* nnzJTJ) const override {
        if (!mat_) return false;
        if (nnzJ) *nnzJ = mat_->nnz();
        if (nnzJTJ) *nnzJTJ = mat_->nnz_jtj();
        return true;
    }
    int eval_jacobian(void** params, int* rowPtr, int* colInd, void* val) override {
        if constexpr (HasDumpJ<Op>::value) {
            if (distributed() || dom_.mem_rows != dom_.H) return 1;
            begin_call();
            prepare(params);
            op_->jtf(r_, diag_, flags_, stream_);   // families whose J reuses J^T F state (optical_flow)
            op_->dump_j(rowPtr, colInd, (T*)val, stream_);
            end_call();
            return 0;
        }
        return Plan::eval_jacobian(params, rowPtr, colInd, val);
    }

private:
    static constexpr int kScCost = 1, kScModel = 0, kScTmp = 2, kScQ0 = 3, kScBase = 8;
    // cost sits right after model cost so one 16-byte copy (and one all-reduce) takes both
    // per PCG iteration: rz[i], q[i] (written together by step2 as a pair), pAp[i]
    // iteration i's slots: rz, q, pAp, then (fused PCG step) r.W Ap, Ap.W Ap, r.W r and
    // step23's identity value of rz
    static constexpr int kSlots = 7;
    int rz(int i) const { return kScBase + kSlots * i; }
    int q(int i) const { return kScBase + kSlots * i + 1; }
    int pap(int i) const { return kScBase + kSlots * i + 2; }
    int nb() const { return op_->stencil_blocks(); }
    int fg() const { return flat_grid(n_, 1); }
    long long pix_lo() const { return dom_.off(0, dom_.y_lo); }
    long long pix_hi() const { return dom_.off(0, dom_.y_hi); }

    void allocate() {
        op_.reset(new Op(spec_, opts_, dom_));
        L_ = op_->layout();
        n_ = L_.off[L_.nimg];
        for (T** v : {&r_, &diag_, &pre_, &p_, &Ap_, &delta_})
            *v = (T*)dmalloc(sizeof(T) * n_);
        if (lm_)
            for (T** v : {&b_, &CtC_, &SSq_, &prev_, &Adelta_})
                *v = (T*)dmalloc(sizeof(T) * n_);
        for (T* v : {r_, diag_, pre_, p_, Ap_, delta_, b_, CtC_, SSq_, prev_, Adelta_})
            if (v) OPT_HIP_CHECK(hipMemset(v, 0, sizeof(T) * n_));
        flags_ = (uint8_t*)dmalloc(dom_.npix_mem());
        OPT_HIP_CHECK(hipMemset(flags_, 0, dom_.npix_mem()));
        red_.ensure(std::max(op_->stencil_blocks(), 4096), 2, 64);
        if constexpr (HasDumpJ<Op>::value) {
            if (opts_.materialized)
                mat_.reset(new MaterializedJacobian<T>(op_->jacobian_rows(), op_->jacobian_nnz(), n_,
                                                       opts_.fused_jtj));
        }
    }
    void release() {
        drop_graph();
        for (T** v : {&r_, &diag_, &pre_, &p_, &Ap_, &delta_, &b_, &CtC_, &SSq_, &prev_, &Adelta_}) {
            dfree(*v);
            *v = nullptr;
        }
        dfree(flags_);
        flags_ = nullptr;
        mat_.reset();
        op_.reset();
    }

    // bind + unknown halo + ComputedArrays, for the standalone entry points
    void prepare(void** params) {
        op_->bind(params, stream_);
        exchange_unknowns();
        op_->precompute(stream_);
        exchange_computed();
    }
    void precompute() {
        tbegin("precompute"); op_->precompute(stream_); tend();
        exchange_computed();
    }

    bool distributed() const { return comm_ && comm_->size() > 1; }
    void allreduce(int idx, int n) {
        if (distributed()) comm_->allreduce_sum(red_.scalars + idx, n, stream_);
    }
    void exchange(const std::vector<HaloPlane>& planes) {
        if (!distributed() || planes.empty()) return;
        tbegin("halo_exchange");
        comm_->halo_exchange(planes, dom_, op_->halo(), stream_);
        tend();
    }
    std::vector<HaloPlane> vec_planes(T* v) const {
        std::vector<HaloPlane> pl;
        for (int k = 0; k < L_.nimg; ++k) pl.push_back({(void*)(v + L_.off[k]), sizeof(T) * L_.ch[k] * dom_.W});
        return pl;
    }
    void exchange_vec(T* v) {
        if (!distributed()) return;
        exchange(vec_planes(v));
    }
    void exchange_unknowns() {
        if (!distributed()) return;
        std::vector<HaloPlane> pl;
        for (int k = 0; k < L_.nimg; ++k) pl.push_back({(void*)op_->unknown(k), sizeof(T) * L_.ch[k] * dom_.W});
        exchange(pl);
    }
    void exchange_computed() {
        if (!distributed()) return;
        std::vector<HaloPlane> pl;
        op_->computed_planes(pl);
        exchange(pl);
    }

    void launch_step2(bool first, int i_num, int i_den, int out, const int* stop, ZetaArgs z = {},
                      bool delta = true) {
        const int g = fg();
        const int use_pre = spec_.use_preconditioner ? 1 : 0;
        auto slot = red_.slot(g, out);
#define S2(F, LMV, D)                                                                                  \
    hipLaunchKernelGGL((step2_kernel<T, F, LMV, D>), dim3(g), dim3(kBlock), 0, stream_, n_, (const T*)p_, \
                       (const T*)Ap_, (const T*)pre_, (const T*)b_, r_, delta_, red_.scalars, i_num,    \
                       i_den, use_pre, stop, slot, z)
        if (first && lm_) S2(true, true, true);
        else if (lm_) S2(false, true, true);
        else if (!delta) S2(false, false, false);
        else if (first) S2(true, false, true);
        else S2(false, false, true);
#undef S2
    }
    UnknownPtrs<T> unknowns() {
        UnknownPtrs<T> X{};
        for (int k = 0; k < L_.nimg && k < 4; ++k) X.x[k] = op_->unknown(k);
        return X;
    }
    void update(bool save) {
        tbegin("update");
        if (save)
            hipLaunchKernelGGL((update_images_kernel<T, true>), dim3(fg()), dim3(kBlock), 0, stream_, L_,
                               (const uint8_t*)flags_, unknowns(), (const T*)delta_, prev_,
                               pix_lo(), pix_hi());
        else
            hipLaunchKernelGGL((update_images_kernel<T, false>), dim3(fg()), dim3(kBlock), 0, stream_, L_,
                               (const uint8_t*)flags_, unknowns(), (const T*)delta_, prev_,
                               pix_lo(), pix_hi());
        OPT_HIP_CHECK(hipGetLastError());
        tend();
        exchange_unknowns();
    }
    void revert() {
        hipLaunchKernelGGL((revert_images_kernel<T>), dim3(fg()), dim3(kBlock), 0, stream_, L_,
                           (const uint8_t*)flags_, unknowns(), (const T*)prev_, pix_lo(),
                           pix_hi());
        OPT_HIP_CHECK(hipGetLastError());
        exchange_unknowns();
    }
    // J at the current unknowns (saveJToCRS), then J^T (+ J^T J) values (cusparseOuter)
    void materialize() {
        if constexpr (HasDumpJ<Op>::value) {
            tbegin("saveJToCRS");
            op_->dump_j(mat_->rowPtrJ(), mat_->colIndJ(), mat_->valJ(), stream_);
            tend();
            mat_->build([this](const char* n, bool b) { if (b) tbegin(n); else tend(); }, stream_);
        }
    }
    void mat_apply(const T* p, T* Ap, const int* stop, int out) {
        PcgMask m{L_, (const uint8_t*)flags_, pix_lo(), pix_hi(), stop};
        mat_->apply(p, Ap, m, red_.slot(mat_->blocks(), out), [this](const char* n, bool b) {
            if (b) tbegin(n); else tend();
        }, stream_);
    }
    double read(int idx) { return read_device_scalar(red_.scalars + idx); }

    Domain dom_;
    std::unique_ptr<Op> op_;
    Comm* comm_ = nullptr;
    bool lm_ = false;
    VecLayout L_;
    long long n_ = 0;
    T *r_ = nullptr, *diag_ = nullptr, *pre_ = nullptr, *p_ = nullptr, *Ap_ = nullptr, *delta_ = nullptr;
    T *b_ = nullptr, *CtC_ = nullptr, *SSq_ = nullptr, *prev_ = nullptr, *Adelta_ = nullptr;
    uint8_t* flags_ = nullptr;
    int* stop_ = nullptr;
    hipGraphExec_t graph_exec_ = nullptr;      // captured PCG loop (pcg_graph_begin)
    std::vector<unsigned long long> graph_key_;
    bool capturing_ = false;
    const bool graph_off_ = getenv("OPT_AMD_NO_GRAPH") && atoi(getenv("OPT_AMD_NO_GRAPH"));
    const bool overlap_ = env_int("OPT_AMD_HALO_OVERLAP", 1) != 0;   // 0: blocking halo before each apply
    const bool fuse3_on_ = env_int("OPT_AMD_FUSE_STEP3", 1) != 0;
    // Ops with apply_sums: OPT_AMD_FUSE23=0 the classic apply / step2 / step3 loop, 1 the
    // fused loop, 2 (default) the fused loop on row slabs only. One GPU, shape_from_shading
    // 4096^2 LM: the apply with the four sums takes 175 us against 131 (r read back, 6
    // instead of 7 waves per SIMD), more than step3's pass saves: 3.56 vs 3.36 ms per step
    // (tools/r03_fuse23.sh). On slabs the fused loop saves an all-reduce per iteration.
    const int fuse23_ = env_int("OPT_AMD_FUSE23", 2);
    const bool delta3_on_ = env_int("OPT_AMD_DELTA_IN_STEP3", 1) != 0;   // 0: delta updated by step2    // 0: step3_kernel + the whole apply
    std::unique_ptr<MaterializedJacobian<T>> mat_;
    float radius_ = 1e4f, decrease_ = 2.0f;
};

// Plan factory for the generic driver: refuses useMaterializedJTJ for a family without
// a J assembly (the reference returns a nil plan on compile errors, o.t:1352,1526).
template <class Op>
std::unique_ptr<Plan> make_stencil_plan(const ProblemSpec& spec, const StateOptions& opts, Domain dom,
                                        std::string* err) {
    if (opts.materialized && !HasDumpJ<Op>::value) {
        *err = std::string(Op::kName) + ": no materialized Jacobian (useMaterializedJTJ) for this energy family";
        return nullptr;
    }
    return std::unique_ptr<Plan>(new StencilPlan<Op>(spec, opts, dom));
}

}  // namespace optamd
