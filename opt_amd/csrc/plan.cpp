// plan.cpp — Plan base class, solver parameters, kernel timer, reduction scratch.
#include <cstdlib>
#include <cstdarg>
#include "plan.h"
#include <cstring>
#include <sstream>
#include <iomanip>

namespace optamd {

void* dmalloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0) bytes = 16;
    OPT_HIP_CHECK(hipMalloc(&p, bytes));
    return p;
}
void dfree(void* p) {
    if (p) OPT_HIP_CHECK(hipFree(p));
}

bool SolverParams::set(const char* name, const void* v) {
#define F(x) if (!strcmp(name, #x)) { x = *(const float*)v; return true; }
#define I(x) if (!strcmp(name, #x)) { x = *(const int*)v; return true; }
    F(min_relative_decrease) F(min_trust_region_radius) F(max_trust_region_radius)
    F(q_tolerance) F(function_tolerance) F(trust_region_radius) F(radius_decrease_factor)
    F(min_lm_diagonal) F(max_lm_diagonal)
    I(residual_reset_period) I(nIterations) I(lIterations)
#undef F
#undef I
    return false;
}

// ---------------------------------------------------------------- KernelTimer
hipEvent_t KernelTimer::get_event() {
    if (!pool_.empty()) { hipEvent_t e = pool_.back(); pool_.pop_back(); return e; }
    hipEvent_t e;
    OPT_HIP_CHECK(hipEventCreate(&e));
    return e;
}
void KernelTimer::begin(hipStream_t s, const char* name) {
    if (mode == 0) return;
    if (mode == 2 && !timed(name)) return;
    open_ = name;
    open_ev_ = get_event();
    OPT_HIP_CHECK(hipEventRecord(open_ev_, s));
}
bool KernelTimer::ext_pair(const char* name, hipEvent_t* a, hipEvent_t* b) {
    if (mode == 0 || (mode == 2 && !timed(name))) return false;
    *a = get_event();
    *b = get_event();
    return true;
}
void KernelTimer::end(hipStream_t s) {
    if (!open_) return;
    hipEvent_t b = get_event();
    OPT_HIP_CHECK(hipEventRecord(b, s));
    pending_.push_back({open_, open_ev_, b});
    open_ = nullptr;
    if (pending_.size() > 4096) flush();
}
void KernelTimer::flush() {
    for (auto& p : pending_) {
        OPT_HIP_CHECK(hipEventSynchronize(p.b));
        float ms = 0.f;
        OPT_HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
        auto& a = acc_[p.name];
        a.first += 1;
        a.second += ms;
        pool_.push_back(p.a);
        pool_.push_back(p.b);
    }
    pending_.clear();
}
void KernelTimer::reset() { flush(); acc_.clear(); }
bool KernelTimer::stat(const std::string& name, long long* n, double* ms) {
    flush();
    auto it = acc_.find(name);
    if (it == acc_.end()) { *n = 0; *ms = 0; return false; }
    *n = it->second.first;
    *ms = it->second.second;
    return true;
}
std::string KernelTimer::report() {
    flush();
    std::ostringstream o;
    o << "--------------------------------------------------------------\n";
    o << std::left << std::setw(34) << "Kernel" << std::right << std::setw(8) << "Count"
      << std::setw(12) << "Total(ms)" << std::setw(12) << "Avg(us)" << "\n";
    double total = 0;
    for (auto& kv : acc_) {
        o << std::left << std::setw(34) << kv.first << std::right << std::setw(8)
          << kv.second.first << std::setw(12) << std::fixed << std::setprecision(3)
          << kv.second.second << std::setw(12) << std::setprecision(2)
          << 1000.0 * kv.second.second / std::max(1LL, kv.second.first) << "\n";
        total += kv.second.second;
    }
    o << "TIMING total " << std::setprecision(3) << total << " ms\n";
    return o.str();
}
KernelTimer::~KernelTimer() {
    for (auto& p : pending_) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : pool_) (void)hipEventDestroy(e);
}

// ------------------------------------------------------------- ReduceScratch
int Plan::scalars(double* out, int n) {
    const int k = std::min(n, red_.n_scalars);
    OPT_HIP_CHECK(hipStreamSynchronize(stream_));
    if (k > 0) OPT_HIP_CHECK(hipMemcpy(out, red_.scalars, sizeof(double) * k, hipMemcpyDeviceToHost));
    return std::max(k, 0);
}

void ReduceScratch::ensure(int mb, int kmax, int ns) {
    (void)kmax;   // partials hold kMaxReduce rows of max_blocks: any K <= kMaxReduce fits
    if (mb > max_blocks || !partials) {
        dfree(partials);
        max_blocks = std::max(mb, max_blocks);
        partials = (double*)dmalloc(sizeof(double) * (size_t)max_blocks * kMaxReduce);
    }
    if (!ticket) {
        ticket = (unsigned*)dmalloc(sizeof(unsigned) * kTicketWords);
        OPT_HIP_CHECK(hipMemset(ticket, 0, sizeof(unsigned) * kTicketWords));
    }
    if (ns > n_scalars) {
        // grown (lIterations raised between Steps): the old values move along
        double* s = (double*)dmalloc(sizeof(double) * ns);
        OPT_HIP_CHECK(hipMemset(s, 0, sizeof(double) * ns));
        if (scalars) {
            OPT_HIP_CHECK(hipDeviceSynchronize());
            OPT_HIP_CHECK(hipMemcpy(s, scalars, sizeof(double) * n_scalars, hipMemcpyDeviceToDevice));
        }
        dfree(scalars);
        scalars = s;
        n_scalars = ns;
    }
}
ReduceScratch::~ReduceScratch() {
    dfree(partials);
    dfree(ticket);
    dfree(scalars);
}

// ----------------------------------------------------------------------- Plan
Plan::Plan(const ProblemSpec& spec, const StateOptions& opts) : spec_(spec), opts_(opts) {
    OPT_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    timer_.mode = opts.kernel_timing ? 1 : 0;
    if (const char* v = getenv("OPT_AMD_HOST_SYNC")) host_sync_ = atoi(v);
}

Plan::~Plan() {
    if (halo_stream_) {
        OPT_HIP_CHECK(hipStreamSynchronize(halo_stream_));
        OPT_HIP_CHECK(hipStreamDestroy(halo_stream_));
    }
    for (hipEvent_t e : halo_ev_)
        if (e) OPT_HIP_CHECK(hipEventDestroy(e));
    if (pinned_) (void)hipHostFree(pinned_);
}

void Plan::halo_mark() {
    if (!halo_stream_) {
        OPT_HIP_CHECK(hipStreamCreateWithFlags(&halo_stream_, hipStreamNonBlocking));
        for (hipEvent_t& e : halo_ev_) OPT_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    OPT_HIP_CHECK(hipEventRecord(halo_ev_[0], stream_));
}
void Plan::halo_begin(Comm* comm, const std::vector<HaloPlane>& planes, const Domain& dom, int halo) {
    OPT_HIP_CHECK(hipStreamWaitEvent(halo_stream_, halo_ev_[0], 0));
    comm->halo_exchange(planes, dom, halo, halo_stream_);
    OPT_HIP_CHECK(hipEventRecord(halo_ev_[1], halo_stream_));
}
void Plan::halo_join() { OPT_HIP_CHECK(hipStreamWaitEvent(stream_, halo_ev_[1], 0)); }

void Plan::set_solver_param(const char* name, const void* value) {
    if (!sp_.set(name, value))
        fprintf(stderr, "Warning: tried to set nonexistent solver parameter %s\n", name);
}

void Plan::begin_call() {
    // Order this plan's stream after everything the caller queued on the default
    // stream (the reference runs all device work on the default stream). Nothing to order
    // after when that stream has finished its work (OPT_AMD_HOST_SYNC bit 0).
    if ((host_sync_ & 1) && hipStreamQuery(nullptr) == hipSuccess) return;
    hipEvent_t e;
    OPT_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    OPT_HIP_CHECK(hipEventRecord(e, 0));
    OPT_HIP_CHECK(hipStreamWaitEvent(stream_, e, 0));
    OPT_HIP_CHECK(hipEventDestroy(e));
}
void Plan::log_solver(const char* fmt, ...) {
    if (opts_.verbosity <= 0) return;
    va_list ap;
    va_start(ap, fmt);
    vprintf(fmt, ap);
    va_end(ap);
    fflush(stdout);
}
void Plan::cleanup_log() {
    if (opts_.verbosity <= 0) return;
    printf("final cost=%.16f\n", prev_cost_);
    if (opts_.kernel_timing) printf("%s", timer_.report().c_str());
    fflush(stdout);
}

double Plan::read_device_scalar(const double* dev) {
    double v = 0.0;
    double* dst = &v;
    if (host_sync_ & 2) {
        if (!pinned_) OPT_HIP_CHECK(hipHostMalloc((void**)&pinned_, sizeof(double), hipHostMallocDefault));
        dst = pinned_;
    }
    OPT_HIP_CHECK(hipMemcpyAsync(dst, dev, sizeof(double), hipMemcpyDeviceToHost, stream_));
    if (host_sync_ & 4) {
        hipError_t q;
        while ((q = hipStreamQuery(stream_)) == hipErrorNotReady) {
        }
        OPT_HIP_CHECK(q);
    } else {
        OPT_HIP_CHECK(hipStreamSynchronize(stream_));
    }
    return *dst;
}
void Plan::end_call() {
    OPT_HIP_CHECK(hipStreamSynchronize(stream_));
    OPT_HIP_CHECK(hipGetLastError());
}
void Plan::drain() noexcept {
    (void)hipStreamSynchronize(stream_);
}

std::unique_ptr<Plan> make_plan(const ProblemSpec& spec, const StateOptions& opts,
                                const unsigned* dims, std::string* err) {
    if (spec.family == "image_warping") return make_image_warping_plan(spec, opts, dims, err);
    if (spec.family == "poisson_image_editing") return make_poisson_plan(spec, opts, dims, err);
    if (spec.family == "optical_flow") return make_optical_flow_plan(spec, opts, dims, err);
    if (spec.family == "shape_from_shading") return make_sfs_plan(spec, opts, dims, err);
    if (spec.family == "arap_mesh_deformation") return make_arap_plan(spec, opts, dims, err);
    if (spec.family == "generic") return make_generic_plan(spec, opts, dims, err);
    *err = "energy family '" + spec.family + "' has no kernels in this build";
    return nullptr;
}

}  // namespace optamd
