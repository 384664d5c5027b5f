// plan.h — the solver plan interface behind Opt_Plan, the GN/LM solver parameters,
// per-kernel timing, and the device scratch every family shares.
#pragma once
#include <hip/hip_runtime.h>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>
#include "comm.h"
#include "common.h"
#include "problem.h"

namespace optamd {

// A problem the plan cannot run, found when the arrays are bound (Init / Step) rather
// than at Opt_ProblemPlan (e.g. an arap graph whose adjacency exceeds the 32-bit index
// range): thrown by the plan, caught at the C ABI (opt_api.cpp), which reports it on
// stderr and through OptAMD_PlanError and stops the solve instead of the process.
struct PlanError : std::runtime_error {
    using std::runtime_error::runtime_error;
};


// Runtime solver parameters with the reference defaults
// (API/src/solverGPUGaussNewton.t:41-55, struct SolverParameters :186-201).
struct SolverParams {
    float min_relative_decrease = 1e-3f;
    float min_trust_region_radius = 1e-32f;
    float max_trust_region_radius = 1e16f;
    float q_tolerance = 0.0001f;
    float function_tolerance = 0.000001f;
    float trust_region_radius = 1e4f;
    float radius_decrease_factor = 2.0f;
    float min_lm_diagonal = 1e-6f;
    float max_lm_diagonal = 1e32f;
    int residual_reset_period = 10;
    int nIterations = 10;
    int lIterations = 10;
    // strcmp dispatch as setSolverParameter (solverGPUGaussNewton.t:2382-2398).
    bool set(const char* name, const void* value);
};

struct StateOptions {
    bool double_precision = false;
    int verbosity = 0;
    bool kernel_timing = false;
    bool host_buffers = false;   // backend_cpu / backend_cpu_mt: params are host pointers
    std::string backend = "backend_cuda";
    // useMaterializedJTJ / useFusedJTJ (Opt.h:32-34): J assembled in CSR every step and
    // the PCG apply done as J^T J p (fused: one SpMV with the assembled J^T J) or
    // J^T (J p) (two SpMVs) — solverGPUGaussNewton.t:1532-1757.
    bool materialized = false;
    bool fused_jtj = false;
};

// hipEvent-pair accounting per kernel name (reference Timer, backend_cuda.t:152-297).
class KernelTimer {
public:
    int mode = 0;  // 0 off, 1 all kernels, 2 apply kernel (+ aux_names) only
    std::string apply_name;
    std::vector<std::string> aux_names;   // more kernels mode 2 times (image_warping: its fused passes)
    bool timed(const char* name) const {
        if (apply_name == name) return true;
        for (auto& n : aux_names) if (n == name) return true;
        return false;
    }
    void begin(hipStream_t s, const char* name);
    void end(hipStream_t s);
    // Event pair to attach to the launch itself (hipExtLaunchKernel): the timestamps come
    // from the kernel's own dispatch, with no marker packets between kernels.
    // Returns false when `name` is not timed; else record() after the launch.
    bool ext_pair(const char* name, hipEvent_t* a, hipEvent_t* b);
    void ext_record(const char* name, hipEvent_t a, hipEvent_t b) { pending_.push_back({name, a, b}); }
    void flush();  // resolve recorded pairs (synchronises)
    void reset();
    bool stat(const std::string& name, long long* n, double* ms);
    std::string report();
    ~KernelTimer();
private:
    struct Pending { std::string name; hipEvent_t a, b; };
    std::vector<Pending> pending_;
    std::vector<hipEvent_t> pool_;
    const char* open_ = nullptr;
    hipEvent_t open_ev_ = nullptr;
    std::map<std::string, std::pair<long long, double>> acc_;
    hipEvent_t get_event();
};

// Device scratch for the deterministic reductions (common.h ReduceSlot).
struct ReduceScratch {
    double* partials = nullptr;
    unsigned* ticket = nullptr;
    double* scalars = nullptr;
    int max_blocks = 0;
    int n_scalars = 0;
    void ensure(int max_blocks, int k_max, int n_scalars);
    ReduceSlot slot(int nblocks, int scalar_index) const {
        return ReduceSlot{partials, ticket, scalars + scalar_index, nblocks};
    }
    ~ReduceScratch();
};

class Plan {
public:
    virtual ~Plan();
    virtual void init(void** params) = 0;
    virtual int step(void** params) = 0;
    virtual double cost() const { return prev_cost_; }
    virtual long long unknown_count() const = 0;
    virtual std::string family() const = 0;
    virtual int eval_jtf(void** params, void* r, void* pre, double* rz) = 0;
    virtual int apply_jtj(void** params, const void* p, void* Ap, double* pAp) = 0;
    virtual double eval_cost(void** params) = 0;
    virtual double time_apply(void** params, const void* p, void* Ap, int reps) = 0;
    virtual std::string apply_kernel_name() const = 0;
    // Row-slab decomposition (image domains): this rank owns global rows [y_lo, y_hi)
    // and the caller's arrays hold rows [y_lo - halo_lo, y_hi + halo_hi) with
    // halo_lo = min(halo, y_lo), halo_hi = min(halo, H - y_hi). Returns an error text
    // (empty on success).
    virtual std::string set_decomposition(Comm* comm, int y_lo, int y_hi) {
        (void)comm; (void)y_lo; (void)y_hi;
        return "this energy family does not support row-slab decomposition";
    }
    virtual int halo() const { return 0; }
    // Materialized Jacobian (saveJToCRS, solverGPUGaussNewton.t:1004-1022): nonzeros
    // (-1: the family has no J assembly) and *rows = residual count.
    virtual long long jacobian_shape(long long* rows) const { if (rows) *rows = 0; return -1; }
    // Sizes of the plan's materialized J and J^T J (0 before the first step); false when
    // the plan runs matrix-free.
    virtual bool materialized_nonzeros(long long* nnzJ, long long* nnzJTJ) const {
        (void)nnzJ; (void)nnzJTJ;
        return false;
    }
    // J at the current unknowns into caller device arrays (rowPtr rows+1, colInd/val nnz).
    virtual int eval_jacobian(void** params, int* rowPtr, int* colInd, void* val) {
        (void)params; (void)rowPtr; (void)colInd; (void)val;
        return 1;
    }

    void set_solver_param(const char* name, const void* value);
    // the device scalar slots (red_.scalars) to the host, up to n; the count copied
    int scalars(double* out, int n);
    int iterations() const { return n_iter_; }
    hipStream_t stream() const { return stream_; }
    KernelTimer& timer() { return timer_; }
    void drain() noexcept;          // end_call after a throw (opt_api.cpp: guarded): waits, reports nothing

protected:
    Plan(const ProblemSpec& spec, const StateOptions& opts);
    void begin_call();              // order after the caller's default-stream work
    void end_call();                // wait for this plan's device work
    // One device double to the host, waiting for stream_'s work (the Step's cost): with
    // OPT_AMD_HOST_SYNC bit 1 through a pinned host word (no staging copy), bit 2 waiting by
    // polling the stream instead of hipStreamSynchronize
    double read_device_scalar(const double* dev);
    // Launch bookkeeping: wraps a kernel launch with the timer when enabled.
    // The reference's cleanup (solverGPUGaussNewton.t:1902-1910), run when Step returns 0:
    // with verbosityLevel > 0 it logs "final cost=%.16f" (the line the examples' test
    // harness parses, examples/test_final_cost.py:100-103) and the per-kernel timing table.
    void cleanup_log();
    // logSolver: printf to stdout when verbosityLevel > 0 (o.t:95-104)
    void log_solver(const char* fmt, ...);
    // Halo refresh overlapped with interior work (row slabs): halo_mark() marks stream_'s
    // work so far; the interior launches follow on stream_ (they read no halo row and
    // write none of the exchanged rows); halo_begin() runs the exchange on a second
    // stream ordered after the mark only (RCCL: queued; LocalGroup: host copies while the
    // interior kernels run); halo_join() makes stream_ wait for it before the boundary
    // launches. The plan's collectives keep one total order (each is ordered after the
    // previous through stream_ and these events), as RCCL requires.
    void halo_mark();
    void halo_begin(Comm* comm, const std::vector<HaloPlane>& planes, const Domain& dom, int halo);
    void halo_join();
    void tbegin(const char* name) { if (timer_.mode) timer_.begin(stream_, name); }
    void tend() { if (timer_.mode) timer_.end(stream_); }

    ProblemSpec spec_;
    StateOptions opts_;
    SolverParams sp_;
    hipStream_t stream_ = nullptr;
    hipStream_t halo_stream_ = nullptr;           // created on first halo_begin
    hipEvent_t halo_ev_[2] = {nullptr, nullptr};  // stream_ -> halo stream, halo stream -> stream_
    KernelTimer timer_;
    ReduceScratch red_;
    double prev_cost_ = 0.0;
    // OPT_AMD_HOST_SYNC: bit 0 begin_call skips the default-stream event when that stream is
    // idle (hipStreamQuery), bit 1 pinned read-back, bit 2 polled wait (read_device_scalar)
    int host_sync_ = 3;   // same box: GN step 3.008 / 3.030 -> 2.986 / 2.993 ms with 3 (7: 2.993 / 2.987)
    double* pinned_ = nullptr;
    int n_iter_ = 0;
    bool initialised_ = false;
};

// Factory: lower a parsed problem to a plan for the given dims (nullptr + message on
// failure, as problemPlan returns nil on compile errors, o.t:1352,1526).
std::unique_ptr<Plan> make_plan(const ProblemSpec& spec, const StateOptions& opts,
                                const unsigned* dims, std::string* err);

// Per-family factories.
std::unique_ptr<Plan> make_image_warping_plan(const ProblemSpec&, const StateOptions&,
                                              const unsigned* dims, std::string* err);

std::unique_ptr<Plan> make_poisson_plan(const ProblemSpec&, const StateOptions&,
                                        const unsigned* dims, std::string* err);

std::unique_ptr<Plan> make_optical_flow_plan(const ProblemSpec&, const StateOptions&,
                                             const unsigned* dims, std::string* err);

std::unique_ptr<Plan> make_sfs_plan(const ProblemSpec&, const StateOptions&, const unsigned* dims,
                                    std::string* err);

std::unique_ptr<Plan> make_arap_plan(const ProblemSpec&, const StateOptions&, const unsigned* dims,
                                     std::string* err);

std::unique_ptr<Plan> make_generic_plan(const ProblemSpec&, const StateOptions&, const unsigned* dims,
                                        std::string* err);

// Device-memory helpers (fail-stop).
void* dmalloc(size_t bytes);
void dfree(void* p);

}  // namespace optamd
