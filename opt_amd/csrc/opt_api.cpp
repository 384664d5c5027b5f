// opt_api.cpp — the Opt.h C ABI (reference API/release/include/Opt.h, implemented in
// the reference by the trampolines of API/src/createwrapper.t:291-305 into
// API/src/o.t:3301-3352) plus the opt_amd.h extension entry points.
#include <algorithm>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>
#include "../../include/Opt.h"
#include "../../include/opt_amd.h"
#include "csr.h"
#include "plan.h"
#include "problem.h"

static_assert(sizeof(Opt_InitializationParameters) == 44,
              "Opt_InitializationParameters must keep the reference layout (Opt.h:10-35)");

struct Opt_State {
    optamd::StateOptions opts;
    int device = 0;
};
struct Opt_Problem {
    optamd::ProblemSpec spec;
};
struct Opt_Plan {
    std::unique_ptr<optamd::Plan> impl;
    std::string error;   // set when Init / Step met an optamd::PlanError; the solve stops
};

namespace {
bool valid_state(Opt_State* s, const char* fn) {
    if (!s) { fprintf(stderr, "[opt_amd] %s: null Opt_State\n", fn); return false; }
    return true;
}
bool valid_plan(Opt_Plan* p, const char* fn) {
    if (!p || !p->impl) { fprintf(stderr, "[opt_amd] %s: null Opt_Plan\n", fn); return false; }
    return true;
}
}  // namespace

// Every entry point that binds the caller's arrays (and so may raise a PlanError, e.g. the
// ARAP adjacency limit found by build_csr inside bind) runs its body through guarded(): no
// C++ exception crosses the extern "C" frame into the caller (ctypes, cgo, C), the plan's
// stream is drained of whatever the call had queued before the throw (its begin_call /
// end_call pair did not complete), and the call returns its error value.
template <typename F, typename R>
static R guarded(Opt_Plan* plan, const char* fn, R err, F&& body) {
    try {
        return body();
    } catch (const std::exception& e) {
        plan->error = e.what();
        fprintf(stderr, "[opt_amd] %s: %s\n", fn, e.what());
        plan->impl->drain();
        return err;
    }
}

extern "C" {

Opt_State* Opt_NewState(Opt_InitializationParameters params) {
    auto* s = new Opt_State();
    char backend[21];
    memcpy(backend, params.backend, 20);
    backend[20] = 0;
    std::string b = backend;
    if (b.empty()) b = "backend_cuda";
    if (b != "backend_cuda" && b != "backend_cpu" && b != "backend_cpu_mt") {
        fprintf(stderr, "[opt_amd] unknown backend '%s' (backend_cuda | backend_cpu | backend_cpu_mt)\n",
                b.c_str());
        delete s;
        return nullptr;
    }
    s->opts.backend = b;
    s->opts.host_buffers = (b != "backend_cuda");
    s->opts.double_precision = params.doublePrecision != 0;
    s->opts.verbosity = params.verbosityLevel;
    s->opts.kernel_timing = params.collectPerKernelTimingInfo != 0;
    s->opts.materialized = params.useMaterializedJTJ != 0;
    s->opts.fused_jtj = params.useFusedJTJ != 0;
    return s;
}

Opt_Problem* Opt_ProblemDefine(Opt_State* state, const char* filename, const char* solverkind) {
    if (!valid_state(state, "Opt_ProblemDefine")) return nullptr;
    std::string kind = solverkind ? solverkind : "";
    if (kind != "gaussNewtonGPU" && kind != "LMGPU" && kind != "gaussNewtonCPU") {
        fprintf(stderr, "[opt_amd] unknown solver kind '%s' (gaussNewtonGPU | LMGPU | gaussNewtonCPU)\n",
                kind.c_str());
        return nullptr;
    }
    std::ifstream in(filename ? filename : "");
    if (!in.good()) {
        fprintf(stderr, "[opt_amd] cannot read energy file '%s'\n", filename ? filename : "(null)");
        return nullptr;
    }
    std::stringstream ss;
    ss << in.rdbuf();
    auto* p = new Opt_Problem();
    p->spec.filename = filename;
    p->spec.solverkind = kind;
    p->spec.text = ss.str();
    std::string err;
    bool ok = optamd::parse_energy(ss.str(), &p->spec, &err) && optamd::classify(&p->spec, &err);
    // A hand-written family serves the file only if the file lowers to exactly that
    // family's residual templates (the reference derives every kernel from the file,
    // o.t:1295-1348); any other energy, and every energy with OPT_AMD_GENERIC=1, goes to
    // the general front end.
    if (ok) {
        std::string why;
        if (!optamd::family_is_canonical(&p->spec, &why)) {
            if (state->opts.verbosity > 0)
                fprintf(stderr, "[opt_amd] %s: not the %s family's energy (%s); using generated kernels\n",
                        filename, p->spec.family.c_str(), why.c_str());
            err = why;
            ok = false;
        }
    }
    if (!ok || optamd::env_int("OPT_AMD_GENERIC", 0)) {
        std::string gerr;
        if (optamd::generic_accepts(ss.str(), &p->spec, &gerr)) {
            ok = true;
        } else if (!ok) {
            err += "; general front end: " + gerr;
        }
    }
    if (!ok) {
        fprintf(stderr, "[opt_amd] %s\n", err.c_str());
        delete p;
        return nullptr;
    }
    return p;
}

void Opt_ProblemDelete(Opt_State*, Opt_Problem* problem) { delete problem; }

Opt_Plan* Opt_ProblemPlan(Opt_State* state, Opt_Problem* problem, unsigned int* dimensions) {
    if (!valid_state(state, "Opt_ProblemPlan")) return nullptr;
    if (!problem || !dimensions) {
        fprintf(stderr, "[opt_amd] Opt_ProblemPlan: null problem or dimensions\n");
        return nullptr;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        fprintf(stderr, "[opt_amd] Opt_ProblemPlan: no HIP device (this runtime has no CPU compute path)\n");
        return nullptr;
    }
    OPT_HIP_CHECK(hipGetDevice(&state->device));
    std::string err;
    auto impl = optamd::make_plan(problem->spec, state->opts, dimensions, &err);
    if (!impl && problem->spec.family != "generic") {
        // a hand-written family that cannot serve these options (e.g. useMaterializedJTJ
        // for shape_from_shading): the generated kernels of the same energy can
        optamd::ProblemSpec g = problem->spec;
        std::string gerr;
        if (optamd::generic_accepts(g.text, &g, &gerr)) {
            impl = optamd::make_plan(g, state->opts, dimensions, &gerr);
            if (impl) err.clear();
            else err += "; generated kernels: " + gerr;
        }
    }
    if (!impl) {
        fprintf(stderr, "[opt_amd] plan failed: %s\n", err.c_str());
        return nullptr;
    }
    auto* p = new Opt_Plan();
    p->impl = std::move(impl);
    return p;
}

void Opt_PlanFree(Opt_State*, Opt_Plan* plan) { delete plan; }

void Opt_SetSolverParameter(Opt_State* state, Opt_Plan* plan, const char* name, void* value) {
    if (!valid_state(state, "Opt_SetSolverParameter") || !valid_plan(plan, "Opt_SetSolverParameter"))
        return;
    if (!name || !value) return;
    plan->impl->set_solver_param(name, value);
}

// A PlanError (a problem the plan cannot run, found when the arrays are bound) stops the
// solve, not the process: Init returns, every later Step returns 0 (the reference's "no
// more steps"), Opt_ProblemCurrentCost returns NaN and OptAMD_PlanError the message.
void Opt_ProblemInit(Opt_State* state, Opt_Plan* plan, void** problemparams) {
    if (!valid_state(state, "Opt_ProblemInit") || !valid_plan(plan, "Opt_ProblemInit")) exit(1);
    plan->error.clear();
    guarded(plan, "Opt_ProblemInit", 0, [&] {
        plan->impl->init(problemparams);
        return 0;
    });
}

int Opt_ProblemStep(Opt_State* state, Opt_Plan* plan, void** problemparams) {
    if (!valid_state(state, "Opt_ProblemStep") || !valid_plan(plan, "Opt_ProblemStep")) exit(1);
    if (!plan->error.empty()) return 0;
    return guarded(plan, "Opt_ProblemStep", 0, [&] { return plan->impl->step(problemparams); });
}

void Opt_ProblemSolve(Opt_State* state, Opt_Plan* plan, void** problemparams) {
    Opt_ProblemInit(state, plan, problemparams);
    while (Opt_ProblemStep(state, plan, problemparams)) {
    }
}

double Opt_ProblemCurrentCost(Opt_State* state, Opt_Plan* plan) {
    if (!valid_state(state, "Opt_ProblemCurrentCost") || !valid_plan(plan, "Opt_ProblemCurrentCost"))
        return 0.0;
    if (!plan->error.empty()) return std::nan("");
    return plan->impl->cost();
}

// ------------------------------------------------------------------ extensions
long long OptAMD_PlanUnknownCount(Opt_Plan* plan) {
    return valid_plan(plan, "OptAMD_PlanUnknownCount") ? plan->impl->unknown_count() : -1;
}
static int copy_name(const std::string& s, char* buf, int n) {
    if (buf && n > 0) {
        strncpy(buf, s.c_str(), n - 1);
        buf[n - 1] = 0;
    }
    return (int)s.size();
}
int OptAMD_PlanFamily(Opt_Plan* plan, char* buf, int n) {
    return valid_plan(plan, "OptAMD_PlanFamily") ? copy_name(plan->impl->family(), buf, n) : -1;
}
int OptAMD_ProblemFamily(Opt_Problem* problem, char* buf, int n) {
    if (!problem) { fprintf(stderr, "[opt_amd] OptAMD_ProblemFamily: null Opt_Problem\n"); return -1; }
    return copy_name(problem->spec.family, buf, n);
}
int OptAMD_EvalJTF(Opt_State* state, Opt_Plan* plan, void** params, void* r, void* pre, double* rz) {
    if (!valid_state(state, "OptAMD_EvalJTF") || !valid_plan(plan, "OptAMD_EvalJTF") || !r || !pre)
        return 1;
    double t = 0;
    int e = guarded(plan, "OptAMD_EvalJTF", 1, [&] { return plan->impl->eval_jtf(params, r, pre, &t); });
    if (rz) *rz = t;
    return e;
}
int OptAMD_ApplyJTJ(Opt_State* state, Opt_Plan* plan, void** params, const void* p, void* Ap,
                    double* pAp) {
    if (!valid_state(state, "OptAMD_ApplyJTJ") || !valid_plan(plan, "OptAMD_ApplyJTJ") || !p || !Ap)
        return 1;
    double t = 0;
    int e = guarded(plan, "OptAMD_ApplyJTJ", 1, [&] { return plan->impl->apply_jtj(params, p, Ap, &t); });
    if (pAp) *pAp = t;
    return e;
}
double OptAMD_EvalCost(Opt_State* state, Opt_Plan* plan, void** params) {
    if (!valid_state(state, "OptAMD_EvalCost") || !valid_plan(plan, "OptAMD_EvalCost")) return -1.0;
    return guarded(plan, "OptAMD_EvalCost", -1.0, [&] { return plan->impl->eval_cost(params); });
}
double OptAMD_TimeApplyJTJ(Opt_State* state, Opt_Plan* plan, void** params, const void* p, void* Ap,
                           int reps) {
    if (!valid_state(state, "OptAMD_TimeApplyJTJ") || !valid_plan(plan, "OptAMD_TimeApplyJTJ"))
        return -1.0;
    return guarded(plan, "OptAMD_TimeApplyJTJ", -1.0, [&] { return plan->impl->time_apply(params, p, Ap, reps); });
}
void OptAMD_SetKernelTiming(Opt_Plan* plan, int mode) {
    if (!valid_plan(plan, "OptAMD_SetKernelTiming")) return;
    plan->impl->timer().reset();
    plan->impl->timer().mode = mode;
}
int OptAMD_KernelStat(Opt_Plan* plan, const char* name, long long* n, double* ms) {
    if (!valid_plan(plan, "OptAMD_KernelStat") || !name) return 1;
    long long nn;
    double mm;
    bool ok = plan->impl->timer().stat(name, &nn, &mm);
    if (n) *n = nn;
    if (ms) *ms = mm;
    return ok ? 0 : 1;
}
int OptAMD_ApplyKernelName(Opt_Plan* plan, char* buf, int n) {
    return valid_plan(plan, "OptAMD_ApplyKernelName") ? copy_name(plan->impl->apply_kernel_name(), buf, n)
                                                      : -1;
}
int OptAMD_KernelReport(Opt_Plan* plan, char* buf, int n) {
    return valid_plan(plan, "OptAMD_KernelReport") ? copy_name(plan->impl->timer().report(), buf, n) : -1;
}
void* OptAMD_PlanStream(Opt_Plan* plan) {
    return valid_plan(plan, "OptAMD_PlanStream") ? (void*)plan->impl->stream() : nullptr;
}
int OptAMD_PlanIterations(Opt_Plan* plan) {
    return valid_plan(plan, "OptAMD_PlanIterations") ? plan->impl->iterations() : -1;
}

int OptAMD_PlanScalars(Opt_Plan* plan, double* out, int n) {
    return valid_plan(plan, "OptAMD_PlanScalars") && out ? plan->impl->scalars(out, n) : -1;
}

struct OptAMD_Comm {
    optamd::Comm* impl;
    bool owned;
};
struct OptAMD_LocalGroup {
    optamd::LocalGroup* impl;
    std::vector<OptAMD_Comm> ranks;
};

int OptAMD_RcclUniqueId(void* out128) {
    std::string err;
    if (!out128 || !optamd::rccl_unique_id(out128, &err)) {
        fprintf(stderr, "[opt_amd] %s\n", err.c_str());
        return 1;
    }
    return 0;
}
OptAMD_Comm* OptAMD_CommCreateRccl(const void* id128, int rank, int nranks) {
    std::string err;
    optamd::Comm* c = optamd::make_rccl_comm(id128, rank, nranks, &err);
    if (!c) {
        fprintf(stderr, "[opt_amd] %s\n", err.c_str());
        return nullptr;
    }
    return new OptAMD_Comm{c, true};
}
void OptAMD_CommDestroy(OptAMD_Comm* comm) {
    if (!comm) return;
    if (comm->owned) { delete comm->impl; delete comm; }
}
int OptAMD_CommSize(OptAMD_Comm* comm) { return comm ? comm->impl->size() : -1; }
int OptAMD_CommRank(OptAMD_Comm* comm) { return comm ? comm->impl->rank() : -1; }
int OptAMD_PlanError(Opt_Plan* plan, char* buf, int n) {
    return valid_plan(plan, "OptAMD_PlanError") ? copy_name(plan->error, buf, n) : -1;
}
int OptAMD_CommKind(OptAMD_Comm* comm, char* buf, int n) { return comm ? copy_name(comm->impl->kind(), buf, n) : -1; }
OptAMD_LocalGroup* OptAMD_LocalGroupCreate(int nranks) {
    if (nranks < 1) return nullptr;
    auto* g = new OptAMD_LocalGroup();
    g->impl = optamd::make_local_group(nranks);
    for (int r = 0; r < nranks; ++r) g->ranks.push_back(OptAMD_Comm{optamd::local_group_rank(g->impl, r), false});
    return g;
}
OptAMD_Comm* OptAMD_LocalGroupRank(OptAMD_LocalGroup* g, int rank) {
    if (!g || rank < 0 || rank >= (int)g->ranks.size()) return nullptr;
    return &g->ranks[rank];
}
void OptAMD_LocalGroupDestroy(OptAMD_LocalGroup* g) {
    if (!g) return;
    optamd::destroy_local_group(g->impl);
    delete g;
}
int OptAMD_PlanHalo(Opt_Plan* plan) {
    return valid_plan(plan, "OptAMD_PlanHalo") ? plan->impl->halo() : -1;
}
int OptAMD_PlanSetDecomposition(Opt_Plan* plan, OptAMD_Comm* comm, int y_lo, int y_hi) {
    if (!valid_plan(plan, "OptAMD_PlanSetDecomposition") || !comm) return 1;
    std::string err = plan->impl->set_decomposition(comm->impl, y_lo, y_hi);
    if (!err.empty()) {
        fprintf(stderr, "[opt_amd] OptAMD_PlanSetDecomposition: %s\n", err.c_str());
        return 1;
    }
    return 0;
}

long long OptAMD_PlanJacobianShape(Opt_Plan* plan, long long* nResiduals) {
    if (!valid_plan(plan, "OptAMD_PlanJacobianShape")) return -1;
    return plan->impl->jacobian_shape(nResiduals);
}
int OptAMD_PlanMaterializedNonzeros(Opt_Plan* plan, long long* nnzJ, long long* nnzJTJ) {
    if (!valid_plan(plan, "OptAMD_PlanMaterializedNonzeros")) return 1;
    return plan->impl->materialized_nonzeros(nnzJ, nnzJTJ) ? 0 : 1;
}
int OptAMD_EvalJacobian(Opt_State* state, Opt_Plan* plan, void** params, int* rowPtr, int* colInd, void* val) {
    if (!valid_state(state, "OptAMD_EvalJacobian") || !valid_plan(plan, "OptAMD_EvalJacobian") || !rowPtr ||
        !colInd || !val)
        return 1;
    return guarded(plan, "OptAMD_EvalJacobian", 1, [&] { return plan->impl->eval_jacobian(params, rowPtr, colInd, val); });
}

// ---- sparse building blocks (synchronous, on the null stream) -------------------
static bool csr_args_ok(const char* fn, int rows, int cols, long long nnz) {
    if (rows < 0 || cols < 0 || nnz < 0 || nnz >= (1LL << 31) - 1) {
        fprintf(stderr, "[opt_amd] %s: invalid CSR shape %d x %d, nnz %lld\n", fn, rows, cols, nnz);
        return false;
    }
    return true;
}
int OptAMD_CsrTranspose(int nRowsA, int nColsA, long long nnz, const int* rowPtrA, const int* colIndA,
                        const void* valA, int* rowPtrAT, int* colIndAT, void* valAT, int doublePrecision) {
    if (!csr_args_ok("OptAMD_CsrTranspose", nRowsA, nColsA, nnz) || !rowPtrA || !rowPtrAT) return 1;
    optamd::DevBuf scratch;
    int* perm = (int*)optamd::dmalloc(sizeof(int) * std::max(nnz, 1LL));
    optamd::csr_transpose_pattern(nRowsA, nColsA, nnz, rowPtrA, colIndA, rowPtrAT, colIndAT, perm, scratch, nullptr);
    if (valA && valAT) {
        if (doublePrecision) optamd::csr_gather<double>(nnz, perm, (const double*)valA, (double*)valAT, nullptr);
        else optamd::csr_gather<float>(nnz, perm, (const float*)valA, (float*)valAT, nullptr);
    }
    OPT_HIP_CHECK(hipDeviceSynchronize());
    optamd::dfree(perm);
    return 0;
}
int OptAMD_CsrATA(int nRowsA, int nColsA, long long nnz, const int* rowPtrA, const int* colIndA, const void* valA,
                  int* rowPtrATA, int* colIndATA, void* valATA, long long* nnzATA, int doublePrecision) {
    if (!csr_args_ok("OptAMD_CsrATA", nRowsA, nColsA, nnz) || !rowPtrA || !rowPtrATA) return 1;
    optamd::DevBuf scratch;
    const size_t vb = doublePrecision ? sizeof(double) : sizeof(float);
    int* rowPtrT = (int*)optamd::dmalloc(sizeof(int) * (nColsA + 1));
    int* colIndT = (int*)optamd::dmalloc(sizeof(int) * std::max(nnz, 1LL));
    int* perm = (int*)optamd::dmalloc(sizeof(int) * std::max(nnz, 1LL));
    void* valT = optamd::dmalloc(vb * std::max(nnz, 1LL));
    optamd::csr_transpose_pattern(nRowsA, nColsA, nnz, rowPtrA, colIndA, rowPtrT, colIndT, perm, scratch, nullptr);
    long long n = optamd::csr_ata_pattern(nColsA, rowPtrA, colIndA, rowPtrT, colIndT, rowPtrATA, nullptr, scratch,
                                          nullptr);
    int rc = n < 0 ? 1 : 0;
    if (!rc && colIndATA) {
        optamd::csr_ata_pattern(nColsA, rowPtrA, colIndA, rowPtrT, colIndT, rowPtrATA, colIndATA, scratch, nullptr);
        if (valA && valATA) {
            if (doublePrecision) {
                optamd::csr_gather<double>(nnz, perm, (const double*)valA, (double*)valT, nullptr);
                optamd::csr_ata_values<double>(nColsA, rowPtrA, colIndA, (const double*)valA, rowPtrT, colIndT,
                                               (const double*)valT, rowPtrATA, colIndATA, (double*)valATA, nullptr);
            } else {
                optamd::csr_gather<float>(nnz, perm, (const float*)valA, (float*)valT, nullptr);
                optamd::csr_ata_values<float>(nColsA, rowPtrA, colIndA, (const float*)valA, rowPtrT, colIndT,
                                              (const float*)valT, rowPtrATA, colIndATA, (float*)valATA, nullptr);
            }
        }
    }
    OPT_HIP_CHECK(hipDeviceSynchronize());
    for (void* v : {(void*)rowPtrT, (void*)colIndT, (void*)perm, valT}) optamd::dfree(v);
    if (nnzATA) *nnzATA = n;
    if (rc) fprintf(stderr, "[opt_amd] OptAMD_CsrATA: A^T A exceeds 2^31 nonzeros\n");
    return rc;
}
int OptAMD_CsrSpMV(int nRowsA, int nColsA, long long nnz, const int* rowPtrA, const int* colIndA, const void* valA,
                   const void* x, void* y, int doublePrecision) {
    if (!csr_args_ok("OptAMD_CsrSpMV", nRowsA, nColsA, nnz) || !rowPtrA || !x || !y) return 1;
    if (doublePrecision)
        optamd::csr_spmv<double>(nRowsA, nnz, rowPtrA, colIndA, (const double*)valA, (const double*)x, (double*)y,
                                 nullptr);
    else
        optamd::csr_spmv<float>(nRowsA, nnz, rowPtrA, colIndA, (const float*)valA, (const float*)x, (float*)y,
                                nullptr);
    OPT_HIP_CHECK(hipDeviceSynchronize());
    return 0;
}

}  // extern "C"

static bool read_file(const char* filename, std::string* text) {
    std::ifstream in(filename ? filename : "");
    if (!in.good()) return false;
    std::stringstream ss;
    ss << in.rdbuf();
    *text = ss.str();
    return true;
}
int OptAMD_GenericSource(const char* filename, int doublePrecision, char* buf, int n) {
    std::string text, out;
    if (!read_file(filename, &text)) return copy_name("cannot read energy file", buf, n), -1;
    const int r = optamd::generic_source(text, (doublePrecision & 1) != 0, &out, (doublePrecision & 2) != 0);
    copy_name(out, buf, n);
    return r;
}
int OptAMD_GenericCompileCheck(const char* filename, int doublePrecision, char* buf, int n) {
    std::string text, log;
    if (!read_file(filename, &text)) return copy_name("cannot read energy file", buf, n), -1;
    const int r = optamd::generic_compile_check(text, doublePrecision != 0, &log);
    copy_name(log, buf, n);
    return r;
}
int OptAMD_GenericDescribe(const char* filename, char* buf, int n) {
    std::string text, out;
    if (!read_file(filename, &text)) return copy_name("cannot read energy file", buf, n), -1;
    const int r = optamd::generic_describe(text, &out);
    copy_name(out, buf, n);
    return r;
}
int OptAMD_GenericSignature(const char* filename, char* buf, int n) {
    std::string text, sig, err;
    if (!read_file(filename, &text)) return copy_name("cannot read energy file", buf, n), -1;
    if (!optamd::generic_signature(text, &sig, nullptr, &err)) return copy_name(err, buf, n), -1;
    return copy_name(sig, buf, n);
}
