// generic.hip — the general energy path: any energy file the front end (gen/) lowers,
// solved by the same GN / LM driver (stencil_plan.h) with kernels generated for that
// energy and compiled at plan time with hiprtc for gfx950.
//
// This is the role of the reference's whole compile pipeline (problemSpecFromFile →
// toenergyspecs → createfunctionset → solverGPUGaussNewton's kernels, API/src/o.t:
// 1295-1348, 2669-3235). The hand-written families (image_warping.hip, ...) remain the
// fast paths for the energies they recognise; this path covers every other energy in
// the DSL subset gen/lua.cpp accepts (centred stencils over 1-3-D index spaces, graph
// residuals, Exclude, Select / InBounds, scalar parameters, up to 4 unknown images).
// OPT_AMD_GENERIC=1 routes recognised families here too (to validate it against the
// hand-written kernels and the reference's known answers).
#include <hip/hiprtc.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include "gen/codegen.h"
#include "graph_util.h"
#include "stencil_plan.h"

namespace optamd {

namespace {

#define OPT_RTC_CHECK(call)                                                                          \
    do {                                                                                             \
        hiprtcResult r_ = (call);                                                                    \
        if (r_ != HIPRTC_SUCCESS) {                                                                  \
            fprintf(stderr, "[opt_amd] hiprtc error %d (%s) in %s\n", (int)r_, hiprtcGetErrorString(r_), #call); \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

// Compile `code` to a gfx950 code object. false + log on a compile error.
bool rtc_compile(const std::string& code, std::string* obj, std::string* log) {
    hiprtcProgram prog;
    OPT_RTC_CHECK(hiprtcCreateProgram(&prog, code.c_str(), "opt_amd_generic.hip", 0, nullptr, nullptr));
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    const hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    if (n > 1) {
        log->resize(n);
        hiprtcGetProgramLog(prog, &(*log)[0]);
    }
    if (rc != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        return false;
    }
    OPT_RTC_CHECK(hiprtcGetCodeSize(prog, &n));
    obj->resize(n);
    OPT_RTC_CHECK(hiprtcGetCode(prog, &(*obj)[0]));
    hiprtcDestroyProgram(&prog);
    return true;
}

// Process-wide cache: one code object per distinct generated source.
std::mutex g_mu;
std::map<std::string, std::string>& code_cache() {
    static std::map<std::string, std::string> m;
    return m;
}

__global__ void incidence_count(const int* keys, int E, int* counts) {
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < E; e += gridDim.x * blockDim.x)
        atomicAdd(&counts[keys[e]], 1);
}
// out[q] = slot[geid[q]]: one slot's vertex of each edge of an incidence list, in its order
__global__ void incidence_gather(const int* slot, const int* geid, int E, int* out) {
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < E; q += gridDim.x * blockDim.x) out[q] = slot[geid[q]];
}
__global__ void iota_kernel(int* v, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v[i] = i;
}

size_t elem_size(const gen::GImage& im, bool dbl) {
    if (im.tvalued) return dbl ? 8 : 4;
    if (im.elem == "uint8") return 1;
    return 4;
}

// gen::generate's off32: every array the graph gathers read is below 2 GiB — the unknown
// vectors, the images (all allocated at the unknowns' domain size), the graph record cache
// (at most 16 fields per vertex in the 32-bit form, codegen.cpp) and the per-edge
// incidence copies. The same answer at the admission compile and in the plan.
bool gather_offsets_fit_32(const gen::GModel& m, const ProblemSpec& s, bool dbl) {
    if (env_int("OPT_AMD_GEN_OFF32", 1) == 0) return false;   // tests: force the 64-bit form
    const long long lim = 1LL << 31, t = dbl ? 8 : 4;
    long long npix = 1, chans = 0;
    for (int d : m.images[m.unknown_images()[0]].dims) npix *= (long long)s.dim_values.at(m.dims[d].index);
    for (int k : m.unknown_images()) chans += m.images[k].channels;
    bool ok = npix * chans * t < lim && npix * 16 * t < lim;
    for (auto& im : m.images) ok &= npix * im.channels * (long long)elem_size(im, dbl) < lim;
    for (auto& g : m.graphs) {
        long long e = 1;
        for (int d : g.dims) e *= (long long)s.dim_values.at(m.dims[d].index);
        ok &= e * 4 < lim;
    }
    return ok;
}

}  // namespace

// Front-end admission check for Opt_ProblemDefine: lower the energy and check it fits the
// generated kernels' limits. Fills the spec fields the driver reads.
bool generic_accepts(const std::string& text, ProblemSpec* spec, std::string* err) {
    gen::GModel m;
    if (!gen::build_model(text, &m, err)) return false;
    if (!m.unsupported.empty()) {
        *err = "the general front end does not lower '" + m.unsupported + "'";
        return false;
    }
    const std::vector<int> unk = m.unknown_images();
    if (unk.empty()) { *err = "no Unknown declared"; return false; }
    if (unk.size() > 4) { *err = "more than 4 unknown images"; return false; }
    if (m.images.size() > 16) { *err = "more than 16 images"; return false; }
    if (m.params.size() > 32) { *err = "more than 32 parameters"; return false; }
    if (m.graphs.size() > 4) { *err = "more than 4 graphs"; return false; }
    size_t slots = 0;
    for (auto& g : m.graphs) slots += g.slot_names.size();
    if (slots > 16) { *err = "more than 16 graph vertex arrays"; return false; }
    const int nd = m.unknown_dims();
    if (nd < 1 || nd > 3) { *err = "unknowns must be 1-, 2- or 3-dimensional"; return false; }
    for (int k : unk)
        if (m.images[k].dims != m.images[unk[0]].dims) { *err = "unknowns over different index spaces"; return false; }
    for (auto& im : m.images)
        if (!im.unknown && im.dims != m.images[unk[0]].dims) {
            *err = std::string(im.internal ? "computed array '" : "array '") + im.name +
                   "' is not over the unknowns' index space";
            return false;
        }
    if (m.residuals.empty()) { *err = "no Energy terms"; return false; }
    spec->text = text;
    spec->use_preconditioner = m.use_preconditioner;
    spec->family = "generic";
    return true;
}

// Structural signature of a lowered energy: every declaration (kind, element type,
// channels, index space, problemparams index — names dropped) and every residual,
// ComputedArray and exclusion template as the hash-consed pool prints it. Two energy
// files with equal signatures define the same problem and the same derivatives
// (the reference derives all kernels from exactly these, o.t:1295-1348, 2669-2715).
bool generic_signature(const std::string& text, std::string* sig, bool* use_pre, std::string* err) {
    gen::GModel m;
    if (!gen::build_model(text, &m, err)) return false;
    if (!m.unsupported.empty()) { *err = "unsupported: " + m.unsupported; return false; }
    std::string s;
    auto ids = [](const std::vector<int>& v) {
        std::string o;
        for (int x : v) o += std::to_string(x) + ",";
        return o;
    };
    for (auto& d : m.dims) s += "D" + std::to_string(d.index) + ";";
    for (auto& im : m.images)
        s += "I" + std::to_string(im.index) + ":" + std::to_string(im.channels) + (im.unknown ? "u" : "a") +
             (im.internal ? "i" : "") + (im.tvalued ? "t" : "") + im.elem + "{" + ids(im.dims) + "};";
    for (auto& p : m.params) s += "P" + std::to_string(p.index) + ":" + p.type + ";";
    for (auto& g : m.graphs) s += "G{" + ids(g.dims) + "}{" + ids(g.slot_index) + "};";
    for (auto& c : m.computed) {
        s += "C" + std::to_string(c.image) + ":";
        for (int e : c.expr) s += m.pool.str(e) + "|";
        std::vector<std::string> gs;   // a set: its order follows traversal, not meaning
        for (auto& g : c.grads)
            gs.push_back("g" + std::to_string(g.ch) + "," + (g.u >= 0 ? m.pool.str(g.u) : std::string("-")) + "," +
                         (g.gimg >= 0 ? "img," : "const,") + (g.expr >= 0 ? m.pool.str(g.expr) : std::string("-")) + "|");
        std::sort(gs.begin(), gs.end());
        for (auto& g : gs) s += g;
        for (int k = 0; k < 3; ++k) s += std::to_string(c.lo[k]) + ":" + std::to_string(c.hi[k]) + ",";
        s += ";";
    }
    s += "X" + (m.exclude >= 0 ? m.pool.str(m.exclude) : std::string("-")) + ";";
    for (auto& r : m.residuals)
        s += "R" + std::to_string(r.graph) + ":" + std::to_string(r.unknowns.size()) + ":" + m.pool.str(r.expr) + ";";
    *sig = s;
    if (use_pre) *use_pre = m.use_preconditioner;
    return true;
}

namespace {
// The energy each hand-written family implements: energies/<family>.t, embedded at build
// time (Makefile: build/gen/family_energies_src.h). Each lowers to exactly the reference
// example's templates (tests/test_generic_frontend.py).
const std::pair<const char*, const char*> kFamilyEnergies[] = {
#include "family_energies_src.h"
};
}  // namespace

bool family_is_canonical(ProblemSpec* spec, std::string* why) {
    static std::mutex mu;
    static std::map<std::string, std::string> canon;   // family -> signature
    std::lock_guard<std::mutex> lk(mu);
    if (!canon.count(spec->family)) {
        for (auto& fe : kFamilyEnergies) {
            if (spec->family != fe.first) continue;
            std::string sig, err;
            if (!generic_signature(fe.second, &sig, nullptr, &err)) {
                *why = "canonical energy of family " + spec->family + " does not lower: " + err;
                return false;
            }
            canon[spec->family] = sig;
        }
        if (!canon.count(spec->family)) { *why = "no canonical energy for family " + spec->family; return false; }
    }
    std::string sig, err;
    bool use_pre = false;
    if (!generic_signature(spec->text, &sig, &use_pre, &err)) {
        *why = err;
        return false;
    }
    if (sig != canon[spec->family]) {
        *why = "the energy's residuals differ from the " + spec->family + " family's";
        return false;
    }
    spec->use_preconditioner = use_pre;
    return true;
}

template <typename TT>
class GenericOp {
public:
    using T = TT;
    static constexpr const char* kName = "generic";
    static constexpr const char* kApplyName = "gen_apply";
    static constexpr bool kSlabs = true;   // decided per energy: slab_refusal()

    GenericOp(const ProblemSpec& spec, const StateOptions& opts, Domain dom) : opts_(opts), dom_(dom) {
        std::string err;
        if (!gen::build_model(spec.text, &m_, &err)) {
            fprintf(stderr, "[opt_amd] generic: %s\n", err.c_str());
            exit(1);
        }
        unk_ = m_.unknown_images();
        const gen::GImage& u0 = m_.images[unk_[0]];
        dims_[0] = dims_[1] = dims_[2] = 1;
        for (size_t k = 0; k < u0.dims.size(); ++k) dims_[k] = (int)spec.dim_values.at(m_.dims[u0.dims[k]].index);
        npix_ = (long long)dims_[0] * dims_[1] * dims_[2];
        own_lo_ = 0;
        own_hi_ = npix_;
        if (u0.dims.size() == 2) {   // a row slab (StencilPlan::set_decomposition) or the whole image
            npix_ = dom.npix_mem();
            ymem0_ = dom.y_mem0;
            own_lo_ = dom.off(0, dom.y_lo);
            own_hi_ = dom.off(0, dom.y_hi);
        }
        halo_ = row_halo();
        for (size_t g = 0; g < m_.graphs.size(); ++g) {
            long long e = 1;
            for (int d : m_.graphs[g].dims) e *= spec.dim_values.at(m_.dims[d].index);
            nedge_[g] = (int)e;
        }
        long long off = 0;
        for (size_t k = 0; k < unk_.size(); ++k) {
            uoff_[k] = off;
            off += npix_ * m_.images[unk_[k]].channels;
        }
        n_ = off;
        src_ = gen::generate(m_, sizeof(T) == 8, gather_offsets_fit_32(m_, spec, sizeof(T) == 8));
        load_module();
        for (size_t i = 0; i < m_.images.size(); ++i)
            if (m_.images[i].internal) {   // ComputedArray values and gradient images
                dimg_[i] = dmalloc(std::max<size_t>(1, image_bytes(i)));
                OPT_HIP_CHECK(hipMemset(dimg_[i], 0, image_bytes(i)));
                a_.img[i] = dimg_[i];
            }
        if (opts_.host_buffers) {
            for (size_t i = 0; i < m_.images.size(); ++i)
                if (!m_.images[i].internal) dimg_[i] = dmalloc(std::max<size_t>(1, image_bytes(i)));
            int sb = 0;
            for (size_t g = 0; g < m_.graphs.size(); ++g)
                for (size_t s = 0; s < m_.graphs[g].slot_names.size(); ++s, ++sb)
                    dslot_[sb] = (int*)dmalloc(sizeof(int) * std::max(1, nedge_[g]));
        }
    }
    ~GenericOp() {
        for (void* p : dimg_) dfree(p);
        for (int* p : dslot_) dfree(p);
        for (int k = 0; k < 16; ++k) { dfree(goff_[k]); dfree(geid_[k]); }
        for (int k = 0; k < 32; ++k) dfree(gnb_[k]);
        dfree(fp_scratch_);
        if (mod_) (void)hipModuleUnload(mod_);
    }

    VecLayout layout() const {
        VecLayout L{};
        L.nimg = (int)unk_.size();
        for (size_t k = 0; k < unk_.size(); ++k) {
            L.ch[k] = m_.images[unk_[k]].channels;
            L.off[k] = uoff_[k];
        }
        L.off[L.nimg] = n_;
        L.N = npix_;
        return L;
    }
    int halo() const { return halo_; }
    // Why this energy cannot run on row slabs ("" = it can). Graph and sampled reads are
    // data-dependent (as the optical_flow / ARAP families), slabs split the 2nd dimension.
    std::string slab_refusal() const {
        if (m_.unknown_dims() != 2) return "generic: row-slab decomposition needs a 2-D energy";
        if (!m_.graphs.empty()) return "generic: no row-slab decomposition for graph energies";
        // (sampled reads may sit in a residual or, cached per Step, in a ComputedArray)
        std::vector<int> roots;
        for (auto& r : m_.residuals) roots.push_back(r.expr);
        for (auto& c : m_.computed) {
            roots.insert(roots.end(), c.expr.begin(), c.expr.end());
            for (auto& g : c.grads) roots.push_back(g.expr);
        }
        for (int e : roots) {
            bool sample = false;
            m_.pool.visit(e, [&](int, const gen::Node& n) { sample |= n.op == gen::Op::Sample; });
            if (sample) return "generic: no row-slab decomposition with sampled images (data-dependent reads)";
        }
        return "";
    }
    int stencil_blocks() const {
        long long w = std::max(npix_, n_);
        for (int e : nedge_) w = std::max<long long>(w, e);
        return (int)std::max<long long>(1, std::min<long long>((w + kBlock - 1) / kBlock, max_blocks_));
    }

    void bind(void** params, hipStream_t s) {
        user_ = params;
        for (size_t i = 0; i < m_.images.size(); ++i) {
            if (m_.images[i].internal) continue;
            void* p = params[m_.images[i].index];
            if (opts_.host_buffers) {
                OPT_HIP_CHECK(hipMemcpyAsync(dimg_[i], p, image_bytes(i), hipMemcpyHostToDevice, s));
                p = dimg_[i];
            }
            a_.img[i] = p;
        }
        // an Array on an Unknown's slot views the (device copy of the) unknown
        for (size_t i = 0; i < m_.images.size(); ++i)
            if (!m_.images[i].unknown && !m_.images[i].internal && m_.images[i].tvalued)
                for (int k : unk_)
                    if (m_.images[k].index == m_.images[i].index) a_.img[i] = a_.img[k];
        for (size_t j = 0; j < m_.params.size(); ++j) {
            const void* p = params[m_.params[j].index];
            const std::string& t = m_.params[j].type;
            a_.prm[j] = t == "double" ? *(const double*)p
                        : (t == "int" || t == "int32") ? (double)*(const int*)p
                        : t == "uint" || t == "uint32" ? (double)*(const unsigned*)p
                                                       : (double)*(const float*)p;
        }
        int sb = 0;
        for (size_t g = 0; g < m_.graphs.size(); ++g) {
            for (size_t k = 0; k < m_.graphs[g].slot_names.size(); ++k, ++sb) {
                const int* v = (const int*)params[m_.graphs[g].slot_index[k]];
                if (opts_.host_buffers) {
                    OPT_HIP_CHECK(hipMemcpyAsync(dslot_[sb], v, sizeof(int) * nedge_[g], hipMemcpyHostToDevice, s));
                    v = dslot_[sb];
                }
                a_.slot[sb] = v;
            }
            a_.nedge[g] = nedge_[g];
        }
        if (sb > 0) check_graphs(s);
        for (int k = 0; k < 3; ++k) a_.dims[k] = dims_[k];
        a_.npix = npix_;
        a_.ymem0 = ymem0_;
        a_.own_lo = own_lo_;
        a_.own_hi = own_hi_;
        for (size_t k = 0; k < unk_.size(); ++k) a_.uoff[k] = uoff_[k];
    }
    // hipGraph replay gate + key (StencilPlan::pcg_graph_begin), from the lowered model:
    // no capture for graph energies (adjacency rebuilt on bind); the key is the argument
    // block every captured launch receives — image / slot / incidence pointers and
    // parameter values as bound by bind().
    bool capture_key(std::vector<unsigned long long>* key) const {
        if (!m_.graphs.empty()) return false;
        unsigned long long w[(sizeof(GenArgs) + 7) / 8] = {};
        memcpy(w, &a_, sizeof(GenArgs));
        key->insert(key->end(), w, w + (sizeof(GenArgs) + 7) / 8);
        return true;
    }
    void unbind(hipStream_t s) {
        if (!opts_.host_buffers) return;
        for (int k : unk_)
            OPT_HIP_CHECK(hipMemcpyAsync(user_[m_.images[k].index], dimg_[k], image_bytes(k), hipMemcpyDeviceToHost, s));
    }
    T* unknown(int k) { return k < (int)unk_.size() ? (T*)a_.img[unk_[k]] : nullptr; }
    void precompute(hipStream_t s) {
        for (hipFunction_t f : k_pre_) launch(f, s, {&a_});
    }
    // The transcendental caches (the precompute kernels after the ComputedArrays' ones:
    // the centred cache image, the graph record cache) from the arrays bound at this Step
    // (StencilPlan::step; HasRefreshCaches). Returns whether any ran.
    bool refresh_caches(hipStream_t s) {
        for (size_t k = m_.computed.size(); k < k_pre_.size(); ++k) launch(k_pre_[k], s, {&a_});
        return k_pre_.size() > m_.computed.size();
    }
    // ComputedArray values and gradient images: exchanged after every precompute
    void computed_planes(std::vector<HaloPlane>& v) const {
        for (size_t i = 0; i < m_.images.size(); ++i)
            if (m_.images[i].internal)
                v.push_back({dimg_[i], (size_t)elem_size(m_.images[i], sizeof(T) == 8) * m_.images[i].channels *
                                           (size_t)dims_[0]});
    }

    void jtf(T* r, T* diag, uint8_t* flags, hipStream_t s) {
        a_.flags = flags;
        launch(k_jtf_, s, {&a_, &r, &diag});   // flags, and r / diag of the centred residuals
        if (src_.has_graph) launch(k_jtf_graph_, s, {&a_, &r, &diag});
    }
    void apply(const T* p, T* Ap, const T* dadd, const int* stop, ReduceSlot rs, hipStream_t s) {
        if (!src_.has_graph) {
            int finish = 1;
            launch(k_apply_, s, {&a_, &p, &Ap, &dadd, &stop, &rs, &finish});
            return;
        }
        int finish = 0, centred = src_.has_centered && !src_.graph_apply_centred ? 1 : 0;
        if (centred) launch(k_apply_, s, {&a_, &p, &Ap, &dadd, &stop, &rs, &finish});
        launch(k_apply_graph_, s, {&a_, &p, &Ap, &dadd, &stop, &rs, &centred});
    }
    void cost(ReduceSlot rs, hipStream_t s) {
        const T* d = nullptr;
        launch(k_cost_, s, {&a_, &d, &rs});
    }
    void model_cost(const T* delta, ReduceSlot rs, hipStream_t s) { launch(k_cost_, s, {&a_, &delta, &rs}); }

    // materialized Jacobian (useMaterializedJTJ, csr.h): the generated saveJToCRS kernels
    long long jacobian_rows() const {
        long long r = 0;
        for (auto& d : src_.dump) r += elements(d.graph) * d.rows;
        return r;
    }
    long long jacobian_nnz() const {
        long long z = 0;
        for (auto& d : src_.dump) z += elements(d.graph) * d.nnz;
        return z;
    }
    void dump_j(int* rowPtr, int* colInd, T* val, hipStream_t s) {
        long long rb = 0, zb = 0;
        for (size_t i = 0; i < src_.dump.size(); ++i) {
            launch(k_dump_[i], s, {&a_, &rowPtr, &colInd, &val, &rb, &zb, &n_});
            rb += elements(src_.dump[i].graph) * src_.dump[i].rows;
            zb += elements(src_.dump[i].graph) * src_.dump[i].nnz;
        }
        OPT_HIP_CHECK(hipMemsetD32Async(rowPtr + rb, (int)zb, 1, s));
    }

    const std::string& source() const { return src_.code; }
    bool tiled_selected() const { return k_apply_ == k_apply_tiled_; }

private:
    long long elements(int graph) const { return graph < 0 ? npix_ : nedge_[graph]; }
    // Rows a slab must hold beyond its own: the widest vertical reach of any residual
    // instance that touches an owned unknown (the span of its reads incl. ComputedArray
    // boxes), of the ComputedArrays' own expressions, and of the exclusion test.
    int row_halo() const {
        if (m_.unknown_dims() != 2) return 0;
        auto reach = [&](int e, int* lo, int* hi) {
            m_.pool.visit(e, [&](int, const gen::Node& n) {
                if (n.op != gen::Op::Read || n.slot >= 0) return;
                int clo = 0, chi = 0;
                for (auto& c : m_.computed)
                    if (c.image == n.i) { clo = c.lo[1]; chi = c.hi[1]; }
                *lo = std::min(*lo, n.off[1] + clo);
                *hi = std::max(*hi, n.off[1] + chi);
            });
        };
        int h = 0;
        for (auto& r : m_.residuals) {
            int lo = 0, hi = 0;
            reach(r.expr, &lo, &hi);
            h = std::max(h, hi - lo);
        }
        for (auto& c : m_.computed) h = std::max({h, -c.lo[1], c.hi[1]});
        if (m_.exclude >= 0) {
            int lo = 0, hi = 0;
            reach(m_.exclude, &lo, &hi);
            h = std::max({h, -lo, hi});
        }
        return std::max(h, 1);
    }
    size_t image_bytes(size_t i) const {
        return (size_t)npix_ * m_.images[i].channels * elem_size(m_.images[i], sizeof(T) == 8);
    }
    void load_module() {
        std::string obj;
        {
            std::lock_guard<std::mutex> lk(g_mu);
            auto it = code_cache().find(src_.code);
            if (it != code_cache().end()) obj = it->second;
        }
        if (obj.empty()) {
            std::string log;
            if (!rtc_compile(src_.code, &obj, &log)) {
                fprintf(stderr, "[opt_amd] generic: generated kernels failed to compile:\n%s\n", log.c_str());
                exit(1);
            }
            std::lock_guard<std::mutex> lk(g_mu);
            code_cache()[src_.code] = obj;
        }
        OPT_HIP_CHECK(hipModuleLoadData(&mod_, obj.data()));
        for (auto kv : {std::make_pair(&k_jtf_, "gen_jtf"), std::make_pair(&k_apply_, "gen_apply"),
                        std::make_pair(&k_cost_, "gen_cost"), std::make_pair(&k_jtf_graph_, "gen_jtf_graph"),
                        std::make_pair(&k_apply_graph_, "gen_apply_graph")})
            OPT_HIP_CHECK(hipModuleGetFunction(kv.first, mod_, kv.second));
        // Centred apply: the register strip where the front end emitted one, else the
        // two-phase LDS tiles where it prefers them (prefer_tiled: many residual instances
        // per pixel), else the gather. OPT_AMD_GEN_APPLY=gather|tiled|strip forces one.
        // (Row slabs use the gather: its reads stay within row_halo() of the owned rows.)
        const bool slab = dom_.mem_rows != dom_.H || dom_.y_lo != 0;
        const char* want = getenv("OPT_AMD_GEN_APPLY");
        const std::string force = want ? want : "";
        if (src_.has_tiled && !slab) {
            OPT_HIP_CHECK(hipModuleGetFunction(&k_apply_tiled_, mod_, "gen_apply_tiled"));
            if (force == "tiled" || (force.empty() && src_.prefer_tiled)) k_apply_ = k_apply_tiled_;
        }
        if (src_.has_strip && !slab) {
            // one wave per (column strip, >= 8-row block): a small image leaves most SIMDs
            // idle (poisson 512^2: 576 waves, 13.7 -> 20.4 us), so below ~2 waves per SIMD
            // the other forms run
            OPT_HIP_CHECK(hipModuleGetFunction(&k_apply_strip_, mod_, "gen_apply_strip"));
            const long long waves = (long long)((dims_[0] + src_.strip_cols - 1) / src_.strip_cols) * ((dims_[1] + 7) / 8);
            if (force == "strip" || (force.empty() && waves >= 2048)) k_apply_ = k_apply_strip_;
        }
        // Strip waves walk whole row blocks, so a grid of 1.33 resident rounds leaves a third
        // of the chip idle in its tail: with the strip apply, launch exactly the blocks that
        // are resident together (its occupancy x CUs; image_warping / shape_from_shading at
        // 80 VGPRs: 1536 blocks; measured 2048 -> 1536: generated image_warping apply
        // 228 -> 204 us, shape_from_shading LM step 4.18 -> 3.82 ms)
        if (k_apply_strip_ && k_apply_ == k_apply_strip_ && !getenv("OPT_AMD_GEN_BLOCKS")) {
            int per_cu = 0, dev = 0, cus = 0;
            OPT_HIP_CHECK(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_apply_strip_, kBlock, 0));
            OPT_HIP_CHECK(hipGetDevice(&dev));
            OPT_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            if (per_cu > 0 && cus > 0) max_blocks_ = std::min(4096, std::max(8, per_cu * cus));
        }
        // J^T F: the register strip under the same rule (OPT_AMD_GEN_JTF=gather|strip forces)
        if (src_.has_jtf_strip && !slab) {
            const char* wj = getenv("OPT_AMD_GEN_JTF");
            const std::string fj = wj ? wj : "";
            const long long waves = (long long)((dims_[0] + src_.jtf_strip_cols - 1) / src_.jtf_strip_cols) * ((dims_[1] + 7) / 8);
            if (fj == "strip" || (fj.empty() && waves >= 2048))
                OPT_HIP_CHECK(hipModuleGetFunction(&k_jtf_, mod_, "gen_jtf_strip"));
        }
        // cost / model cost: the register strip under the same rule (OPT_AMD_GEN_COST forces)
        if (src_.has_cost_strip && !slab) {
            const char* wc = getenv("OPT_AMD_GEN_COST");
            const std::string fc = wc ? wc : "";
            const long long waves = (long long)((dims_[0] + src_.cost_strip_cols - 1) / src_.cost_strip_cols) * ((dims_[1] + 7) / 8);
            if (fc == "strip" || (fc.empty() && waves >= 2048))
                OPT_HIP_CHECK(hipModuleGetFunction(&k_cost_, mod_, "gen_cost_strip"));
        }
        k_dump_.resize(src_.dump.size());
        for (size_t k = 0; k < src_.dump.size(); ++k)
            OPT_HIP_CHECK(hipModuleGetFunction(&k_dump_[k], mod_, ("gen_dump_j_" + std::to_string(k)).c_str()));
        k_pre_.resize(src_.n_precompute);
        for (int k = 0; k < src_.n_precompute; ++k)
            OPT_HIP_CHECK(hipModuleGetFunction(&k_pre_[k], mod_, ("gen_precompute_" + std::to_string(k)).c_str()));
    }
    void launch(hipFunction_t f, hipStream_t s, std::initializer_list<const void*> args) {
        std::vector<void*> a;
        for (const void* p : args) a.push_back(const_cast<void*>(p));
        OPT_HIP_CHECK(hipModuleLaunchKernel(f, stencil_blocks(), 1, 1, kBlock, 1, 1, 0, s, a.data(), nullptr));
    }
    // vertex indices must lie in [0, N) (fail-stop, as the reference does on bad input)
    void check_graphs(hipStream_t s) {
        if (!fp_scratch_)
            fp_scratch_ = (unsigned long long*)dmalloc(sizeof(unsigned long long) * (1 + kFingerprintGrid));
        int sb = 0;
        for (size_t g = 0; g < m_.graphs.size(); ++g) {
            const int ns = (int)m_.graphs[g].slot_names.size();
            const unsigned long long h = graph_fingerprint(a_.slot + sb, ns, nedge_[g], s, fp_scratch_);
            if (!(goff_[sb] && h == fingerprint_[g])) {
                fingerprint_[g] = h;
                for (int k = 0; k < ns; ++k) {
                    if (nedge_[g] > 0) {
                        std::vector<int> hv(nedge_[g]);
                        OPT_HIP_CHECK(hipMemcpyAsync(hv.data(), a_.slot[sb + k], sizeof(int) * nedge_[g],
                                                     hipMemcpyDeviceToHost, s));
                        OPT_HIP_CHECK(hipStreamSynchronize(s));
                        for (int v : hv)
                            if (v < 0 || v >= npix_) {
                                fprintf(stderr, "[opt_amd] generic: graph '%s' vertex index %d outside [0, %lld)\n",
                                        m_.graphs[g].name.c_str(), v, npix_);
                                exit(1);
                            }
                    }
                    build_incidence(sb + k, nedge_[g], s);
                }
                for (int k = 0; k < ns; ++k) build_neighbours(sb + k, nedge_[g], s);
            }
            sb += ns;
        }
        for (int k = 0; k < sb; ++k) {
            a_.goff[k] = goff_[k];
            a_.geid[k] = geid_[k];
        }
        for (size_t i = 0; i < src_.nb_pairs.size() && i < 32; ++i) a_.gnb[i] = gnb_[i];
    }
    // GenArgs::gnb of every (slot k, other slot) pair whose incidence list was rebuilt:
    // the other slot's vertex of each incident edge, in the incidence order
    void build_neighbours(int sb, int E, hipStream_t s) {
        for (size_t i = 0; i < src_.nb_pairs.size() && i < 32; ++i) {
            if (src_.nb_pairs[i].first != sb) continue;
            dfree(gnb_[i]);
            gnb_[i] = (int*)dmalloc(sizeof(int) * std::max(E, 1));
            if (E == 0) continue;
            const int grid = std::min((E + 255) / 256, 4096);
            hipLaunchKernelGGL(incidence_gather, dim3(grid), dim3(256), 0, s, a_.slot[src_.nb_pairs[i].second],
                               (const int*)geid_[sb], E, gnb_[i]);
            OPT_HIP_CHECK(hipGetLastError());
        }
    }
    // Edges by vertex for slot array sb: a stable radix sort of (vertex, edge id) pairs and
    // a histogram + exclusive scan of the vertex counts.
    void build_incidence(int sb, int E, hipStream_t s) {
        dfree(goff_[sb]);
        dfree(geid_[sb]);
        goff_[sb] = (int*)dmalloc(sizeof(int) * (npix_ + 1));
        geid_[sb] = (int*)dmalloc(sizeof(int) * std::max(E, 1));
        OPT_HIP_CHECK(hipMemsetAsync(goff_[sb], 0, sizeof(int) * (npix_ + 1), s));
        if (E == 0) return;
        int* keys = (int*)dmalloc(sizeof(int) * E);
        int* ids = (int*)dmalloc(sizeof(int) * E);
        const int grid = std::min((E + 255) / 256, 4096);
        hipLaunchKernelGGL(iota_kernel, dim3(grid), dim3(256), 0, s, ids, E);
        int bits = 1;
        while ((1LL << bits) < npix_) ++bits;
        size_t need = 0, need2 = 0;
        OPT_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, a_.slot[sb], keys, ids, geid_[sb], E, 0, bits, s));
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, need2, goff_[sb], goff_[sb], (int)npix_ + 1, s));
        need = std::max(need, need2);
        void* tmp = dmalloc(std::max<size_t>(need, 1));
        OPT_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, need, a_.slot[sb], keys, ids, geid_[sb], E, 0, bits, s));
        hipLaunchKernelGGL(incidence_count, dim3(grid), dim3(256), 0, s, a_.slot[sb], E, goff_[sb]);
        size_t n2 = need;
        OPT_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, n2, goff_[sb], goff_[sb], (int)npix_ + 1, s));
        OPT_HIP_CHECK(hipStreamSynchronize(s));
        dfree(tmp);
        dfree(keys);
        dfree(ids);
    }

    StateOptions opts_;
    Domain dom_;
    int ymem0_ = 0, halo_ = 0;
    long long own_lo_ = 0, own_hi_ = 0;
    gen::GModel m_;
    gen::GenSource src_;
    std::vector<int> unk_;
    int dims_[3];
    long long npix_ = 0, n_ = 0;
    long long uoff_[4] = {0, 0, 0, 0};
    std::vector<int> nedge_ = std::vector<int>(4, 0);
    GenArgs a_{};
    void** user_ = nullptr;
    void* dimg_[16] = {};
    int* dslot_[16] = {};
    unsigned long long fingerprint_[4] = {0, 0, 0, 0};
    unsigned long long* fp_scratch_ = nullptr;
    int* goff_[16] = {};
    int* geid_[16] = {};
    int* gnb_[32] = {};
    // grid of every generic kernel (all walk their work grid-stride); a register-strip apply
    // sets it to the blocks the chip holds at once (below), OPT_AMD_GEN_BLOCKS overrides
    int max_blocks_ = std::min(4096, std::max(8, env_int("OPT_AMD_GEN_BLOCKS", 2048)));
    hipModule_t mod_ = nullptr;
    std::vector<hipFunction_t> k_pre_, k_dump_;
    hipFunction_t k_apply_tiled_{}, k_apply_strip_{};
    hipFunction_t k_jtf_{}, k_apply_{}, k_cost_{}, k_jtf_graph_{}, k_apply_graph_{};
};

std::unique_ptr<Plan> make_generic_plan(const ProblemSpec& spec, const StateOptions& opts, const unsigned* dims,
                                        std::string* err) {
    ProblemSpec s = spec;
    gen::GModel m;
    if (!gen::build_model(spec.text, &m, err)) return nullptr;
    int maxidx = -1;
    for (auto& d : m.dims) maxidx = std::max(maxidx, d.index);
    s.dim_values.assign(dims, dims + maxidx + 1);
    long long npix = 1;
    const std::vector<int>& ud = m.images[m.unknown_images()[0]].dims;
    for (int d : ud) npix *= s.dim_values[m.dims[d].index];
    if (npix <= 0 || npix > (1LL << 31) / 16) { *err = "generic: unknown index space empty or too large"; return nullptr; }
    // compile (and cache) the kernels here so that a compile error is a NULL plan, as the
    // reference returns nil on errors in the energy (o.t:1526), not a fail-stop
    {
        gen::GModel mc;
        std::string e2;
        gen::build_model(spec.text, &mc, &e2);
        const std::string code = gen::generate(mc, opts.double_precision, gather_offsets_fit_32(mc, s, opts.double_precision)).code;
        std::lock_guard<std::mutex> lk(g_mu);
        if (!code_cache().count(code)) {
            std::string obj, log;
            if (!rtc_compile(code, &obj, &log)) {
                *err = "generic: generated kernels failed to compile:\n" + log;
                return nullptr;
            }
            code_cache()[code] = obj;
        }
    }
    Domain dom{(int)npix, 1, 0, 1, 0, 1};
    if (ud.size() == 2) {   // image rows: StencilPlan may split them into slabs
        const int W = (int)s.dim_values[m.dims[ud[0]].index], H = (int)s.dim_values[m.dims[ud[1]].index];
        dom = Domain{W, H, 0, H, 0, H};
    }
    if (opts.double_precision) return make_stencil_plan<GenericOp<double>>(s, opts, dom, err);
    return make_stencil_plan<GenericOp<float>>(s, opts, dom, err);
}

// Generated source for `text` (tests / inspection): length, or -1 + message in buf.
int generic_source(const std::string& text, bool dbl, std::string* out, bool off32) {
    gen::GModel m;
    std::string err;
    if (!gen::build_model(text, &m, &err)) { *out = err; return -1; }
    if (!m.unsupported.empty()) { *out = "unsupported: " + m.unsupported; return -1; }
    *out = gen::generate(m, dbl, off32).code;
    return (int)out->size();
}

// One line per residual template: "<domain> <support size> <expression>" (tests).
int generic_describe(const std::string& text, std::string* out) {
    gen::GModel m;
    std::string err;
    if (!gen::build_model(text, &m, &err)) { *out = err; return -1; }
    std::string s;
    for (auto& r : m.residuals) {
        s += (r.graph < 0 ? std::string("centred") : "graph" + std::to_string(r.graph)) + " " +
             std::to_string(r.unknowns.size()) + " " + m.pool.str(r.expr) + "\n";
    }
    *out = s;
    return (int)m.residuals.size();
}

// Compile check without a device (hiprtc only): 0 ok, else -1 + log.
int generic_compile_check(const std::string& text, bool dbl, std::string* log) {
    std::string code;
    if (generic_source(text, dbl, &code) < 0) { *log = code; return -1; }
    std::string obj;
    if (!rtc_compile(code, &obj, log)) return -1;
    // graph energies: also the 32-bit gather form plans take below 2 GiB
    if (code.find("a.gnb[") == std::string::npos) return 0;
    if (generic_source(text, dbl, &code, true) < 0) { *log = code; return -1; }
    return rtc_compile(code, &obj, log) ? 0 : -1;
}

}  // namespace optamd
