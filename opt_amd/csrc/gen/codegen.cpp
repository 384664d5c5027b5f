// gen/codegen.cpp — HIP kernels for a lowered energy (gen/model.h), compiled at plan
// time with hiprtc (generic.hip).
//
// Kernel semantics follow the reference's derived functions (API/src/o.t):
//   gen_jtf        createjtfcentered (:2870-2913): for every unknown x of a pixel, the sum
//                  over the centred residual instances containing x of dr/dx * r and
//                  (dr/dx)^2 (the instances are the residual templates shifted by the
//                  inverse of each support offset, residualsincludingX00 :2723-2733);
//                  writes r = -J^T F (0 on excluded unknowns), diag, and the exclude flags
//   gen_apply      createjtjcentered (:2770-2830): sum over the same instances of
//                  dr/dx * sum_u dr/du p(u); with `finish`, masks excluded unknowns, adds
//                  the LM diagonal and reduces p.Ap (PCGStep1, solverGPUGaussNewton.t:607-632)
//   gen_cost       createcost / createmodelcost (:3119-3129, :2915-2966): 1/2 sum r^2 (or
//                  (r + J delta)^2) over non-excluded centres, plus every graph edge
//   gen_*_graph    createjtfgraph / createjtjgraph (:2969-2994, :2833-2867): per edge,
//                  scattered to the edge's vertices with atomics as the reference does
//                  (Image:atomicAddChannel, backend_cuda.t:751-759)
// Reads outside the index space are zero (Image:get, o.t:856-862); centred residuals are
// wrapped in their bounding-box test at classification time.
#include "codegen.h"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <set>
#include <sstream>
#include <tuple>
#include "reduce_dev_src.h"

#define OPTAMD_STR2(...) #__VA_ARGS__
#define OPTAMD_STR(x) OPTAMD_STR2(x)

namespace optamd {
namespace gen {
namespace {

std::string lit(double v) {
    if (std::isinf(v)) return v < 0 ? "(-(T)HUGE_VAL)" : "((T)HUGE_VAL)";
    char b[64];
    snprintf(b, sizeof(b), "%.17g", v);
    std::string s = b;
    if (s.find_first_of(".eEn") == std::string::npos) s += ".0";
    return "((T)" + s + ")";
}

const char* elem_type(const std::string& e, bool unknown) {
    if (unknown) return "T";
    if (e == "uint8") return "unsigned char";
    if (e == "int") return "int";
    return "float";
}

// One kernel body's emitter: every pool node becomes at most one local temporary.
// Per-step caches of single-pixel transcendentals: (op, image, channel) -> internal image
// holding op(image(x).channel) for every pixel, refreshed by the last precompute kernel.
// While set, the emitter reads f(image(x + o)) from the cache at offset o instead of
// evaluating it (the gather evaluates each residual instance, so an angle's sin/cos would
// otherwise be recomputed at every neighbour that reads it). Same function, same input:
// the cached values are the bits the kernels would compute.
using CacheMap = std::map<std::tuple<int, int, int>, int>;
const CacheMap* g_cache = nullptr;
// Per-step predicate cache (the register strips): comparisons of a centred read of a user
// array with a constant (Mask == 0, Constraints >= 0, ...) packed as bits of one uint8
// image, filled by a precompute kernel once per Step — a strip reads one byte per pixel
// instead of the arrays the masks test. Bit k holds pred_k(v) XOR pred_k(0), so the 0 a
// window reads outside the image decodes to pred_k(0), the value the uncached expression
// gives there. Key: (op, image, channel, constant, read on the left).
struct PredCache {
    int img = -1;
    std::vector<std::tuple<int, int, int, double, bool>> keys;
    std::vector<bool> at0;   // pred_k(0)
};
const PredCache* g_pred = nullptr;
// bit index of predicate node n (and its Read child), -1 when n is not a cached predicate
int pred_bit(const Pool& P, const Node& n, int* rd) {
    if (!g_pred) return -1;
    if (n.op != Op::Lt && n.op != Op::Le && n.op != Op::Gt && n.op != Op::Ge && n.op != Op::Eq && n.op != Op::Ne) return -1;
    double c;
    bool left;
    if (P.is_const(n.b, &c) && P.at(n.a).op == Op::Read) { left = true; *rd = n.a; }
    else if (P.is_const(n.a, &c) && P.at(n.b).op == Op::Read) { left = false; *rd = n.b; }
    else return -1;
    const Node& r = P.at(*rd);
    if (r.slot >= 0) return -1;
    for (size_t k = 0; k < g_pred->keys.size(); ++k)
        if (g_pred->keys[k] == std::make_tuple((int)n.op, r.i, r.ch, c, left)) return (int)k;
    return -1;
}
// Graph energies: the same values for slot reads, packed per vertex into one record image
// (channel k of the record = key k) — a gather pass evaluates every incident edge, so the
// other slot's sin / cos would be re-evaluated once per edge (ARAP's angles: three
// sincos per edge in the reverse pass); the record is one 32-byte line per vertex.
struct GraphCache {
    int img = -1, width = 0;
    std::map<std::tuple<int, int, int>, int> ch;
};
const GraphCache* g_gcache = nullptr;
// Slot reads (graph gathers) as uniform base + 32-bit byte offset (generate's off32): the
// saddr form of global_load, one 32-bit multiply per neighbour instead of a 64-bit address
// per gathered array
bool g_off32 = false;
// the register-strip kernels' row loads / stores through 32-bit offsets (with off32):
// OPT_AMD_GEN_STRIP32=0 64-bit element indices, 1 32-bit, 2 32-bit kept opaque (opt_o32),
// 4 (default) opaque in the kernels without two-channel pair reads
int g_strip32 = 4;
// OPT_AMD_GEN_WIDU: the strip kernels' wave index through readfirstlane (row indices and
// bounds in SGPRs): 0 never, 1 always, 2 (default) in the kernels without pair windows
int g_widu = 2;
// OPT_AMD_GEN_FACTOR=0: the strip apply masks every partial of a masked residual (else the
// residual's mask once, on Jp)
bool g_factor = true;

bool transcendental(const Node& n) {
    return n.op == Op::Sin || n.op == Op::Cos || n.op == Op::Exp || n.op == Op::Log || n.op == Op::Sqrt;
}
bool cacheable(const Pool& P, const Node& n) {
    if (!transcendental(n)) return false;
    const Node c = P.at(n.a);
    return c.op == Op::Read && c.slot < 0;
}
bool cacheable_slot(const Pool& P, const Node& n) {
    if (!transcendental(n)) return false;
    const Node c = P.at(n.a);
    return c.op == Op::Read && c.slot >= 0;
}

class Body {
public:
    Body(GModel& m, std::ostringstream& o, int ndims, const std::vector<int>& unk_slot)
        : M_(m), P_(m.pool), o_(o), nd_(ndims), uslot_(unk_slot) {}

    // Graph gathers: nodes that read only the gathering vertex's own slot (`self`), params
    // and constants are the same for every incident edge; they go to `pre`, emitted before
    // the edge loop (the vertex's own sin/cos, unknowns and knowns once per vertex instead
    // of once per edge).
    void hoist_to(std::ostringstream* pre, int self, int graph) { pre_ = pre; self_ = self; graph_ = graph; }
    bool invariant(int id) {
        if (!pre_) return false;
        auto it = inv_.find(id);
        if (it != inv_.end()) return it->second;
        const Node n = P_.at(id);
        bool r = true;
        switch (n.op) {
            case Op::Const: case Op::Param: r = true; break;
            case Op::Read: r = n.slot == self_ && (n.g < 0 || n.g == graph_); break;
            case Op::InBox: case Op::Coord: case Op::Sample: r = false; break;
            default:
                r = (n.a < 0 || invariant(n.a)) && (n.b < 0 || invariant(n.b)) && (n.d < 0 || invariant(n.d));
        }
        inv_[id] = r;
        return r;
    }
    std::ostream& out(int id) { return invariant(id) ? static_cast<std::ostream&>(*pre_) : o_; }

    std::string v(int id) {
        auto it = done_.find(id);
        if (it != done_.end()) return it->second;
        const Node n = P_.at(id);
        if (g_gcache && cacheable_slot(P_, n)) {
            const Node c = P_.at(n.a);
            auto ci = g_gcache->ch.find(std::make_tuple((int)n.op, c.i, c.ch));
            if (ci != g_gcache->ch.end()) {
                const int W = g_gcache->width, k = ci->second;
                const std::string rec = "((const T*)a.img[" + std::to_string(g_gcache->img) + "]) + (long long)v" +
                                        std::to_string(c.slot) + " * " + std::to_string(W);
                const std::string rec32 = "opt_g32((const T*)a.img[" + std::to_string(g_gcache->img) + "], v" +
                                          std::to_string(c.slot) + ", " + std::to_string(W) + ", ";
                std::string name;
                // the slot's whole record once as 16-byte vectors (per-edge kernels: gen_cost
                // 51.7 -> 41.5 us on 1M-vertex ARAP); the vertex gathers read the fields they use
                // (their edge loops: 83.8 us scalar, 90.0 us as records)
                if (W >= 4 && !pre_) {
                    const std::string kr = "kr" + std::to_string(c.slot);
                    if (!rec_.count(c.slot)) {
                        for (int g = 0; g < W; g += 4)
                            out(id) << "        const OptV4 " << kr << "_" << g / 4 << " = *(const OptV4*)(" << rec << " + "
                                    << g << ");\n";
                        rec_.insert(c.slot);
                    }
                    name = kr + "_" + std::to_string(k / 4) + "." + "xyzw"[k % 4];
                } else {
                    name = "k" + std::to_string(id);
                    if (g_off32 && W <= 16)   // (the plan's size check assumes <= 16 fields)
                        out(id) << "        const T " << name << " = " << rec32 << k << ");\n";
                    else
                        out(id) << "        const T " << name << " = (" << rec << ")[" << k << "];\n";
                }
                done_[id] = name;
                return name;
            }
        }
        if (g_cache && cacheable(P_, n)) {
            const Node c = P_.at(n.a);
            auto ci = g_cache->find(std::make_tuple((int)n.op, c.i, c.ch));
            if (ci != g_cache->end()) {
                // outside the image the argument reads 0: f(0), as the evaluated form
                const double f0 = n.op == Op::Cos || n.op == Op::Exp ? 1.0 : n.op == Op::Log ? -HUGE_VAL : 0.0;
                const std::string name = "k" + std::to_string(id);
                o_ << "        const T " << name << " = (" << inb(c.off) << ") ? ((const T*)a.img[" << ci->second
                   << "])[li + " << rel(c.off) << "] : " << lit(f0) << ";\n";
                done_[id] = name;
                return name;
            }
        }
        std::string e;
        if (n.op != Op::Const && is_bool(id)) {   // a 0 / 1 value: its bool, as a number
            e = "(T)(" + bv(id) + ")";
            const std::string name = "t" + std::to_string(id);
            out(id) << "        const T " << name << " = " << e << ";\n";
            done_[id] = name;
            return name;
        }
        switch (n.op) {
            case Op::Const: done_[id] = lit(n.c); return done_[id];
            case Op::Param: e = "(T)a.prm[" + std::to_string(n.i) + "]"; break;
            case Op::Read: e = read(n, nullptr); break;
            case Op::InBox: e = "(T)(" + inbox(n.off, n.off2) + ")"; break;
            case Op::Coord: e = "(T)(" + std::string(1, "xyz"[n.i]) + " + " + std::to_string(n.off[n.i]) + ")"; break;
            case Op::Add: e = v(n.a) + " + " + v(n.b); break;
            case Op::Sub: e = v(n.a) + " - " + v(n.b); break;
            case Op::Mul: e = v(n.a) + " * " + v(n.b); break;
            case Op::Div: e = v(n.a) + " / " + v(n.b); break;
            case Op::Neg: e = "-" + v(n.a); break;
            case Op::Sqrt: e = "sqrt(" + v(n.a) + ")"; break;
            case Op::Sin:
            case Op::Cos: {   // one sincos per angle: both halves share the range reduction
                const std::string x = v(n.a), sn = "s" + std::to_string(n.a), cn = "c" + std::to_string(n.a);
                if (!sincos_.count(n.a)) {
                    out(n.a) << "        T " << sn << ", " << cn << "; opt_sincos(" << x << ", &" << sn << ", &" << cn << ");\n";
                    sincos_.insert(n.a);
                }
                done_[id] = n.op == Op::Sin ? sn : cn;
                return done_[id];
            }
            case Op::Exp: e = "exp(" + v(n.a) + ")"; break;
            case Op::Log: e = "log(" + v(n.a) + ")"; break;
            case Op::Abs: e = "fabs(" + v(n.a) + ")"; break;
            case Op::Pow: e = "pow(" + v(n.a) + ", " + v(n.b) + ")"; break;
            case Op::Select: e = cond(n.a) + " ? " + v(n.b) + " : " + v(n.d); break;
            case Op::Sample:
                e = "opt_sample(" + img_ptr(n.i) + ", " + std::to_string(M_.images[n.i].channels) + ", " +
                    std::to_string(n.ch) + ", " + v(n.a) + ", " + v(n.b) + ", W, H)";
                break;
            case Op::Lt: e = "(T)(" + v(n.a) + " < " + v(n.b) + ")"; break;
            case Op::Le: e = "(T)(" + v(n.a) + " <= " + v(n.b) + ")"; break;
            case Op::Gt: e = "(T)(" + v(n.a) + " > " + v(n.b) + ")"; break;
            case Op::Ge: e = "(T)(" + v(n.a) + " >= " + v(n.b) + ")"; break;
            case Op::Eq: e = "(T)(" + v(n.a) + " == " + v(n.b) + ")"; break;
            case Op::Ne: e = "(T)(" + v(n.a) + " != " + v(n.b) + ")"; break;
            case Op::And: e = "(T)((" + v(n.a) + " != (T)0) && (" + v(n.b) + " != (T)0))"; break;
            case Op::Or: e = "(T)((" + v(n.a) + " != (T)0) || (" + v(n.b) + " != (T)0))"; break;
            case Op::Not: e = "(T)(" + v(n.a) + " == (T)0)"; break;
        }
        const std::string name = "t" + std::to_string(id);
        out(id) << "        const T " << name << " = " << e << ";\n";
        done_[id] = name;
        return name;
    }
    // Boolean-valued nodes — comparisons, And / Or / Not, InBox, products of booleans, the
    // constants 0 and 1 — are emitted as `bool` and turned into T only where a number is
    // needed: the energies' validity masks (inside * (Mask == 0) * ...) become one && chain
    // instead of float compares, conversions and multiplies, and a Select reads them directly
    // (the same 0 / 1 values: a product of 0 / 1 numbers is their logical and).
    bool is_bool(int id) {
        auto it = isb_.find(id);
        if (it != isb_.end()) return it->second;
        const Node n = P_.at(id);
        bool r = false;
        switch (n.op) {
            case Op::Lt: case Op::Le: case Op::Gt: case Op::Ge: case Op::Eq: case Op::Ne:
            case Op::And: case Op::Or: case Op::Not: case Op::InBox: r = true; break;
            case Op::Const: r = n.c == 0.0 || n.c == 1.0; break;
            case Op::Mul: r = is_bool(n.a) && is_bool(n.b); break;
            default: r = false;
        }
        isb_[id] = r;
        return r;
    }
    // node `id` as a C++ condition (nonzero)
    std::string cond(int id) { return is_bool(id) ? bv(id) : "(" + v(id) + " != (T)0)"; }
    // the strip kernels read cached predicates (g_pred) from the bit image's row windows
    void use_pred(bool on) { use_pred_ = on; }
    // the bool value of boolean node `id`
    std::string bv(int id) {
        auto it = bdone_.find(id);
        if (it != bdone_.end()) return it->second;
        const Node n = P_.at(id);
        std::string e;
        int rd = -1;
        const int k = use_pred_ ? pred_bit(P_, n, &rd) : -1;
        if (k >= 0) {
            const int pr = P_.read(g_pred->img, 0, P_.at(rd).off);
            const std::string w = read(P_.at(pr), nullptr);
            e = "((((int)(" + w + ")) >> " + std::to_string(k) + ") & 1) " + (g_pred->at0[k] ? "== 0" : "!= 0");
            const std::string name = "b" + std::to_string(id);
            out(id) << "        const bool " << name << " = " << e << ";\n";
            bdone_[id] = name;
            return name;
        }
        switch (n.op) {
            case Op::Const: bdone_[id] = n.c != 0.0 ? "true" : "false"; return bdone_[id];
            case Op::Lt: e = v(n.a) + " < " + v(n.b); break;
            case Op::Le: e = v(n.a) + " <= " + v(n.b); break;
            case Op::Gt: e = v(n.a) + " > " + v(n.b); break;
            case Op::Ge: e = v(n.a) + " >= " + v(n.b); break;
            case Op::Eq: e = v(n.a) + " == " + v(n.b); break;
            case Op::Ne: e = v(n.a) + " != " + v(n.b); break;
            case Op::And: case Op::Mul: e = cond(n.a) + " && " + cond(n.b); break;
            case Op::Or: e = cond(n.a) + " || " + cond(n.b); break;
            case Op::Not: e = "!" + cond(n.a); break;
            case Op::InBox: e = inbox(n.off, n.off2); break;
            default: e = "false";
        }
        const std::string name = "b" + std::to_string(id);
        out(id) << "        const bool " << name << " = " << e << ";\n";
        bdone_[id] = name;
        return name;
    }
    // the search direction / step vector at unknown access `u` (a Read of an unknown)
    std::string vec(int u, const char* vname) {
        const std::string key = std::string(vname) + std::to_string(u);
        auto it = vdone_.find(key);
        if (it != vdone_.end()) return it->second;
        const Node n = P_.at(u);
        const std::string name = std::string(vname) + "_" + std::to_string(u);
        out(u) << "        const T " << name << " = " << read(n, vname) << ";\n";
        vdone_[key] = name;
        return name;
    }
    void line(const std::string& s) { o_ << "        " << s << "\n"; }
    // register-strip emission (gen_apply_strip): centred reads come from the caller's
    // row windows instead of memory
    void centred_reads(std::function<std::string(const Node&, const char*)> f) { centred_ = std::move(f); }

private:
    std::string coord(int k, int off) const {
        const char c = "xyz"[k];
        return off == 0 ? std::string(1, c) : "(" + std::string(1, c) + (off > 0 ? " + " : " - ") +
                                                   std::to_string(off > 0 ? off : -off) + ")";
    }
    std::string inb(const int* off) const {
        std::string s;
        for (int k = 0; k < nd_; ++k) {
            if (off[k] == 0) continue;   // the thread's own coordinate is always inside
            if (!s.empty()) s += " && ";
            const char* dim = k == 0 ? "W" : k == 1 ? "H" : "D";
            s += coord(k, off[k]) + " >= 0 && " + coord(k, off[k]) + " < " + dim;
        }
        return s.empty() ? "true" : s;
    }
    std::string inbox(const int* lo, const int* hi) const {
        return "(" + inb(lo) + ") && (" + inb(hi) + ")";
    }
    std::string lin(const int* off) const {
        if (nd_ == 1) return "(long long)" + coord(0, off[0]);
        if (nd_ == 2) return "((long long)(" + coord(1, off[1]) + " - a.ymem0) * W + " + coord(0, off[0]) + ")";
        return "(((long long)" + coord(2, off[2]) + " * H + " + coord(1, off[1]) + ") * W + " + coord(0, off[0]) + ")";
    }
    // offset of a centred access from the thread's pixel, in pixels (32-bit: the
    // front end limits the index space, generic_accepts)
    std::string rel(const int* off) const {
        std::string r = std::to_string(off[0]);
        if (nd_ > 1 && off[1]) r += " + " + std::to_string(off[1]) + " * W";
        if (nd_ > 2 && off[2]) r += " + " + std::to_string(off[2]) + " * W * H";
        return "(" + r + ")";
    }
    std::string img_ptr(int i) const {
        const GImage& im = M_.images[i];
        return "((const " + std::string(elem_type(im.elem, im.tvalued)) + "*)a.img[" + std::to_string(i) + "])";
    }
    std::string read(const Node& n, const char* vname) {
        const GImage& im = M_.images[n.i];
        const std::string ch = std::to_string(im.channels), c = std::to_string(n.ch);
        std::string base, idx;
        if (vname) {
            base = std::string(vname) + " + a.uoff[" + std::to_string(uslot_[n.i]) + "]";
        } else {
            base = "((const " + std::string(elem_type(im.elem, im.tvalued)) + "*)a.img[" + std::to_string(n.i) + "])";
        }
        if (n.slot >= 0) {
            if (g_off32) return "(T)opt_g32(" + base + ", v" + std::to_string(n.slot) + ", " + ch + ", " + c + ")";
            idx = "(long long)v" + std::to_string(n.slot) + " * " + ch + " + " + c;
            return "(T)(" + base + ")[" + idx + "]";
        }
        if (centred_) return centred_(n, vname);
        idx ="(li + " + rel(n.off) + ") * " + ch + " + " + c;
        return "opt_ldm(" + base + ", " + idx + ", " + inb(n.off) + ")";
    }

    GModel& M_;
    Pool& P_;
    std::ostringstream& o_;
    int nd_;
    const std::vector<int>& uslot_;
    std::map<int, std::string> done_, bdone_;
    std::map<int, bool> isb_;
    bool use_pred_ = false;
    std::set<int> sincos_, rec_;
    std::map<std::string, std::string> vdone_;
    std::ostringstream* pre_ = nullptr;
    int self_ = -1, graph_ = -1;
    std::map<int, bool> inv_;
    std::function<std::string(const Node&, const char*)> centred_;
};

struct Instance {   // a centred residual shifted so that it contains unknown (image, ch) at 0
    int res;
    int s[3];
};

}  // namespace

GenSource generate(GModel& m, bool dbl, bool off32) {
    GenSource gs;
    g_off32 = off32;
    {
        const char* sv = getenv("OPT_AMD_GEN_STRIP32");
        g_strip32 = sv ? atoi(sv) : 4;
        const char* wv = getenv("OPT_AMD_GEN_WIDU");
        g_widu = wv ? atoi(wv) : 2;
        const char* fv = getenv("OPT_AMD_GEN_FACTOR");
        g_factor = !fv || atoi(fv) != 0;
    }
    const bool s32 = off32 && g_strip32 != 0;
    Pool& P = m.pool;
    const int nd = m.unknown_dims();
    const std::vector<int> unk = m.unknown_images();
    std::vector<int> uslot(m.images.size(), -1);
    for (size_t k = 0; k < unk.size(); ++k) uslot[unk[k]] = (int)k;
    int sb = 0;
    for (size_t g = 0; g < m.graphs.size() && g < 4; ++g) {
        gs.slot_base[g] = sb;
        sb += (int)m.graphs[g].slot_names.size();
    }
    for (auto& r : m.residuals) (r.graph < 0 ? gs.has_centered : gs.has_graph) = true;
    // graph edge loops: vertex ids one edge ahead (OPT_AMD_GEN_NB_PREFETCH=0: at use);
    // OPT_AMD_GEN_EDGE_UNROLL=k: unroll the gathers' edge loops k times
    const char* pfv = getenv("OPT_AMD_GEN_NB_PREFETCH");
    const bool prefetch_nb = !pfv || atoi(pfv) != 0;
    // (generated ARAP 1M vertices, profiles/r03_unroll_ab.json: apply 89 / 82-83 / 81 us at
    // 1 / 2 / 4, GN step 1.63 / 1.63 / 1.56-1.58 ms; 4 by default, 1 = no pragma)
    const char* urv = getenv("OPT_AMD_GEN_EDGE_UNROLL");
    const int unr = urv ? atoi(urv) : 4;
    const std::string unroll = unr > 1 ? "#pragma unroll " + std::to_string(unr) + "\n" : "";

    std::ostringstream o;
    o << "// generated by opt_amd's energy front end (gen/codegen.cpp)\n";
    o << "typedef " << (dbl ? "double" : "float") << " T;\n";
    o << "typedef T OptV4 __attribute__((ext_vector_type(4)));\n";
    o << OPTAMD_STR(OPTAMD_GENARGS_BODY) << "\n";
    o << kReduceDevSrc << "\n";
    o << "#define OPT_COORDS const int W = a.dims[0], H = a.dims[1], D = a.dims[2]; (void)D;\n";
    o << "__device__ __forceinline__ void opt_sincos(float x, float* s, float* c) { sincosf(x, s, c); }\n"
         "__device__ __forceinline__ void opt_sincos(double x, double* s, double* c) { sincos(x, s, c); }\n";
    // whole-wave DPP lane shifts (wave_shl:1 / wave_shr:1): opt_sh(v, d) is v of lane l + d
    // (0 past the wave's ends); d is a literal at every use, so the loops unroll away
    // (bound_ctrl: the hardware shifts 0 into the end lane, no register set to 0 first)
    o << "__device__ __forceinline__ float opt_lr(float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true)); }\n"
         "__device__ __forceinline__ float opt_ll(float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true)); }\n"
         "__device__ __forceinline__ double opt_dd(double v, bool r) {\n"
         "    const long long b = __double_as_longlong(v);\n"
         "    const int lo = r ? __builtin_amdgcn_update_dpp(0, (int)b, 0x130, 0xf, 0xf, true) : __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xf, 0xf, true);\n"
         "    const int hi = r ? __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x130, 0xf, 0xf, true) : __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xf, 0xf, true);\n"
         "    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);\n}\n"
         "__device__ __forceinline__ double opt_lr(double v) { return opt_dd(v, true); }\n"
         "__device__ __forceinline__ double opt_ll(double v) { return opt_dd(v, false); }\n"
         "__device__ __forceinline__ T opt_sh(T v, int d) { for (; d > 0; --d) v = opt_lr(v); for (; d < 0; ++d) v = opt_ll(v); return v; }\n";
    // masked read without a branch: the load always issues (at element 0 of the array when
    // the access is outside), the value is selected afterwards
    // XCD-contiguous block order for the graph kernels and the register strips: the
    // hardware deals blocks to the 8 XCDs round robin, so with blockIdx order a vertex's
    // mesh neighbours (v +- 1, v +- a row) are gathered on several XCDs and cached in each
    // one's L2; with this order each XCD walks one contiguous eighth of the vertices (of
    // each grid-stride pass), and neighbouring strips, which share their halo columns, run
    // on the same XCD (generated image_warping / shape_from_shading GN / LM steps 6.91-6.92 ->
    // 6.86 / 3.87-3.89 -> 3.84-3.85 ms, same box; the grid-stride centred kernels gained
    // nothing, poisson's lost: they keep blockIdx order)
    o << "__device__ __forceinline__ long long opt_xcd_block() {\n"
         "    const int nb = gridDim.x, b = blockIdx.x, q = nb / 8, r = nb % 8, x = b % 8;\n"
         "    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;\n}\n";
    // element v * stride + c of b, addressed as b + a 32-bit byte offset to element v's
    // record (generate's off32) + c: the channel stays a constant offset of the same
    // address, so a record's channels merge into one multi-dword load (a channel inside
    // the 32-bit sum cannot: the compiler must allow for its wrap-around)
    o << "template <typename E> __device__ __forceinline__ E opt_g32(const E* b, int v, unsigned stride, unsigned c) {\n"
         "    return ((const E*)((const char*)b + (unsigned)v * (stride * (unsigned)sizeof(E))))[c];\n}\n";
    // the same reads and element access through a 32-bit byte offset from a uniform base
    // (generate's off32: every array below 2 GiB): global_load / global_store with an SGPR
    // base and one VGPR offset, no 64-bit address arithmetic per access
    // O: the byte offset passes through an empty asm (opt_o32). Left visible, the compiler
    // shares one 64-bit extension of it between arrays and adds each base in 64 bits per
    // access; kept opaque, every access takes the SGPR-base form — which measured faster for
    // kernels whose windows are all single-channel (generated shape_from_shading 161 ->
    // 150 us) and slower where two-channel pair reads share the offsets (image_warping 192 ->
    // 205 us), so the strip kernels choose per kernel (OPT_AMD_GEN_STRIP32)
    o << "__device__ __forceinline__ unsigned opt_o32(unsigned o) { asm(\"\" : \"+v\"(o)); return o; }\n"
         "template <bool O, typename E> __device__ __forceinline__ const E& opt_at32(const E* b, unsigned i) {\n"
         "    const unsigned o = i * (unsigned)sizeof(E); return *(const E*)((const char*)b + (O ? opt_o32(o) : o));\n}\n"
         "template <bool O, typename E> __device__ __forceinline__ E& opt_at32(E* b, unsigned i) {\n"
         "    const unsigned o = i * (unsigned)sizeof(E); return *(E*)((char*)b + (O ? opt_o32(o) : o));\n}\n"
         "template <bool O, typename E> __device__ __forceinline__ T opt_ldm32(const E* b, unsigned i, bool c) {\n"
         "    const E v = opt_at32<O>(b, c ? i : 0u); return c ? (T)v : (T)0;\n}\n"
         "template <bool O, typename E> __device__ __forceinline__ void opt_ldm2_32(const E* b, unsigned i, bool c, T& v0, T& v1) {\n"
         "    const unsigned j = c ? i : 0u;\n"
         "    E x, y;\n"
         "    if ((((unsigned long long)b) & (2 * sizeof(E) - 1)) == 0) {\n"
         "        struct alignas(2 * sizeof(E)) P2 { E x, y; };\n"
         "        const unsigned o = j * (unsigned)sizeof(E);\n"
         "        const P2 v = *(const P2*)((const char*)b + (O ? opt_o32(o) : o)); x = v.x; y = v.y;\n"
         "    } else { x = opt_at32<O>(b, j); y = opt_at32<O>(b, j + 1); }\n"
         "    v0 = c ? (T)x : (T)0; v1 = c ? (T)y : (T)0;\n}\n";
    o << "template <typename E> __device__ __forceinline__ T opt_ldm(const E* b, long long i, bool c) {\n"
         "    const E v = b[c ? i : 0]; return c ? (T)v : (T)0;\n}\n"
         // both channels of a 2-channel element (i = its first channel) in one access when
         // the array is aligned for it (a uniform branch), else two
         "template <typename E> __device__ __forceinline__ void opt_ldm2(const E* b, long long i, bool c, T& v0, T& v1) {\n"
         "    const long long j = c ? i : 0;\n"
         "    E x, y;\n"
         "    if ((((unsigned long long)b) & (2 * sizeof(E) - 1)) == 0) {\n"
         "        struct alignas(2 * sizeof(E)) P2 { E x, y; };\n"
         "        const P2 v = *reinterpret_cast<const P2*>(b + j); x = v.x; y = v.y;\n"
         "    } else { x = b[j]; y = b[j + 1]; }\n"
         "    v0 = c ? (T)x : (T)0; v1 = c ? (T)y : (T)0;\n}\n";
    // Image:get / Image:sample (o.t:856-876): floor / ceil taps, zero outside, lerps in T
    o << "template <typename E> __device__ __forceinline__ T opt_tap(const E* im, int nch, int c, int x, int y, int W, int H) {\n"
         "    return (x >= 0 && x < W && y >= 0 && y < H) ? (T)im[((long long)y * W + x) * nch + c] : (T)0;\n}\n"
         "template <typename E> __device__ __forceinline__ T opt_sample(const E* im, int nch, int c, T x, T y, int W, int H) {\n"
         "    const int x0 = (int)floor(x), x1 = (int)ceil(x), y0 = (int)floor(y), y1 = (int)ceil(y);\n"
         "    const T xn = x - (T)x0, yn = y - (T)y0;\n"
         "    const T u = ((T)1 - xn) * opt_tap(im, nch, c, x0, y0, W, H) + xn * opt_tap(im, nch, c, x1, y0, W, H);\n"
         "    const T b = ((T)1 - xn) * opt_tap(im, nch, c, x0, y1, W, H) + xn * opt_tap(im, nch, c, x1, y1, W, H);\n"
         "    return ((T)1 - yn) * u + yn * b;\n}\n";
    // memory pixel index -> coordinates; 2-D energies may hold a row slab whose memory row 0
    // is global row a.ymem0 (coordinates, bounds and Index(1) are global)
    // (32-bit unsigned divisions: the pixel index fits an int, as `li` assumes; a 64-bit
    // division is a ~100-instruction sequence per pixel)
    const char* coords = nd == 2
        ? "        const unsigned ul = (unsigned)lin, uq = ul / (unsigned)W;\n"
          "        const int x = (int)(ul - uq * (unsigned)W); const int y = (int)uq + a.ymem0; const int z = 0;\n"
          "        const int li = (int)lin; (void)x; (void)y; (void)z; (void)li;\n"
        : "        const unsigned ul = (unsigned)lin, uq = ul / (unsigned)W, uz = uq / (unsigned)H;\n"
          "        const int x = (int)(ul - uq * (unsigned)W); const int y = (int)(uq - uz * (unsigned)H); const int z = (int)uz;\n"
          "        const int li = (int)lin; (void)x; (void)y; (void)z; (void)li;\n";

    // centred instances per output (unknown image, channel)
    std::map<std::pair<int, int>, std::vector<std::pair<Instance, int>>> inst;   // -> (instance, support node)
    for (size_t ri = 0; ri < m.residuals.size(); ++ri) {
        const GResidual& r = m.residuals[ri];
        if (r.graph >= 0) continue;
        for (int u : r.unknowns) {
            const Node n = P.at(u);
            Instance I{(int)ri, {-n.off[0], -n.off[1], -n.off[2]}};
            inst[{n.i, n.ch}].push_back({I, u});
        }
    }
    auto shifted = [&](int id, const int* s) { return P.shift(id, s); };
    const int zero3[3] = {0, 0, 0};

    // --------------------------------------------- gen_precompute_<k> (ComputedArrays)
    // One kernel per ComputedArray, launched in declaration order (a later one may read an
    // earlier one at an offset): the values and the non-constant gradient images
    // (createprecomputed, o.t:3131-3153).
    for (size_t k = 0; k < m.computed.size(); ++k) {
        const GComputed& c = m.computed[k];
        o << "extern \"C\" __global__ __launch_bounds__(256) void gen_precompute_" << k << "(GenArgs a) {\n"
             "    OPT_COORDS\n"
             "    for (long long lin = a.own_lo + (long long)blockIdx.x * 256 + threadIdx.x; lin < a.own_hi; lin += (long long)gridDim.x * 256) {\n"
          << coords;
        Body b(m, o, nd, uslot);
        const int nch = (int)c.expr.size();
        for (int ch = 0; ch < nch; ++ch)
            b.line("((T*)a.img[" + std::to_string(c.image) + "])[lin * " + std::to_string(nch) + " + " + std::to_string(ch) +
                   "] = " + b.v(c.expr[ch]) + ";");
        for (const GGrad& g : c.grads)
            if (g.gimg >= 0) b.line("((T*)a.img[" + std::to_string(g.gimg) + "])[lin] = " + b.v(g.expr) + ";");
        o << "    }\n}\n";
    }
    gs.n_precompute = (int)m.computed.size();

    // ------------------------------------------------ transcendental caches (see g_cache)
    // Worth it when residuals have instances at several shifts (each would re-evaluate
    // its neighbours' transcendentals): cache every sin / cos / exp / log / sqrt of a
    // centred read the residuals use, one internal image each, filled by one extra
    // precompute kernel after the ComputedArrays.
    CacheMap cache;
    {
        bool multi = false;
        for (auto& r : m.residuals) {
            if (r.graph >= 0) continue;
            std::set<std::string> offs;
            for (int u : r.unknowns) {
                const Node n = P.at(u);
                offs.insert(std::to_string(n.off[0]) + "," + std::to_string(n.off[1]) + "," + std::to_string(n.off[2]));
            }
            multi |= offs.size() > 1;
        }
        std::vector<std::pair<std::tuple<int, int, int>, int>> want;   // key -> a node with offset 0 form
        if (multi)
            for (auto& r : m.residuals) {
                if (r.graph >= 0) continue;
                P.visit(r.expr, [&](int, const Node& n) {
                    if (!cacheable(P, n)) return;
                    const Node c = P.at(n.a);
                    auto key = std::make_tuple((int)n.op, c.i, c.ch);
                    for (auto& w : want)
                        if (w.first == key) return;
                    const int z0[3] = {0, 0, 0};
                    want.push_back({key, P.un(n.op, P.read(c.i, c.ch, z0))});
                });
            }
        if (!want.empty()) {
            o << "extern \"C\" __global__ __launch_bounds__(256) void gen_precompute_" << gs.n_precompute << "(GenArgs a) {\n"
                 "    OPT_COORDS\n"
                 "    for (long long lin = a.own_lo + (long long)blockIdx.x * 256 + threadIdx.x; lin < a.own_hi; lin += (long long)gridDim.x * 256) {\n"
              << coords;
            Body b(m, o, nd, uslot);
            const int uimg = unk.empty() ? 0 : unk[0];
            for (auto& w : want) {
                if (m.images.size() >= 16) break;   // GenArgs::img capacity
                GImage ci;
                ci.name = "cache_" + std::to_string(std::get<0>(w.first)) + "_" + std::to_string(std::get<1>(w.first)) +
                          "_" + std::to_string(std::get<2>(w.first));
                ci.dims = m.images[uimg].dims;
                ci.internal = ci.tvalued = true;
                m.images.push_back(ci);
                const int id = (int)m.images.size() - 1;
                cache[w.first] = id;
                b.line("((T*)a.img[" + std::to_string(id) + "])[lin] = " + b.v(w.second) + ";");
            }
            o << "    }\n}\n";
            if (!cache.empty()) ++gs.n_precompute;
        }
    }
    g_cache = cache.empty() ? nullptr : &cache;

    // predicate cache (see g_pred): up to 8 comparisons of a user array on the unknowns'
    // domain with a constant, from the centred residuals and the Exclude expression
    PredCache pcache;
    {
        const char* pv = getenv("OPT_AMD_GEN_PRED");
        const bool on = !pv || atoi(pv) != 0;
        const int uimg = unk.empty() ? -1 : unk[0];
        auto cmp0 = [](Op op, double l, double r) {
            switch (op) {
                case Op::Lt: return l < r;
                case Op::Le: return l <= r;
                case Op::Gt: return l > r;
                case Op::Ge: return l >= r;
                case Op::Eq: return l == r;
                default: return l != r;
            }
        };
        auto consider = [&](int root) {
            P.visit(root, [&](int, const Node& n) {
                if (n.op != Op::Lt && n.op != Op::Le && n.op != Op::Gt && n.op != Op::Ge && n.op != Op::Eq &&
                    n.op != Op::Ne)
                    return;
                double c;
                bool left;
                int rd;
                if (P.is_const(n.b, &c) && P.at(n.a).op == Op::Read) { left = true; rd = n.a; }
                else if (P.is_const(n.a, &c) && P.at(n.b).op == Op::Read) { left = false; rd = n.b; }
                else return;
                const Node r = P.at(rd);
                if (r.slot >= 0) return;
                const GImage& im = m.images[r.i];
                if (im.unknown || im.internal || im.dims != m.images[uimg].dims) return;
                const auto key = std::make_tuple((int)n.op, r.i, r.ch, c, left);
                for (auto& k : pcache.keys)
                    if (k == key) return;
                if (pcache.keys.size() >= 8) return;
                pcache.keys.push_back(key);
                pcache.at0.push_back(left ? cmp0(n.op, 0.0, c) : cmp0(n.op, c, 0.0));
            });
        };
        if (on && uimg >= 0 && m.images.size() < 16 && nd == 2) {
            for (auto& r : m.residuals)
                if (r.graph < 0) consider(r.expr);
            if (m.exclude >= 0) consider(m.exclude);
        }
        if (!pcache.keys.empty()) {
            GImage pi;
            pi.name = "pred_bits";
            pi.dims = m.images[uimg].dims;
            pi.internal = true;
            pi.tvalued = false;
            pi.elem = "uint8";
            pi.channels = 1;
            m.images.push_back(pi);
            pcache.img = (int)m.images.size() - 1;
            o << "extern \"C\" __global__ __launch_bounds__(256) void gen_precompute_" << gs.n_precompute << "(GenArgs a) {\n"
                 "    OPT_COORDS\n"
                 "    for (long long lin = a.own_lo + (long long)blockIdx.x * 256 + threadIdx.x; lin < a.own_hi; lin += (long long)gridDim.x * 256) {\n"
              << coords;
            Body b(m, o, nd, uslot);
            b.line("unsigned bits = 0;");
            const int z0[3] = {0, 0, 0};
            for (size_t k = 0; k < pcache.keys.size(); ++k) {
                const auto& key = pcache.keys[k];
                const Op op = (Op)std::get<0>(key);
                const int rd0 = P.read(std::get<1>(key), std::get<2>(key), z0), cn = P.cnst(std::get<3>(key));
                const int pn = std::get<4>(key) ? P.bin(op, rd0, cn) : P.bin(op, cn, rd0);
                b.line("bits |= (" + b.cond(pn) + (pcache.at0[k] ? " ? 0u : 1u" : " ? 1u : 0u") + ") << " +
                       std::to_string(k) + ";");
            }
            b.line("((unsigned char*)a.img[" + std::to_string(pcache.img) + "])[lin] = (unsigned char)bits;");
            o << "    }\n}\n";
            ++gs.n_precompute;
        }
    }
    g_pred = pcache.keys.empty() ? nullptr : &pcache;

    // graph record cache (see g_gcache): transcendentals of slot reads of arrays on the
    // unknowns' domain, one record per vertex, filled by one more precompute kernel
    GraphCache gcache;
    {
        const char* ev = getenv("OPT_AMD_GEN_GRAPH_CACHE");
        const bool on = !ev || atoi(ev) != 0;
        const int uimg = unk.empty() ? -1 : unk[0];
        std::vector<std::pair<std::tuple<int, int, int>, int>> want;
        if (on && uimg >= 0 && m.images.size() < 16)
            for (auto& r : m.residuals) {
                if (r.graph < 0) continue;
                P.visit(r.expr, [&](int, const Node& n) {
                    if (!cacheable_slot(P, n)) return;
                    const Node c = P.at(n.a);
                    if (m.images[c.i].dims != m.images[uimg].dims) return;
                    auto key = std::make_tuple((int)n.op, c.i, c.ch);
                    for (auto& w : want)
                        if (w.first == key) return;
                    const int z0[3] = {0, 0, 0};
                    want.push_back({key, P.un(n.op, P.read(c.i, c.ch, z0))});
                });
            }
        if (!want.empty()) {
            int width = 1;
            while (width < (int)want.size()) width *= 2;   // aligned records
            GImage ci;
            ci.name = "graph_cache";
            ci.dims = m.images[uimg].dims;
            ci.channels = width;
            ci.internal = ci.tvalued = true;
            m.images.push_back(ci);
            gcache.img = (int)m.images.size() - 1;
            gcache.width = width;
            o << "extern \"C\" __global__ __launch_bounds__(256) void gen_precompute_" << gs.n_precompute << "(GenArgs a) {\n"
                 "    OPT_COORDS\n"
                 "    for (long long lin = a.own_lo + (long long)blockIdx.x * 256 + threadIdx.x; lin < a.own_hi; lin += (long long)gridDim.x * 256) {\n"
              << coords;
            Body b(m, o, nd, uslot);
            std::vector<std::string> val(width, "(T)0");
            for (size_t k = 0; k < want.size(); ++k) {
                gcache.ch[want[k].first] = (int)k;
                val[k] = b.v(want[k].second);
            }
            // whole 16-byte vectors per record (width >= 4), scalar stores below that
            const std::string base = "((T*)a.img[" + std::to_string(gcache.img) + "]) + lin * " + std::to_string(width);
            if (width >= 4) {
                for (int g = 0; g < width; g += 4)
                    b.line("*(OptV4*)(" + base + " + " + std::to_string(g) + ") = OptV4{" + val[g] + ", " + val[g + 1] + ", " +
                           val[g + 2] + ", " + val[g + 3] + "};");
            } else {
                for (int k = 0; k < width; ++k) b.line("(" + base + ")[" + std::to_string(k) + "] = " + val[k] + ";");
            }
            o << "    }\n}\n";
            ++gs.n_precompute;
        }
    }
    g_gcache = gcache.img < 0 ? nullptr : &gcache;

    // ---------------------------------------------------------------- gen_jtf
    {
        o << "extern \"C\" __global__ __launch_bounds__(256) void gen_jtf(GenArgs a, T* __restrict__ r, T* __restrict__ diag) {\n"
             "    OPT_COORDS\n"
             "    for (long long lin = a.own_lo + (long long)blockIdx.x * 256 + threadIdx.x; lin < a.own_hi; lin += (long long)gridDim.x * 256) {\n"
          << coords;
        Body b(m, o, nd, uslot);
        const std::string act = m.exclude >= 0 ? "(" + b.v(m.exclude) + " == (T)0)" : "true";
        b.line("const bool act = " + act + ";");
        b.line("a.flags[lin] = act ? 1 : 0;");
        for (int k : unk) {
            const GImage& im = m.images[k];
            for (int c = 0; c < im.channels; ++c) {
                std::vector<std::string> F, Dg;
                for (auto& ent : inst[{k, c}]) {
                    const GResidual& r = m.residuals[ent.first.res];
                    const int R = shifted(r.expr, ent.first.s);
                    const int g = shifted(P.diff(r.expr, ent.second), ent.first.s);
                    if (P.is_const(g)) {
                        double gv;
                        P.is_const(g, &gv);
                        if (gv == 0.0) continue;
                    }
                    const std::string gn = b.v(g), rn = b.v(R);
                    F.push_back(gn + " * " + rn);
                    Dg.push_back(gn + " * " + gn);
                }
                const std::string e = "a.uoff[" + std::to_string(uslot[k]) + "] + lin * " + std::to_string(im.channels) +
                                      " + " + std::to_string(c);
                std::string fs = "(T)0", ds = "(T)0";
                for (auto& t : F) fs += " + " + t;
                for (auto& t : Dg) ds += " + " + t;
                b.line("{ const T F = " + fs + "; const T Dg = " + ds + ";");
                b.line("  r[" + e + "] = act ? -F : (T)0; diag[" + e + "] = Dg; }");
            }
        }
        o << "    }\n}\n";
    }

    // ------------------------------------------------------------ gen_apply_tiled
    // Two-phase J^T J p over 2-D output tiles whose tile + halo region is 32 x 8 or 16 x 16.
    // Phase 1 evaluates every centred residual ONCE per centre q of the tile and the halo
    // its outputs gather from: the non-constant partials d(r, u)(q) and Jp_r(q) = sum_u
    // d(r, u)(q) p(q + off(u)), kept in LDS. Phase 2 gathers each output x from
    // d(r, u)(x - off(u)) * Jp_r(x - off(u)). The gather form of createjtjcentered
    // (o.t:2770-2830, what gen_apply does) re-evaluates each residual instance's partials
    // for every pixel that reads it; here each is computed once per centre (plus the halo).
    struct Entry { int r; int u; int dnode; int slot; int ox, oy; };   // slot -1: constant partial
    std::vector<int> cres;                                           // centred residual ids
    std::vector<Entry> ents;
    int nd_slots = 0;
    int minx = 0, maxx = 0, miny = 0, maxy = 0;
    int PX = 32, PY = 8, TX = 0, TY = 0, nf = 0;
    size_t lds = 0;
    bool tiled = false;
    if (gs.has_centered && nd == 2) {
        for (size_t ri = 0; ri < m.residuals.size(); ++ri) {
            const GResidual& r = m.residuals[ri];
            if (r.graph >= 0 || r.unknowns.empty()) continue;
            cres.push_back((int)ri);
            for (int u : r.unknowns) {
                const Node n = P.at(u);
                const int d = P.diff(r.expr, u);
                double gv;
                if (P.is_const(d, &gv) && gv == 0.0) continue;
                Entry e{(int)cres.size() - 1, u, d, P.is_const(d) ? -1 : nd_slots++, n.off[0], n.off[1]};
                ents.push_back(e);
                minx = std::min(minx, n.off[0]); maxx = std::max(maxx, n.off[0]);
                miny = std::min(miny, n.off[1]); maxy = std::max(maxy, n.off[1]);
            }
        }
        // phase 1 covers the tile + halo in exactly one pass of the 256 threads: pick the
        // region shape (32 x 8 or 16 x 16) that leaves the most output pixels
        const int sx = maxx - minx, sy = maxy - miny;
        if ((16 - sx) * (16 - sy) > (32 - sx) * (8 - sy)) PX = PY = 16;
        TX = PX - sx;
        TY = PY - sy;
        nf = (int)cres.size() + nd_slots;
        lds = (size_t)nf * PX * PY * (dbl ? 8 : 4);
        tiled = !cres.empty() && TX > 0 && TY > 0 && lds <= 64 * 1024;
        // the gather evaluates every distinct (residual, shift) instance per pixel; the
        // tiled form evaluates each residual once per centre (+ halo) but pays LDS traffic
        // and barriers. Measured: the gather wins at ~2 instances per
        // residual (image_warping, poisson, optical_flow), the tiles at ~4.7
        // (shape_from_shading, radius-2 supports through ComputedArray gradient images).
        std::set<std::string> inst_keys;
        for (const Entry& e : ents)
            inst_keys.insert(std::to_string(e.r) + ":" + std::to_string(e.ox) + "," + std::to_string(e.oy));
        gs.instances_per_residual = cres.empty() ? 0.0 : (double)inst_keys.size() / cres.size();
        gs.prefer_tiled = tiled && gs.instances_per_residual > 3.0;
    }


    // -------------------------------------------------------------- gen_apply
    // The gather form of the centred J^T J p at pixel `lin` (coordinates in scope). fused:
    // inside gen_apply_graph, the sum of output (k, c) goes to cacc<slot>_<c> (declared by
    // the caller) instead of Ap
    auto centred_apply = [&](Body& b, bool fused) {
        if (!fused) b.line("const bool act = (a.flags[lin] & 1) != 0;");
        std::map<std::string, std::string> jp;   // (residual, shift) -> J p of that instance
        for (int k : unk) {
            const GImage& im = m.images[k];
            for (int c = 0; c < im.channels; ++c) {
                std::vector<std::string> terms;
                for (auto& ent : inst[{k, c}]) {
                    const GResidual& r = m.residuals[ent.first.res];
                    const int* s = ent.first.s;
                    const int g = shifted(P.diff(r.expr, ent.second), s);
                    double gv;
                    if (P.is_const(g, &gv) && gv == 0.0) continue;
                    const std::string key = std::to_string(ent.first.res) + ":" + std::to_string(s[0]) + "," +
                                            std::to_string(s[1]) + "," + std::to_string(s[2]);
                    if (!jp.count(key)) {
                        std::string sum = "(T)0";
                        for (int u : r.unknowns) {
                            const int gu = shifted(P.diff(r.expr, u), s);
                            if (P.is_const(gu, &gv) && gv == 0.0) continue;
                            sum += " + " + b.v(gu) + " * " + b.vec(shifted(u, s), "p");
                        }
                        const std::string nm = "jp" + std::to_string(jp.size());
                        b.line("const T " + nm + " = " + sum + ";");
                        jp[key] = nm;
                    }
                    terms.push_back(b.v(g) + " * " + jp[key]);
                }
                std::string acc = "(T)0";
                for (auto& t : terms) acc += " + " + t;
                if (fused) {
                    b.line("cacc" + std::to_string(uslot[k]) + "_" + std::to_string(c) + " = " + acc + ";");
                    continue;
                }
                const std::string e = "a.uoff[" + std::to_string(uslot[k]) + "] + lin * " + std::to_string(im.channels) +
                                      " + " + std::to_string(c);
                b.line("{ const long long e = " + e + "; const T acc = " + acc + ";");
                b.line("  if (finish) { const T pe = p[e]; const T o = act ? acc + (dadd ? dadd[e] * pe : (T)0) : (T)0; Ap[e] = o; dot += pe * o; }");
                b.line("  else Ap[e] = acc; }");
            }
        }
    };
    {
        o << "extern \"C\" __global__ __launch_bounds__(256) void gen_apply(GenArgs a, const T* __restrict__ p, T* __restrict__ Ap,\n"
             "        const T* __restrict__ dadd, const int* stop, ReduceSlot rs, int finish) {\n"
             "    if (stop && *stop) return;\n"
             "    OPT_COORDS\n"
             "    T dot = 0;\n";
        o << "    for (long long lin = a.own_lo + (long long)blockIdx.x * 256 + threadIdx.x; lin < a.own_hi; lin += (long long)gridDim.x * 256) {\n"
              << coords;
        Body b(m, o, nd, uslot);
        centred_apply(b, false);
        o << "    }\n"
             "    if (finish) { double v[1] = {(double)dot}; block_reduce_publish<1>(v, rs, blockIdx.x); }\n}\n";
    }

    if (tiled) {
            gs.has_tiled = true;
            gs.tiles_x = TX;
            gs.tiles_y = TY;
            gs.tiled_lds = lds;
            const int PXY = PX * PY;
            o << "extern \"C\" __global__ __launch_bounds__(256) void gen_apply_tiled(GenArgs a, const T* __restrict__ p, T* __restrict__ Ap,\n"
                 "        const T* __restrict__ dadd, const int* stop, ReduceSlot rs, int finish) {\n"
                 "    if (stop && *stop) return;\n"
                 "    OPT_COORDS\n"
                 "    __shared__ T lds[" << nf * PXY << "];\n"
                 "    T dot = 0;\n"
                 "    const int ntx = (W + " << TX - 1 << ") / " << TX << ", nty = (H + " << TY - 1 << ") / " << TY << ";\n"
                 "    for (int t = blockIdx.x; t < ntx * nty; t += gridDim.x) {\n"
                 "        const int X0 = (t % ntx) * " << TX << ", Y0 = (t / ntx) * " << TY << ";\n"
                 "        for (int idx = threadIdx.x; idx < " << PXY << "; idx += 256) {   // one pass\n"
                 "        const int x = X0 - " << maxx << " + idx % " << PX << ", y = Y0 - " << maxy << " + idx / " << PX << ";\n"
                 "        const int z = 0; (void)z;\n"
                 "        const int li = (y - a.ymem0) * W + x; (void)li;\n"
                 "        if (x >= 0 && x < W && y >= 0 && y < H) {\n";
            {
                Body b(m, o, nd, uslot);
                std::vector<std::string> dname(ents.size());
                for (size_t ci = 0; ci < cres.size(); ++ci) {
                    const GResidual& r = m.residuals[cres[ci]];
                    std::string sum = "(T)0";
                    for (size_t ei = 0; ei < ents.size(); ++ei) {
                        if (ents[ei].r != (int)ci) continue;
                        const std::string dn = b.v(ents[ei].dnode);
                        if (ents[ei].slot >= 0)
                            b.line("lds[" + std::to_string((cres.size() + ents[ei].slot) * PXY) + " + idx] = " + dn + ";");
                        sum += " + " + dn + " * " + b.vec(ents[ei].u, "p");
                    }
                    (void)r;
                    b.line("lds[" + std::to_string(ci * PXY) + " + idx] = " + sum + ";");
                }
            }
            o << "        } else {   // no residual is centred outside the domain (and 0 * stale LDS could be NaN)\n";
            for (int fi = 0; fi < nf; ++fi)
                o << "            lds[" << fi * PXY << " + idx] = (T)0;\n";
            o << "        }\n"
                 "        }\n"
                 "        __syncthreads();\n"
                 "        {\n"
                 "        const int lx = threadIdx.x % " << TX << ", ly = threadIdx.x / " << TX << ";\n"
                 "        const int x = X0 + lx, y = Y0 + ly;\n"
                 "        if (threadIdx.x < " << TX * TY << " && x < W && y < H) {\n"
                 "        const long long lin = (long long)(y - a.ymem0) * W + x;\n"
                 "        const bool act = (a.flags[lin] & 1) != 0;\n";
            for (int k : unk) {
                const GImage& im = m.images[k];
                for (int c = 0; c < im.channels; ++c) {
                    std::string acc = "(T)0";
                    for (const Entry& e : ents) {
                        const Node n = P.at(e.u);
                        if (n.i != k || n.ch != c) continue;
                        // centre q = x - off(u), local index in the tile + halo region
                        const std::string qi = "(lx + " + std::to_string(maxx - e.ox) + ") + (ly + " +
                                               std::to_string(maxy - e.oy) + ") * " + std::to_string(PX);
                        std::string dv;
                        if (e.slot >= 0) {
                            dv = "lds[" + std::to_string((cres.size() + e.slot) * PXY) + " + " + qi + "]";
                        } else {
                            double cv;
                            P.is_const(e.dnode, &cv);
                            dv = lit(cv);
                        }
                        acc += " + " + dv + " * lds[" + std::to_string(e.r * PXY) + " + " + qi + "]";
                    }
                    const std::string el = "a.uoff[" + std::to_string(uslot[k]) + "] + lin * " + std::to_string(im.channels) +
                                           " + " + std::to_string(c);
                    o << "        { const long long e = " << el << "; const T acc = " << acc << ";\n"
                         "          if (finish) { const T pe = p[e]; const T o = act ? acc + (dadd ? dadd[e] * pe : (T)0) : (T)0; Ap[e] = o; dot += pe * o; }\n"
                         "          else Ap[e] = acc; }\n";
                }
            }
            o << "        }\n"
                 "        }\n"
                 "        __syncthreads();\n"
                 "    }\n"
                 "    if (finish) { double v[1] = {(double)dot}; block_reduce_publish<1>(v, rs, blockIdx.x); }\n}\n";
        }

    // ------------------------------------------------------------ gen_apply_strip
    // J^T J p in registers: each wave owns a column strip (one pixel per lane, halo lanes
    // at both ends) and walks down a block of rows. Every centred residual is evaluated
    // ONCE per centre (as the tiled form), its reads served from per-array row windows
    // (the rows centre + dy the residuals touch; a column offset dx is a DPP lane shift);
    // each centre's contributions d(r, u) Jp_r are summed per output offset (u's offset),
    // lane-shifted to the output column and added to rolling per-row accumulators; an
    // output row is finished once the last centre row that reaches it has been evaluated.
    // No LDS and no barriers: the hand-written image_warping / SFS applies work this way.
    // Same instance set as createjtjcentered (o.t:2770-2830): centres outside the image
    // contribute nothing (gen_apply_tiled's rule).
    // gen_jtf_strip: the same walk for J^T F + diag(J^T J) + flags: each centre's residual
    // values R_r and partials d(r, u) once, d R and d^2 accumulated per output offset; the
    // output's Exclude is evaluated at the output row (shifted by miny). Same instance set.
    auto strip_kernel = [&](bool jtf) {
        bool ok = true;
        for (int ci : cres)
            P.visit(m.residuals[ci].expr, [&](int, const Node& n) { ok &= n.op != Op::Sample; });
        if (jtf && m.exclude >= 0)
            P.visit(m.exclude, [&](int, const Node& n) { ok &= n.op != Op::Sample && !(n.op == Op::Read && n.slot >= 0); });
        // rows each (p?, image, channel) window must hold, lane reach of the reads
        std::map<std::tuple<int, int, int>, std::pair<int, int>> win;
        int rxlo = 0, rxhi = 0;
        auto wname = [](const std::tuple<int, int, int>& k, int dy) {
            return std::string(std::get<0>(k) ? "wp" : "wi") + std::to_string(std::get<1>(k)) + "c" +
                   std::to_string(std::get<2>(k)) + (dy < 0 ? "m" : "p") + std::to_string(std::abs(dy));
        };
        std::ostringstream body, fin;
        const CacheMap* saved = g_cache;
        g_cache = nullptr;   // sin / cos of a window value: no cache images
        {
            Body b(m, body, nd, uslot);
            b.use_pred(true);
            b.centred_reads([&](const Node& n, const char* vname) {
                const auto key = std::make_tuple(vname ? 1 : 0, n.i, n.ch);
                auto it = win.find(key);
                if (it == win.end()) win[key] = {n.off[1], n.off[1]};
                else it->second = {std::min(it->second.first, n.off[1]), std::max(it->second.second, n.off[1])};
                rxlo = std::min(rxlo, n.off[0]);
                rxhi = std::max(rxhi, n.off[0]);
                const std::string w = wname(key, n.off[1]);
                return n.off[0] == 0 ? w : "opt_sh(" + w + ", " + std::to_string(n.off[0]) + ")";
            });
            std::vector<std::string> dname(ents.size());
            for (size_t ci = 0; ci < cres.size(); ++ci) {
                // A residual Select(c1, Select(c2, e, 0), 0) has partials Select(c1, Select(c2,
                // de, 0), 0): its mask is evaluated once (m<ci>) and applied to Jp alone — each
                // partial's contribution d * Jp is then 0 with it — instead of a select per
                // partial; only when every partial is free of operations that can be non-finite
                // where the mask is off (division, sqrt, log, pow, exp), where 0 * d could be NaN.
                std::vector<int> conds;
                std::vector<int> de(ents.size(), -1);
                bool factor = !jtf && g_factor;
                if (factor) {
                    int core = m.residuals[cres[ci]].expr;
                    double z;
                    while (P.at(core).op == Op::Select && P.is_const(P.at(core).d, &z) && z == 0.0) {
                        conds.push_back(P.at(core).a);
                        core = P.at(core).b;
                    }
                    factor = !conds.empty();
                    for (size_t ei = 0; ei < ents.size() && factor; ++ei) {
                        if (ents[ei].r != (int)ci || ents[ei].slot < 0) continue;
                        int x = ents[ei].dnode;
                        for (int c : conds) {
                            const Node& n = P.at(x);
                            if (n.op == Op::Select && n.a == c && P.is_const(n.d, &z) && z == 0.0) x = n.b;
                            else { factor = false; break; }
                        }
                        P.visit(x, [&](int, const Node& n) {
                            factor = factor && n.op != Op::Div && n.op != Op::Sqrt && n.op != Op::Log &&
                                     n.op != Op::Pow && n.op != Op::Exp && n.op != Op::Sample;
                        });
                        de[ei] = x;
                    }
                }
                if (factor) {
                    std::string mc = "qin";
                    for (int c : conds) mc += " && " + b.cond(c);
                    b.line("const bool m" + std::to_string(ci) + " = " + mc + ";");
                    std::string fsum = "(T)0";
                    for (size_t ei = 0; ei < ents.size(); ++ei) {
                        if (ents[ei].r != (int)ci) continue;
                        if (ents[ei].slot >= 0) {
                            dname[ei] = "d" + std::to_string(ei);
                            b.line("const T " + dname[ei] + " = " + b.v(de[ei]) + ";");
                        } else {
                            double cv;
                            P.is_const(ents[ei].dnode, &cv);
                            dname[ei] = lit(cv);
                        }
                        fsum += " + " + dname[ei] + " * " + b.vec(ents[ei].u, "p");
                    }
                    b.line("const T jp" + std::to_string(ci) + " = m" + std::to_string(ci) + " ? " + fsum + " : (T)0;");
                    // A partial that reads a known array (or a ComputedArray) may be non-finite
                    // where the mask is off — NaN / Inf is a common "no data" value there — and
                    // d * jp would then be NaN * 0. The reference's Select discards that branch,
                    // so those partials keep the mask on their transpose contribution;
                    // partials over unknowns, parameters and constants alone need none.
                    for (size_t ei = 0; ei < ents.size(); ++ei) {
                        if (ents[ei].r != (int)ci || ents[ei].slot < 0) continue;
                        bool data = false;
                        P.visit(de[ei], [&](int, const Node& n) {
                            data = data || (n.op == Op::Read && !(n.i >= 0 && n.i < (int)m.images.size() &&
                                                                   m.images[n.i].unknown));
                        });
                        if (!data) continue;
                        const std::string dm = "dm" + std::to_string(ei);
                        b.line("const T " + dm + " = m" + std::to_string(ci) + " ? " + dname[ei] + " : (T)0;");
                        dname[ei] = dm;
                    }
                    continue;
                }
                std::string sum = "(T)0";
                for (size_t ei = 0; ei < ents.size(); ++ei) {
                    if (ents[ei].r != (int)ci) continue;
                    const std::string dn = b.v(ents[ei].dnode);
                    if (ents[ei].slot >= 0) {
                        dname[ei] = "d" + std::to_string(ei);
                        b.line("const T " + dname[ei] + " = qin ? " + dn + " : (T)0;");
                    } else {
                        double cv;
                        P.is_const(ents[ei].dnode, &cv);
                        dname[ei] = lit(cv);
                    }
                    if (!jtf) sum += " + " + dn + " * " + b.vec(ents[ei].u, "p");
                }
                if (jtf) b.line("const T jp" + std::to_string(ci) + " = qin ? " + b.v(m.residuals[cres[ci]].expr) + " : (T)0;");
                else b.line("const T jp" + std::to_string(ci) + " = qin ? " + sum + " : (T)0;");
            }
            // contributions per output (image, channel, offset): one lane shift each
            // (jtf: jp holds the residual value; dg the squared partials)
            std::map<std::tuple<int, int, int, int>, std::pair<std::string, std::string>> grp;
            for (size_t ei = 0; ei < ents.size(); ++ei) {
                const Node n = P.at(ents[ei].u);
                auto& s = grp[std::make_tuple(n.i, n.ch, ents[ei].oy, ents[ei].ox)];
                s.first += (s.first.empty() ? "" : " + ") + dname[ei] + " * jp" + std::to_string(ents[ei].r);
                if (jtf) {
                    // a constant partial still only counts where its centre is inside
                    const std::string d = ents[ei].slot >= 0 ? dname[ei] : "(qin ? " + dname[ei] + " : (T)0)";
                    s.second += (s.second.empty() ? "" : " + ") + d + " * " + d;
                }
            }
            for (auto& g : grp) {
                const int k = std::get<0>(g.first), c = std::get<1>(g.first), oy = std::get<2>(g.first),
                          ox = std::get<3>(g.first);
                const std::string sfx = std::to_string(uslot[k]) + "_" + std::to_string(c) + "_" + std::to_string(oy - miny);
                auto add = [&](const std::string& acc, const std::string& e) {
                    b.line(acc + " += " + (ox == 0 ? "(" + e + ")" : "opt_sh(" + e + ", " + std::to_string(-ox) + ")") + ";");
                };
                add("ac" + sfx, g.second.first);
                if (jtf) add("dq" + sfx, g.second.second);
            }
            if (jtf) {
                // the output row's Exclude, read from the same windows
                Body bf(m, fin, nd, uslot);
                bf.use_pred(true);
                bf.centred_reads([&](const Node& n, const char* vname) {
                    const auto key = std::make_tuple(vname ? 1 : 0, n.i, n.ch);
                    auto it = win.find(key);
                    if (it == win.end()) win[key] = {n.off[1], n.off[1]};
                    else it->second = {std::min(it->second.first, n.off[1]), std::max(it->second.second, n.off[1])};
                    rxlo = std::min(rxlo, n.off[0]);
                    rxhi = std::max(rxhi, n.off[0]);
                    const std::string w = wname(key, n.off[1]);
                    return n.off[0] == 0 ? w : "opt_sh(" + w + ", " + std::to_string(n.off[0]) + ")";
                });
                const int sh[3] = {0, miny, 0};
                const std::string act = m.exclude >= 0 ? "(" + bf.v(shifted(m.exclude, sh)) + " == (T)0)" : "true";
                bf.line("const bool act = " + act + ";");
            }
        }
        g_cache = saved;
        int regs = 0;
        for (auto& w : win) regs += w.second.second - w.second.first + 2;   // + the prefetched row
        int nacc = 0;
        for (int k : unk) nacc += m.images[k].channels;
        regs += nacc * (maxy - miny + 1) * (jtf ? 2 : 1);
        const int loff = -rxlo + maxx, nout = 64 + rxlo - rxhi - (maxx - minx);
        ok = ok && nout >= 16 && regs <= 96 * (dbl ? 1 : 2) / 2;
        if (!ok) return;
        if (jtf) {
            gs.has_jtf_strip = true;
            gs.jtf_strip_cols = nout;
            o << "extern \"C\" __global__ __launch_bounds__(256) void gen_jtf_strip(GenArgs a, T* __restrict__ r, T* __restrict__ diag) {\n"
                 "    OPT_COORDS\n";
        } else {
            gs.has_strip = true;
            gs.strip_cols = nout;
            o << "extern \"C\" __global__ __launch_bounds__(256) void gen_apply_strip(GenArgs a, const T* __restrict__ p, T* __restrict__ Ap,\n"
                 "        const T* __restrict__ dadd, const int* stop, ReduceSlot rs, int finish) {\n"
                 "    if (stop && *stop) return;\n"
                 "    OPT_COORDS\n"
                 "    T dot = 0;\n";
        }
        o << "    const int lane = threadIdx.x & 63, z = 0; (void)z;\n"
             "    const int nsx = (W + " << nout - 1 << ") / " << nout << ", G = gridDim.x * 4;\n"
             "    const int RB = max(8, (int)(((long long)H * nsx + G - 1) / G)), nby = (H + RB - 1) / RB;\n";
        auto base_of = [&](const std::tuple<int, int, int>& k) {
            const int i = std::get<1>(k);
            return std::get<0>(k) ? "(p + a.uoff[" + std::to_string(uslot[i]) + "])"
                                  : "((const " + std::string(elem_type(m.images[i].elem, m.images[i].tvalued)) +
                                        "*)a.img[" + std::to_string(i) + "])";
        };
        // the two channels of a 2-channel array whose windows span the same rows are
        // read as one 8 / 16-byte access (opt_ldm2)
        auto partner = [&](const std::tuple<int, int, int>& k) -> const std::pair<int, int>* {
            const int i = std::get<1>(k);
            if (m.images[i].channels != 2) return nullptr;
            auto a0 = win.find(std::make_tuple(std::get<0>(k), i, 0));
            auto a1 = win.find(std::make_tuple(std::get<0>(k), i, 1));
            if (a0 == win.end() || a1 == win.end() || a0->second != a1->second) return nullptr;
            return &a1->second;
        };
        bool pairs = false;
        for (auto& w : win) pairs = pairs || (std::get<2>(w.first) == 0 && partner(w.first));
        const bool opq = g_strip32 == 2 || (g_strip32 == 4 && !pairs);   // opt_at32<O>
        // the wave loop (emitted once pairs is known): the wave index through readfirstlane
        // in the kernels without pair windows (OPT_AMD_GEN_WIDU=2, the default; 1 always, 0 never)
        o << "    for (int wid = " << (g_widu == 1 || (g_widu == 2 && !pairs)
                                          ? "__builtin_amdgcn_readfirstlane((int)opt_xcd_block() * 4 + (threadIdx.x >> 6))"
                                          : "(int)opt_xcd_block() * 4 + (threadIdx.x >> 6)") << "; wid < nsx * nby; wid += G) {\n"
             "        const int x = (wid % nsx) * " << nout << " + lane - " << loff << ";\n"
             "        const int y0 = (wid / nsx) * RB, y1 = min(H, y0 + RB);\n"
             "        const bool xin = x >= 0 && x < W, xout = xin && lane >= " << loff << " && lane < " << loff + nout << ";\n";
        // statement loading row yy of window k into `dst` (and of its partner channel)
        auto load = [&](const std::tuple<int, int, int>& k, const std::string& yy, int dy, const char* sfx) {
            const int i = std::get<1>(k), c = std::get<2>(k), ch = m.images[i].channels;
            const std::string cond = "xin && " + yy + " >= 0 && " + yy + " < H";
            const std::string pix = s32 ? "(unsigned)(" + yy + " * W + x) * " + std::to_string(ch) + "u"
                                            : "(long long)(" + yy + " * W + x) * " + std::to_string(ch);
            const std::string sf = s32 ? (opq ? "_32<true>(" : "_32<false>(") : "(";
            if (partner(k)) {
                if (c == 1) return std::string();
                const auto k1 = std::make_tuple(std::get<0>(k), i, 1);
                return "opt_ldm2" + sf + base_of(k) + ", " + pix + ", " + cond + ", " + wname(k, dy) + sfx + ", " +
                       wname(k1, dy) + sfx + ");";
            }
            return wname(k, dy) + sfx + " = opt_ldm" + (s32 ? std::string(opq ? "32<true>(" : "32<false>(") : std::string("(")) + base_of(k) +
                   ", " + pix + " + " + std::to_string(c) + ", " + cond + ");";
        };
        const std::string qy0 = "(y0 - " + std::to_string(maxy) + ")";
        // each window's next top row is loaded one row ahead (<window>_n): its loads are
        // in flight during a whole row of residual arithmetic before they are consumed
        for (auto& w : win) {
            o << "        T " << wname(w.first, w.second.second) << "_n = 0";
            for (int dy = w.second.first; dy <= w.second.second; ++dy) o << ", " << wname(w.first, dy) << " = 0";
            o << ";\n";
        }
        for (auto& w : win) {
            for (int dy = w.second.first + 1; dy <= w.second.second; ++dy) {
                const std::string st = load(w.first, "(" + qy0 + " - 1 + " + std::to_string(dy) + ")", dy, "");
                if (!st.empty()) o << "        " << st << "\n";
            }
            const std::string st = load(w.first, "(" + qy0 + " + " + std::to_string(w.second.second) + ")",
                                        w.second.second, "_n");
            if (!st.empty()) o << "        " << st << "\n";
        }
        for (int k : unk)
            for (int c = 0; c < m.images[k].channels; ++c)
                for (int j = 0; j <= maxy - miny; ++j) {
                    o << "        T ac" << uslot[k] << "_" << c << "_" << j << " = 0;\n";
                    if (jtf) o << "        T dq" << uslot[k] << "_" << c << "_" << j << " = 0;\n";
                }
        o << "        for (int y = " << qy0 << "; y < y1 - " << miny << "; ++y) {\n";
        for (auto& w : win) {
            for (int dy = w.second.first; dy < w.second.second; ++dy)
                o << "        " << wname(w.first, dy) << " = " << wname(w.first, dy + 1) << ";\n";
            o << "        " << wname(w.first, w.second.second) << " = " << wname(w.first, w.second.second) << "_n;\n";
        }
        for (auto& w : win) {
            const std::string st = load(w.first, "(y + " + std::to_string(w.second.second + 1) + ")", w.second.second, "_n");
            if (!st.empty()) o << "        " << st << "\n";
        }
        o << "        const bool qin = xin && y >= 0 && y < H;\n" << body.str();
        // output row y + miny has all its centres
        // (off32: the element index as a 32-bit byte offset from the array's base, opt_at32)
        const std::string ity = s32 ? "unsigned" : "long long";
        auto at = [&](const std::string& arr, const std::string& e) {
            return s32 ? std::string(opq ? "opt_at32<true>(" : "opt_at32<false>(") + arr + ", " + e + ")" : arr + "[" + e + "]";
        };
        o << "        const int yo = y + " << miny << ";\n"
             "        if (xout && yo >= y0 && yo < y1) {\n"
             "        const " << ity << " lin = (" << ity << ")yo * W + x;\n";
        if (jtf) o << fin.str() << "        " << at("a.flags", "lin") << " = act ? 1 : 0;\n";
        else o << "        const bool act = (" << at("a.flags", "lin") << " & 1) != 0;\n";
        for (int k : unk)
            for (int c = 0; c < m.images[k].channels; ++c) {
                const std::string el = "(" + ity + ")a.uoff[" + std::to_string(uslot[k]) + "] + lin * " +
                                       std::to_string(m.images[k].channels) + " + " + std::to_string(c);
                const std::string sfx = std::to_string(uslot[k]) + "_" + std::to_string(c) + "_0";
                if (jtf) {
                    o << "        { const " << ity << " e = " << el << "; " << at("r", "e") << " = act ? -ac" << sfx
                      << " : (T)0; " << at("diag", "e") << " = dq" << sfx << "; }\n";
                    continue;
                }
                // p at the output pixel: its row window when one holds row yo (same load)
                std::string pe = at("p", "e");
                auto wi = win.find(std::make_tuple(1, k, c));
                if (wi != win.end() && wi->second.first <= miny && miny <= wi->second.second)
                    pe = wname(wi->first, miny);
                o << "        { const " << ity << " e = " << el << "; const T acc = ac" << sfx << ";\n"
                     "          if (finish) { const T pe = " << pe << "; const T o = act ? acc + (dadd ? " << at("dadd", "e")
                  << " * pe : (T)0) : (T)0; " << at("Ap", "e") << " = o; dot += pe * o; }\n"
                     "          else " << at("Ap", "e") << " = acc; }\n";
            }
        o << "        }\n";
        for (int k : unk)
            for (int c = 0; c < m.images[k].channels; ++c)
                for (const char* an : {"ac", "dq"}) {
                    if (!jtf && an[0] == 'd') continue;
                    const std::string a0 = an + std::to_string(uslot[k]) + "_" + std::to_string(c) + "_";
                    for (int j = 0; j < maxy - miny; ++j) o << "        " << a0 << j << " = " << a0 << j + 1 << ";\n";
                    o << "        " << a0 << maxy - miny << " = 0;\n";
                }
        o << "        }\n"
             "    }\n";
        if (jtf) o << "}\n";
        else o << "    if (finish) { double v[1] = {(double)dot}; block_reduce_publish<1>(v, rs, blockIdx.x); }\n}\n";
    };
    // gen_cost_strip: cost / model cost (gen_cost's per-centre expression: excluded centres
    // skipped, 1/2 sum r^2, or with delta the linearised residuals r + sum_u dr/du delta_u)
    // with every read served from row windows (unknowns, knowns, delta) walked down a
    // column strip, one pixel per lane and centre; no scatter, so no row lag.
    auto cost_strip = [&]() {
        bool ok = !cres.empty();
        for (int ci : cres)
            P.visit(m.residuals[ci].expr, [&](int, const Node& n) { ok &= n.op != Op::Sample; });
        if (m.exclude >= 0)
            P.visit(m.exclude, [&](int, const Node& n) { ok &= n.op != Op::Sample && !(n.op == Op::Read && n.slot >= 0); });
        for (auto& r : m.residuals) ok &= r.graph < 0;   // graph terms: gen_cost
        if (!ok) return;
        // window key: (0 known / unknown image, 2 delta; image; channel)
        std::map<std::tuple<int, int, int>, std::pair<int, int>> win;
        int rxlo = 0, rxhi = 0;
        auto wname = [](const std::tuple<int, int, int>& k, int dy) {
            return std::string(std::get<0>(k) ? "wd" : "wi") + std::to_string(std::get<1>(k)) + "c" +
                   std::to_string(std::get<2>(k)) + (dy < 0 ? "m" : "p") + std::to_string(std::abs(dy));
        };
        std::ostringstream body;
        const CacheMap* saved = g_cache;
        g_cache = nullptr;
        {
            Body b(m, body, nd, uslot);
            b.use_pred(true);
            b.centred_reads([&](const Node& n, const char* vname) {
                const auto key = std::make_tuple(vname ? 2 : 0, n.i, n.ch);
                auto it = win.find(key);
                if (it == win.end()) win[key] = {n.off[1], n.off[1]};
                else it->second = {std::min(it->second.first, n.off[1]), std::max(it->second.second, n.off[1])};
                rxlo = std::min(rxlo, n.off[0]);
                rxhi = std::max(rxhi, n.off[0]);
                const std::string w = wname(key, n.off[1]);
                return n.off[0] == 0 ? w : "opt_sh(" + w + ", " + std::to_string(n.off[0]) + ")";
            });
            b.line("bool on = xout && y >= y0 && y < y1;");
            if (m.exclude >= 0) b.line("on = on && " + b.v(m.exclude) + " == (T)0;");
            std::string sum = "(T)0";
            for (int ci : cres) {
                const std::string R = b.v(m.residuals[ci].expr);
                sum += " + " + R + " * " + R;
            }
            b.line("T s = " + sum + ";");
            b.line("if (delta) {");
            std::string ms = "(T)0";
            int idx = 0;
            for (int ci : cres) {
                const GResidual& r = m.residuals[ci];
                std::string e = b.v(r.expr);
                for (int u : r.unknowns) {
                    const int gu = P.diff(r.expr, u);
                    double gv;
                    if (P.is_const(gu, &gv) && gv == 0.0) continue;
                    e += " + " + b.v(gu) + " * " + b.vec(u, "delta");
                }
                b.line("  const T m" + std::to_string(idx) + " = " + e + ";");
                ms += " + m" + std::to_string(idx) + " * m" + std::to_string(idx);
                ++idx;
            }
            b.line("  s = " + ms + ";");
            b.line("}");
            b.line("if (on) acc += (T)0.5 * s;");
        }
        g_cache = saved;
        int regs = 0;
        for (auto& w : win) regs += w.second.second - w.second.first + 2;
        const int loff = -rxlo, nout = 64 + rxlo - rxhi;
        if (nout < 16 || regs > 96 * (dbl ? 1 : 2) / 2) return;
        gs.has_cost_strip = true;
        gs.cost_strip_cols = nout;
        o << "extern \"C\" __global__ __launch_bounds__(256) void gen_cost_strip(GenArgs a, const T* __restrict__ delta, ReduceSlot rs) {\n"
             "    OPT_COORDS\n"
             "    T acc = 0;\n"
             "    const int lane = threadIdx.x & 63, z = 0; (void)z;\n"
             "    const int nsx = (W + " << nout - 1 << ") / " << nout << ", G = gridDim.x * 4;\n"
             "    const int RB = max(8, (int)(((long long)H * nsx + G - 1) / G)), nby = (H + RB - 1) / RB;\n";
        auto base_of = [&](const std::tuple<int, int, int>& k) {
            const int i = std::get<1>(k);
            const std::string own = "((const " + std::string(elem_type(m.images[i].elem, m.images[i].tvalued)) +
                                    "*)a.img[" + std::to_string(i) + "])";
            // delta may be null (the cost): the image itself stands in as a valid address
            return std::get<0>(k) ? "(delta ? delta + a.uoff[" + std::to_string(uslot[i]) + "] : " + own + ")" : own;
        };
        auto partner = [&](const std::tuple<int, int, int>& k) {
            const int i = std::get<1>(k);
            if (m.images[i].channels != 2) return false;
            auto a0 = win.find(std::make_tuple(std::get<0>(k), i, 0));
            auto a1 = win.find(std::make_tuple(std::get<0>(k), i, 1));
            return a0 != win.end() && a1 != win.end() && a0->second == a1->second;
        };
        bool pairs = false;
        for (auto& w : win) pairs = pairs || (std::get<2>(w.first) == 0 && partner(w.first));
        const bool opq = g_strip32 == 2 || (g_strip32 == 4 && !pairs);   // opt_at32<O>
        // the wave loop (emitted once pairs is known): the wave index through readfirstlane
        // in the kernels without pair windows (OPT_AMD_GEN_WIDU=2, the default; 1 always, 0 never)
        o << "    for (int wid = " << (g_widu == 1 || (g_widu == 2 && !pairs)
                                          ? "__builtin_amdgcn_readfirstlane((int)opt_xcd_block() * 4 + (threadIdx.x >> 6))"
                                          : "(int)opt_xcd_block() * 4 + (threadIdx.x >> 6)") << "; wid < nsx * nby; wid += G) {\n"
             "        const int x = (wid % nsx) * " << nout << " + lane - " << loff << ";\n"
             "        const int y0 = (wid / nsx) * RB, y1 = min(H, y0 + RB);\n"
             "        const bool xin = x >= 0 && x < W, xout = xin && lane >= " << loff << " && lane < " << loff + nout << ";\n";
        auto load = [&](const std::tuple<int, int, int>& k, const std::string& yy, int dy, const char* sfx) {
            const int i = std::get<1>(k), c = std::get<2>(k), ch = m.images[i].channels;
            const std::string cond = "xin && " + yy + " >= 0 && " + yy + " < H" + (std::get<0>(k) ? " && delta" : "");
            const std::string pix = s32 ? "(unsigned)(" + yy + " * W + x) * " + std::to_string(ch) + "u"
                                            : "(long long)(" + yy + " * W + x) * " + std::to_string(ch);
            const std::string sf = s32 ? (opq ? "_32<true>(" : "_32<false>(") : "(";
            if (partner(k)) {
                if (c == 1) return std::string();
                const auto k1 = std::make_tuple(std::get<0>(k), i, 1);
                return "opt_ldm2" + sf + base_of(k) + ", " + pix + ", " + cond + ", " + wname(k, dy) + sfx + ", " +
                       wname(k1, dy) + sfx + ");";
            }
            return wname(k, dy) + sfx + " = opt_ldm" + (s32 ? std::string(opq ? "32<true>(" : "32<false>(") : std::string("(")) + base_of(k) +
                   ", " + pix + " + " + std::to_string(c) + ", " + cond + ");";
        };
        for (auto& w : win) {
            o << "        T " << wname(w.first, w.second.second) << "_n = 0";
            for (int dy = w.second.first; dy <= w.second.second; ++dy) o << ", " << wname(w.first, dy) << " = 0";
            o << ";\n";
        }
        for (auto& w : win) {
            for (int dy = w.second.first + 1; dy <= w.second.second; ++dy) {
                const std::string st = load(w.first, "(y0 - 1 + " + std::to_string(dy) + ")", dy, "");
                if (!st.empty()) o << "        " << st << "\n";
            }
            const std::string st = load(w.first, "(y0 + " + std::to_string(w.second.second) + ")", w.second.second, "_n");
            if (!st.empty()) o << "        " << st << "\n";
        }
        o << "        for (int y = y0; y < y1; ++y) {\n";
        for (auto& w : win) {
            for (int dy = w.second.first; dy < w.second.second; ++dy)
                o << "        " << wname(w.first, dy) << " = " << wname(w.first, dy + 1) << ";\n";
            o << "        " << wname(w.first, w.second.second) << " = " << wname(w.first, w.second.second) << "_n;\n";
        }
        for (auto& w : win) {
            const std::string st = load(w.first, "(y + " + std::to_string(w.second.second + 1) + ")", w.second.second, "_n");
            if (!st.empty()) o << "        " << st << "\n";
        }
        o << "        const bool qin = xin; (void)qin;\n" << body.str() << "        }\n    }\n"
             "    double v[1] = {(double)acc}; block_reduce_publish<1>(v, rs, blockIdx.x);\n}\n";
    };
    if (tiled) {
        strip_kernel(false);
        strip_kernel(true);
        cost_strip();
    }

    // ------------------------------------------------------------ gen_dump_j_<i>
    // saveJToCRS / saveJToCRS_Graph (solverGPUGaussNewton.t:1004-1022, 1287-1305) with
    // generateDumpJ (:385-442): the residuals grouped into energy specs by domain in order
    // of first appearance (toenergyspecs); element e of spec i owns rows row_base + e R_i +
    // r and nonzeros nnz_base + e NNZ_i + ...; each row lists every unknown access of its
    // template (zero partials included), column = image offset + channels * tooffset +
    // channel wrapped into [0, nUnknowns) (wrap, :365-381), sorted by column (sortCol).
    // Every element is written, excluded ones included, as the reference does.
    {
        std::vector<int> order;   // spec domains in order of first appearance
        for (auto& r : m.residuals)
            if (std::find(order.begin(), order.end(), r.graph) == order.end()) order.push_back(r.graph);
        for (size_t si = 0; si < order.size(); ++si) {
            const int g = order[si];
            std::vector<const GResidual*> rs;
            int npe = 0;
            for (auto& r : m.residuals)
                if (r.graph == g) { rs.push_back(&r); npe += (int)r.unknowns.size(); }
            gs.dump.push_back({g, (int)rs.size(), npe});
            o << "extern \"C\" __global__ __launch_bounds__(256) void gen_dump_j_" << si
              << "(GenArgs a, int* __restrict__ rowPtr, int* __restrict__ colInd, T* __restrict__ val,\n"
                 "        long long row_base, long long nnz_base, long long nunk) {\n"
                 "    OPT_COORDS\n";
            if (g < 0) {
                o << "    for (long long lin = a.own_lo + (long long)blockIdx.x * 256 + threadIdx.x; lin < a.own_hi; lin += (long long)gridDim.x * 256) {\n"
                  << coords << "        const long long el = lin;\n";
            } else {
                o << "    for (long long el = (long long)blockIdx.x * 256 + threadIdx.x; el < a.nedge[" << g
                  << "]; el += (long long)gridDim.x * 256) {\n";
                for (size_t sl = 0; sl < m.graphs[g].slot_names.size(); ++sl)
                    o << "        const int v" << sl << " = a.slot[" << gs.slot_base[g] + sl << "][el];\n";
            }
            Body b(m, o, nd, uslot);
            int nz = 0;
            for (size_t ri = 0; ri < rs.size(); ++ri) {
                const GResidual& r = *rs[ri];
                const int K = (int)r.unknowns.size();
                b.line("rowPtr[row_base + el * " + std::to_string(rs.size()) + " + " + std::to_string(ri) +
                       "] = (int)(nnz_base + el * " + std::to_string(npe) + " + " + std::to_string(nz) + ");");
                if (K == 0) continue;
                const std::string cc = "cc" + std::to_string(ri), vv = "vv" + std::to_string(ri);
                b.line("long long " + cc + "[" + std::to_string(K) + "]; T " + vv + "[" + std::to_string(K) + "];");
                int q = 0;
                for (int u : r.unknowns) {
                    const Node n = P.at(u);
                    const int ch = m.images[n.i].channels;
                    std::string idx;
                    if (n.slot >= 0) {
                        idx = "(long long)v" + std::to_string(n.slot);
                    } else {   // tooffset of the (possibly outside) access
                        idx = "(el + " + std::to_string(n.off[0]) + "LL";
                        if (nd > 1) idx += " + " + std::to_string(n.off[1]) + "LL * W";
                        if (nd > 2) idx += " + " + std::to_string(n.off[2]) + "LL * W * H";
                        idx += ")";
                    }
                    const int d = P.diff(r.expr, u);
                    const std::string dv = b.v(d);
                    b.line(cc + "[" + std::to_string(q) + "] = a.uoff[" + std::to_string(uslot[n.i]) + "] + " +
                           std::to_string(ch) + " * " + idx + " + " + std::to_string(n.ch) + "; " + vv + "[" +
                           std::to_string(q) + "] = " + dv + ";");
                    ++q;
                }
                const std::string Ks = std::to_string(K);
                b.line("for (int i = 0; i < " + Ks + "; ++i) { const long long c = " + cc + "[i]; " + cc +
                       "[i] = c < 0 ? c + nunk : (c >= nunk ? c - nunk : c); }");
                b.line("for (int i = 1; i < " + Ks + "; ++i) for (int j = i; j > 0 && " + cc + "[j] < " + cc +
                       "[j - 1]; --j) { const long long tc = " + cc + "[j]; " + cc + "[j] = " + cc + "[j - 1]; " + cc +
                       "[j - 1] = tc; const T tv = " + vv + "[j]; " + vv + "[j] = " + vv + "[j - 1]; " + vv + "[j - 1] = tv; }");
                b.line("for (int i = 0; i < " + Ks + "; ++i) { colInd[nnz_base + el * " + std::to_string(npe) + " + " +
                       std::to_string(nz) + " + i] = (int)" + cc + "[i]; val[nnz_base + el * " + std::to_string(npe) +
                       " + " + std::to_string(nz) + " + i] = " + vv + "[i]; }");
                nz += K;
            }
            o << "    }\n}\n";
        }
    }

    // ------------------------------------------------------- cost (centres + edges)
    {
        o << "extern \"C\" __global__ __launch_bounds__(256) void gen_cost(GenArgs a, const T* __restrict__ delta, ReduceSlot rs) {\n"
             "    OPT_COORDS\n"
             "    T acc = 0;\n";
        if (gs.has_centered) {
            o << "    for (long long lin = a.own_lo + (long long)blockIdx.x * 256 + threadIdx.x; lin < a.own_hi; lin += (long long)gridDim.x * 256) {\n"
              << coords;
            Body b(m, o, nd, uslot);
            if (m.exclude >= 0) b.line("if (" + b.v(m.exclude) + " != (T)0) continue;");
            std::string sum = "(T)0", msum = "(T)0";
            for (auto& r : m.residuals) {
                if (r.graph >= 0) continue;
                const std::string R = b.v(r.expr);
                sum += " + " + R + " * " + R;
            }
            b.line("T s = " + sum + ";");
            b.line("if (delta) {");
            {
                int idx = 0;
                std::string ms = "(T)0";
                for (auto& r : m.residuals) {
                    if (r.graph >= 0) continue;
                    std::string e = b.v(r.expr);
                    for (int u : r.unknowns) {
                        const int gu = P.diff(r.expr, u);
                        double gv;
                        if (P.is_const(gu, &gv) && gv == 0.0) continue;
                        e += " + " + b.v(gu) + " * " + b.vec(u, "delta");
                    }
                    b.line("  const T m" + std::to_string(idx) + " = " + e + ";");
                    ms += " + m" + std::to_string(idx) + " * m" + std::to_string(idx);
                    ++idx;
                }
                b.line("  s = " + ms + ";");
            }
            b.line("}");
            b.line("acc += (T)0.5 * s;");
            o << "    }\n";
        }
        for (size_t g = 0; g < m.graphs.size(); ++g) {
            bool any = false;
            for (auto& r : m.residuals) any |= r.graph == (int)g;
            if (!any) continue;
            // the next edge's vertex ids are loaded one edge ahead (as the gathers' edge loops)
            const size_t ns = m.graphs[g].slot_names.size();
            auto sl = [&](size_t s) { return "a.slot[" + std::to_string(gs.slot_base[g] + s) + "]"; };
            o << "    {\n    const long long es = (long long)gridDim.x * 256, ne = a.nedge[" << g << "];\n"
              << "    long long e = opt_xcd_block() * 256 + threadIdx.x;\n";
            if (prefetch_nb)
                for (size_t s = 0; s < ns; ++s) o << "    int n" << s << " = e < ne ? " << sl(s) << "[e] : 0;\n";
            o << "    for (; e < ne; e += es) {\n";
            for (size_t s = 0; s < ns; ++s)
                o << "        const int v" << s << " = " << (prefetch_nb ? "n" + std::to_string(s) : sl(s) + "[e]") << ";\n";
            if (prefetch_nb) {
                o << "        if (e + es < ne) {";
                for (size_t s = 0; s < ns; ++s) o << " n" << s << " = " << sl(s) << "[e + es];";
                o << " }\n";
            }
            Body b(m, o, nd, uslot);
            std::string sum = "(T)0";
            int idx = 0;
            for (auto& r : m.residuals) {
                if (r.graph != (int)g) continue;
                std::string e = b.v(r.expr);
                b.line("T q" + std::to_string(idx) + " = " + e + ";");
                sum += " + q" + std::to_string(idx) + " * q" + std::to_string(idx);
                ++idx;
            }
            b.line("if (delta) {");
            idx = 0;
            for (auto& r : m.residuals) {
                if (r.graph != (int)g) continue;
                std::string e;
                for (int u : r.unknowns) {
                    const int gu = P.diff(r.expr, u);
                    double gv;
                    if (P.is_const(gu, &gv) && gv == 0.0) continue;
                    e += " + " + b.v(gu) + " * " + b.vec(u, "delta");
                }
                if (!e.empty()) b.line("  q" + std::to_string(idx) + " = q" + std::to_string(idx) + e + ";");
                ++idx;
            }
            b.line("}");
            b.line("acc += (T)0.5 * (" + sum + ");");
            o << "    }\n    }\n";
        }
        o << "    double v[1] = {(double)acc};\n    block_reduce_publish<1>(v, rs, blockIdx.x);\n}\n";
    }

    // ------------------------------------------------------------- graph gathers
    // The reference scatters every edge's J^T F / J^T J p contributions to the edge's
    // vertices with float atomics (createjtfgraph / createjtjgraph, o.t:2833-2867,
    // 2969-2994; Image:atomicAddChannel, backend_cuda.t:751-759). Here each vertex gathers
    // them instead, over per-slot incidence lists built once per bind (a.goff / a.geid:
    // the edges whose slot k is this vertex, ascending): no atomics, a fixed summation
    // order (bitwise reproducible), each edge evaluated once per incident slot. The same
    // kernel finishes the element (exclusion mask, LM diagonal, p.Ap).
    auto graph_gather = [&](bool apply) {
        // accumulators per output (unknown image, channel)
        for (int k : unk)
            for (int c = 0; c < m.images[k].channels; ++c)
                o << "        T acc" << uslot[k] << "_" << c << " = 0, dg" << uslot[k] << "_" << c << " = 0;\n";
        o << "        (void)0;\n";
        for (size_t g = 0; g < m.graphs.size(); ++g) {
            const size_t nslots = m.graphs[g].slot_names.size();
            for (size_t k = 0; k < nslots; ++k) {
                // residuals of graph g reading an unknown at slot k
                bool any = false;
                for (auto& r : m.residuals)
                    if (r.graph == (int)g)
                        for (int u : r.unknowns) any |= P.at(u).slot == (int)k;
                if (!any) continue;
                const int sbk = gs.slot_base[g] + (int)k;
                std::ostringstream pre, body;
                Body b(m, body, nd, uslot);
                b.hoist_to(&pre, (int)k, (int)g);
                int idx = 0;
                for (auto& r : m.residuals) {
                    if (r.graph != (int)g) continue;
                    std::vector<int> mine;
                    for (int u : r.unknowns)
                        if (P.at(u).slot == (int)k) mine.push_back(u);
                    if (mine.empty()) continue;
                    std::string R;
                    if (apply) {
                        std::string sum = "(T)0";
                        for (int u : r.unknowns) {
                            const int gu = P.diff(r.expr, u);
                            double gv;
                            if (P.is_const(gu, &gv) && gv == 0.0) continue;
                            sum += " + " + b.v(gu) + " * " + b.vec(u, "p");
                        }
                        R = "jp" + std::to_string(idx++);
                        b.line("const T " + R + " = " + sum + ";");
                    } else {
                        R = b.v(r.expr);
                    }
                    for (int u : mine) {
                        const int gu = P.diff(r.expr, u);
                        double gv;
                        if (P.is_const(gu, &gv) && gv == 0.0) continue;
                        const Node n = P.at(u);
                        const std::string gn = b.v(gu);
                        const std::string a_ = "acc" + std::to_string(uslot[n.i]) + "_" + std::to_string(n.ch);
                        const std::string d_ = "dg" + std::to_string(uslot[n.i]) + "_" + std::to_string(n.ch);
                        b.line(a_ + " += " + gn + " * " + R + ";" + (apply ? "" : " " + d_ + " += " + gn + " * " + gn + ";"));
                    }
                }
                // { own-vertex values; for each incident edge { the other slots; the rest } }
                // the other slots' vertices come from per-incidence-order copies (one load
                // each instead of the edge id, then the slot array)
                // the next edge's other-slot vertex ids are loaded one edge ahead (prefetch_nb),
                // so an edge's gathers do not wait behind its id load
                std::ostringstream head, loop;
                for (size_t s2 = 0; s2 < nslots; ++s2)
                    if (s2 != k) {
                        const std::pair<int, int> key(sbk, gs.slot_base[g] + (int)s2);
                        auto it = std::find(gs.nb_pairs.begin(), gs.nb_pairs.end(), key);
                        int idx = (int)(it - gs.nb_pairs.begin());
                        if (it == gs.nb_pairs.end()) gs.nb_pairs.push_back(key);
                        const std::string vs = "v" + std::to_string(s2), ns = "n" + std::to_string(s2);
                        const std::string gnb = "a.gnb[" + std::to_string(idx) + "]";
                        auto at = [&](const std::string& q) {
                            return off32 ? "opt_g32(" + gnb + ", " + q + ", 1, 0)" : gnb + "[" + q + "]";
                        };
                        if (idx < 32 && prefetch_nb) {
                            head << "        int " << ns << " = q0 < q1 ? " << at("q0") << " : 0;\n";
                            loop << "        const int " << vs << " = " << ns << ";\n"
                                 << "        if (q + 1 < q1) " << ns << " = " << at("q + 1") << ";\n";
                        } else if (idx < 32) {   // GenArgs::gnb capacity; past it, through the edge id
                            loop << "        const int " << vs << " = " << at("q") << ";\n";
                        } else {
                            loop << "        const int " << vs << " = a.slot[" << key.second << "][a.geid[" << sbk
                                 << "][q]];\n";
                        }
                    }
                o << "        {\n        const int v" << k << " = (int)vtx;\n" << pre.str()
                  << "        const int q0 = a.goff[" << sbk << "][vtx], q1 = a.goff[" << sbk << "][vtx + 1];\n"
                  << head.str() << unroll << "        for (int q = q0; q < q1; ++q) {\n" << loop.str();
                o << body.str() << "        }\n        }\n";
            }
        }
    };
    {
        o << "extern \"C\" __global__ __launch_bounds__(256) void gen_jtf_graph(GenArgs a, T* __restrict__ r, T* __restrict__ diag) {\n"
             "    OPT_COORDS\n"
             "    for (long long vtx = opt_xcd_block() * 256 + threadIdx.x; vtx < a.npix; vtx += (long long)gridDim.x * 256) {\n";
        graph_gather(false);
        o << "        const bool act = (a.flags[vtx] & 1) != 0;\n";
        for (int k : unk)
            for (int c = 0; c < m.images[k].channels; ++c) {
                const std::string e = "a.uoff[" + std::to_string(uslot[k]) + "] + vtx * " +
                                      std::to_string(m.images[k].channels) + " + " + std::to_string(c);
                const std::string sfx = std::to_string(uslot[k]) + "_" + std::to_string(c);
                o << "        { const long long i = " << e << "; r[i] = act ? r[i] - acc" << sfx
                  << " : (T)0; diag[i] += dg" << sfx << "; }\n";
            }
        o << "    }\n}\n";
        o << "extern \"C\" __global__ __launch_bounds__(256) void gen_apply_graph(GenArgs a, const T* __restrict__ p, T* __restrict__ Ap,\n"
             "        const T* __restrict__ dadd, const int* stop, ReduceSlot rs, int has_centred) {\n"
             "    if (stop && *stop) return;\n"
             "    OPT_COORDS\n"
             "    T dot = 0;\n"
             "    for (long long vtx = opt_xcd_block() * 256 + threadIdx.x; vtx < a.npix; vtx += (long long)gridDim.x * 256) {\n";
        graph_gather(true);
        // 1-D vertex domains: the centred terms at this vertex too (after the edge loops,
        // whose registers are free by then), instead of a gen_apply pass that stores them
        // for this kernel to read back
        gs.graph_apply_centred = gs.has_centered && nd == 1;
        if (gs.graph_apply_centred) {
            std::string decl = "        T";
            for (int k : unk)
                for (int c = 0; c < m.images[k].channels; ++c)
                    decl += std::string(decl.size() > 9 ? "," : "") + " cacc" + std::to_string(uslot[k]) + "_" + std::to_string(c) + " = 0";
            o << decl << ";\n        {\n        const long long lin = vtx;\n" << coords;
            Body b(m, o, nd, uslot);
            centred_apply(b, true);
            o << "        }\n";
        }
        o << "        const bool act = (a.flags[vtx] & 1) != 0;\n";
        for (int k : unk)
            for (int c = 0; c < m.images[k].channels; ++c) {
                const std::string e = "a.uoff[" + std::to_string(uslot[k]) + "] + vtx * " +
                                      std::to_string(m.images[k].channels) + " + " + std::to_string(c);
                const std::string sfx = std::to_string(uslot[k]) + "_" + std::to_string(c);
                const std::string cen = gs.graph_apply_centred ? "cacc" + sfx : "(has_centred ? Ap[i] : (T)0)";
                o << "        { const long long i = " << e << "; const T pe = p[i];\n"
                  << "          const T o = act ? " << cen << " + acc" << sfx
                  << " + (dadd ? dadd[i] * pe : (T)0) : (T)0;\n"
                  << "          Ap[i] = o; dot += pe * o; }\n";
            }
        o << "    }\n"
             "    double v[1] = {(double)dot};\n    block_reduce_publish<1>(v, rs, blockIdx.x);\n}\n";
    }
    (void)zero3;
    g_cache = nullptr;
    g_gcache = nullptr;
    g_pred = nullptr;
    char note[128];
    snprintf(note, sizeof(note), "// apply: %s (%.2f residual instances per centred residual)\n",
             gs.has_strip ? "gen_apply_strip" : gs.prefer_tiled ? "gen_apply_tiled" : "gen_apply",
             gs.instances_per_residual);
    gs.code = note + o.str();
    return gs;
}

}  // namespace gen
}  // namespace optamd
