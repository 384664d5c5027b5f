// problem.cpp — reads an Opt energy file (a Lua program in the reference,
// API/src/o.t:1295-1348 runs it with the lib.t environment) far enough to recover
// the declarations that define the problemparams binding (util.t:677-721) and the
// operators that identify the kernel family.
#include "problem.h"
#include <algorithm>
#include <cctype>
#include <map>
#include <set>
#include <sstream>

namespace optamd {
namespace {

enum class Tk { Name, Number, String, Op, End };
struct Token { Tk kind; std::string text; int line; };

// Lua lexer: names, numbers, short and long strings, operators; drops `--` line
// comments and `--[[ ... ]]` / `--[==[ ... ]==]` block comments.
bool lex(const std::string& s, std::vector<Token>* out, std::string* err) {
    size_t i = 0, n = s.size();
    int line = 1;
    auto long_bracket = [&](size_t at, int* level) -> bool {
        // at points to '['; matches [=*[
        size_t j = at + 1;
        int lv = 0;
        while (j < n && s[j] == '=') { ++lv; ++j; }
        if (j < n && s[j] == '[') { *level = lv; return true; }
        return false;
    };
    auto skip_long = [&](size_t at, int level) -> size_t {
        // returns index after the closing ]=*]
        std::string close = "]" + std::string(level, '=') + "]";
        size_t start = at + 2 + level;
        size_t e = s.find(close, start);
        if (e == std::string::npos) return std::string::npos;
        for (size_t k = at; k < e; ++k) if (s[k] == '\n') ++line;
        return e + close.size();
    };
    while (i < n) {
        char c = s[i];
        if (c == '\n') { ++line; ++i; continue; }
        if (isspace((unsigned char)c)) { ++i; continue; }
        if (c == '-' && i + 1 < n && s[i + 1] == '-') {
            int lv;
            if (i + 2 < n && s[i + 2] == '[' && long_bracket(i + 2, &lv)) {
                size_t e = skip_long(i + 2, lv);
                if (e == std::string::npos) { *err = "unterminated block comment"; return false; }
                i = e;
            } else {
                while (i < n && s[i] != '\n') ++i;
            }
            continue;
        }
        if (isalpha((unsigned char)c) || c == '_') {
            size_t j = i;
            while (j < n && (isalnum((unsigned char)s[j]) || s[j] == '_')) ++j;
            out->push_back({Tk::Name, s.substr(i, j - i), line});
            i = j;
            continue;
        }
        if (isdigit((unsigned char)c) || (c == '.' && i + 1 < n && isdigit((unsigned char)s[i + 1]))) {
            size_t j = i;
            while (j < n && (isalnum((unsigned char)s[j]) || s[j] == '.' ||
                             ((s[j] == '-' || s[j] == '+') && (s[j - 1] == 'e' || s[j - 1] == 'E'))))
                ++j;
            out->push_back({Tk::Number, s.substr(i, j - i), line});
            i = j;
            continue;
        }
        if (c == '"' || c == '\'') {
            size_t j = i + 1;
            std::string v;
            while (j < n && s[j] != c) {
                if (s[j] == '\\' && j + 1 < n) { v += s[j + 1]; j += 2; continue; }
                if (s[j] == '\n') { *err = "unterminated string"; return false; }
                v += s[j++];
            }
            if (j >= n) { *err = "unterminated string"; return false; }
            out->push_back({Tk::String, v, line});
            i = j + 1;
            continue;
        }
        int lv;
        if (c == '[' && long_bracket(i, &lv)) {
            size_t e = skip_long(i, lv);
            if (e == std::string::npos) { *err = "unterminated long string"; return false; }
            out->push_back({Tk::String, s.substr(i + 2 + lv, e - (i + 2 + lv) - 2 - lv), line});
            i = e;
            continue;
        }
        static const char* ops3[] = {"..."};
        static const char* ops2[] = {"==", "~=", "<=", ">=", "..", "::"};
        bool done = false;
        for (auto o : ops3) if (s.compare(i, 3, o) == 0) { out->push_back({Tk::Op, o, line}); i += 3; done = true; break; }
        if (done) continue;
        for (auto o : ops2) if (s.compare(i, 2, o) == 0) { out->push_back({Tk::Op, o, line}); i += 2; done = true; break; }
        if (done) continue;
        out->push_back({Tk::Op, std::string(1, c), line});
        ++i;
    }
    out->push_back({Tk::End, "", line});
    return true;
}

struct Parser {
    const std::vector<Token>& t;
    ProblemSpec* spec;
    std::string* err;
    std::map<std::string, std::string> dimvar;   // local variable -> Dim name

    // Split the argument list of a call whose '(' is at index `open`; returns index of
    // the matching ')' and fills args with [begin,end) token ranges at depth 0.
    size_t args(size_t open, std::vector<std::pair<size_t, size_t>>* a) {
        int depth = 0;
        size_t start = open + 1;
        for (size_t i = open; i < t.size(); ++i) {
            const std::string& x = t[i].text;
            if (t[i].kind == Tk::Op && (x == "(" || x == "{" || x == "[")) { ++depth; continue; }
            if (t[i].kind == Tk::Op && (x == ")" || x == "}" || x == "]")) {
                --depth;
                if (depth == 0) {
                    if (i > start) a->push_back({start, i});
                    return i;
                }
                continue;
            }
            if (depth == 1 && t[i].kind == Tk::Op && x == ",") {
                a->push_back({start, i});
                start = i + 1;
            }
        }
        return t.size() - 1;
    }
    bool is_single(std::pair<size_t, size_t> r, Tk k) const {
        return r.second == r.first + 1 && t[r.first].kind == k;
    }
    std::string str_arg(std::pair<size_t, size_t> r) const {
        return is_single(r, Tk::String) ? t[r.first].text : "";
    }
    int int_arg(std::pair<size_t, size_t> r) const {
        if (!is_single(r, Tk::Number)) return -1;
        return atoi(t[r.first].text.c_str());
    }
    std::vector<std::string> table_names(std::pair<size_t, size_t> r) const {
        std::vector<std::string> v;
        if (r.second <= r.first || t[r.first].text != "{") return v;
        for (size_t i = r.first + 1; i + 1 < r.second; ++i)
            if (t[i].kind == Tk::Name) v.push_back(t[i].text);
        return v;
    }
    static bool image_type(const std::string& ty, std::string* elem, int* ch) {
        static const std::map<std::string, std::pair<std::string, int>> m = {
            {"opt_float", {"float", 1}},  {"opt_float2", {"float", 2}},
            {"opt_float3", {"float", 3}}, {"opt_float4", {"float", 4}},
            {"float", {"float", 1}},      {"float2", {"float", 2}},
            {"float3", {"float", 3}},     {"float4", {"float", 4}},
            {"double", {"double", 1}},    {"uint8", {"uint8", 1}},
            {"int", {"int", 1}},          {"int32", {"int", 1}}};
        auto it = m.find(ty);
        if (it == m.end()) return false;
        *elem = it->second.first;
        *ch = it->second.second;
        return true;
    }

    bool run() {
        std::set<std::string> known_ops = {"Rotate2D", "Rotate3D", "Stencil", "InBounds",
                                           "InBoundsExpanded", "Select", "Index", "Energy",
                                           "All", "Sqrt", "sqrt", "abs", "Dot3", "Matrix3x3Mul",
                                           "normalize", "length", "Slice", "L_p", "greatereq",
                                           "greater", "less", "eq", "Not", "And", "Or"};
        for (size_t i = 0; i + 1 < t.size(); ++i) {
            // local a, b, c = e1, e2, e3   (bind Dim variables)
            if (t[i].kind == Tk::Name && t[i].text == "local") {
                std::vector<std::string> names;
                size_t j = i + 1;
                while (j < t.size() && t[j].kind == Tk::Name) {
                    names.push_back(t[j].text);
                    if (t[j + 1].text == ",") j += 2; else { ++j; break; }
                }
                if (j < t.size() && t[j].text == "=" && !names.empty()) {
                    // walk expressions: record Dim(...) calls in order
                    size_t k = j + 1;
                    for (size_t v = 0; v < names.size() && k < t.size(); ++v) {
                        size_t call = k;
                        if (t[call].text == "opt" && t[call + 1].text == ".") call += 2;
                        if (t[call].kind == Tk::Name && t[call].text == "Dim" && t[call + 1].text == "(") {
                            std::vector<std::pair<size_t, size_t>> a;
                            size_t close = args(call + 1, &a);
                            if (a.size() >= 1) dimvar[names[v]] = str_arg(a[0]);
                            k = close + 1;
                            if (t[k].text == ",") ++k; else break;
                        } else break;
                    }
                }
            }
            if (t[i].kind == Tk::Name && t[i + 1].text == "{" && known_ops.count(t[i].text) &&
                std::find(spec->ops.begin(), spec->ops.end(), t[i].text) == spec->ops.end())
                spec->ops.push_back(t[i].text);   // Stencil { ... } call form
            if (t[i].kind != Tk::Name || t[i + 1].text != "(") continue;
            const std::string& f = t[i].text;
            if (i > 0 && t[i - 1].text == "." && !(i > 1 && t[i - 2].text == "opt")) continue;
            if (i > 0 && t[i - 1].text == "function") continue;
            std::vector<std::pair<size_t, size_t>> a;
            if (known_ops.count(f)) {
                if (std::find(spec->ops.begin(), spec->ops.end(), f) == spec->ops.end())
                    spec->ops.push_back(f);
                continue;
            }
            if (f == "Dim") {
                args(i + 1, &a);
                if (a.size() != 2 || str_arg(a[0]).empty() || int_arg(a[1]) < 0)
                    return fail(i, "Dim(name, index) expected");
                spec->dims.push_back({str_arg(a[0]), int_arg(a[1])});
            } else if (f == "Unknown" || f == "Array") {
                args(i + 1, &a);
                if (a.size() != 4) return fail(i, f + "(name, type, {dims}, index) expected");
                DeclImage im;
                im.name = str_arg(a[0]);
                im.unknown = (f == "Unknown");
                if (!is_single(a[1], Tk::Name) || !image_type(t[a[1].first].text, &im.elem, &im.channels))
                    return fail(i, "unsupported element type for " + im.name);
                for (auto& d : table_names(a[2]))
                    im.dims.push_back(dimvar.count(d) ? dimvar[d] : d);
                im.index = int_arg(a[3]);
                if (im.name.empty() || im.index < 0) return fail(i, f + " needs a name and an index");
                spec->images.push_back(im);
            } else if (f == "Param") {
                args(i + 1, &a);
                if (a.size() != 3) return fail(i, "Param(name, type, index) expected");
                DeclParam p;
                p.name = str_arg(a[0]);
                p.type = is_single(a[1], Tk::Name) ? t[a[1].first].text : "";
                p.index = int_arg(a[2]);
                if (p.index < 0) {
                    // Param("L_" .. i .. "", float, 6+i) inside a numeric for: expand below
                    if (!expand_param_loop(i, a)) return false;
                } else {
                    spec->params.push_back(p);
                }
            } else if (f == "Graph") {
                args(i + 1, &a);
                if (a.size() < 2) return fail(i, "Graph(name, ...) expected");
                DeclGraph g;
                g.name = str_arg(a[0]);
                size_t k = 1;
                if (t[a[1].first].text == "{") {
                    for (auto& d : table_names(a[1])) g.dims.push_back(dimvar.count(d) ? dimvar[d] : d);
                    k = 2;
                } else {
                    k = 2;  // legacy form: edge-count param index
                }
                while (k + 2 < a.size()) {  // (slot name, {dims}, index) triples
                    g.vertices.push_back({str_arg(a[k]), int_arg(a[k + 2])});
                    k += 3;
                }
                spec->graphs.push_back(g);
            } else if (f == "UsePreconditioner") {
                args(i + 1, &a);
                if (a.size() == 1 && is_single(a[0], Tk::Name))
                    spec->use_preconditioner = (t[a[0].first].text == "true");
            } else if (f == "Exclude") {
                spec->n_exclude++;
            } else if (f == "ComputedArray") {
                args(i + 1, &a);
                if (!a.empty()) spec->computed_arrays.push_back(str_arg(a[0]));
            } else if (f == "SampledImage") {
                spec->uses_sampled_image = true;
            }
        }
        return true;
    }

    // `for i=A,B do L[i] = Param("L_" .. i .. "", float, C+i) end` (shape_from_shading.t)
    bool expand_param_loop(size_t at, const std::vector<std::pair<size_t, size_t>>& a) {
        // find the enclosing numeric for: scan back for `for NAME = A , B do`
        for (size_t j = at; j-- > 0;) {
            if (t[j].text == "for" && t[j + 1].kind == Tk::Name && t[j + 2].text == "=" &&
                t[j + 3].kind == Tk::Number && t[j + 4].text == "," && t[j + 5].kind == Tk::Number) {
                std::string var = t[j + 1].text;
                int lo = atoi(t[j + 3].text.c_str()), hi = atoi(t[j + 5].text.c_str());
                // index expression: NUMBER + var   or   var + NUMBER
                int base = 0;
                for (size_t k = a[2].first; k < a[2].second; ++k)
                    if (t[k].kind == Tk::Number) base = atoi(t[k].text.c_str());
                std::string prefix;
                for (size_t k = a[0].first; k < a[0].second; ++k)
                    if (t[k].kind == Tk::String) { prefix = t[k].text; break; }
                for (int v = lo; v <= hi; ++v) {
                    DeclParam p;
                    p.name = prefix + std::to_string(v);
                    p.type = is_single(a[1], Tk::Name) ? t[a[1].first].text : "";
                    p.index = base + v;
                    spec->params.push_back(p);
                }
                return true;
            }
        }
        return fail(at, "Param index must be a number or a loop expression");
    }

    bool fail(size_t i, const std::string& m) {
        *err = spec->filename + ":" + std::to_string(t[i].line) + ": " + m;
        return false;
    }
};

std::vector<const DeclImage*> sorted(const ProblemSpec& s, bool unknown) {
    std::vector<const DeclImage*> v;
    for (auto& im : s.images) if (im.unknown == unknown) v.push_back(&im);
    std::sort(v.begin(), v.end(), [](auto a, auto b) { return a->index < b->index; });
    return v;
}

}  // namespace

bool ProblemSpec::uses_op(const std::string& op) const {
    return std::find(ops.begin(), ops.end(), op) != ops.end();
}
const DeclImage* ProblemSpec::unknown(int i) const {
    auto v = sorted(*this, true);
    return i < (int)v.size() ? v[i] : nullptr;
}
const DeclImage* ProblemSpec::array(int i) const {
    auto v = sorted(*this, false);
    return i < (int)v.size() ? v[i] : nullptr;
}
int ProblemSpec::n_unknowns() const { return (int)sorted(*this, true).size(); }
int ProblemSpec::n_arrays() const { return (int)sorted(*this, false).size(); }

bool parse_energy(const std::string& text, ProblemSpec* spec, std::string* err) {
    std::vector<Token> toks;
    if (!lex(text, &toks, err)) { *err = spec->filename + ": " + *err; return false; }
    Parser p{toks, spec, err, {}};
    if (!p.run()) return false;
    int mx = -1;
    for (auto& im : spec->images) mx = std::max(mx, im.index);
    for (auto& pr : spec->params) mx = std::max(mx, pr.index);
    for (auto& g : spec->graphs) for (auto& v : g.vertices) mx = std::max(mx, v.second);
    spec->n_params_total = mx + 1;
    return true;
}

// Family recognition from the declaration signature (unknown/array channel counts
// and domains) and the DSL operators used. Every family's kernels restate the
// derivation the reference would generate for that energy file.
bool classify(ProblemSpec* s, std::string* err) {
    auto dims_of = [](const DeclImage* im) { return im ? (int)im->dims.size() : -1; };
    const int nu = s->n_unknowns(), na = s->n_arrays();
    auto ch = [](const DeclImage* im) { return im ? im->channels : -1; };
    if (s->graphs.empty() && nu == 2 && na == 3 && s->params.size() == 2 &&
        s->uses_op("Rotate2D") && ch(s->unknown(0)) == 2 && ch(s->unknown(1)) == 1 &&
        dims_of(s->unknown(0)) == 2 && ch(s->array(0)) == 2 && ch(s->array(1)) == 2 &&
        ch(s->array(2)) == 1 && s->n_exclude == 1) {
        s->family = "image_warping";
        return true;
    }
    if (s->graphs.empty() && nu == 1 && na == 2 && s->params.empty() &&
        dims_of(s->unknown(0)) == 2 && ch(s->array(0)) == ch(s->unknown(0)) &&
        ch(s->array(1)) == 1 && s->n_exclude == 1 && s->uses_op("Stencil") &&
        !s->uses_op("Rotate2D")) {
        s->family = "poisson_image_editing";
        return true;
    }
    if (s->graphs.empty() && nu == 1 && s->uses_sampled_image && ch(s->unknown(0)) == 2) {
        s->family = "optical_flow";
        return true;
    }
    if (s->graphs.empty() && nu == 1 && !s->computed_arrays.empty() && ch(s->unknown(0)) == 1) {
        s->family = "shape_from_shading";
        return true;
    }
    if (s->graphs.size() == 1 && nu == 2 && s->uses_op("Rotate3D")) {
        s->family = "arap_mesh_deformation";
        return true;
    }
    *err = s->filename + ": energy does not match any kernel family this runtime lowers "
           "(image_warping, poisson_image_editing, optical_flow, shape_from_shading, "
           "arap_mesh_deformation)";
    return false;
}

}  // namespace optamd
