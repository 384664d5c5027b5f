// problem.h — the parsed energy specification (what Opt_ProblemDefine records).
//
// The reference runs the energy file as a Lua program inside Terra
// (problemSpecFromFile, API/src/o.t:1295-1348) and derives every kernel symbolically
// (o.t:2669-3235). This runtime reads the file's declarations (Dim, Unknown, Array,
// Param, Graph, UsePreconditioner, Exclude, ComputedArray, SampledImage) and lowers
// the energy to one of the hand-written HIP kernel families it recognises from the
// declaration signature and the DSL operators the energy uses. A general Lua-subset
// front-end with symbolic AD is a later row.
#pragma once
#include <string>
#include <vector>

namespace optamd {

struct DeclDim { std::string name; int index = -1; };

struct DeclImage {
    std::string name;
    std::string elem;        // "float" / "uint8" ... scalar element type
    int channels = 1;        // opt_float2 -> 2 ...
    std::vector<std::string> dims;
    int index = -1;          // position in problemparams
    bool unknown = false;
};

struct DeclParam { std::string name; std::string type; int index = -1; };

struct DeclGraph {
    std::string name;
    std::vector<std::string> dims;                       // edge-count dims
    std::vector<std::pair<std::string, int>> vertices;   // (slot name, param index)
};

struct ProblemSpec {
    std::string filename;
    std::string solverkind;      // gaussNewtonGPU | LMGPU | gaussNewtonCPU
    std::vector<DeclDim> dims;
    std::vector<DeclImage> images;
    std::vector<DeclParam> params;
    std::vector<DeclGraph> graphs;
    bool use_preconditioner = false;  // default: opt.ProblemSpec, API/src/o.t:258
    int n_exclude = 0;
    std::vector<std::string> computed_arrays;
    bool uses_sampled_image = false;
    std::vector<std::string> ops;     // DSL operators seen (Rotate2D, Stencil, ...)
    std::string family;               // set by classify()
    int n_params_total = 0;           // highest declared index + 1
    std::string text;                 // the energy file (family "generic": re-lowered per plan)
    std::vector<unsigned> dim_values; // generic plans: Opt_ProblemPlan's dimensions

    bool uses_op(const std::string& op) const;
    const DeclImage* unknown(int i) const;   // i-th unknown by declared index order
    const DeclImage* array(int i) const;     // i-th Array by declared index order
    int n_unknowns() const;
    int n_arrays() const;
    bool lm() const { return solverkind == "LMGPU"; }
};

// Parse `text` (contents of an Opt energy file). Returns false + message on error.
bool parse_energy(const std::string& text, ProblemSpec* spec, std::string* err);
// Decide which kernel family lowers this energy; false + message if none.
bool classify(ProblemSpec* spec, std::string* err);
// General front end (generic.hip): accept any energy gen/ lowers; sets family "generic".
bool generic_accepts(const std::string& text, ProblemSpec* spec, std::string* err);
int generic_source(const std::string& text, bool dbl, std::string* out, bool off32 = false);
int generic_describe(const std::string& text, std::string* out);
int generic_compile_check(const std::string& text, bool dbl, std::string* log);
// Structural signature of the lowered energy (declarations + residual templates, names
// dropped); false + message if the front end cannot lower it.
bool generic_signature(const std::string& text, std::string* sig, bool* use_pre, std::string* err);
// true iff spec->text lowers to exactly the energy spec->family's kernels implement
// (then also takes UsePreconditioner from the lowered model); else false + reason.
bool family_is_canonical(ProblemSpec* spec, std::string* why);

}  // namespace optamd
