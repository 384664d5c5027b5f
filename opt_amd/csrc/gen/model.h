// gen/model.h — an energy file lowered to declarations + scalar residual templates.
//
// The reference runs the energy file as a Lua program against lib.t / ProblemSpecAD
// (API/src/o.t:1295-1348) and turns every Energy term into residual templates grouped by
// domain (toenergyspecs / classifyexpression, o.t:2669-2715). build_model() does the same
// with a Lua-subset interpreter (gen/lua.cpp): the result lists the declarations in
// problemparams order and one template per scalar residual, each with its domain
// (centred over the unknowns' index space, or a graph) and its unknown support.
#pragma once
#include <string>
#include <vector>
#include "ir.h"

namespace optamd {
namespace gen {

struct GDim { std::string name; int index = -1; };
struct GImage {
    std::string name;
    int index = -1;              // position in problemparams
    int channels = 1;
    bool unknown = false;
    std::vector<int> dims;       // GDim ids
    std::string elem = "float";  // element type of a known array ("float", "uint8", ...)
    bool internal = false;       // ComputedArray value / gradient image: allocated by the plan
    bool tvalued = false;        // stored in the solver precision T (unknowns, internal
                                 // images, arrays aliasing an unknown's parameter slot)
};
// d(computed channel)/d(unknown access u): a gradient image (gimg) or a constant (gimg -1)
struct GGrad { int ch = 0; int u = -1; int expr = -1; int gimg = -1; };
// ComputedArray (ProblemSpecAD:ComputedImage, o.t:1686-1718): evaluated per pixel by the
// precompute kernel (createprecomputed, o.t:3131-3153) with its gradient images.
struct GComputed {
    int image = -1;
    std::vector<int> expr;         // per channel
    std::vector<GGrad> grads;
    int lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};   // bbox of the expression (bboxforexpression)
};
struct GParam { std::string name; std::string type; int index = -1; };
struct GGraph {
    std::string name;
    std::vector<int> dims;                // edge-count GDim ids
    std::vector<std::string> slot_names;
    std::vector<int> slot_index;          // problemparams index of each vertex array
};
struct GResidual {
    int expr = -1;                 // scalar expression (centred: wrapped in its bbox select)
    int graph = -1;                // -1: centred over the unknowns' index space
    std::vector<int> unknowns;     // distinct unknown Read nodes (the support)
};

struct GModel {
    Pool pool;
    std::vector<GDim> dims;
    std::vector<GImage> images;
    std::vector<GParam> params;
    std::vector<GGraph> graphs;
    std::vector<GResidual> residuals;
    std::vector<GComputed> computed;   // declaration order (= precompute order)
    int exclude = -1;              // Exclude(expr): centred scalar, -1 = none
    bool use_preconditioner = false;
    std::string unsupported;       // first construct the generic path cannot lower
    int n_params_total = 0;

    int unknown_dims() const;      // dimensionality of the unknowns' index space
    std::vector<int> unknown_images() const;   // image ids of the unknowns, declaration order
};

// Run `text` (an Opt energy file). false + message on a Lua or DSL error.
bool build_model(const std::string& text, GModel* m, std::string* err);

}  // namespace gen
}  // namespace optamd
