// gen/codegen.h — HIP source for a lowered energy (the role of the reference's
// createjtfcentered / createjtjcentered / createjtfgraph / createjtjgraph / createcost /
// createmodelcost, o.t:2770-3129, and of the Terra emitter, o.t:1949-2665).
#pragma once
#include <string>
#include <vector>
#include "model.h"

// Kernel argument block shared by the host (generic.hip) and the generated source: the
// macro body is compiled on the host and pasted, stringised, into the generated code.
#define OPTAMD_GENARGS_BODY                                                                 \
    struct GenArgs {                                                                        \
        int dims[3];                /* unknowns' index space, unused dims = 1 */            \
        long long npix;             /* elements of that space */                            \
        const void* img[16];        /* by image id: unknowns (T) and known arrays */        \
        double prm[32];             /* by parameter id, at full width (cast to T on use) */ \
        const int* slot[16];        /* graph vertex arrays, graph-major */                  \
        const int* goff[16];        /* per slot: incidence offsets by vertex (N+1) */       \
        const int* geid[16];        /* per slot: incident edge ids, ascending */            \
        const int* gnb[32];         /* per (slot k, other slot): its vertex per incident edge */ \
        int nedge[4];               /* edges per graph */                                   \
        unsigned char* flags;       /* bit0: active (not excluded) */                       \
        long long uoff[4];          /* offset of each unknown image in the vector */        \
        int ymem0;                  /* 2-D row slabs: global row of memory row 0 */          \
        long long own_lo, own_hi;   /* owned pixels (memory indices) */                      \
    };

namespace optamd {
OPTAMD_GENARGS_BODY
namespace gen {

struct GenSource {
    std::string code;
    bool has_centered = false;   // centred residuals present
    bool has_graph = false;      // graph residuals present
    int slot_base[4] = {0, 0, 0, 0};   // GenArgs::slot index of graph g's first vertex array
    int n_precompute = 0;              // kernels gen_precompute_0 .. n-1 (ComputedArrays)
    bool has_tiled = false;            // gen_apply_tiled emitted (2-D centred energies)
    int tiles_x = 32, tiles_y = 8;     // its output tile
    size_t tiled_lds = 0;              // its LDS bytes
    double instances_per_residual = 0; // distinct (residual, shift) instances / centred residuals
    bool prefer_tiled = false;         // the plan's default apply (static rule, codegen.cpp)
    bool has_strip = false;            // gen_apply_strip emitted (2-D centred, no sampled reads)
    int strip_cols = 64;               // its output columns per wave
    bool has_jtf_strip = false;        // gen_jtf_strip emitted (the same walk for J^T F)
    int jtf_strip_cols = 64;
    bool has_cost_strip = false;       // gen_cost_strip emitted (centred-only 2-D energies)
    int cost_strip_cols = 64;
    // materialized J (saveJToCRS): one kernel gen_dump_j_<i> per energy spec, in order;
    // spec i: domain (-1 centred, else graph id), residual rows and nonzeros per element
    struct DumpSpec { int graph; int rows; int nnz; };
    std::vector<DumpSpec> dump;
    // GenArgs::gnb[i] = slot nb_pairs[i].second's vertex of each edge in slot
    // nb_pairs[i].first's incidence order (the graph gathers read neighbours through it)
    std::vector<std::pair<int, int>> nb_pairs;
    // gen_apply_graph adds the centred residuals' terms itself (1-D vertex domains): the
    // plan launches no gen_apply before it
    bool graph_apply_centred = false;
};

// Generate the kernels for `m` in float (dbl = false) or double. off32: every array a
// graph gather reads (the unknown vectors, known and internal images, the incidence
// copies) is below 2 GiB, so slot reads address it as a uniform base plus a 32-bit byte
// offset (the plan checks the sizes).
GenSource generate(GModel& m, bool dbl, bool off32 = false);

}  // namespace gen
}  // namespace optamd
