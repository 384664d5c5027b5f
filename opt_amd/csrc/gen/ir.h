// gen/ir.h — scalar expression IR of the general energy front end.
//
// The reference builds energies as symbolic expressions (API/src/ad.t: Exp / Var /
// Apply / Const, with :d for derivatives and a simplifier) over image accesses
// (ImageAccess with an Offset or a graph index, o.t:2669-2710) and bounds tests
// (BoundsAccess). Here every scalar expression is a node of one hash-consed pool
// (structurally equal expressions share an id, so the code generator's common
// subexpressions fall out of the pool), built with light algebraic simplification
// (constant folding, 0 / 1 identities) and differentiated symbolically.
#pragma once
#include <array>
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace optamd {
namespace gen {

enum class Op : uint8_t {
    Const,    // c
    Param,    // scalar problem parameter #i
    Read,     // image i, channel ch, at offset off (centred) or graph slot `slot`
    InBox,    // all of [off, off2] (per dimension) inside the domain
    Coord,    // index coordinate i (Index(i)), shifted by off[i]
    Add, Sub, Mul, Div, Neg,
    Sqrt, Sin, Cos, Exp, Log, Abs, Pow,
    Select,   // a ? b : c
    Lt, Le, Gt, Ge, Eq, Ne, And, Or, Not,
    Sample,   // bilinear sample of image i, channel ch, at (a, b); off2[0] / off2[1] = the
              // images sampled for d/dx and d/dy (-1: none) (ad.sampledimage, o.t:3266-3280)
};

struct Node {
    Op op = Op::Const;
    double c = 0.0;
    int a = -1, b = -1, d = -1;     // children
    int i = -1;                     // Param index / image index / coordinate dimension
    int ch = 0;                     // Read channel
    int slot = -1;                  // Read: graph slot (-1: offset access)
    int g = -1;                     // Read: graph id for slot accesses
    int off[3] = {0, 0, 0};
    int off2[3] = {0, 0, 0};        // InBox upper corner
};

class Pool {
public:
    const Node& at(int id) const { return nodes_[id]; }
    int size() const { return (int)nodes_.size(); }

    int cnst(double c);
    int param(int i);
    int read(int image, int ch, const int* off, int slot = -1, int graph = -1);
    int inbox(const int* lo, const int* hi);
    int coord(int dim, int off = 0);
    int un(Op op, int a);
    int bin(Op op, int a, int b);
    int select(int c, int a, int b);
    int sample(int image, int ch, int x, int y, int dx_image, int dy_image);

    bool is_const(int id, double* v = nullptr) const;
    // d(id)/d(var) where var is a Read node (an unknown access)
    int diff(int id, int var);
    // id with every centred access / bounds test / coordinate moved by `s`
    int shift(int id, const int* s);
    // id with every node in `repl` replaced by its image (children rebuilt, hash-consed)
    int substitute(int id, const std::map<int, int>& repl);
    // Visit every node reachable from id once.
    template <class F>
    void visit(int id, F&& f) const {
        std::vector<char> seen(nodes_.size(), 0);
        std::vector<int> st{id};
        while (!st.empty()) {
            const int n = st.back();
            st.pop_back();
            if (n < 0 || seen[n]) continue;
            seen[n] = 1;
            const Node nd = nodes_[n];   // copy: f may grow the pool
            f(n, nd);
            for (int c : {nd.a, nd.b, nd.d}) st.push_back(c);
        }
    }
    std::string str(int id) const;
    // Register d(image ch)/d(u) = gnode for a ComputedArray image (ImageAccess:gradient,
    // o.t:1551-1562): diff() of a read of that image at offset o yields gnode shifted by o
    // for the unknown access u shifted by o.
    void add_computed_grad(int image, int ch, int u, int gnode) { comp_[image].push_back({ch, u, gnode}); }
    const std::map<int, std::vector<std::array<int, 3>>>& computed_grads() const { return comp_; }

private:
    int intern(const Node& n);
    std::vector<Node> nodes_;
    std::unordered_map<std::string, int> index_;
    std::map<std::pair<int, int>, int> dmemo_;
    std::map<std::pair<int, std::string>, int> smemo_;
    std::map<int, std::vector<std::array<int, 3>>> comp_;   // image -> (ch, u, gnode)
};

}  // namespace gen
}  // namespace optamd
