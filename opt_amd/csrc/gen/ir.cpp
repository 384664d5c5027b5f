// gen/ir.cpp — expression pool, simplification, symbolic derivative, shifting
// (the roles of API/src/ad.t's constructors, simplifier and :d, and of o.t's shiftexp).
#include "ir.h"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <sstream>

namespace optamd {
namespace gen {

static std::string key_of(const Node& n) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%d|%.17g|%d|%d|%d|%d|%d|%d|%d|%d,%d,%d|%d,%d,%d", (int)n.op, n.c, n.a, n.b, n.d, n.i,
             n.ch, n.slot, n.g, n.off[0], n.off[1], n.off[2], n.off2[0], n.off2[1], n.off2[2]);
    return buf;
}

int Pool::intern(const Node& n) {
    const std::string k = key_of(n);
    auto it = index_.find(k);
    if (it != index_.end()) return it->second;
    nodes_.push_back(n);
    const int id = (int)nodes_.size() - 1;
    index_.emplace(k, id);
    return id;
}

bool Pool::is_const(int id, double* v) const {
    if (nodes_[id].op != Op::Const) return false;
    if (v) *v = nodes_[id].c;
    return true;
}

int Pool::cnst(double c) {
    Node n;
    n.op = Op::Const;
    n.c = c == 0.0 ? 0.0 : c;   // no -0 constants
    return intern(n);
}
int Pool::param(int i) {
    Node n;
    n.op = Op::Param;
    n.i = i;
    return intern(n);
}
int Pool::read(int image, int ch, const int* off, int slot, int graph) {
    Node n;
    n.op = Op::Read;
    n.i = image;
    n.ch = ch;
    n.slot = slot;
    n.g = graph;
    if (slot < 0)
        for (int k = 0; k < 3; ++k) n.off[k] = off ? off[k] : 0;
    return intern(n);
}
int Pool::inbox(const int* lo, const int* hi) {
    Node n;
    n.op = Op::InBox;
    for (int k = 0; k < 3; ++k) { n.off[k] = lo[k]; n.off2[k] = hi[k]; }
    return intern(n);
}
int Pool::coord(int dim, int off) {
    Node n;
    n.op = Op::Coord;
    n.i = dim;
    n.off[dim] = off;
    return intern(n);
}

static double fold1(Op op, double a) {
    switch (op) {
        case Op::Neg: return -a;
        case Op::Sqrt: return std::sqrt(a);
        case Op::Sin: return std::sin(a);
        case Op::Cos: return std::cos(a);
        case Op::Exp: return std::exp(a);
        case Op::Log: return std::log(a);
        case Op::Abs: return std::fabs(a);
        case Op::Not: return a == 0.0 ? 1.0 : 0.0;
        default: return 0.0;
    }
}
static double fold2(Op op, double a, double b) {
    switch (op) {
        case Op::Add: return a + b;
        case Op::Sub: return a - b;
        case Op::Mul: return a * b;
        case Op::Div: return a / b;
        case Op::Pow: return std::pow(a, b);
        case Op::Lt: return a < b;
        case Op::Le: return a <= b;
        case Op::Gt: return a > b;
        case Op::Ge: return a >= b;
        case Op::Eq: return a == b;
        case Op::Ne: return a != b;
        case Op::And: return (a != 0.0 && b != 0.0) ? 1.0 : 0.0;
        case Op::Or: return (a != 0.0 || b != 0.0) ? 1.0 : 0.0;
        default: return 0.0;
    }
}

int Pool::un(Op op, int a) {
    double va;
    if (is_const(a, &va)) return cnst(fold1(op, va));
    if (op == Op::Neg && nodes_[a].op == Op::Neg) return nodes_[a].a;
    Node n;
    n.op = op;
    n.a = a;
    return intern(n);
}

int Pool::bin(Op op, int a, int b) {
    double va, vb;
    const bool ca = is_const(a, &va), cb = is_const(b, &vb);
    if (ca && cb) return cnst(fold2(op, va, vb));
    switch (op) {
        case Op::Add:
            if (ca && va == 0.0) return b;
            if (cb && vb == 0.0) return a;
            break;
        case Op::Sub:
            if (cb && vb == 0.0) return a;
            if (ca && va == 0.0) return un(Op::Neg, b);
            if (a == b) return cnst(0.0);
            break;
        case Op::Mul:
            if ((ca && va == 0.0) || (cb && vb == 0.0)) return cnst(0.0);
            if (ca && va == 1.0) return b;
            if (cb && vb == 1.0) return a;
            if (ca && va == -1.0) return un(Op::Neg, b);
            if (cb && vb == -1.0) return un(Op::Neg, a);
            break;
        case Op::Div:
            if (ca && va == 0.0) return cnst(0.0);
            if (cb && vb == 1.0) return a;
            break;
        case Op::Pow:
            if (cb && vb == 1.0) return a;
            if (cb && vb == 0.0) return cnst(1.0);
            break;
        case Op::And:
            if ((ca && va == 0.0) || (cb && vb == 0.0)) return cnst(0.0);
            if (ca) return b;
            if (cb) return a;
            break;
        case Op::Or:
            if ((ca && va != 0.0) || (cb && vb != 0.0)) return cnst(1.0);
            if (ca) return b;
            if (cb) return a;
            break;
        default: break;
    }
    Node n;
    n.op = op;
    n.a = a;
    n.b = b;
    return intern(n);
}

int Pool::select(int c, int a, int b) {
    double vc;
    if (is_const(c, &vc)) return vc != 0.0 ? a : b;
    if (a == b) return a;
    Node n;
    n.op = Op::Select;
    n.a = c;
    n.b = a;
    n.d = b;
    return intern(n);
}

int Pool::sample(int image, int ch, int x, int y, int dx_image, int dy_image) {
    Node n;
    n.op = Op::Sample;
    n.i = image;
    n.ch = ch;
    n.a = x;
    n.b = y;
    n.off2[0] = dx_image;
    n.off2[1] = dy_image;
    return intern(n);
}

int Pool::substitute(int id, const std::map<int, int>& repl) {
    if (id < 0) return id;
    auto it = repl.find(id);
    if (it != repl.end()) return it->second;
    Node n = nodes_[id];
    if (n.a < 0 && n.b < 0 && n.d < 0) return id;
    Node m = n;
    m.a = substitute(n.a, repl);
    m.b = substitute(n.b, repl);
    m.d = substitute(n.d, repl);
    if (m.a == n.a && m.b == n.b && m.d == n.d) return id;
    return intern(m);
}

int Pool::diff(int id, int var) {
    auto it = dmemo_.find({id, var});
    if (it != dmemo_.end()) return it->second;
    const Node n = nodes_[id];   // copy: the pool may grow below
    int r;
    switch (n.op) {
        case Op::Read: {
            r = cnst(id == var ? 1.0 : 0.0);
            auto it = comp_.find(n.i);
            if (it != comp_.end() && n.slot < 0) {   // chain rule through a ComputedArray
                r = cnst(0.0);
                for (const auto& e : it->second)
                    if (e[0] == n.ch && shift(e[1], n.off) == var) r = bin(Op::Add, r, shift(e[2], n.off));
            }
            break;
        }
        case Op::Add: r = bin(Op::Add, diff(n.a, var), diff(n.b, var)); break;
        case Op::Sub: r = bin(Op::Sub, diff(n.a, var), diff(n.b, var)); break;
        case Op::Neg: r = un(Op::Neg, diff(n.a, var)); break;
        case Op::Mul:
            r = bin(Op::Add, bin(Op::Mul, diff(n.a, var), n.b), bin(Op::Mul, n.a, diff(n.b, var)));
            break;
        case Op::Div: {   // (a' b - a b') / b^2
            const int da = diff(n.a, var), db = diff(n.b, var);
            r = bin(Op::Sub, bin(Op::Div, da, n.b), bin(Op::Div, bin(Op::Mul, n.a, db), bin(Op::Mul, n.b, n.b)));
            break;
        }
        case Op::Sqrt:   // a' / (2 sqrt a)
            r = bin(Op::Div, diff(n.a, var), bin(Op::Mul, cnst(2.0), id));
            break;
        case Op::Sin: r = bin(Op::Mul, diff(n.a, var), un(Op::Cos, n.a)); break;
        case Op::Cos: r = un(Op::Neg, bin(Op::Mul, diff(n.a, var), un(Op::Sin, n.a))); break;
        case Op::Exp: r = bin(Op::Mul, diff(n.a, var), id); break;
        case Op::Log: r = bin(Op::Div, diff(n.a, var), n.a); break;
        case Op::Abs:
            r = bin(Op::Mul, diff(n.a, var), select(bin(Op::Lt, n.a, cnst(0.0)), cnst(-1.0), cnst(1.0)));
            break;
        case Op::Pow: {   // constant exponent: e a^(e-1) a'; general: a^b (b' ln a + b a'/a)
            double e;
            if (is_const(n.b, &e))
                r = bin(Op::Mul, bin(Op::Mul, cnst(e), bin(Op::Pow, n.a, cnst(e - 1.0))), diff(n.a, var));
            else
                r = bin(Op::Mul, id,
                        bin(Op::Add, bin(Op::Mul, diff(n.b, var), un(Op::Log, n.a)),
                            bin(Op::Div, bin(Op::Mul, n.b, diff(n.a, var)), n.a)));
            break;
        }
        case Op::Select: r = select(n.a, diff(n.b, var), diff(n.d, var)); break;
        case Op::Sample: {   // op:getpartials (o.t:3274-3278): the derivative images, sampled
            const int da = diff(n.a, var), db = diff(n.b, var);
            if (n.off2[0] < 0) { r = cnst(0.0); break; }   // rejected by the front end if used
            r = bin(Op::Add, bin(Op::Mul, sample(n.off2[0], n.ch, n.a, n.b, -1, -1), da),
                    bin(Op::Mul, sample(n.off2[1], n.ch, n.a, n.b, -1, -1), db));
            break;
        }
        default: r = cnst(0.0); break;   // constants, parameters, bounds, comparisons, logic
    }
    dmemo_[{id, var}] = r;
    return r;
}

int Pool::shift(int id, const int* s) {
    const std::string sk = std::to_string(s[0]) + "," + std::to_string(s[1]) + "," + std::to_string(s[2]);
    auto it = smemo_.find({id, sk});
    if (it != smemo_.end()) return it->second;
    const Node n = nodes_[id];
    int r;
    switch (n.op) {
        case Op::Read:
            if (n.slot >= 0) { r = id; break; }
            {
                int o[3] = {n.off[0] + s[0], n.off[1] + s[1], n.off[2] + s[2]};
                r = read(n.i, n.ch, o);
            }
            break;
        case Op::InBox: {
            int lo[3], hi[3];
            for (int k = 0; k < 3; ++k) { lo[k] = n.off[k] + s[k]; hi[k] = n.off2[k] + s[k]; }
            r = inbox(lo, hi);
            break;
        }
        case Op::Coord: r = coord(n.i, n.off[n.i] + s[n.i]); break;
        case Op::Const:
        case Op::Param: r = id; break;
        case Op::Select: r = select(shift(n.a, s), shift(n.b, s), shift(n.d, s)); break;
        case Op::Sample: r = sample(n.i, n.ch, shift(n.a, s), shift(n.b, s), n.off2[0], n.off2[1]); break;
        default:
            if (n.b < 0) r = un(n.op, shift(n.a, s));
            else r = bin(n.op, shift(n.a, s), shift(n.b, s));
            break;
    }
    smemo_[{id, sk}] = r;
    return r;
}

std::string Pool::str(int id) const {
    const Node& n = nodes_[id];
    std::ostringstream o;
    switch (n.op) {
        case Op::Const: o << n.c; break;
        case Op::Param: o << "P" << n.i; break;
        case Op::Read:
            o << "I" << n.i << "[" << n.ch << "]";
            if (n.slot >= 0) o << "@g" << n.g << "." << n.slot;
            else o << "(" << n.off[0] << "," << n.off[1] << "," << n.off[2] << ")";
            break;
        case Op::InBox: o << "inbox"; break;
        case Op::Coord:
            o << "idx" << n.i;
            if (n.off[n.i]) o << (n.off[n.i] > 0 ? "+" : "") << n.off[n.i];
            break;
        case Op::Select: o << "(" << str(n.a) << " ? " << str(n.b) << " : " << str(n.d) << ")"; break;
        case Op::Sample: o << "sample_I" << n.i << "[" << n.ch << "](" << str(n.a) << ", " << str(n.b) << ")"; break;
        default: {
            static const char* names[] = {"", "", "", "", "", "+", "-", "*", "/", "neg", "sqrt", "sin", "cos",
                                          "exp", "log", "abs", "pow", "", "<", "<=", ">", ">=", "==", "!=", "&&",
                                          "||", "!"};
            if (n.b < 0) o << names[(int)n.op] << "(" << str(n.a) << ")";
            else o << "(" << str(n.a) << " " << names[(int)n.op] << " " << str(n.b) << ")";
        }
    }
    return o.str();
}

}  // namespace gen
}  // namespace optamd
