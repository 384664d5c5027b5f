// gen/lua.cpp — a Lua-subset interpreter for Opt energy files, with the DSL of the
// reference's API/src/lib.t and ProblemSpecAD (o.t:251-475) as builtins.
//
// Supported Lua: local / global assignment (multiple targets and values), function
// definitions (global, local, closures, varargs not needed), return, calls and method
// calls (incl. f{...} / f"..." sugar), tables (array and hash parts, nested), field and
// index access, numeric and generic for, while, if / elseif / else, and / or / not,
// comparisons, arithmetic, string concatenation, and the few library functions energy
// files use (print, pairs, ipairs, tostring, type, unpack, math.*).
// DSL: Dim, Param, Unknown, Array / Image, Graph (+ G.slot), UsePreconditioner, Exclude,
// Energy, Select, InBounds, InBoundsExpanded, Index, Stencil, eq / greater / greatereq /
// less / lesseq / notEq, And / Or / Not / All, Dot3, Sqrt, normalize, length, Vector,
// Rotate2D, Rotate3D, Matrix3x3Mul, sin / cos / exp / log / abs / pow; image access
// X(dx, dy[, ch]), X(G.v) and component access e(i), e:dot(f).
// Not lowered by the generic path: ComputedArray, SampledImage, L_p, Slice (they record
// GModel::unsupported; the hand-written families cover the examples that use them).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include "model.h"

namespace optamd {
namespace gen {
namespace {

// ======================================================================== lexer
enum class T { Name, Num, Str, Op, Eof };
struct Tok { T k; std::string s; double v = 0; int line = 0; };

struct LuaError : std::runtime_error {
    explicit LuaError(const std::string& m) : std::runtime_error(m) {}
};
[[noreturn]] void fail(int line, const std::string& m) {
    throw LuaError("line " + std::to_string(line) + ": " + m);
}

std::vector<Tok> lex(const std::string& s) {
    std::vector<Tok> out;
    size_t i = 0, n = s.size();
    int line = 1;
    auto longbr = [&](size_t at, int* lv) {
        size_t j = at + 1;
        int l = 0;
        while (j < n && s[j] == '=') { ++l; ++j; }
        if (j < n && s[j] == '[') { *lv = l; return true; }
        return false;
    };
    auto skiplong = [&](size_t at, int lv, std::string* body) {
        const std::string close = "]" + std::string(lv, '=') + "]";
        const size_t st = at + 2 + lv;
        const size_t e = s.find(close, st);
        if (e == std::string::npos) fail(line, "unterminated long bracket");
        if (body) *body = s.substr(st, e - st);
        for (size_t k = at; k < e; ++k) if (s[k] == '\n') ++line;
        return e + close.size();
    };
    static const char* ops3[] = {"..."};
    static const char* ops2[] = {"==", "~=", "<=", ">=", "..", "::"};
    while (i < n) {
        const char c = s[i];
        if (c == '\n') { ++line; ++i; continue; }
        if (isspace((unsigned char)c)) { ++i; continue; }
        if (c == '-' && i + 1 < n && s[i + 1] == '-') {
            int lv;
            if (i + 2 < n && s[i + 2] == '[' && longbr(i + 2, &lv)) i = skiplong(i + 2, lv, nullptr);
            else while (i < n && s[i] != '\n') ++i;
            continue;
        }
        Tok t;
        t.line = line;
        if (isalpha((unsigned char)c) || c == '_') {
            size_t j = i;
            while (j < n && (isalnum((unsigned char)s[j]) || s[j] == '_')) ++j;
            t.k = T::Name;
            t.s = s.substr(i, j - i);
            i = j;
        } else if (isdigit((unsigned char)c) || (c == '.' && i + 1 < n && isdigit((unsigned char)s[i + 1]))) {
            size_t j = i;
            if (c == '0' && i + 1 < n && (s[i + 1] == 'x' || s[i + 1] == 'X')) {
                j += 2;
                while (j < n && isxdigit((unsigned char)s[j])) ++j;
                t.v = (double)strtoll(s.substr(i, j - i).c_str(), nullptr, 16);
            } else {
                while (j < n && (isdigit((unsigned char)s[j]) || s[j] == '.')) ++j;
                if (j < n && (s[j] == 'e' || s[j] == 'E')) {
                    ++j;
                    if (j < n && (s[j] == '+' || s[j] == '-')) ++j;
                    while (j < n && isdigit((unsigned char)s[j])) ++j;
                }
                t.v = strtod(s.substr(i, j - i).c_str(), nullptr);
            }
            t.k = T::Num;
            i = j;
        } else if (c == '"' || c == '\'') {
            size_t j = i + 1;
            std::string v;
            while (j < n && s[j] != c) {
                if (s[j] == '\\' && j + 1 < n) {
                    const char e = s[j + 1];
                    v += e == 'n' ? '\n' : e == 't' ? '\t' : e;
                    j += 2;
                    continue;
                }
                if (s[j] == '\n') fail(line, "unterminated string");
                v += s[j++];
            }
            if (j >= n) fail(line, "unterminated string");
            t.k = T::Str;
            t.s = v;
            i = j + 1;
        } else if (c == '[' && i + 1 < n && (s[i + 1] == '[' || s[i + 1] == '=')) {
            int lv;
            if (!longbr(i, &lv)) { t.k = T::Op; t.s = "["; ++i; }
            else { t.k = T::Str; i = skiplong(i, lv, &t.s); }
        } else {
            t.k = T::Op;
            bool done = false;
            for (const char* o : ops3)
                if (s.compare(i, 3, o) == 0) { t.s = o; i += 3; done = true; break; }
            if (!done)
                for (const char* o : ops2)
                    if (s.compare(i, 2, o) == 0) { t.s = o; i += 2; done = true; break; }
            if (!done) { t.s = std::string(1, c); ++i; }
        }
        out.push_back(t);
    }
    Tok e;
    e.k = T::Eof;
    e.line = line;
    out.push_back(e);
    return out;
}

// ========================================================================== AST
struct Expr;
struct Stat;
using EP = std::shared_ptr<Expr>;
using SP = std::shared_ptr<Stat>;
using Block = std::vector<SP>;

struct FuncBody { std::vector<std::string> params; bool vararg = false; Block body; };

enum class EK { Nil, True, False, Num, Str, Vararg, Func, Table, Bin, Un, Name, Index, Call, Method };
struct Expr {
    EK k;
    int line = 0;
    double num = 0;
    std::string str;                  // Str / Name / operator / method name
    EP a, b;                          // Bin, Un, Index (a[b]), Call (a), Method (a)
    std::vector<EP> args;             // Call / Method arguments
    std::vector<std::pair<EP, EP>> fields;   // Table: (key or null, value)
    std::shared_ptr<FuncBody> fn;
};

enum class SK { Local, Assign, Call, Do, While, Repeat, NumFor, GenFor, If, Func, LocalFunc, Return, Break };
struct Stat {
    SK k;
    int line = 0;
    std::vector<std::string> names;   // Local / NumFor / GenFor / LocalFunc
    std::vector<EP> targets, values;  // Assign (targets), Local/Assign/Return/GenFor (values)
    EP e, e2, e3;                     // Call expr; While cond; NumFor start/stop/step; Func target
    std::vector<EP> conds;            // If
    std::vector<Block> blocks;        // If branches (+ else), loop / do bodies
    std::shared_ptr<FuncBody> fn;
};

class Parser {
public:
    explicit Parser(std::vector<Tok> t) : t_(std::move(t)) {}
    Block chunk() {
        Block b = block();
        if (peek().k != T::Eof) fail(peek().line, "unexpected '" + peek().s + "'");
        return b;
    }

private:
    std::vector<Tok> t_;
    size_t p_ = 0;
    const Tok& peek(int o = 0) const { return t_[std::min(p_ + o, t_.size() - 1)]; }
    bool isop(const char* s, int o = 0) const { return peek(o).k == T::Op && peek(o).s == s; }
    bool isname(const char* s, int o = 0) const { return peek(o).k == T::Name && peek(o).s == s; }
    Tok next() { return t_[p_ < t_.size() - 1 ? p_++ : p_]; }
    void expectop(const char* s) {
        if (!isop(s)) fail(peek().line, std::string("expected '") + s + "' near '" + peek().s + "'");
        ++p_;
    }
    void expectname(const char* s) {
        if (!isname(s)) fail(peek().line, std::string("expected '") + s + "' near '" + peek().s + "'");
        ++p_;
    }
    std::string name() {
        if (peek().k != T::Name) fail(peek().line, "expected a name near '" + peek().s + "'");
        return next().s;
    }
    bool block_end() const {
        return peek().k == T::Eof || isname("end") || isname("else") || isname("elseif") || isname("until");
    }
    Block block() {
        Block b;
        while (!block_end()) {
            if (isop(";")) { ++p_; continue; }
            if (isname("return")) {
                auto s = std::make_shared<Stat>();
                s->k = SK::Return;
                s->line = next().line;
                if (!block_end() && !isop(";")) s->values = exprlist();
                if (isop(";")) ++p_;
                b.push_back(s);
                break;
            }
            b.push_back(statement());
        }
        return b;
    }
    SP statement() {
        auto s = std::make_shared<Stat>();
        s->line = peek().line;
        if (isname("local")) {
            ++p_;
            if (isname("function")) {
                ++p_;
                s->k = SK::LocalFunc;
                s->names.push_back(name());
                s->fn = funcbody();
                return s;
            }
            s->k = SK::Local;
            s->names.push_back(name());
            while (isop(",")) { ++p_; s->names.push_back(name()); }
            if (isop("=")) { ++p_; s->values = exprlist(); }
            return s;
        }
        if (isname("function")) {
            ++p_;
            s->k = SK::Func;
            auto tgt = std::make_shared<Expr>();
            tgt->k = EK::Name;
            tgt->str = name();
            tgt->line = s->line;
            bool method = false;
            while (isop(".") || isop(":")) {
                method = isop(":");
                ++p_;
                auto ix = std::make_shared<Expr>();
                ix->k = EK::Index;
                ix->a = tgt;
                ix->b = std::make_shared<Expr>();
                ix->b->k = EK::Str;
                ix->b->str = name();
                tgt = ix;
                if (method) break;
            }
            s->e = tgt;
            s->fn = funcbody();
            if (method) s->fn->params.insert(s->fn->params.begin(), "self");
            return s;
        }
        if (isname("for")) {
            ++p_;
            const std::string n1 = name();
            if (isop("=")) {
                ++p_;
                s->k = SK::NumFor;
                s->names.push_back(n1);
                s->e = expr();
                expectop(",");
                s->e2 = expr();
                if (isop(",")) { ++p_; s->e3 = expr(); }
            } else {
                s->k = SK::GenFor;
                s->names.push_back(n1);
                while (isop(",")) { ++p_; s->names.push_back(name()); }
                expectname("in");
                s->values = exprlist();
            }
            expectname("do");
            s->blocks.push_back(block());
            expectname("end");
            return s;
        }
        if (isname("while")) {
            ++p_;
            s->k = SK::While;
            s->e = expr();
            expectname("do");
            s->blocks.push_back(block());
            expectname("end");
            return s;
        }
        if (isname("repeat")) {
            ++p_;
            s->k = SK::Repeat;
            s->blocks.push_back(block());
            expectname("until");
            s->e = expr();
            return s;
        }
        if (isname("do")) {
            ++p_;
            s->k = SK::Do;
            s->blocks.push_back(block());
            expectname("end");
            return s;
        }
        if (isname("if")) {
            ++p_;
            s->k = SK::If;
            s->conds.push_back(expr());
            expectname("then");
            s->blocks.push_back(block());
            while (isname("elseif")) {
                ++p_;
                s->conds.push_back(expr());
                expectname("then");
                s->blocks.push_back(block());
            }
            if (isname("else")) { ++p_; s->blocks.push_back(block()); }
            expectname("end");
            return s;
        }
        if (isname("break")) { ++p_; s->k = SK::Break; return s; }
        // assignment or call
        EP first = suffixed();
        if (isop("=") || isop(",")) {
            s->k = SK::Assign;
            s->targets.push_back(first);
            while (isop(",")) { ++p_; s->targets.push_back(suffixed()); }
            expectop("=");
            s->values = exprlist();
            return s;
        }
        if (first->k != EK::Call && first->k != EK::Method) fail(s->line, "syntax error (expression statement)");
        s->k = SK::Call;
        s->e = first;
        return s;
    }
    std::shared_ptr<FuncBody> funcbody() {
        auto f = std::make_shared<FuncBody>();
        expectop("(");
        if (!isop(")")) {
            do {
                if (isop("...")) { ++p_; f->vararg = true; break; }
                f->params.push_back(name());
            } while (isop(",") && (++p_, true));
        }
        expectop(")");
        f->body = block();
        expectname("end");
        return f;
    }
    std::vector<EP> exprlist() {
        std::vector<EP> v{expr()};
        while (isop(",")) { ++p_; v.push_back(expr()); }
        return v;
    }
    EP primary() {
        auto e = std::make_shared<Expr>();
        e->line = peek().line;
        if (peek().k == T::Name) { e->k = EK::Name; e->str = next().s; return e; }
        if (isop("(")) {
            ++p_;
            EP in = expr();
            expectop(")");
            // parentheses truncate to one value: wrap as a unary "()"
            auto w = std::make_shared<Expr>();
            w->k = EK::Un;
            w->str = "()";
            w->a = in;
            w->line = e->line;
            return w;
        }
        fail(peek().line, "unexpected '" + peek().s + "'");
    }
    EP suffixed() {
        EP e = primary();
        for (;;) {
            if (isop(".")) {
                ++p_;
                auto ix = std::make_shared<Expr>();
                ix->k = EK::Index;
                ix->line = e->line;
                ix->a = e;
                ix->b = std::make_shared<Expr>();
                ix->b->k = EK::Str;
                ix->b->str = name();
                e = ix;
            } else if (isop("[")) {
                ++p_;
                auto ix = std::make_shared<Expr>();
                ix->k = EK::Index;
                ix->line = e->line;
                ix->a = e;
                ix->b = expr();
                expectop("]");
                e = ix;
            } else if (isop(":")) {
                ++p_;
                auto m = std::make_shared<Expr>();
                m->k = EK::Method;
                m->line = e->line;
                m->a = e;
                m->str = name();
                m->args = callargs();
                e = m;
            } else if (isop("(") || isop("{") || peek().k == T::Str) {
                auto c = std::make_shared<Expr>();
                c->k = EK::Call;
                c->line = e->line;
                c->a = e;
                c->args = callargs();
                e = c;
            } else {
                return e;
            }
        }
    }
    std::vector<EP> callargs() {
        if (peek().k == T::Str) {
            auto s = std::make_shared<Expr>();
            s->k = EK::Str;
            s->str = next().s;
            return {s};
        }
        if (isop("{")) return {table()};
        expectop("(");
        std::vector<EP> a;
        if (!isop(")")) a = exprlist();
        expectop(")");
        return a;
    }
    EP table() {
        auto t = std::make_shared<Expr>();
        t->k = EK::Table;
        t->line = peek().line;
        expectop("{");
        while (!isop("}")) {
            if (isop("[")) {
                ++p_;
                EP k = expr();
                expectop("]");
                expectop("=");
                t->fields.push_back({k, expr()});
            } else if (peek().k == T::Name && isop("=", 1)) {
                auto k = std::make_shared<Expr>();
                k->k = EK::Str;
                k->str = next().s;
                ++p_;
                t->fields.push_back({k, expr()});
            } else {
                t->fields.push_back({nullptr, expr()});
            }
            if (isop(",") || isop(";")) ++p_;
            else break;
        }
        expectop("}");
        return t;
    }
    EP simple() {
        auto e = std::make_shared<Expr>();
        e->line = peek().line;
        if (peek().k == T::Num) { e->k = EK::Num; e->num = next().v; return e; }
        if (peek().k == T::Str) { e->k = EK::Str; e->str = next().s; return e; }
        if (isname("nil")) { ++p_; e->k = EK::Nil; return e; }
        if (isname("true")) { ++p_; e->k = EK::True; return e; }
        if (isname("false")) { ++p_; e->k = EK::False; return e; }
        if (isop("...")) { ++p_; e->k = EK::Vararg; return e; }
        if (isname("function")) { ++p_; e->k = EK::Func; e->fn = funcbody(); return e; }
        if (isop("{")) return table();
        return suffixed();
    }
    static int lprec(const std::string& o) {
        if (o == "or") return 1;
        if (o == "and") return 2;
        if (o == "<" || o == ">" || o == "<=" || o == ">=" || o == "~=" || o == "==") return 3;
        if (o == "..") return 9;   // right assoc
        if (o == "+" || o == "-") return 10;
        if (o == "*" || o == "/" || o == "%") return 11;
        if (o == "^") return 14;   // right assoc
        return -1;
    }
    std::string binop() const {
        if (peek().k == T::Op) return peek().s;
        if (isname("and") || isname("or")) return peek().s;
        return "";
    }
    EP expr(int limit = 0) {
        EP left;
        if (isname("not") || isop("-") || isop("#")) {
            const std::string o = next().s;
            auto u = std::make_shared<Expr>();
            u->k = EK::Un;
            u->str = o;
            u->line = peek().line;
            u->a = expr(12);
            left = u;
        } else {
            left = simple();
        }
        for (;;) {
            const std::string o = binop();
            const int pr = lprec(o);
            if (pr < 0 || pr <= limit) break;
            ++p_;
            const int rp = (o == ".." || o == "^") ? pr - 1 : pr;
            auto b = std::make_shared<Expr>();
            b->k = EK::Bin;
            b->str = o;
            b->line = left->line;
            b->a = left;
            b->b = expr(rp);
            left = b;
        }
        return left;
    }
};

// ======================================================================== values
struct Value;
using VList = std::vector<Value>;
struct Table;
struct Closure;
using Builtin = std::function<VList(VList&)>;

enum class V { Nil, Bool, Num, Str, Table, Closure, Builtin, Expr, Dim, Image, Graph, Slot, Type, Opaque };
struct Value {
    V k = V::Nil;
    bool b = false;
    double n = 0;
    std::string s;
    std::shared_ptr<Table> t;
    std::shared_ptr<Closure> f;
    std::shared_ptr<Builtin> bf;
    std::vector<int> e;    // Expr components (node ids)
    int id = -1;           // Dim / Image / Graph id; Slot: graph id; Type: channel count
    int slot = -1;         // Slot index
};
struct Table {
    std::map<std::string, Value> h;   // string keys
    std::vector<Value> a;             // 1..n
};
struct Scope {
    std::map<std::string, std::shared_ptr<Value>> vars;
    std::shared_ptr<Scope> parent;
    std::shared_ptr<Value> find(const std::string& n) {
        for (Scope* s = this; s; s = s->parent.get()) {
            auto it = s->vars.find(n);
            if (it != s->vars.end()) return it->second;
        }
        return nullptr;
    }
};
struct Closure { std::shared_ptr<FuncBody> fn; std::shared_ptr<Scope> env; };

Value num(double d) { Value v; v.k = V::Num; v.n = d; return v; }
Value boolean(bool b) { Value v; v.k = V::Bool; v.b = b; return v; }
Value str(const std::string& s) { Value v; v.k = V::Str; v.s = s; return v; }
Value expr(std::vector<int> e) { Value v; v.k = V::Expr; v.e = std::move(e); return v; }
Value builtin(Builtin f) { Value v; v.k = V::Builtin; v.bf = std::make_shared<Builtin>(std::move(f)); return v; }
Value table() { Value v; v.k = V::Table; v.t = std::make_shared<Table>(); return v; }
bool truthy(const Value& v) { return !(v.k == V::Nil || (v.k == V::Bool && !v.b)); }

struct BreakSignal {};
struct ReturnSignal { VList vals; };

// ================================================================== interpreter
class Interp {
public:
    explicit Interp(GModel* m) : m_(m) {
        globals_ = std::make_shared<Scope>();
        install();
    }
    void run(const Block& b) { exec_block(b, std::make_shared<Scope>(Scope{{}, globals_})); }
    void finish();

private:
    GModel* m_;
    std::shared_ptr<Scope> globals_;
    std::vector<int> energy_terms_;   // scalar residual expressions, in Energy order
    std::vector<std::pair<int, int>> sample_cache_;   // cached Sample node (offset 0) -> its image
    int cache_samples(int e);
    int line_ = 0;

    Pool& P() { return m_->pool; }
    [[noreturn]] void err(const std::string& msg) { fail(line_, msg); }

    // ---------------------------------------------------------------- statements
    void exec_block(const Block& b, std::shared_ptr<Scope> sc) {
        for (auto& s : b) exec(*s, sc);
    }
    void assign(const Expr& t, const Value& v, std::shared_ptr<Scope> sc) {
        if (t.k == EK::Name) {
            auto slot = sc->find(t.str);
            if (slot) *slot = v;
            else globals_->vars[t.str] = std::make_shared<Value>(v);
            return;
        }
        if (t.k == EK::Index) {
            Value obj = eval1(*t.a, sc), key = eval1(*t.b, sc);
            if (obj.k != V::Table) err("indexing assignment into a non-table");
            setidx(*obj.t, key, v);
            return;
        }
        err("cannot assign to this expression");
    }
    static void setidx(Table& t, const Value& key, const Value& v) {
        if (key.k == V::Num && key.n >= 1 && key.n == std::floor(key.n)) {
            const size_t i = (size_t)key.n;
            if (i <= t.a.size()) { t.a[i - 1] = v; return; }
            if (i == t.a.size() + 1) { t.a.push_back(v); return; }
            t.h["#" + std::to_string(i)] = v;
            return;
        }
        if (key.k == V::Str) { t.h[key.s] = v; return; }
        t.h["?" + std::to_string((long long)key.n)] = v;
    }
    void exec(const Stat& s, std::shared_ptr<Scope> sc) {
        line_ = s.line;
        switch (s.k) {
            case SK::Local: {
                VList vals = evallist(s.values, sc);
                for (size_t i = 0; i < s.names.size(); ++i)
                    sc->vars[s.names[i]] = std::make_shared<Value>(i < vals.size() ? vals[i] : Value{});
                break;
            }
            case SK::Assign: {
                VList vals = evallist(s.values, sc);
                for (size_t i = 0; i < s.targets.size(); ++i) assign(*s.targets[i], i < vals.size() ? vals[i] : Value{}, sc);
                break;
            }
            case SK::Call: eval(*s.e, sc); break;
            case SK::Do: exec_block(s.blocks[0], std::make_shared<Scope>(Scope{{}, sc})); break;
            case SK::While:
                try {
                    while (truthy(eval1(*s.e, sc))) exec_block(s.blocks[0], std::make_shared<Scope>(Scope{{}, sc}));
                } catch (BreakSignal&) {}
                break;
            case SK::Repeat:   // the condition sees the body's locals
                try {
                    for (;;) {
                        auto in = std::make_shared<Scope>(Scope{{}, sc});
                        exec_block(s.blocks[0], in);
                        if (truthy(eval1(*s.e, in))) break;
                    }
                } catch (BreakSignal&) {}
                break;
            case SK::NumFor: {
                const Value a = eval1(*s.e, sc), b = eval1(*s.e2, sc);
                const Value st = s.e3 ? eval1(*s.e3, sc) : num(1);
                if (a.k != V::Num || b.k != V::Num || st.k != V::Num) err("numeric for needs numbers");
                try {
                    for (double i = a.n; st.n > 0 ? i <= b.n : i >= b.n; i += st.n) {
                        auto in = std::make_shared<Scope>(Scope{{}, sc});
                        in->vars[s.names[0]] = std::make_shared<Value>(num(i));
                        exec_block(s.blocks[0], in);
                    }
                } catch (BreakSignal&) {}
                break;
            }
            case SK::GenFor: {
                VList it = evallist(s.values, sc);
                Value f = it.size() > 0 ? it[0] : Value{}, st = it.size() > 1 ? it[1] : Value{},
                      ctl = it.size() > 2 ? it[2] : Value{};
                try {
                    for (;;) {
                        VList args{st, ctl};
                        VList r = call(f, args);
                        if (r.empty() || r[0].k == V::Nil) break;
                        ctl = r[0];
                        auto in = std::make_shared<Scope>(Scope{{}, sc});
                        for (size_t i = 0; i < s.names.size(); ++i)
                            in->vars[s.names[i]] = std::make_shared<Value>(i < r.size() ? r[i] : Value{});
                        exec_block(s.blocks[0], in);
                    }
                } catch (BreakSignal&) {}
                break;
            }
            case SK::If: {
                size_t i = 0;
                for (; i < s.conds.size(); ++i)
                    if (truthy(eval1(*s.conds[i], sc))) {
                        exec_block(s.blocks[i], std::make_shared<Scope>(Scope{{}, sc}));
                        return;
                    }
                if (s.blocks.size() > s.conds.size())
                    exec_block(s.blocks.back(), std::make_shared<Scope>(Scope{{}, sc}));
                break;
            }
            case SK::Func: {
                Value f;
                f.k = V::Closure;
                f.f = std::make_shared<Closure>(Closure{s.fn, sc});
                assign(*s.e, f, sc);
                break;
            }
            case SK::LocalFunc: {
                auto slot = std::make_shared<Value>();
                sc->vars[s.names[0]] = slot;
                slot->k = V::Closure;
                slot->f = std::make_shared<Closure>(Closure{s.fn, sc});
                break;
            }
            case SK::Return: throw ReturnSignal{evallist(s.values, sc)};
            case SK::Break: throw BreakSignal{};
        }
    }

    // --------------------------------------------------------------- expressions
    VList evallist(const std::vector<EP>& es, std::shared_ptr<Scope> sc) {
        VList out;
        for (size_t i = 0; i < es.size(); ++i) {
            VList v = eval(*es[i], sc);
            if (i + 1 == es.size()) out.insert(out.end(), v.begin(), v.end());
            else out.push_back(v.empty() ? Value{} : v[0]);
        }
        return out;
    }
    Value eval1(const Expr& e, std::shared_ptr<Scope> sc) {
        VList v = eval(e, sc);
        return v.empty() ? Value{} : v[0];
    }
    VList eval(const Expr& e, std::shared_ptr<Scope> sc) {
        line_ = e.line ? e.line : line_;
        switch (e.k) {
            case EK::Nil: return {Value{}};
            case EK::True: return {boolean(true)};
            case EK::False: return {boolean(false)};
            case EK::Num: return {num(e.num)};
            case EK::Str: return {str(e.str)};
            case EK::Vararg: {
                auto va = sc->find("...");
                if (!va || va->k != V::Table) return {};
                return va->t->a;
            }
            case EK::Func: {
                Value f;
                f.k = V::Closure;
                f.f = std::make_shared<Closure>(Closure{e.fn, sc});
                return {f};
            }
            case EK::Table: {
                Value t = table();
                for (size_t i = 0; i < e.fields.size(); ++i) {
                    auto& fd = e.fields[i];
                    if (fd.first) setidx(*t.t, eval1(*fd.first, sc), eval1(*fd.second, sc));
                    else if (i + 1 == e.fields.size()) {
                        for (auto& v : eval(*fd.second, sc)) t.t->a.push_back(v);
                    } else {
                        t.t->a.push_back(eval1(*fd.second, sc));
                    }
                }
                return {t};
            }
            case EK::Name: {
                auto v = sc->find(e.str);
                return {v ? *v : Value{}};
            }
            case EK::Index: return {index(eval1(*e.a, sc), eval1(*e.b, sc))};
            case EK::Call: {
                Value f = eval1(*e.a, sc);
                VList args = evallist(e.args, sc);
                return call(f, args);
            }
            case EK::Method: {
                Value obj = eval1(*e.a, sc);
                VList args = evallist(e.args, sc);
                return method(obj, e.str, args);
            }
            case EK::Un: {
                Value a = eval1(*e.a, sc);
                if (e.str == "()") return {a};
                if (e.str == "not") return {boolean(!truthy(a))};
                if (e.str == "#") {
                    if (a.k == V::Table) return {num((double)a.t->a.size())};
                    if (a.k == V::Str) return {num((double)a.s.size())};
                    if (a.k == V::Expr) return {num((double)a.e.size())};
                    err("length of a non-table");
                }
                return {arith("-u", a, Value{})};
            }
            case EK::Bin: {
                if (e.str == "and") {
                    Value a = eval1(*e.a, sc);
                    return {truthy(a) ? eval1(*e.b, sc) : a};
                }
                if (e.str == "or") {
                    Value a = eval1(*e.a, sc);
                    return {truthy(a) ? a : eval1(*e.b, sc)};
                }
                return {arith(e.str, eval1(*e.a, sc), eval1(*e.b, sc))};
            }
        }
        return {};
    }
    Value index(const Value& o, const Value& k) {
        if (o.k == V::Table) {
            if (k.k == V::Num && k.n >= 1 && k.n == std::floor(k.n) && (size_t)k.n <= o.t->a.size())
                return o.t->a[(size_t)k.n - 1];
            if (k.k == V::Str) {
                auto it = o.t->h.find(k.s);
                return it == o.t->h.end() ? Value{} : it->second;
            }
            if (k.k == V::Num) {
                auto it = o.t->h.find("#" + std::to_string((long long)k.n));
                return it == o.t->h.end() ? Value{} : it->second;
            }
            return Value{};
        }
        if (o.k == V::Graph && k.k == V::Str) {
            const GGraph& g = m_->graphs[o.id];
            for (size_t i = 0; i < g.slot_names.size(); ++i)
                if (g.slot_names[i] == k.s) {
                    Value v;
                    v.k = V::Slot;
                    v.id = o.id;
                    v.slot = (int)i;
                    return v;
                }
            err("graph " + g.name + " has no vertex slot '" + k.s + "'");
        }
        if (o.k == V::Expr && k.k == V::Num) {   // ExpVector:__index, 0-based (ad.t:312-317)
            const int i = (int)k.n;
            if (i < 0 || i >= (int)o.e.size()) err("index out of bounds");
            return expr({o.e[i]});
        }
        // internals of DSL objects (the reference's debug printing walks .data / .key_ ...):
        // an opaque value that absorbs further indexing and calls
        if (o.k == V::Opaque || ((o.k == V::Image || o.k == V::Dim || o.k == V::Expr || o.k == V::Slot) && k.k == V::Str)) {
            Value v;
            v.k = V::Opaque;
            return v;
        }
        err("attempt to index a non-table value");
    }

    // ------------------------------------------------------------------ calls
    VList call(const Value& f, VList& args) {
        if (f.k == V::Builtin) return (*f.bf)(args);
        if (f.k == V::Closure) {
            auto sc = std::make_shared<Scope>(Scope{{}, f.f->env});
            const auto& ps = f.f->fn->params;
            for (size_t i = 0; i < ps.size(); ++i)
                sc->vars[ps[i]] = std::make_shared<Value>(i < args.size() ? args[i] : Value{});
            if (f.f->fn->vararg) {
                Value va = table();
                for (size_t i = ps.size(); i < args.size(); ++i) va.t->a.push_back(args[i]);
                sc->vars["..."] = std::make_shared<Value>(va);
            }
            const int saved = line_;
            try {
                exec_block(f.f->fn->body, sc);
            } catch (ReturnSignal& r) {
                line_ = saved;
                return r.vals;
            }
            line_ = saved;
            return {};
        }
        if (f.k == V::Image) return {image_access(f.id, args)};
        if (f.k == V::Expr) {   // component access e(i)
            if (args.size() != 1 || args[0].k != V::Num) err("expression call expects one component index");
            const int i = (int)args[0].n;
            if (i < 0 || i >= (int)f.e.size()) err("component index out of range");
            return {expr({f.e[i]})};
        }
        if (f.k == V::Opaque) return {f};
        err("attempt to call a non-function value");
    }
    VList method(const Value& o, const std::string& name, VList& args) {
        if (o.k == V::Expr && name == "dot") {
            if (args.size() != 1) err(":dot expects one argument");
            return {dot(o, args[0])};
        }
        if (o.k == V::Expr && name == "size") return {num((double)o.e.size())};
        Value f = index(o, str(name));
        VList a{o};
        a.insert(a.end(), args.begin(), args.end());
        return call(f, a);
    }

    // ------------------------------------------------------- expression algebra
    std::vector<int> as_expr(const Value& v) {
        if (v.k == V::Expr) return v.e;
        if (v.k == V::Num) return {P().cnst(v.n)};
        if (v.k == V::Bool) return {P().cnst(v.b ? 1.0 : 0.0)};
        err("expected a number or an expression");
    }
    Value zip(Op op, const Value& a, const Value& b) {
        std::vector<int> x = as_expr(a), y = as_expr(b);
        if (x.size() != y.size() && x.size() != 1 && y.size() != 1)
            err("vector size mismatch (" + std::to_string(x.size()) + " vs " + std::to_string(y.size()) + ")");
        const size_t n = std::max(x.size(), y.size());
        std::vector<int> r(n);
        for (size_t i = 0; i < n; ++i) r[i] = P().bin(op, x[x.size() == 1 ? 0 : i], y[y.size() == 1 ? 0 : i]);
        return expr(r);
    }
    Value map1(Op op, const Value& a) {
        std::vector<int> x = as_expr(a);
        for (int& c : x) c = P().un(op, c);
        return expr(x);
    }
    Value arith(const std::string& o, const Value& a, const Value& b) {
        const bool nums = a.k == V::Num && (b.k == V::Num || o == "-u");
        if (nums) {
            if (o == "-u") return num(-a.n);
            if (o == "+") return num(a.n + b.n);
            if (o == "-") return num(a.n - b.n);
            if (o == "*") return num(a.n * b.n);
            if (o == "/") return num(a.n / b.n);
            if (o == "%") return num(a.n - std::floor(a.n / b.n) * b.n);
            if (o == "^") return num(std::pow(a.n, b.n));
            if (o == "<") return boolean(a.n < b.n);
            if (o == ">") return boolean(a.n > b.n);
            if (o == "<=") return boolean(a.n <= b.n);
            if (o == ">=") return boolean(a.n >= b.n);
            if (o == "==") return boolean(a.n == b.n);
            if (o == "~=") return boolean(a.n != b.n);
            if (o == "..") return str(numstr(a.n) + numstr(b.n));
        }
        if (o == "..") return str(tostr(a) + tostr(b));
        if (o == "==" || o == "~=") {
            bool eqv;
            if (a.k != b.k) eqv = false;
            else if (a.k == V::Str) eqv = a.s == b.s;
            else if (a.k == V::Bool) eqv = a.b == b.b;
            else if (a.k == V::Nil) eqv = true;
            else if (a.k == V::Table) eqv = a.t == b.t;
            else if (a.k == V::Expr) eqv = a.e == b.e;
            else eqv = a.id == b.id && a.slot == b.slot;
            return boolean(o == "==" ? eqv : !eqv);
        }
        if ((o == "<" || o == ">" || o == "<=" || o == ">=") && a.k == V::Str && b.k == V::Str) {
            const int c = a.s.compare(b.s);
            return boolean(o == "<" ? c < 0 : o == ">" ? c > 0 : o == "<=" ? c <= 0 : c >= 0);
        }
        if (o == "-u") return map1(Op::Neg, a);
        if (o == "+") return zip(Op::Add, a, b);
        if (o == "-") return zip(Op::Sub, a, b);
        if (o == "*") return zip(Op::Mul, a, b);
        if (o == "/") return zip(Op::Div, a, b);
        if (o == "^") return zip(Op::Pow, a, b);
        err("unsupported operator '" + o + "' on these values");
    }
    static std::string numstr(double d) {
        char b[64];
        if (d == std::floor(d) && std::fabs(d) < 1e15) snprintf(b, sizeof(b), "%lld", (long long)d);
        else snprintf(b, sizeof(b), "%.14g", d);
        return b;
    }
    std::string tostr(const Value& v) {
        switch (v.k) {
            case V::Nil: return "nil";
            case V::Bool: return v.b ? "true" : "false";
            case V::Num: return numstr(v.n);
            case V::Str: return v.s;
            case V::Expr: return v.e.size() == 1 ? P().str(v.e[0]) : "vector";
            default: return "object";
        }
    }
    Value dot(const Value& a, const Value& b) {
        std::vector<int> x = as_expr(a), y = as_expr(b);
        if (x.size() != y.size()) err("dot of vectors of different sizes");
        int s = P().cnst(0.0);
        for (size_t i = 0; i < x.size(); ++i) s = P().bin(Op::Add, s, P().bin(Op::Mul, x[i], y[i]));
        return expr({s});
    }
    int comp(const Value& v, int i) {
        std::vector<int> x = as_expr(v);
        if (i >= (int)x.size()) err("component " + std::to_string(i) + " of a " + std::to_string(x.size()) + "-vector");
        return x[i];
    }

    // ---------------------------------------------------------- DSL: declarations
    int dim_of(const Value& v) {
        if (v.k != V::Dim) err("expected a Dim");
        return v.id;
    }
    int lp_counter_ = 0;
    void note_index(int idx) { m_->n_params_total = std::max(m_->n_params_total, idx + 1); }
    int channels_of(const Value& t) {
        if (t.k == V::Type) return t.id;
        err("expected an element type (opt_float, opt_float2, ...)");
    }
    Value decl_image(VList& a, bool unknown) {
        if (a.size() < 4) err("Unknown/Array(name, type, {dims}, index)");
        GImage im;
        im.name = a[0].s;
        im.channels = channels_of(a[1]);
        im.elem = a[1].s.empty() ? "float" : a[1].s;
        if (a[2].k != V::Table) err("image dims must be a table of Dims");
        for (auto& d : a[2].t->a) im.dims.push_back(dim_of(d));
        im.index = (int)a[3].n;
        im.unknown = unknown;
        im.tvalued = unknown;
        note_index(im.index);
        m_->images.push_back(im);
        Value v;
        v.k = V::Image;
        v.id = (int)m_->images.size() - 1;
        return v;
    }
    // ProblemSpecAD:ComputedImage (o.t:1686-1718): a T-valued internal image holding exp,
    // plus one gradient image per (channel, unknown access) whose derivative is not constant.
    Value computed_array(VList& a) {
        if (a.size() < 3 || a[1].k != V::Table) err("ComputedArray(name, {dims}, expression)");
        GImage im;
        im.name = a[0].s;
        for (auto& d : a[1].t->a) im.dims.push_back(dim_of(d));
        const std::vector<int> ex = as_expr(a[2]);
        im.channels = (int)ex.size();
        im.internal = im.tvalued = true;
        m_->images.push_back(im);
        const int id = (int)m_->images.size() - 1;
        GComputed c;
        c.image = id;
        c.expr = ex;
        bool bounds = false;
        for (int e : ex)
            P().visit(e, [&](int, const Node& n) {
                if (n.op == Op::Read && n.slot < 0) {
                    const GComputed* inner = computed_of(n.i);
                    for (int k = 0; k < 3; ++k) {
                        c.lo[k] = std::min(c.lo[k], n.off[k] + (inner ? inner->lo[k] : 0));
                        c.hi[k] = std::max(c.hi[k], n.off[k] + (inner ? inner->hi[k] : 0));
                    }
                } else if (n.op == Op::InBox) {
                    bounds = true;
                }
            });
        if (bounds)
            for (int k = 0; k < 3; ++k) c.lo[k] = c.hi[k] = 0;
        for (int ch = 0; ch < (int)ex.size(); ++ch) {
            std::set<int> unk;
            P().visit(ex[ch], [&](int nid, const Node& n) {
                if (n.op == Op::Read && m_->images[n.i].unknown) {
                    if (n.slot >= 0) err("ComputedArray over a graph access is not supported (NYI in the reference)");
                    unk.insert(nid);
                }
            });
            for (int u : unk) {
                GGrad g;
                g.ch = ch;
                g.u = u;
                g.expr = P().diff(ex[ch], u);
                int gnode = g.expr;
                if (!P().is_const(g.expr)) {
                    GImage gi;
                    gi.name = im.name + "_d_" + std::to_string(u);
                    gi.dims = m_->images[id].dims;
                    gi.internal = gi.tvalued = true;
                    m_->images.push_back(gi);
                    g.gimg = (int)m_->images.size() - 1;
                    const int z[3] = {0, 0, 0};
                    gnode = P().read(g.gimg, 0, z);
                }
                P().add_computed_grad(id, ch, u, gnode);
                c.grads.push_back(g);
            }
        }
        m_->computed.push_back(c);
        Value v;
        v.k = V::Image;
        v.id = id;
        return v;
    }
    const GComputed* computed_of(int image) const {
        for (auto& c : m_->computed)
            if (c.image == image) return &c;
        return nullptr;
    }
    Value image_access(int id, VList& a) {
        const GImage& im = m_->images[id];
        const int nd = (int)im.dims.size();
        if (!a.empty() && a[0].k == V::Slot) {   // X(G.v)
            int ch = -1;
            if (a.size() == 2) ch = (int)a[1].n;
            else if (a.size() != 1) err("graph access X(G.v[, channel])");
            std::vector<int> out;
            for (int c = 0; c < im.channels; ++c)
                if (ch < 0 || c == ch) out.push_back(P().read(id, c, nullptr, a[0].slot, a[0].id));
            return expr(out);
        }
        int off[3] = {0, 0, 0};
        int ch = -1;
        if ((int)a.size() == nd || (int)a.size() == nd + 1) {
            for (int k = 0; k < nd; ++k) {
                if (a[k].k != V::Num) err("image offsets must be numbers (SampledImage is not lowered)");
                off[k] = (int)a[k].n;
            }
            if ((int)a.size() == nd + 1) ch = (int)a[nd].n;
        } else {
            err("image " + im.name + " accessed with " + std::to_string(a.size()) + " arguments");
        }
        std::vector<int> out;
        for (int c = 0; c < im.channels; ++c)
            if (ch < 0 || c == ch) out.push_back(P().read(id, c, off));
        if (ch >= im.channels) err("channel out of range");
        return expr(out);
    }
    Value inbounds(VList& a, int expand) {
        int lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
        const int n = (int)a.size() - (expand ? 1 : 0);
        const int e = expand ? (int)a.back().n : 0;
        for (int k = 0; k < n && k < 3; ++k) {
            lo[k] = (int)a[k].n - e;
            hi[k] = (int)a[k].n + e;
        }
        return expr({P().inbox(lo, hi)});
    }

    void install();
    void def(const std::string& n, Builtin f) { globals_->vars[n] = std::make_shared<Value>(builtin(std::move(f))); }
    void unsupported(const std::string& what) {
        if (m_->unsupported.empty()) m_->unsupported = what;
    }
};

void Interp::install() {
    // element types
    auto type = [&](const std::string& n, int ch, const std::string& elem) {
        Value v;
        v.k = V::Type;
        v.id = ch;
        v.s = elem;
        globals_->vars[n] = std::make_shared<Value>(v);
    };
    type("float", 1, "float");
    type("double", 1, "float");
    type("int", 1, "int");
    type("uint8", 1, "uint8");
    type("opt_float", 1, "float");
    for (int c = 2; c <= 16; ++c) type("opt_float" + std::to_string(c), c, "float");

    def("print", [](VList&) { return VList{}; });
    def("tostring", [this](VList& a) { return VList{str(a.empty() ? "nil" : tostr(a[0]))}; });
    def("type", [](VList& a) {
        static const char* n[] = {"nil", "boolean", "number", "string", "table", "function", "function",
                                  "userdata", "userdata", "userdata", "userdata", "userdata", "userdata", "userdata"};
        return VList{str(a.empty() ? "nil" : n[(int)a[0].k])};
    });
    def("error", [this](VList& a) -> VList { err(a.empty() ? "error" : tostr(a[0])); });
    def("assert", [this](VList& a) -> VList {
        if (a.empty() || !truthy(a[0])) err(a.size() > 1 ? tostr(a[1]) : "assertion failed");
        return a;
    });
    auto ipairs_next = builtin([](VList& a) -> VList {
        const int i = (int)a[1].n + 1;
        if (a[0].k != V::Table || i > (int)a[0].t->a.size()) return {Value{}};
        return {num(i), a[0].t->a[i - 1]};
    });
    def("ipairs", [ipairs_next](VList& a) { return VList{ipairs_next, a.empty() ? Value{} : a[0], num(0)}; });
    def("pairs", [](VList& a) {
        // snapshot the table's entries (DSL objects iterate as empty)
        auto keys = std::make_shared<VList>(), vals = std::make_shared<VList>();
        if (!a.empty() && a[0].k == V::Table) {
            for (size_t i = 0; i < a[0].t->a.size(); ++i) { keys->push_back(num((double)i + 1)); vals->push_back(a[0].t->a[i]); }
            for (auto& kv : a[0].t->h) { keys->push_back(str(kv.first)); vals->push_back(kv.second); }
        }
        auto pos = std::make_shared<size_t>(0);
        Value it = builtin([keys, vals, pos](VList&) -> VList {
            if (*pos >= keys->size()) return {Value{}};
            const size_t i = (*pos)++;
            return {(*keys)[i], (*vals)[i]};
        });
        return VList{it, Value{}, Value{}};
    });
    auto unpack = [](VList& a) { return a.empty() || a[0].k != V::Table ? VList{} : a[0].t->a; };
    def("unpack", unpack);
    {
        Value tb = table();
        tb.t->h["unpack"] = builtin(unpack);
        tb.t->h["insert"] = builtin([](VList& a) {
            if (!a.empty() && a[0].k == V::Table && a.size() > 1) a[0].t->a.push_back(a.back());
            return VList{};
        });
        globals_->vars["table"] = std::make_shared<Value>(tb);
    }
    {
        Value mt = table();
        auto m1 = [&](const char* n, double (*f)(double)) {
            mt.t->h[n] = builtin([f](VList& a) { return VList{num(f(a.at(0).n))}; });
        };
        m1("sqrt", std::sqrt); m1("sin", std::sin); m1("cos", std::cos); m1("exp", std::exp);
        m1("log", std::log); m1("abs", std::fabs); m1("floor", std::floor); m1("ceil", std::ceil);
        mt.t->h["pi"] = num(M_PI);
        mt.t->h["huge"] = num(HUGE_VAL);
        mt.t->h["max"] = builtin([](VList& a) { double r = a.at(0).n; for (auto& v : a) r = std::max(r, v.n); return VList{num(r)}; });
        mt.t->h["min"] = builtin([](VList& a) { double r = a.at(0).n; for (auto& v : a) r = std::min(r, v.n); return VList{num(r)}; });
        globals_->vars["math"] = std::make_shared<Value>(mt);
    }

    // ---- declarations (ProblemSpecAD, o.t:251-475; lib.t)
    def("Dim", [this](VList& a) {
        if (a.size() < 2) err("Dim(name, index)");
        m_->dims.push_back(GDim{a[0].s, (int)a[1].n});
        Value v;
        v.k = V::Dim;
        v.id = (int)m_->dims.size() - 1;
        return VList{v};
    });
    def("Param", [this](VList& a) {
        if (a.size() < 3) err("Param(name, type, index)");
        GParam p{a[0].s, a[1].s.empty() ? "float" : a[1].s, (int)a[2].n};
        note_index(p.index);
        m_->params.push_back(p);
        return VList{expr({P().param((int)m_->params.size() - 1)})};
    });
    def("Unknown", [this](VList& a) { return VList{decl_image(a, true)}; });
    def("Array", [this](VList& a) { return VList{decl_image(a, false)}; });
    def("Image", [this](VList& a) { return VList{decl_image(a, false)}; });
    def("Graph", [this](VList& a) {
        if (a.size() < 5 || (a.size() - 2) % 3 != 0) err("Graph(name, {dims}, slot, {dims}, index, ...)");
        GGraph g;
        g.name = a[0].s;
        if (a[1].k == V::Table) for (auto& d : a[1].t->a) g.dims.push_back(dim_of(d));
        for (size_t i = 2; i + 2 < a.size(); i += 3) {
            g.slot_names.push_back(a[i].s);
            g.slot_index.push_back((int)a[i + 2].n);
            note_index((int)a[i + 2].n);
        }
        m_->graphs.push_back(g);
        Value v;
        v.k = V::Graph;
        v.id = (int)m_->graphs.size() - 1;
        return VList{v};
    });
    def("UsePreconditioner", [this](VList& a) {
        m_->use_preconditioner = !a.empty() && truthy(a[0]);
        return VList{};
    });
    def("Exclude", [this](VList& a) {
        if (a.empty()) err("Exclude(expr)");
        m_->exclude = comp(a[0], 0);
        return VList{};
    });
    def("Energy", [this](VList& a) {
        for (auto& v : a)
            for (int c : as_expr(v)) energy_terms_.push_back(c);
        return VList{};
    });
    def("Result", [](VList&) { return VList{}; });
    def("ComputedArray", [this](VList& a) { return VList{computed_array(a)}; });
    def("ComputedImage", [this](VList& a) { return VList{computed_array(a)}; });
    def("L_p", [this](VList& a) {   // lib.t:113-122
        if (a.size() < 4) err("L_p(val, val_const, p, dims)");
        const std::vector<int> vc = as_expr(a[1]);
        int dot = P().cnst(0.0);
        for (int c : vc) dot = P().bin(Op::Add, dot, P().bin(Op::Mul, c, c));
        const int dist = P().un(Op::Sqrt, dot);
        const int C = P().bin(Op::Pow, P().bin(Op::Add, dist, P().cnst(0.0000001)),
                              P().bin(Op::Sub, comp(a[2], 0), P().cnst(2.0)));
        VList ca{str("L_p" + std::to_string(++lp_counter_)), a[3], expr({P().un(Op::Sqrt, C)})};
        Value im = computed_array(ca);
        VList z;
        for (size_t k = 0; k < m_->images[im.id].dims.size(); ++k) z.push_back(num(0));
        return VList{zip(Op::Mul, image_access(im.id, z), a[0])};
    });
    def("Slice", [this](VList& a) {   // lib.t:70-82: channels [s, e) of an image access
        if (a.size() < 3 || a[0].k != V::Image) err("Slice(image, s, e)");
        const int id = a[0].id, s0 = (int)a[1].n, e0 = (int)a[2].n;
        return VList{builtin([this, id, s0, e0](VList& args) {
            const Value v = image_access(id, args);
            std::vector<int> out;
            for (int c = s0; c < e0; ++c) out.push_back(comp(v, c));
            return VList{expr(out)};
        })};
    });
    // ad.sampledimage (o.t:3243-3282): I(x, y[, c]) bilinear at data-dependent coordinates,
    // differentiated through the sampled derivative images
    def("SampledImage", [this](VList& a) {
        if (a.empty() || a[0].k != V::Image) err("SampledImage(image[, image_dx, image_dy])");
        const int im = a[0].id;
        int dx = -1, dy = -1;
        if (a.size() >= 3) {
            if (a[1].k != V::Image || a[2].k != V::Image) err("SampledImage derivatives must be images");
            dx = a[1].id;
            dy = a[2].id;
        }
        if (m_->images[im].dims.size() != 2) err("sampled images must be 2D");
        return VList{builtin([this, im, dx, dy](VList& args) {
            if (args.size() < 2) err("sampled image expects (x, y[, channel])");
            const int x = comp(args[0], 0), y = comp(args[1], 0);
            const int nch = m_->images[im].channels;
            std::vector<int> out;
            if (args.size() > 2) {
                const int c = (int)args[2].n;
                if (c < 0 || c >= nch) err("index out of bounds");
                out.push_back(P().sample(im, c, x, y, dx, dy));
            } else {
                for (int c = 0; c < nch; ++c) out.push_back(P().sample(im, c, x, y, dx, dy));
            }
            return VList{expr(out)};
        })};
    });
    // ---- expression library (lib.t, ad.t)
    def("Select", [this](VList& a) {
        if (a.size() != 3) err("Select(cond, a, b)");
        std::vector<int> c = as_expr(a[0]), x = as_expr(a[1]), y = as_expr(a[2]);
        const size_t n = std::max({c.size(), x.size(), y.size()});
        std::vector<int> r(n);
        for (size_t i = 0; i < n; ++i)
            r[i] = P().select(c[c.size() == 1 ? 0 : i], x[x.size() == 1 ? 0 : i], y[y.size() == 1 ? 0 : i]);
        return VList{expr(r)};
    });
    auto cmp = [this](const char* n, Op op) { def(n, [this, op](VList& a) { return VList{zip(op, a.at(0), a.at(1))}; }); };
    cmp("eq", Op::Eq); cmp("notEq", Op::Ne); cmp("greater", Op::Gt); cmp("greatereq", Op::Ge);
    cmp("less", Op::Lt); cmp("lesseq", Op::Le); cmp("and_", Op::And); cmp("or_", Op::Or);
    def("Not", [this](VList& a) { return VList{map1(Op::Not, a.at(0))}; });
    def("not_", [this](VList& a) { return VList{map1(Op::Not, a.at(0))}; });
    def("And", [this](VList& a) {
        Value r = num(1);
        for (auto& v : a) r = zip(Op::And, r, v);
        return VList{r};
    });
    def("Or", [this](VList& a) {
        Value r = num(0);
        for (auto& v : a) r = zip(Op::Or, r, v);
        return VList{r};
    });
    def("All", [this](VList& a) {   // lib.t L.All: product of the components
        std::vector<int> x = as_expr(a.at(0));
        int r = P().cnst(1.0);
        for (int c : x) r = P().bin(Op::Mul, r, c);
        return VList{expr({r})};
    });
    def("InBounds", [this](VList& a) { return VList{inbounds(a, 0)}; });
    def("InBoundsExpanded", [this](VList& a) { return VList{inbounds(a, 1)}; });
    def("Index", [this](VList& a) { return VList{expr({P().coord((int)a.at(0).n)})}; });
    def("Stencil", [this](VList& a) {
        if (a.empty() || a[0].k != V::Table) err("Stencil { {dx, dy}, ... }");
        auto lst = a[0].t;
        auto i = std::make_shared<size_t>(0);
        return VList{builtin([lst, i](VList&) -> VList {
            if (*i >= lst->a.size()) return {Value{}};
            const Value& e = lst->a[(*i)++];
            return e.k == V::Table ? e.t->a : VList{e};
        })};
    });
    def("Vector", [this](VList& a) {
        std::vector<int> r;
        for (auto& v : a) for (int c : as_expr(v)) r.push_back(c);
        return VList{expr(r)};
    });
    auto f1 = [this](const char* n, Op op) { def(n, [this, op](VList& a) { return VList{map1(op, a.at(0))}; }); };
    f1("Sqrt", Op::Sqrt); f1("sqrt", Op::Sqrt); f1("sin", Op::Sin); f1("cos", Op::Cos); f1("exp", Op::Exp);
    f1("log", Op::Log); f1("abs", Op::Abs);
    def("pow", [this](VList& a) { return VList{zip(Op::Pow, a.at(0), a.at(1))}; });
    def("Dot3", [this](VList& a) {
        int s = P().bin(Op::Add, P().bin(Op::Add, P().bin(Op::Mul, comp(a.at(0), 0), comp(a.at(1), 0)),
                                          P().bin(Op::Mul, comp(a[0], 1), comp(a[1], 1))),
                        P().bin(Op::Mul, comp(a[0], 2), comp(a[1], 2)));
        return VList{expr({s})};
    });
    def("normalize", [this](VList& a) {
        Value v = a.at(0);
        VList d{v, v};
        Value n = (*globals_->vars["Dot3"]->bf)(d)[0];
        return VList{zip(Op::Div, v, map1(Op::Sqrt, n))};
    });
    def("length", [this](VList& a) {
        Value diff = zip(Op::Sub, a.at(0), a.at(1));
        VList d{diff, diff};
        return VList{map1(Op::Sqrt, (*globals_->vars["Dot3"]->bf)(d)[0])};
    });
    def("Matrix3x3Mul", [this](VList& a) {
        const Value& M = a.at(0);
        const Value& v = a.at(1);
        std::vector<int> r(3);
        for (int i = 0; i < 3; ++i)
            r[i] = P().bin(Op::Add,
                           P().bin(Op::Add, P().bin(Op::Mul, comp(M, 3 * i), comp(v, 0)),
                                   P().bin(Op::Mul, comp(M, 3 * i + 1), comp(v, 1))),
                           P().bin(Op::Mul, comp(M, 3 * i + 2), comp(v, 2)));
        return VList{expr(r)};
    });
    def("Rotate2D", [this](VList& a) {   // lib.t:99-103
        const int ang = comp(a.at(0), 0);
        const int c = P().un(Op::Cos, ang), s = P().un(Op::Sin, ang);
        const int v0 = comp(a.at(1), 0), v1 = comp(a[1], 1);
        return VList{expr({P().bin(Op::Add, P().bin(Op::Mul, c, v0), P().bin(Op::Mul, P().un(Op::Neg, s), v1)),
                           P().bin(Op::Add, P().bin(Op::Mul, s, v0), P().bin(Op::Mul, c, v1))})};
    });
    def("Rotate3D", [this](VList& a) {   // lib.t:84-98
        const int al = comp(a.at(0), 0), be = comp(a[0], 1), ga = comp(a[0], 2);
        const int ca = P().un(Op::Cos, al), cb = P().un(Op::Cos, be), cg = P().un(Op::Cos, ga);
        const int sa = P().un(Op::Sin, al), sb = P().un(Op::Sin, be), sg = P().un(Op::Sin, ga);
        auto mul = [&](int x, int y) { return P().bin(Op::Mul, x, y); };
        auto add = [&](int x, int y) { return P().bin(Op::Add, x, y); };
        auto neg = [&](int x) { return P().un(Op::Neg, x); };
        std::vector<int> M = {mul(cg, cb),
                              add(mul(neg(sg), ca), mul(mul(cg, sb), sa)),
                              add(mul(sg, sa), mul(mul(cg, sb), ca)),
                              mul(sg, cb),
                              add(mul(cg, ca), mul(mul(sg, sb), sa)),
                              add(mul(neg(cg), sa), mul(mul(sg, sb), ca)),
                              neg(sb),
                              mul(cb, sa),
                              mul(cb, ca)};
        VList mm{expr(M), a.at(1)};
        return (*globals_->vars["Matrix3x3Mul"]->bf)(mm);
    });
    // `opt` namespace (opt.Dim etc.) and ad aliases
    {
        Value opt = table();
        for (const char* n : {"Dim", "Param", "Unknown", "Array", "Image", "Graph", "InBounds"}) opt.t->h[n] = *globals_->vars[n];
        globals_->vars["opt"] = std::make_shared<Value>(opt);
        Value ad = table();
        for (const char* n : {"sqrt", "sin", "cos", "exp", "log", "abs", "pow", "select"}) {
            auto it = globals_->vars.find(std::string(n) == "select" ? "Select" : n);
            if (it != globals_->vars.end()) ad.t->h[n] = *it->second;
        }
        globals_->vars["ad"] = std::make_shared<Value>(ad);
    }
}

// Per-step sample cache (round 6): a SampledImage read whose coordinates use the unknowns
// and coordinates of ONE pixel (offset o) — optical_flow's I_hat(x + u(0,0), y + v(0,0)) — is
// fixed while the PCG loop runs (the unknowns change only at the update). It becomes a
// T-valued ComputedArray of its own (value + one gradient image per unknown access: the
// sampled derivative images times the coordinates' derivatives, the same expressions
// diff() forms for the Sample node, ad.sampledimage / o.t:3266-3280), evaluated once per
// Step by the precompute kernels, and the residual reads it at offset o. The applies then
// read two cached partials per pixel instead of re-sampling eight taps in every PCG
// iteration (the reference re-samples, as the generic path did before). The values are
// the same expressions on the same inputs. OPT_AMD_GEN_SAMPLE_CACHE=0 keeps the samples
// in the residuals.
int Interp::cache_samples(int e) {
    const char* sv = getenv("OPT_AMD_GEN_SAMPLE_CACHE");
    if (sv && atoi(sv) == 0) return e;
    std::map<int, int> repl;
    P().visit(e, [&](int id, const Node& n) {
        // (a sample without derivative images stays: the residual check below names it when
        // its coordinates use the unknowns)
        if (n.op != Op::Sample || n.off2[0] < 0 || n.off2[1] < 0 || repl.count(id)) return;
        int off[3] = {0, 0, 0};
        bool set[3] = {false, false, false}, ok = true, reads = false;
        auto want = [&](int d, int v) {
            if (set[d] && off[d] != v) ok = false;
            set[d] = true;
            off[d] = v;
        };
        for (int c : {n.a, n.b})
            P().visit(c, [&](int, const Node& q) {
                if (q.op == Op::Read) {
                    if (q.slot >= 0 || computed_of(q.i)) { ok = false; return; }
                    reads = true;
                    for (int d = 0; d < 3; ++d) want(d, q.off[d]);
                } else if (q.op == Op::Coord) {
                    want(q.i, q.off[q.i]);
                } else if (q.op == Op::Sample || q.op == Op::InBox) {
                    ok = false;
                }
            });
        if (!ok || !reads || m_->images.size() + 3 > 16) return;   // GenArgs::img holds 16 images
        const int neg[3] = {-off[0], -off[1], -off[2]};
        const int s0 = P().shift(id, neg);
        int img = -1;
        for (auto& c : sample_cache_)
            if (c.first == s0) img = c.second;
        if (img < 0) {
            GImage im;
            im.name = "sample_cache_" + std::to_string(sample_cache_.size());
            const std::vector<int> unk = m_->unknown_images();
            if (unk.empty()) return;
            im.dims = m_->images[unk[0]].dims;
            im.channels = 1;
            im.internal = im.tvalued = true;
            m_->images.push_back(im);
            img = (int)m_->images.size() - 1;
            GComputed c;
            c.image = img;
            c.expr = {s0};
            std::set<int> unkr;
            P().visit(s0, [&](int nid, const Node& q) {
                if (q.op == Op::Read && q.slot < 0 && m_->images[q.i].unknown) unkr.insert(nid);
            });
            for (int u : unkr) {
                GGrad g;
                g.ch = 0;
                g.u = u;
                g.expr = P().diff(s0, u);
                int gnode = g.expr;
                if (!P().is_const(g.expr)) {
                    GImage gi;
                    gi.name = im.name + "_d_" + std::to_string(u);
                    gi.dims = im.dims;
                    gi.internal = gi.tvalued = true;
                    m_->images.push_back(gi);
                    g.gimg = (int)m_->images.size() - 1;
                    const int z[3] = {0, 0, 0};
                    gnode = P().read(g.gimg, 0, z);
                }
                P().add_computed_grad(img, 0, u, gnode);
                c.grads.push_back(g);
            }
            m_->computed.push_back(c);
            sample_cache_.push_back({s0, img});
        }
        repl[id] = P().read(img, 0, off);
    });
    return repl.empty() ? e : P().substitute(e, repl);
}

// Classify and finish the residual templates (classifyexpression + bbox, o.t:2669-2715).
void Interp::finish() {
    // an Array declared on an Unknown's parameter slot is a view of that unknown
    // (intrinsic_image_decomposition's r_const): stored in the solver precision
    for (auto& im : m_->images)
        if (!im.unknown && !im.internal)
            for (auto& u : m_->images)
                if (u.unknown && u.index == im.index) im.tvalued = true;
    for (int& e : energy_terms_) e = cache_samples(e);
    for (int e : energy_terms_) {
        GResidual r;
        bool any = false;
        int graph = -1;
        bool bounds = false;
        int lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
        std::set<int> unk;
        P().visit(e, [&](int id, const Node& n) {
            if (n.op == Op::Read) {
                any = true;
                if (n.slot >= 0) {
                    if (graph >= 0 && graph != n.g) throw LuaError("residual reads from two graphs");
                    graph = n.g;
                } else if (const GComputed* c = computed_of(n.i)) {
                    // a ComputedArray read: its bbox moved by the access offset, and the
                    // unknown accesses behind its gradient images (o.t:2683-2687, 1686-1700)
                    for (int k = 0; k < 3; ++k) {
                        lo[k] = std::min(lo[k], n.off[k] + c->lo[k]);
                        hi[k] = std::max(hi[k], n.off[k] + c->hi[k]);
                    }
                    for (const GGrad& g : c->grads)
                        if (g.ch == n.ch) unk.insert(P().shift(g.u, n.off));
                } else {
                    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], n.off[k]); hi[k] = std::max(hi[k], n.off[k]); }
                }
                if (m_->images[n.i].unknown) unk.insert(id);
            } else if (n.op == Op::InBox) {
                bounds = true;
            } else if (n.op == Op::Sample && n.off2[0] < 0) {
                bool dep = false;
                for (int c : {n.a, n.b})
                    P().visit(c, [&](int, const Node& q) { dep |= q.op == Op::Read && m_->images[q.i].unknown; });
                if (dep) throw LuaError("image derivatives are not defined for sampled image " + m_->images[n.i].name);
            }
        });
        if (!any) throw LuaError("residual must actually use some image");
        r.graph = graph;
        if (graph < 0) {
            // by default zero any residual that reads out of bounds (usesbounds: only the centre)
            if (bounds) for (int k = 0; k < 3; ++k) lo[k] = hi[k] = 0;
            r.expr = P().select(P().inbox(lo, hi), e, P().cnst(0.0));
        } else {
            r.expr = e;
        }
        r.unknowns.assign(unk.begin(), unk.end());
        m_->residuals.push_back(r);
    }
}

}  // namespace

int GModel::unknown_dims() const {
    for (auto& im : images)
        if (im.unknown) return (int)im.dims.size();
    return 0;
}
std::vector<int> GModel::unknown_images() const {
    std::vector<int> u;
    for (size_t i = 0; i < images.size(); ++i)
        if (images[i].unknown) u.push_back((int)i);
    std::sort(u.begin(), u.end(), [&](int a, int b) { return images[a].index < images[b].index; });
    return u;
}

bool build_model(const std::string& text, GModel* m, std::string* err) {
    try {
        Parser p(lex(text));
        Block b = p.chunk();
        Interp in(m);
        in.run(b);
        in.finish();
    } catch (LuaError& e) {
        *err = e.what();
        return false;
    } catch (ReturnSignal&) {
    } catch (BreakSignal&) {
        *err = "break outside a loop";
        return false;
    } catch (std::exception& e) {
        *err = e.what();
        return false;
    }
    if (m->images.empty()) { *err = "no Unknown declared"; return false; }
    return true;
}

}  // namespace gen
}  // namespace optamd
