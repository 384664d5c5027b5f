// comm.cpp — RCCL and in-process transports for row-slab decomposition (comm.h).
#include "comm.h"
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <cstdlib>
#include <cstring>

namespace optamd {

// Row span helpers. Rows exchanged with the neighbour above: my first `h` owned rows
// go up (they are its bottom halo), and my top halo comes from its last owned rows.
namespace {
struct Span { int y0, n; };   // global rows [y0, y0+n)
inline Span send_up(const Domain& d, int h) { return {d.y_lo, h}; }
inline Span recv_up(const Domain& d, int h) { return {d.y_lo - h, h}; }
inline Span send_dn(const Domain& d, int h) { return {d.y_hi - h, h}; }
inline Span recv_dn(const Domain& d, int h) { return {d.y_hi, h}; }
inline char* row_ptr(const HaloPlane& p, const Domain& d, int y) {
    return (char*)p.base + (size_t)(y - d.y_mem0) * p.row_bytes;
}
}  // namespace

// ======================================================================= RCCL
// librccl is resolved at run time so that single-GPU users need no RCCL and a host
// process that already loaded one (e.g. PyTorch's) shares it.
namespace {
struct RcclApi {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errStr = nullptr;
    // optional (RCCL >= 2.18): a second communicator for the halo traffic
    ncclResult_t (*commSplit)(ncclComm_t, int, int, ncclComm_t*, void*) = nullptr;
    bool load(std::string* err) {
        if (h) return true;
        // OPT_AMD_RCCL_LIB: an explicit library (the tests' multi-process stand-in,
        // tests/rccl_stub), loaded privately so a process's own RCCL (PyTorch's) is untouched
        if (const char* lib = getenv("OPT_AMD_RCCL_LIB"); lib && *lib) {
            h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
            if (!h) { *err = std::string("cannot load OPT_AMD_RCCL_LIB=") + lib + ": " + dlerror(); return false; }
        }
        if (!h) for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
            if (!h) h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
            if (h) break;
        }
        if (!h) { *err = "cannot load librccl"; return false; }
#define SYM(f, name) f = (decltype(f))dlsym(h, name); if (!f) { *err = std::string("missing ") + name; return false; }
        SYM(getUniqueId, "ncclGetUniqueId") SYM(commInitRank, "ncclCommInitRank")
        SYM(commDestroy, "ncclCommDestroy") SYM(allReduce, "ncclAllReduce") SYM(send, "ncclSend")
        SYM(recv, "ncclRecv") SYM(groupStart, "ncclGroupStart") SYM(groupEnd, "ncclGroupEnd")
        SYM(errStr, "ncclGetErrorString")
#undef SYM
        commSplit = (decltype(commSplit))dlsym(h, "ncclCommSplit");
        return true;
    }
};
RcclApi g_rccl;

#define RCCL_CHECK(call)                                                                     \
    do {                                                                                     \
        ncclResult_t r_ = (call);                                                            \
        if (r_ != ncclSuccess) {                                                             \
            fprintf(stderr, "[opt_amd] RCCL error %s in %s\n", g_rccl.errStr(r_), #call);    \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

// Two communicators when RCCL can split one: c_ carries the scalar all-reduces (plan
// stream), ch_ the halo send/recv (the plan's halo stream when it overlaps halos with the
// interior apply). Each is then used from one stream, in the same order on every rank;
// without a split both share c_ and the plans exchange halos on the plan stream.
class RcclComm final : public Comm {
public:
    RcclComm(ncclComm_t c, ncclComm_t ch, int rank, int n) : c_(c), ch_(ch), rank_(rank), n_(n) {}
    ~RcclComm() override {
        if (ch_ && ch_ != c_) g_rccl.commDestroy(ch_);
        if (c_) g_rccl.commDestroy(c_);
    }
    int rank() const override { return rank_; }
    int size() const override { return n_; }
    std::string kind() const override { return "rccl"; }
    bool concurrent_halo() const override { return ch_ != c_; }
    void allreduce_sum(double* dev, int n, hipStream_t s) override {
        RCCL_CHECK(g_rccl.allReduce(dev, dev, (size_t)n, ncclFloat64, ncclSum, c_, s));
    }
    void halo_exchange(const std::vector<HaloPlane>& planes, const Domain& d, int h,
                       hipStream_t s) override {
        if (n_ == 1 || h == 0) return;
        RCCL_CHECK(g_rccl.groupStart());
        for (const auto& p : planes) {
            const size_t bytes = (size_t)h * p.row_bytes;
            if (rank_ > 0) {
                RCCL_CHECK(g_rccl.send(row_ptr(p, d, send_up(d, h).y0), bytes, ncclChar, rank_ - 1, ch_, s));
                RCCL_CHECK(g_rccl.recv(row_ptr(p, d, recv_up(d, h).y0), bytes, ncclChar, rank_ - 1, ch_, s));
            }
            if (rank_ < n_ - 1) {
                RCCL_CHECK(g_rccl.send(row_ptr(p, d, send_dn(d, h).y0), bytes, ncclChar, rank_ + 1, ch_, s));
                RCCL_CHECK(g_rccl.recv(row_ptr(p, d, recv_dn(d, h).y0), bytes, ncclChar, rank_ + 1, ch_, s));
            }
        }
        RCCL_CHECK(g_rccl.groupEnd());
    }

private:
    ncclComm_t c_, ch_;
    int rank_, n_;
};
}  // namespace

bool rccl_unique_id(void* out, std::string* err) {
    if (!g_rccl.load(err)) return false;
    ncclUniqueId id;
    if (g_rccl.getUniqueId(&id) != ncclSuccess) { *err = "ncclGetUniqueId failed"; return false; }
    memcpy(out, &id, sizeof(id));
    return true;
}

Comm* make_rccl_comm(const void* id128, int rank, int nranks, std::string* err) {
    if (!g_rccl.load(err)) return nullptr;
    ncclUniqueId id;
    memcpy(&id, id128, sizeof(id));
    ncclComm_t c;
    ncclResult_t r = g_rccl.commInitRank(&c, nranks, id, rank);
    if (r != ncclSuccess) { *err = std::string("ncclCommInitRank: ") + g_rccl.errStr(r); return nullptr; }
    ncclComm_t ch = c;   // collective over all ranks: every rank takes the same branch
    if (g_rccl.commSplit && nranks > 1 && g_rccl.commSplit(c, 0, rank, &ch, nullptr) != ncclSuccess) ch = c;
    return new RcclComm(c, ch, rank, nranks);
}

// ================================================================ local group
// Ranks are host threads of one process. Every collective is a rendezvous: each rank
// makes its data ready (stream sync), publishes it, waits at a barrier, then the
// reduction is summed in rank order (deterministic) or each rank copies its boundary
// rows straight into its neighbours' halo rows (device-to-device, peer if needed).
class LocalGroup {
public:
    explicit LocalGroup(int n) : n_(n), vals_(n), planes_(n), doms_(n) {
        for (int r = 0; r < n; ++r) ranks_.emplace_back(new Rank(this, r));
    }
    Comm* rank(int r) { return ranks_[r].get(); }

    void barrier() {
        std::unique_lock<std::mutex> lk(m_);
        const unsigned long gen = gen_;
        if (++arrived_ == n_) {
            arrived_ = 0;
            ++gen_;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen_ != gen; });
        }
    }

    class Rank final : public Comm {
    public:
        Rank(LocalGroup* g, int r) : g_(g), r_(r) {}
        int rank() const override { return r_; }
        int size() const override { return g_->n_; }
        std::string kind() const override { return "local"; }
        void allreduce_sum(double* dev, int n, hipStream_t s) override {
            if (g_->n_ == 1) return;
            std::vector<double> mine(n);
            OPT_HIP_CHECK(hipMemcpyAsync(mine.data(), dev, sizeof(double) * n, hipMemcpyDeviceToHost, s));
            OPT_HIP_CHECK(hipStreamSynchronize(s));
            g_->vals_[r_] = mine;
            g_->barrier();
            std::vector<double> sum(n, 0.0);
            for (int q = 0; q < g_->n_; ++q)
                for (int k = 0; k < n; ++k) sum[k] += g_->vals_[q][k];
            g_->barrier();
            OPT_HIP_CHECK(hipMemcpyAsync(dev, sum.data(), sizeof(double) * n, hipMemcpyHostToDevice, s));
            OPT_HIP_CHECK(hipStreamSynchronize(s));
        }
        void halo_exchange(const std::vector<HaloPlane>& planes, const Domain& d, int h,
                           hipStream_t s) override {
            if (g_->n_ == 1 || h == 0) return;
            OPT_HIP_CHECK(hipStreamSynchronize(s));
            g_->planes_[r_] = planes;
            g_->doms_[r_] = d;
            g_->barrier();
            for (int nb : {r_ - 1, r_ + 1}) {
                if (nb < 0 || nb >= g_->n_) continue;
                const Domain& nd = g_->doms_[nb];
                const Span sp = (nb < r_) ? send_up(d, h) : send_dn(d, h);
                for (size_t k = 0; k < planes.size(); ++k) {
                    const HaloPlane& src = planes[k];
                    const HaloPlane& dst = g_->planes_[nb][k];
                    OPT_HIP_CHECK(hipMemcpyAsync(row_ptr(dst, nd, sp.y0), row_ptr(src, d, sp.y0),
                                                 (size_t)sp.n * src.row_bytes, hipMemcpyDefault, s));
                }
            }
            OPT_HIP_CHECK(hipStreamSynchronize(s));
            g_->barrier();
        }

    private:
        LocalGroup* g_;
        int r_;
    };

private:
    int n_;
    std::vector<std::unique_ptr<Rank>> ranks_;
    std::vector<std::vector<double>> vals_;
    std::vector<std::vector<HaloPlane>> planes_;
    std::vector<Domain> doms_;
    std::mutex m_;
    std::condition_variable cv_;
    int arrived_ = 0;
    unsigned long gen_ = 0;
};

LocalGroup* make_local_group(int nranks) { return new LocalGroup(nranks); }
Comm* local_group_rank(LocalGroup* g, int r) { return g->rank(r); }
void destroy_local_group(LocalGroup* g) { delete g; }

}  // namespace optamd
