// rccl_stub.cpp — TEST INFRASTRUCTURE: a stand-in for librccl with the ten entry points
// opt_amd's RcclComm resolves (opt_amd/csrc/comm.cpp, RcclApi::load), so that the RCCL
// transport code — grouped ncclSend/ncclRecv halo exchanges, the split halo communicator,
// the ncclAllReduce of the PCG scalars — executes with 2..8 rank PROCESSES on a box whose
// one GPU real RCCL refuses to give to two ranks of one communicator
// (tests/test_rccl_multirank_gpu.py). Loaded through OPT_AMD_RCCL_LIB=<this .so>.
//
// Transport: one POSIX shared-memory segment per communicator (named from the unique id;
// ncclCommSplit derives a second one) holding a process-shared barrier, per-rank scalar
// slots and per-(sender, receiver) send mailboxes. Every call is stream-ordered by
// synchronising the caller's stream first and then runs on the host:
//   * ncclAllReduce (double, sum): each rank publishes its values, and every rank sums the
//     slots in rank order 0..n-1 from 0.0 — the order OptAMD_LocalGroup sums in, so a
//     solve over this transport is bitwise the LocalGroup solve;
//   * ncclSend / ncclRecv inside ncclGroupStart/End: a send publishes the IPC handle
//     (hipIpcGetMemHandle of the allocation's base) and offset of its buffer; the matching
//     receive (in posting order per peer) opens the handle and copies device to device;
//     the sender returns once every receive of its buffers has completed (its buffer may
//     then be overwritten).
// Not a performance path, and not part of the product: only the tests load it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

namespace {
constexpr int kMaxRanks = 16;
constexpr int kMaxOps = 64;       // sends in flight per (sender, receiver) pair
constexpr int kMaxScalars = 64;   // doubles per all-reduce

struct Mail {
    hipIpcMemHandle_t h;
    uint64_t off, bytes;
};
struct Shm {
    std::atomic<int> arrive;
    std::atomic<int> gen;
    double red[kMaxRanks][kMaxScalars];
    Mail box[kMaxRanks][kMaxRanks][kMaxOps];
    std::atomic<uint64_t> posted[kMaxRanks][kMaxRanks];     // sends posted src -> dst
    std::atomic<uint64_t> consumed[kMaxRanks][kMaxRanks];   // of those, received by dst
};
}  // namespace

struct ncclComm {
    std::string name;
    int rank = 0, n = 1, splits = 0;
    Shm* shm = nullptr;
    uint64_t sent[kMaxRanks] = {}, recvd[kMaxRanks] = {};
    std::map<std::string, char*> opened;   // IPC handle bytes -> mapped base
};

namespace {
struct Op {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
    ncclComm* comm;
    hipStream_t stream;
};
thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;

bool hip_ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    fprintf(stderr, "[rccl_stub] %s: %s\n", what, hipGetErrorString(e));
    return false;
}

// spin with a deadline: a peer that never arrives is an error, not a hang
template <typename F>
bool wait_for(F ready, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    while (!ready()) {
        sched_yield();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
            fprintf(stderr, "[rccl_stub] timeout waiting for %s\n", what);
            return false;
        }
    }
    return true;
}

bool barrier(ncclComm* c) {
    Shm* s = c->shm;
    const int g = s->gen.load(std::memory_order_acquire);
    if (s->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == c->n) {
        s->arrive.store(0, std::memory_order_relaxed);
        s->gen.fetch_add(1, std::memory_order_acq_rel);
        return true;
    }
    return wait_for([&] { return s->gen.load(std::memory_order_acquire) != g; }, "barrier");
}

ncclResult_t attach(ncclComm* c) {
    const int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) return ncclSystemError;
    if (ftruncate(fd, sizeof(Shm)) != 0) { close(fd); return ncclSystemError; }
    void* p = mmap(nullptr, sizeof(Shm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return ncclSystemError;
    c->shm = static_cast<Shm*>(p);
    return barrier(c) ? ncclSuccess : ncclSystemError;   // every rank has the segment
}

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

ncclResult_t run_group(std::vector<Op>& ops) {
    for (auto& o : ops)
        if (!hip_ok(hipStreamSynchronize(o.stream), "hipStreamSynchronize")) return ncclUnhandledCudaError;
    // post every send
    for (auto& o : ops) {
        if (!o.send) continue;
        ncclComm* c = o.comm;
        void* base = nullptr;
        size_t size = 0;
        if (!hip_ok(hipMemGetAddressRange(&base, &size, o.buf), "hipMemGetAddressRange")) return ncclInvalidArgument;
        const uint64_t k = c->sent[o.peer];
        if (k - c->shm->consumed[c->rank][o.peer].load(std::memory_order_acquire) >= (uint64_t)kMaxOps)
            return ncclInternalError;
        Mail& m = c->shm->box[c->rank][o.peer][k % kMaxOps];
        if (!hip_ok(hipIpcGetMemHandle(&m.h, base), "hipIpcGetMemHandle")) return ncclUnhandledCudaError;
        m.off = (uint64_t)((char*)o.buf - (char*)base);
        m.bytes = o.bytes;
        c->sent[o.peer] = k + 1;
        c->shm->posted[c->rank][o.peer].store(k + 1, std::memory_order_release);
    }
    // receive in posting order per peer
    for (auto& o : ops) {
        if (o.send) continue;
        ncclComm* c = o.comm;
        const uint64_t k = c->recvd[o.peer];
        auto& posted = c->shm->posted[o.peer][c->rank];
        if (!wait_for([&] { return posted.load(std::memory_order_acquire) > k; }, "a send")) return ncclSystemError;
        const Mail& m = c->shm->box[o.peer][c->rank][k % kMaxOps];
        if (m.bytes != o.bytes) {
            fprintf(stderr, "[rccl_stub] size mismatch: send %llu, recv %zu bytes\n", (unsigned long long)m.bytes,
                    o.bytes);
            return ncclInvalidArgument;
        }
        const std::string key(reinterpret_cast<const char*>(&m.h), sizeof(m.h));
        char*& mapped = c->opened[key];
        if (!mapped) {
            void* p = nullptr;
            if (!hip_ok(hipIpcOpenMemHandle(&p, m.h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle"))
                return ncclUnhandledCudaError;
            mapped = static_cast<char*>(p);
        }
        // on the caller's stream (a synchronous hipMemcpy runs on the null stream, which a
        // non-blocking plan stream does not order against)
        if (!hip_ok(hipMemcpyAsync(o.buf, mapped + m.off, o.bytes, hipMemcpyDeviceToDevice, o.stream), "hipMemcpyAsync") ||
            !hip_ok(hipStreamSynchronize(o.stream), "hipStreamSynchronize"))
            return ncclUnhandledCudaError;
        c->recvd[o.peer] = k + 1;
        c->shm->consumed[o.peer][c->rank].store(k + 1, std::memory_order_release);
    }
    // a send buffer is free once its receiver has copied it
    for (auto& o : ops) {
        if (!o.send) continue;
        ncclComm* c = o.comm;
        auto& done = c->shm->consumed[c->rank][o.peer];
        const uint64_t want = c->sent[o.peer];
        if (!wait_for([&] { return done.load(std::memory_order_acquire) >= want; }, "a receive"))
            return ncclSystemError;
    }
    return ncclSuccess;
}

ncclResult_t enqueue(const Op& o) {
    g_ops.push_back(o);
    if (g_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(g_ops);
    return run_group(ops);
}
}  // namespace

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (rccl_stub)";
        case ncclUnhandledCudaError: return "HIP call failed (rccl_stub)";
        case ncclSystemError: return "system error: shared memory or a peer timed out (rccl_stub)";
        case ncclInternalError: return "internal error (rccl_stub)";
        case ncclInvalidArgument: return "invalid argument (rccl_stub)";
        default: return "error (rccl_stub)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::random_device rd;
    char name[64];
    snprintf(name, sizeof(name), "/optamd_rccl_stub_%d_%08x%08x", (int)getpid(), rd(), rd());
    memset(id->internal, 0, sizeof(id->internal));
    strncpy(id->internal, name, sizeof(id->internal) - 1);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    auto* c = new ncclComm();
    c->name.assign(id.internal, strnlen(id.internal, sizeof(id.internal)));
    c->rank = rank;
    c->n = nranks;
    const ncclResult_t r = attach(c);
    if (r != ncclSuccess) { delete c; return r; }
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm, ncclConfig_t*) {
    // every rank in one color, ranked as before (the only split RcclComm makes)
    if (!comm || !newcomm || color != 0 || key != comm->rank) return ncclInvalidArgument;
    auto* c = new ncclComm();
    c->name = comm->name + "_s" + std::to_string(++comm->splits);
    c->rank = comm->rank;
    c->n = comm->n;
    const ncclResult_t r = attach(c);
    if (r != ncclSuccess) { delete c; return r; }
    *newcomm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    barrier(comm);   // no peer still reads our buffers or our segment
    for (auto& kv : comm->opened) (void)hipIpcCloseMemHandle(kv.second);
    munmap(comm->shm, sizeof(Shm));
    if (comm->rank == 0) shm_unlink(comm->name.c_str());
    delete comm;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_depth <= 0) return ncclInvalidArgument;
    if (--g_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(g_ops);
    return run_group(ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
    const size_t es = type_size(t);
    if (!comm || !es || peer < 0 || peer >= comm->n || peer == comm->rank) return ncclInvalidArgument;
    return enqueue(Op{true, const_cast<void*>(buf), count * es, peer, comm, s});
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
    const size_t es = type_size(t);
    if (!comm || !es || peer < 0 || peer >= comm->n || peer == comm->rank) return ncclInvalidArgument;
    return enqueue(Op{false, buf, count * es, peer, comm, s});
}

ncclResult_t ncclAllReduce(const void* sendbuf, void* recvbuf, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t s) {
    if (!comm || t != ncclFloat64 || op != ncclSum || count > (size_t)kMaxScalars) return ncclInvalidArgument;
    if (g_depth > 0) return ncclInvalidArgument;   // RcclComm never groups a collective
    if (!hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize")) return ncclUnhandledCudaError;
    double mine[kMaxScalars];
    if (!hip_ok(hipMemcpyAsync(mine, sendbuf, sizeof(double) * count, hipMemcpyDeviceToHost, s), "hipMemcpyAsync") ||
        !hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize"))
        return ncclUnhandledCudaError;
    memcpy(comm->shm->red[comm->rank], mine, sizeof(double) * count);
    if (!barrier(comm)) return ncclSystemError;
    double sum[kMaxScalars];
    for (size_t k = 0; k < count; ++k) sum[k] = 0.0;
    for (int q = 0; q < comm->n; ++q)   // rank order, as OptAMD_LocalGroup sums
        for (size_t k = 0; k < count; ++k) sum[k] += comm->shm->red[q][k];
    if (!barrier(comm)) return ncclSystemError;   // every rank has read the slots
    // ordered on s and complete before returning: `sum` is a stack buffer
    if (!hip_ok(hipMemcpyAsync(recvbuf, sum, sizeof(double) * count, hipMemcpyHostToDevice, s), "hipMemcpyAsync") ||
        !hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize"))
        return ncclUnhandledCudaError;
    return ncclSuccess;
}

}  // extern "C"
