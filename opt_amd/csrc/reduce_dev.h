// reduce_dev.h — deterministic device-wide sums (device code only, no includes).
// Included by common.h inside namespace optamd, and pasted verbatim into the HIP source
// the general energy front end generates (gen/codegen.cpp) so both share one
// implementation.
#ifndef OPTAMD_HAVE_KBLOCK
#define OPTAMD_HAVE_KBLOCK
constexpr int kWave = 64;
constexpr int kBlock = 256;
#endif

// ---- deterministic device-wide sums ---------------------------------------------
// The reference sums every PCG scalar with one float atomic per 32-lane warp into a
// single address (unknownWideReduction, solverGPUGaussNewton.t:466-472;
// backend_cuda.t:366-375,447-495): order-dependent and contended. Here each block
// reduces its values in a fixed tree (fp64), publishes ONE partial per scalar with an
// agent-scope (sc1, write-through) store, drains it, and takes a ticket; the block
// that draws the last ticket sums all partials in block-index order and writes the
// scalars. Bitwise reproducible for any dispatch order or XCD placement
// (MI355X_MICROARCH.md "Valid forms", row 1; cdna_hip_programming.md G16).
struct ReduceSlot {
    double* partials;     // [K][nblocks]
    unsigned* ticket;     // kTicketShards shard counters + 1 top counter, 64 B apart, zero between launches
    double* out;          // K results
    int nblocks;
};
// Ordering of the hand-off. The partials go out as sc1 (write-through) stores, every
// storing lane drains them (s_waitcnt vmcnt(0)) before its agent-scope ticket add, and
// the last block reads them back with sc1 loads after an agent acquire: the guide's
// validated "one lane per workgroup, agent-scope add, last adder" row
// (MI355X_MICROARCH.md, Valid forms). A release on every ticket add
// (-DOPTAMD_REDUCE_ORDER=__ATOMIC_ACQ_REL: buffer_wbl2 sc1 per block) writes back the
// XCD L2's freshly dirtied output lines before each add; measured on MI355X it takes
// the image_warping JᵀJ·p apply from 142 to 236 µs and the GN step from 4.76 to
// 7.04 ms (profiles/r02b_reduce_order.json), so the tickets stay relaxed.
#ifndef OPTAMD_REDUCE_ORDER
#define OPTAMD_REDUCE_ORDER __ATOMIC_RELAXED
#endif
constexpr int kTicketShards = 32;     // arrival counters (b % 32: each fed by one XCD)
constexpr int kTicketStride = 16;     // unsigned words between counters (64 B)
constexpr int kTicketWords = (kTicketShards + 1) * kTicketStride;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, kWave);
    return v;
}

// Called by every thread of a kBlock-thread block exactly once, after all the
// block's stores of the kernel's outputs. v[k] is this thread's contribution.
// Returns 1 in thread 0 of the block that summed the partials (after it stored the K
// results; with `tot`, also copied there), 0 elsewhere: an epilogue that needs the
// launch's totals (the LM zeta test) runs there once every block has published.
// Arrivals are counted per shard (shard = block % 32, ~nblocks/32 adds per counter
// instead of nblocks on one word: a single hot counter costs ~12 ns per add,
// MI355X_MICROARCH.md row "fanin"); the last arriver of each shard then adds to a
// top counter, and the last of those sums every partial in block order.
template <int K>
__device__ __forceinline__ int block_reduce_publish(const double (&v)[K], const ReduceSlot& rs,
                                                    int block_linear, double* tot = nullptr) {
    __shared__ double red[kBlock / kWave][K];
    __shared__ int last_flag;
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double s = wave_sum(v[k]);
        if (lane == 0) red[wid][k] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double s = red[0][k];
#pragma unroll
            for (int w = 1; w < kBlock / kWave; ++w) s += red[w][k];
            __hip_atomic_store(&rs.partials[(long long)k * rs.nblocks + block_linear], s,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int shard = block_linear % kTicketShards;
        const int shards = rs.nblocks < kTicketShards ? rs.nblocks : kTicketShards;
        const unsigned in_shard = (unsigned)((rs.nblocks - shard + kTicketShards - 1) / kTicketShards);
        unsigned* sc = rs.ticket + shard * kTicketStride;
        const unsigned t = __hip_atomic_fetch_add(sc, 1u, OPTAMD_REDUCE_ORDER, __HIP_MEMORY_SCOPE_AGENT);
        int last = 0;
        if (t == in_shard - 1) {
            __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsigned* top = rs.ticket + kTicketShards * kTicketStride;
            const unsigned t2 = __hip_atomic_fetch_add(top, 1u, OPTAMD_REDUCE_ORDER, __HIP_MEMORY_SCOPE_AGENT);
            if (t2 == (unsigned)(shards - 1)) {
                __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
        last_flag = last;
    }
    __syncthreads();
    if (!last_flag) return 0;
    // one block per launch: the agent acquire (buffer_inv sc1) is cheap here
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // Last arriver: fixed-order sum of all partials (sc1 loads bypass the stale L1).
    __shared__ double acc[kBlock];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double s = 0.0;
        for (int i = threadIdx.x; i < rs.nblocks; i += kBlock)
            s += __hip_atomic_load(&rs.partials[(long long)k * rs.nblocks + i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        acc[threadIdx.x] = s;
        __syncthreads();
        for (int stride = kBlock / 2; stride > 0; stride >>= 1) {
            if (threadIdx.x < stride) acc[threadIdx.x] += acc[threadIdx.x + stride];
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            __hip_atomic_store(&rs.out[k], acc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tot) tot[k] = acc[0];
        }
        __syncthreads();
    }
    return threadIdx.x == 0;
}

