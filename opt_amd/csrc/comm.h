// comm.h — inter-rank transport for row-slab decomposed image domains.
//
// The reference has no multi-device code at all; this is the
// MI355X-side design of §8e: each rank owns a slab of image rows plus `halo` rows of
// its neighbours' data. Per PCG iteration the solver needs two scalar all-reduces
// (p.Ap, r.z) and one halo refresh of the vectors the next stencil apply reads.
//   RcclComm        one process per GPU, RCCL over xGMI (librccl loaded lazily)
//   LocalGroupComm  all ranks as threads of one process (devices shared or peer),
//                   used to test the decomposition on a single GPU
#pragma once
#include <hip/hip_runtime.h>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>
#include "common.h"

namespace optamd {

// One exchanged array: `base` points at memory row 0 of this rank's slab (global
// row dom.y_mem0); a row is `row_bytes` contiguous bytes.
struct HaloPlane {
    void* base;
    size_t row_bytes;
};

class Comm {
public:
    virtual ~Comm() {}
    virtual int rank() const = 0;
    virtual int size() const = 0;
    // In-place sum over ranks of n doubles in device memory, ordered on `s`.
    virtual void allreduce_sum(double* dev, int n, hipStream_t s) = 0;
    // Refresh the `halo` rows above and below this rank's owned rows in every plane
    // from the neighbouring ranks' owned rows, ordered on `s`.
    virtual void halo_exchange(const std::vector<HaloPlane>& planes, const Domain& dom, int halo,
                               hipStream_t s) = 0;
    virtual std::string kind() const = 0;
    // May a halo exchange on a second stream run concurrently with all-reduces on the
    // plan stream? (RCCL: only when the halos have a communicator of their own, so each
    // communicator is used from one stream in one order on every rank.)
    virtual bool concurrent_halo() const { return true; }
};

// ------------------------------------------------------------------ RCCL
bool rccl_unique_id(void* out128, std::string* err);
Comm* make_rccl_comm(const void* id128, int rank, int nranks, std::string* err);

// ----------------------------------------------------------- local group
class LocalGroup;
LocalGroup* make_local_group(int nranks);
Comm* local_group_rank(LocalGroup* g, int rank);   // owned by the group
void destroy_local_group(LocalGroup* g);

}  // namespace optamd
