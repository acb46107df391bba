// The learner's gradient exchange at the C-ABI (SURVEY.md 8(b) msat_comm_init / msat_allreduce; the
// reference's counterpart is the single-device optax update at learner:647-650, so there is no
// reference collective to mirror -- this is the MI355X data-parallel design of 8(e)).
//
// One communicator per process (one process per GPU), created from a 128-byte unique id that rank 0
// draws and the host broadcasts by any means (the Python facade uses the torch.distributed store;
// a cgo / JNI host its own channel).  The all-reduce is RCCL in place on the caller's stream: a ring
// over the xGMI links for the ~2.8 MB flat gradient, and the fp64 moment / metric sums.  No device
// memory is allocated here; the communicator is the library's only global state.
#include <rccl/rccl.h>

#include <cstring>

#include "common.h"
#include "marlsat_net.h"

namespace {

int comm_fail(ncclResult_t r, const char *what) {
    return msat::fail(MSAT_ECOMM, "%s: %s", what, ncclGetErrorString(r));
}

}  // namespace

extern "C" size_t msat_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

extern "C" int msat_comm_unique_id(uint8_t *id_out) {
    MSAT_REQUIRE(id_out, "NULL id buffer");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return comm_fail(r, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
    return MSAT_OK;
}

extern "C" int msat_comm_init(const uint8_t *id, int32_t rank, int32_t world, void **comm_out) {
    MSAT_REQUIRE(id && comm_out, "NULL pointer");
    MSAT_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank %d / world %d", rank, world);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, world, uid, rank);
    if (r != ncclSuccess) return comm_fail(r, "ncclCommInitRank");
    *comm_out = c;
    return MSAT_OK;
}

extern "C" int msat_allreduce_sum(void *comm, void *buf, size_t count, int32_t dtype, void *stream) {
    MSAT_REQUIRE(comm, "NULL communicator");
    MSAT_REQUIRE(buf || count == 0, "NULL buffer");
    MSAT_REQUIRE(dtype == 0 || dtype == 1, "dtype must be 0 (fp32) or 1 (fp64), got %d", dtype);
    if (count == 0) return MSAT_OK;
    const ncclResult_t r = ncclAllReduce(buf, buf, count, dtype ? ncclFloat64 : ncclFloat32, ncclSum,
                                         static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(stream));
    if (r != ncclSuccess) return comm_fail(r, "ncclAllReduce");
    return MSAT_OK;
}

extern "C" int msat_comm_destroy(void *comm) {
    if (!comm) return MSAT_OK;
    const ncclResult_t r = ncclCommDestroy(static_cast<ncclComm_t>(comm));
    if (r != ncclSuccess) return comm_fail(r, "ncclCommDestroy");
    return MSAT_OK;
}
