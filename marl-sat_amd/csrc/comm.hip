// The learner's gradient exchange at the C-ABI (SURVEY.md 8(b) msat_comm_init / msat_allreduce; the
// reference's counterpart is the single-device optax update at learner:647-650, so there is no
// reference collective to mirror -- this is the MI355X data-parallel design of 8(e)).
//
// One communicator per process (one process per GPU), created from a 128-byte unique id that rank 0
// draws and the host broadcasts by any means (the Python facade uses the torch.distributed store;
// a cgo / JNI host its own channel).  The all-reduce is RCCL in place on the caller's stream: a ring
// over the xGMI links for the ~2.8 MB flat gradient, and the fp64 moment / metric sums.  No device
// memory is allocated here; the communicator is the library's only global state.
//
// RCCL is resolved lazily (dlopen of the soname librccl.so.1 on the first msat_comm_* call), so
// libmarlsat.so has no load-time dependency on it: a host that only steps environments loads the
// library without RCCL installed, and msat_comm_* then fail with MSAT_ECOMM.  Opening by soname
// returns the copy already mapped into the process when there is one (torch's bundled RCCL in a
// Python host), so the library and torch.distributed share one RCCL instance there.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "common.h"
#include "marlsat_net.h"

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    const char *error = nullptr;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            r.error = "librccl.so.1 not found";
            return;
        }
        r.get_unique_id = reinterpret_cast<decltype(&ncclGetUniqueId)>(dlsym(h, "ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(&ncclCommInitRank)>(dlsym(h, "ncclCommInitRank"));
        r.all_reduce = reinterpret_cast<decltype(&ncclAllReduce)>(dlsym(h, "ncclAllReduce"));
        r.comm_destroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(h, "ncclCommDestroy"));
        r.error_string = reinterpret_cast<decltype(&ncclGetErrorString)>(dlsym(h, "ncclGetErrorString"));
        if (!(r.get_unique_id && r.comm_init_rank && r.all_reduce && r.comm_destroy && r.error_string))
            r.error = "librccl.so.1 lacks an nccl* entry point";
    });
    return r;
}

#define MSAT_RCCL(r)                                                                   \
    const Rccl &r = rccl();                                                            \
    if (r.error) return msat::fail(MSAT_ECOMM, "RCCL unavailable: %s", r.error)

int comm_fail(const Rccl &r, ncclResult_t e, const char *what) {
    return msat::fail(MSAT_ECOMM, "%s: %s", what, r.error_string(e));
}

}  // namespace

extern "C" size_t msat_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

extern "C" int msat_comm_unique_id(uint8_t *id_out) {
    MSAT_REQUIRE(id_out, "NULL id buffer");
    MSAT_RCCL(lib);
    ncclUniqueId id;
    const ncclResult_t r = lib.get_unique_id(&id);
    if (r != ncclSuccess) return comm_fail(lib, r, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
    return MSAT_OK;
}

extern "C" int msat_comm_init(const uint8_t *id, int32_t rank, int32_t world, void **comm_out) {
    MSAT_REQUIRE(id && comm_out, "NULL pointer");
    MSAT_REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank %d / world %d", rank, world);
    MSAT_RCCL(lib);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    const ncclResult_t r = lib.comm_init_rank(&c, world, uid, rank);
    if (r != ncclSuccess) return comm_fail(lib, r, "ncclCommInitRank");
    *comm_out = c;
    return MSAT_OK;
}

extern "C" int msat_allreduce_sum(void *comm, void *buf, size_t count, int32_t dtype, void *stream) {
    MSAT_REQUIRE(comm, "NULL communicator");
    MSAT_REQUIRE(buf || count == 0, "NULL buffer");
    MSAT_REQUIRE(dtype == 0 || dtype == 1, "dtype must be 0 (fp32) or 1 (fp64), got %d", dtype);
    if (count == 0) return MSAT_OK;
    MSAT_RCCL(lib);
    const ncclResult_t r = lib.all_reduce(buf, buf, count, dtype ? ncclFloat64 : ncclFloat32, ncclSum,
                                          static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(stream));
    if (r != ncclSuccess) return comm_fail(lib, r, "ncclAllReduce");
    return MSAT_OK;
}

extern "C" int msat_comm_destroy(void *comm) {
    if (!comm) return MSAT_OK;
    MSAT_RCCL(lib);
    const ncclResult_t r = lib.comm_destroy(static_cast<ncclComm_t>(comm));
    if (r != ncclSuccess) return comm_fail(lib, r, "ncclCommDestroy");
    return MSAT_OK;
}
