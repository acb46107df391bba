// Shared helpers for libmarlsat: error channel, launch checks, Philox RNG,
// wave/block reductions.  gfx950 only (wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <limits.h>

#include "marlsat.h"
#include "marlsat_net.h"  // every extern "C" definition is checked against its declaration

namespace msat {

// ---------------------------------------------------------------- errors ----
int fail(int code, const char *fmt, ...);  // sets the thread-local message, returns code
int check_launch_plain(const char *what);  // hipGetLastError -> MSAT_EHIP

// ------------------------------------------------------------- debug build ----
// libmarlsat_debug.so is every kernel built with -DMSAT_DEBUG: MSAT_DCHECK(idx, bound) records the first
// index outside [0, bound) (source line, index, bound) in this translation unit's g_msat_dbg, and
// check_launch() synchronises after every launch and turns a recorded failure into MSAT_EHIP naming the
// launch and the line.  The kernels carry on after a failed check (no trap: the message is the result).
// In the product build both compile to nothing.
#ifdef MSAT_DEBUG
struct MsatDbg {
    int failed, line;
    long long idx, bound;
};
static __device__ MsatDbg g_msat_dbg;

#define MSAT_DCHECK(idx_, bound_)                                                                \
    do {                                                                                         \
        const long long _i = (long long)(idx_), _b = (long long)(bound_);                        \
        if (_i < 0 || _i >= _b) {                                                                \
            if (atomicCAS(&::msat::g_msat_dbg.failed, 0, 1) == 0) {                              \
                ::msat::g_msat_dbg.line = __LINE__;                                              \
                ::msat::g_msat_dbg.idx = _i;                                                     \
                ::msat::g_msat_dbg.bound = _b;                                                   \
            }                                                                                    \
        }                                                                                        \
    } while (0)

static inline int check_launch(const char *what) {
    int rc = check_launch_plain(what);
    if (rc) return rc;
    if (hipDeviceSynchronize() != hipSuccess) return check_launch_plain(what);
    MsatDbg h{};
    if (hipMemcpyFromSymbol(&h, HIP_SYMBOL(g_msat_dbg), sizeof(h)) != hipSuccess) return check_launch_plain(what);
    if (h.failed) {
        const MsatDbg z{};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_msat_dbg), &z, sizeof(z));
        return fail(MSAT_EHIP, "MSAT_DEBUG: %s: index %lld outside [0, %lld) at line %d of its source", what, h.idx,
                    h.bound, h.line);
    }
    return MSAT_OK;
}
#define MSAT_DEBUG_BUILD 1
#else
#define MSAT_DCHECK(idx_, bound_) ((void)0)
static inline int check_launch(const char *what) { return check_launch_plain(what); }
#define MSAT_DEBUG_BUILD 0
#endif

// Debug builds: the number of elements of size `elem` from p to the end of p's device allocation (for a
// torch tensor: the end of its caching-allocator segment, so an index past the tensor but inside the segment
// is not caught -- an index past the segment is).  The bounds the kernels' MSAT_DCHECKs compare against.
// Product builds: 0 without a driver call (the checks compile to nothing).
// (A pointer the runtime does not know -- NULL, host memory -- gets no bound: LLONG_MAX.)
static inline long long dbg_extent(const void *p, size_t elem) {
    if (!MSAT_DEBUG_BUILD) return 0;
    hipDeviceptr_t base = nullptr;
    size_t bytes = 0;
    if (p == nullptr || hipMemGetAddressRange(&base, &bytes, (hipDeviceptr_t)p) != hipSuccess) return LLONG_MAX;
    return (long long)(((const char *)base + bytes - (const char *)p) / (long long)elem);
}

#define MSAT_REQUIRE(cond, ...)                      \
    do {                                             \
        if (!(cond)) return ::msat::fail(MSAT_EBADARG, __VA_ARGS__); \
    } while (0)

// --------------------------------------------------------------- Philox ----
// Philox4x32-10 (Salmon et al., SC'11).  Mirrored bit-exactly by
// oracle/rng.py so RNG-driven resets can be replayed on the host.
__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
        const uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// Stream layout used for resets of env b at call counter `ctr`:
//   word block w=0, lane 0 -> problem index  ((u64)r * N) >> 32
//   word block w=1+v/128, lane (v%128)/32, bit v%32 -> assignment of var v
__host__ __device__ __forceinline__ uint4 reset_rng_block(uint64_t seed, uint64_t ctr, uint32_t env,
                                                          uint32_t w) {
    return philox4x32_10(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), env, w), (uint32_t)seed,
                         (uint32_t)(seed >> 32));
}

// ------------------------------------------------------------- LDS-DMA ----
// global_load_lds_dwordx4 issued from inline asm: 16 bytes per lane from `src` into LDS at
// the wave-uniform byte address `lds` + 16 * lane.  The builtin form is tracked by hipcc, which
// then waits vmcnt(0) before EVERY later ds_read (it cannot tell the DMA's target buffer from
// the one being read), so the next slab's load never overlaps the current slab's MFMAs.  The
// asm form is invisible to hipcc's wait bookkeeping: the caller retires it with a counted
// wait_vmcnt<N>() and a barrier before reading the buffer.  M0 is saved and restored in the
// same statement (it is compiler-reserved).
__device__ __forceinline__ void glds16_async(const void *src, const void *lds) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(dst)
        : "memory");
}

// Same, with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset (the saddr
// form): no 64-bit per-lane address arithmetic in the issuing loop.
__device__ __forceinline__ void glds16_async_s(const void *sbase, unsigned voff, const void *lds) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(dst)
        : "memory");
}

// Two pieces: sbase0 -> lds, sbase1 -> lds + STEP bytes, same per-lane offset, M0 written once per pair.
template <int STEP>
__device__ __forceinline__ void glds16_async_s2(const void *sbase0, const void *sbase1, unsigned voff,
                                                const void *lds) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
        "s_add_u32 m0, m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase0), "s"(sbase1), "s"(dst), "n"(STEP)
        : "memory");
}

// 4 bytes per lane (global_load_lds_dword): LDS at the wave-uniform byte address `lds` + 4 * lane, saddr form.
__device__ __forceinline__ void glds4_async_s(const void *sbase, unsigned voff, const void *lds) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(dst)
        : "memory");
}

// s_waitcnt vmcnt(N): all but this wave's N youngest vector-memory operations are done.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// workgroup barrier that waits only for this wave's LDS operations (not for vector memory)
__device__ __forceinline__ void barrier_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ----------------------------------------------------------- reductions ----
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max_f32(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

}  // namespace msat
