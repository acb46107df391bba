// Diagnostics (not on the product path): a pure 16 B-per-lane streaming-store
// kernel that prices the HBM write ceiling the obs pass is measured against.
#include "common.h"
#include "marlsat_debug.h"

namespace msat {
template <bool kNt>
__global__ void __launch_bounds__(256) fill_kernel(int4 *__restrict__ dst, size_t n16, int value) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i v = {value, value, value, value};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        if (kNt)
            __builtin_nontemporal_store(v, reinterpret_cast<v4i *>(dst + i));
        else
            *reinterpret_cast<v4i *>(dst + i) = v;
    }
}
// pattern 1: each block owns one contiguous chunk (like one env's obs block per workgroup)
template <bool kNt>
__global__ void __launch_bounds__(256) fill_chunk_kernel(int4 *__restrict__ dst, size_t n16, size_t per_block, int value) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i v = {value, value, value, value};
    const size_t lo = (size_t)blockIdx.x * per_block;
    const size_t hi = lo + per_block < n16 ? lo + per_block : n16;
    for (size_t i = lo + threadIdx.x; i < hi; i += 256) {
        if (kNt)
            __builtin_nontemporal_store(v, reinterpret_cast<v4i *>(dst + i));
        else
            *reinterpret_cast<v4i *>(dst + i) = v;
    }
}
}  // namespace msat

extern "C" int msat_debug_fill_chunked(void *dst, size_t bytes, int32_t value, int32_t nontemporal, int32_t grid,
                                       void *stream) {
    MSAT_REQUIRE(dst && bytes % 16 == 0 && grid > 0, "bad fill args");
    const size_t n16 = bytes / 16, per = (n16 + grid - 1) / grid;
    if (nontemporal)
        hipLaunchKernelGGL(msat::fill_chunk_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int4 *)dst,
                           n16, per, value);
    else
        hipLaunchKernelGGL(msat::fill_chunk_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int4 *)dst,
                           n16, per, value);
    return msat::check_launch("fill_chunk_kernel");
}

extern "C" int msat_debug_fill(void *dst, size_t bytes, int32_t value, int32_t nontemporal, int32_t grid,
                               void *stream) {
    MSAT_REQUIRE(dst && bytes % 16 == 0 && grid > 0, "bad fill args");
    const size_t n16 = bytes / 16;
    if (nontemporal)
        hipLaunchKernelGGL(msat::fill_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int4 *)dst, n16,
                           value);
    else
        hipLaunchKernelGGL(msat::fill_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int4 *)dst, n16,
                           value);
    return msat::check_launch("fill_kernel");
}
