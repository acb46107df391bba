// Diagnostics (not on the product path): a pure 16 B-per-lane streaming-store
// kernel that prices the HBM write ceiling the obs pass is measured against.
#include "common.h"
#include "marlsat_probe.h"

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
// pattern 2: obs expansion from compact bit images (two-phase env-step prototype).
// Quad q covers obs elements 4q..4q+3 of the flat [E][A][D] array (D % 4 == 0, so a quad
// stays in one row and one 32-bit image word). vimg[e][Dw]: bit d = value of element d;
// mimg[inst][a][Dw]: bit d = element visible to agent a (else -1).
__global__ void __launch_bounds__(256) obs_expand_kernel(int4 *__restrict__ dst, uint32_t nq, uint32_t D,
                                                         uint32_t A, uint32_t Dw, const int *__restrict__ inst,
                                                         const uint32_t *__restrict__ vimg,
                                                         const uint32_t *__restrict__ mimg) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < nq; q += gridDim.x * 256) {
        const uint32_t i = q * 4, row = i / D, d = i - row * D, e = row / A, a = row - e * A;
        const uint32_t w = d >> 5, sh = d & 31;
        const uint32_t vb = vimg[(size_t)e * Dw + w] >> sh;
        const uint32_t mb = mimg[((size_t)inst[e] * A + a) * Dw + w] >> sh;
        v4i o;
        o.x = (mb & 1) ? (int)(vb & 1) : -1;
        o.y = (mb & 2) ? (int)((vb >> 1) & 1) : -1;
        o.z = (mb & 4) ? (int)((vb >> 2) & 1) : -1;
        o.w = (mb & 8) ? (int)((vb >> 3) & 1) : -1;
        *reinterpret_cast<v4i *>(dst + q) = o;
    }
}
// Same expansion, one wave per obs row (e, a): the row's image words sit one per lane
// (Dw <= 64) and each quad takes its word by lane shuffle, so the loop is stores only.
__global__ void __launch_bounds__(256) obs_expand_rows_kernel(int4 *__restrict__ dst, uint32_t rows, uint32_t D,
                                                              uint32_t A, uint32_t Dw,
                                                              const int *__restrict__ inst,
                                                              const uint32_t *__restrict__ vimg,
                                                              const uint32_t *__restrict__ mimg) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const uint32_t lane = threadIdx.x & 63, nq = D / 4, nw = gridDim.x * 4;
    for (uint32_t r = (blockIdx.x * 256 + threadIdx.x) >> 6; r < rows; r += nw) {
        const uint32_t e = r / A, a = r - e * A;
        uint32_t vw = 0, mw = 0;
        if (lane < Dw) {
            vw = vimg[(size_t)e * Dw + lane];
            mw = mimg[((size_t)inst[e] * A + a) * Dw + lane];
        }
        int4 *o = dst + (size_t)r * nq;
        for (uint32_t q = lane; q < nq; q += 64) {
            const uint32_t d = q * 4, w = d >> 5, sh = d & 31;
            const uint32_t vb = (uint32_t)__shfl((int)vw, (int)w) >> sh, mb = (uint32_t)__shfl((int)mw, (int)w) >> sh;
            v4i v;
            v.x = (mb & 1) ? (int)(vb & 1) : -1;
            v.y = (mb & 2) ? (int)((vb >> 1) & 1) : -1;
            v.z = (mb & 4) ? (int)((vb >> 2) & 1) : -1;
            v.w = (mb & 8) ? (int)((vb >> 3) & 1) : -1;
            *reinterpret_cast<v4i *>(o + q) = v;
        }
    }
}
// pattern 3: one workgroup per env writes its A obs rows of D16 x 16 B, env-major ([E][A][D], the
// product layout) or agent-major ([A][E][D]: agent a's rows of all envs contiguous)
template <int NT>
__global__ void __launch_bounds__(NT) fill_rows_kernel(int4 *__restrict__ dst, int E, int A, int D16, int amajor,
                                                       int value) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i v = {value, value, value, value};
    for (int e = blockIdx.x; e < E; e += gridDim.x)
        for (int a = 0; a < A; ++a) {
            const size_t row = amajor ? (size_t)a * E + e : (size_t)e * A + a;
            for (int i = threadIdx.x; i < D16; i += NT) *reinterpret_cast<v4i *>(dst + row * D16 + i) = v;
        }
}

// Read-pattern probe for the data gradient's activation stream: the same bytes (M rows x K floats of a
// row-major buffer with leading dimension ld) read (0) as register-A column strips -- per 128-row workgroup
// and 32-column step, lane (l16, g) loads two float4 of row l16 + 16 i, columns 32 d + 8 g .. + 7, i < 2 --
// (1) as contiguous rows (each wave-instruction 1 KiB of one row), (2) as (0) with three workgroups per
// row block (the per-tile kernel's three column tiles re-reading from L2).
template <int MODE>
__global__ void __launch_bounds__(256) strip_read_kernel(const float *__restrict__ D, int M, int ld, int K,
                                                         float *__restrict__ out) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63, l16 = lane & 15, g = lane >> 4;
    const int blk = MODE == 2 ? blockIdx.x / 3 : blockIdx.x;
    const int m0 = blk * 128 + w * 32;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (MODE == 1) {
        for (int r = 0; r < 32; ++r) {
            const float *row = D + (size_t)min(m0 + r, M - 1) * ld;
            for (int c = 4 * lane; c < K; c += 256) {
                const float4 v = *reinterpret_cast<const float4 *>(row + c);
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
        }
    } else {
        const float *a0 = D + (size_t)min(m0 + l16, M - 1) * ld + 8 * g;
        const float *a1 = D + (size_t)min(m0 + 16 + l16, M - 1) * ld + 8 * g;
        for (int d = 0; d < K / 32; ++d) {
            const float4 u0 = *reinterpret_cast<const float4 *>(a0 + 32 * d);
            const float4 u1 = *reinterpret_cast<const float4 *>(a0 + 32 * d + 4);
            const float4 v0 = *reinterpret_cast<const float4 *>(a1 + 32 * d);
            const float4 v1 = *reinterpret_cast<const float4 *>(a1 + 32 * d + 4);
            s.x += u0.x + u1.x + v0.x + v1.x; s.y += u0.y + u1.y + v0.y + v1.y;
            s.z += u0.z + u1.z + v0.z + v1.z; s.w += u0.w + u1.w + v0.w + v1.w;
        }
    }
    out[(size_t)blockIdx.x * 256 + t] = s.x + s.y + s.z + s.w;
}

// Texture-path probe: L2-resident reads at full occupancy (three 256-thread workgroups per CU, as the data
// gradient runs), 1 KiB per wave-instruction, in four forms -- plain loads into registers (0: lane-linear,
// 2: the register-A pattern, 16 rows x 64 B at a 2 KiB row stride) and LDS-DMA pieces (1: lane-linear,
// 3: the weight-piece pattern, 16 rows x 64 B at a 768 B stride) -- so the TA / TD counters of each can be
// read against its byte rate.
template <int MODE>
__global__ void __launch_bounds__(256, 3) l2_read_kernel(const char *__restrict__ buf, int window, int iters,
                                                         int stride, float *__restrict__ out) {
    __shared__ uint4 ring[4][8][64];  // per wave: eight 1 KiB pieces
    const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6), l16 = lane & 15, g = lane >> 4;
    const int wid = blockIdx.x * 4 + w;
    unsigned lo;
    if (MODE == 0 || MODE == 1) lo = 16u * lane;
    else if (MODE == 2) lo = (unsigned)stride * l16 + 32u * g;
    else if (MODE == 4) lo = (unsigned)stride * (lane >> 3) + 16u * (lane & 7);  // 8 rows x 128 B
    else lo = (unsigned)stride * (lane >> 2) + 16u * (lane & 3);                // 16 rows x 64 B
    const unsigned span = (MODE == 0 || MODE == 1) ? 1024u : 16u * (unsigned)stride;
    const unsigned nwin = (unsigned)window > span ? (unsigned)window - span : 0u;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int it = 0; it < iters; it += 8) {
        if constexpr (MODE == 0 || MODE == 2 || MODE == 4 || MODE == 5) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const unsigned off = ((unsigned)(wid * 8 + it + u) * 4096u) % (nwin + 1u);
                v[u] = *reinterpret_cast<const float4 *>(buf + off + lo);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
            }
        } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const unsigned off = ((unsigned)(wid * 8 + it + u) * 4096u) % (nwin + 1u);
                glds16_async_s(buf + off, lo, &ring[w][u][0]);
            }
            wait_vmcnt<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const uint4 q = ring[w][it & 7][lane];
            acc.x += __uint_as_float(q.x);
        }
    }
    out[(size_t)blockIdx.x * 256 + t] = acc.x + acc.y + acc.z + acc.w;
}
}  // namespace msat

extern "C" int msat_probe_l2_read(const void *buf, int32_t window, int32_t mode, int32_t iters, int32_t grid,
                                  int32_t stride, float *out, void *stream) {
    MSAT_REQUIRE(buf && out && window >= 65536 && iters > 0 && iters % 8 == 0 && grid > 0 && mode >= 0 && mode <= 5 &&
                     stride >= 128 && stride % 16 == 0 && 16 * stride < window,
                 "bad l2_read args");
    const char *b = static_cast<const char *>(buf);
    hipStream_t s = (hipStream_t)stream;
    if (mode == 0) hipLaunchKernelGGL(msat::l2_read_kernel<0>, dim3(grid), dim3(256), 0, s, b, window, iters, stride, out);
    else if (mode == 1) hipLaunchKernelGGL(msat::l2_read_kernel<1>, dim3(grid), dim3(256), 0, s, b, window, iters, stride, out);
    else if (mode == 2) hipLaunchKernelGGL(msat::l2_read_kernel<2>, dim3(grid), dim3(256), 0, s, b, window, iters, stride, out);
    else if (mode == 3) hipLaunchKernelGGL(msat::l2_read_kernel<3>, dim3(grid), dim3(256), 0, s, b, window, iters, stride, out);
    else if (mode == 4) hipLaunchKernelGGL(msat::l2_read_kernel<4>, dim3(grid), dim3(256), 0, s, b, window, iters, stride, out);
    else hipLaunchKernelGGL(msat::l2_read_kernel<5>, dim3(grid), dim3(256), 0, s, b, window, iters, stride, out);
    return msat::check_launch("l2_read_kernel");
}


extern "C" int msat_probe_strip_read(const float *D, int32_t M, int32_t ld, int32_t K, int32_t mode, float *out,
                                     void *stream) {
    MSAT_REQUIRE(D && out && M > 0 && K % 32 == 0 && ld >= K && ld % 4 == 0 && mode >= 0 && mode <= 2,
                 "bad strip_read args");
    const int nb = (M + 127) / 128;
    if (mode == 0)
        hipLaunchKernelGGL(msat::strip_read_kernel<0>, dim3(nb), dim3(256), 0, (hipStream_t)stream, D, M, ld, K, out);
    else if (mode == 1)
        hipLaunchKernelGGL(msat::strip_read_kernel<1>, dim3(nb), dim3(256), 0, (hipStream_t)stream, D, M, ld, K, out);
    else
        hipLaunchKernelGGL(msat::strip_read_kernel<2>, dim3(3 * nb), dim3(256), 0, (hipStream_t)stream, D, M, ld, K,
                           out);
    return msat::check_launch("strip_read_kernel");
}


extern "C" int msat_probe_obs_expand(void *dst, int32_t E, int32_t A, int32_t D, const int32_t *inst,
                                     const uint32_t *vimg, const uint32_t *mimg, int32_t grid, void *stream) {
    MSAT_REQUIRE(dst && inst && vimg && mimg && E > 0 && A > 0 && D > 0 && D % 4 == 0 && grid != 0,
                 "bad expand args");
    const uint64_t nq = (uint64_t)E * A * D / 4;
    MSAT_REQUIRE(nq * 4 < (1ull << 32), "expand: too many elements");
    if (grid < 0) {  // one wave per row
        MSAT_REQUIRE((D + 31) / 32 <= 64, "expand rows: D too large");
        hipLaunchKernelGGL(msat::obs_expand_rows_kernel, dim3(-grid), dim3(256), 0, (hipStream_t)stream,
                           (int4 *)dst, (uint32_t)(E * A), (uint32_t)D, (uint32_t)A, (uint32_t)((D + 31) / 32),
                           inst, vimg, mimg);
        return msat::check_launch("obs_expand_rows_kernel");
    }
    hipLaunchKernelGGL(msat::obs_expand_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int4 *)dst,
                       (uint32_t)nq, (uint32_t)D, (uint32_t)A, (uint32_t)((D + 31) / 32), inst, vimg, mimg);
    return msat::check_launch("obs_expand_kernel");
}

extern "C" int msat_probe_fill_chunked(void *dst, size_t bytes, int32_t value, int32_t nontemporal, int32_t grid,
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

extern "C" int msat_probe_fill(void *dst, size_t bytes, int32_t value, int32_t nontemporal, int32_t grid,
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

extern "C" int msat_probe_fill_rows(void *dst, int32_t E, int32_t A, int32_t D16, int32_t amajor, int32_t value,
                                    int32_t threads, int32_t grid, void *stream) {
    MSAT_REQUIRE(dst && E > 0 && A > 0 && D16 > 0 && grid > 0 && (threads == 256 || threads == 512), "bad fill args");
    if (threads == 512)
        hipLaunchKernelGGL(msat::fill_rows_kernel<512>, dim3(grid), dim3(512), 0, (hipStream_t)stream, (int4 *)dst, E,
                           A, D16, amajor, value);
    else
        hipLaunchKernelGGL(msat::fill_rows_kernel<256>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (int4 *)dst, E,
                           A, D16, amajor, value);
    return msat::check_launch("fill_rows_kernel");
}
