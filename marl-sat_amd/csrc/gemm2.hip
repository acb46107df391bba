// fp32 MFMA GEMM, LDS-DMA pipeline (the fast path of msat_gemm / msat_gemm_wgrad).
//
// 128x128 output tile per 256-thread workgroup (4 waves, 64x64 each = 2x2 MFMA 32x32x2
// tiles), reduction staged through LDS D = 32 (or 16) deep, double-buffered, filled straight from
// global memory by global_load_lds_dwordx4 (no VGPR staging, no transpose pass).
//
// Operand images (one 32-deep slab x 128 output indices o):
//   * "k-major" operand (rows [o][k], k contiguous: activations; W[n][k] when transposed):
//     [o][32] with the 16-byte chunk c of row o stored at slot c ^ ((o >> 1) & 7).  Lane l
//     of a 32-row MFMA tile reads one chunk -- 4 reduction values -- with ds_read_b128;
//     the swizzle spreads every ds_read_b128 lane group over all 64 banks.
//   * "o-major" operand (rows [k][o], o contiguous: W[k][n], and both wgrad operands):
//     plain [32][128], read with ds_read_b32 (32 consecutive words per half-wave).
// Reduction order inside a slab (both operands use it): MFMA step j = 4q + r feeds
// k = 8q + r (lanes 0-31) and k = 8q + 4 + r (lanes 32-63), so a k-major lane's 4-wide
// chunk 2q + h covers steps 4q..4q+3.  Per output element the sum is still one fixed-
// order fmaf chain (bitwise reproducible), just in a permuted k order.
//
// Edge handling: output rows/cols past M/N read clamped (valid, finite) addresses and are
// not stored; the reduction tail must be zero on both operands, so the GEMM requires
// K % 32 == 0 and the weight-gradient kernel loads its last partial slab through
// registers with zero fill.
#include <stdlib.h>

#include <algorithm>

#include "common.h"

namespace msat {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kG2T = 256;
constexpr int kG2M = 128;  // tile rows / cols

// bijective XCD-aware remap (blocks sharing an XCD get consecutive logical ids)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__device__ __forceinline__ void glds16(const float *src, float *dst) { glds16_async(src, dst); }

// chunk swizzle of a k-major image row o (D/4 chunks of 4 floats per row)
template <int D>
__device__ __forceinline__ int kswz(int o) {
    return D == 32 ? (o >> 1) & 7 : (o >> 2) & 3;
}

// k-major image fill: src rows o (ld), columns k0..k0+D-1; rows >= omax clamped.
template <int D>
__device__ __forceinline__ void fill_kmajor(float *img, const float *__restrict__ src, int ld, int o0, int omax, int k0) {
    constexpr int RPI = 256 / D;          // rows per wave-instruction (1 KiB)
    constexpr int NI = kG2M / RPI / 4;    // instructions per wave
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int base = (w * NI + i) * RPI;
        const int o = base + lane / (D / 4), slot = lane % (D / 4);
        const int c = slot ^ kswz<D>(o);
        const int row = min(o0 + o, omax - 1);
        glds16(src + (size_t)row * ld + k0 + 4 * c, img + base * D);
    }
}

// o-major image fill: src rows k (ld), columns o0..o0+127; rows >= kmax / cols >= omax clamped.
template <int D>
__device__ __forceinline__ void fill_omajor(float *img, const float *__restrict__ src, int ld, int o0, int omax, int k0,
                                            int kmax) {
    constexpr int NI = D / 8;  // (D x 128 floats) / 1 KiB / 4 waves
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int f = (w * NI + i) * 64 + lane;  // float4 index in the image
        const int k = f >> 5, o4 = (f & 31) * 4;
        const int row = min(k0 + k, kmax - 1);
        const int col = min(o0 + o4, omax - 4);
        glds16(src + (size_t)row * ld + col, img + (w * NI + i) * 256);
    }
}

// o-major image through registers with zero fill (reduction tail of the weight gradient).
template <int D>
__device__ __forceinline__ void fill_omajor_zero(float *img, const float *__restrict__ src, int ld, int o0, int omax,
                                                 int k0, int kend) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < D / 8; ++i) {
        const int f = i * kG2T + t;
        const int k = f >> 5, o4 = (f & 31) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k0 + k < kend && o0 + o4 < omax) v = *reinterpret_cast<const float4 *>(src + (size_t)(k0 + k) * ld + o0 + o4);
        *reinterpret_cast<float4 *>(img + 4 * f) = v;
    }
}

// One D-deep slab of MFMAs for wave (wr, wc) from images Ai (A-operand, o = m) / Bi (o = n).
template <int D, bool AK, bool BK>
__device__ __forceinline__ void mfma_slab(const float *Ai, const float *Bi, int wr, int wc, f32x16 (&acc)[2][2]) {
    const int lane = threadIdx.x & 63, li = lane & 31, h = lane >> 5;
#pragma unroll
    for (int q = 0; q < D / 8; ++q) {
        float4 af[2], bf[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            if (AK) {
                const int o = wr + 32 * t + li;
                af[t] = *reinterpret_cast<const float4 *>(Ai + o * D + 4 * ((2 * q + h) ^ kswz<D>(o)));
            } else {
                const float *p = Ai + (8 * q + 4 * h) * kG2M + wr + 32 * t + li;
                af[t] = make_float4(p[0], p[kG2M], p[2 * kG2M], p[3 * kG2M]);
            }
            if (BK) {
                const int o = wc + 32 * t + li;
                bf[t] = *reinterpret_cast<const float4 *>(Bi + o * D + 4 * ((2 * q + h) ^ kswz<D>(o)));
            } else {
                const float *p = Bi + (8 * q + 4 * h) * kG2M + wc + 32 * t + li;
                bf[t] = make_float4(p[0], p[kG2M], p[2 * kG2M], p[3 * kG2M]);
            }
        }
#define MSAT_STEP(C)                                                                                   \
    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[0].C, bf[0].C, acc[0][0], 0, 0, 0);             \
    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[0].C, bf[1].C, acc[0][1], 0, 0, 0);             \
    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[1].C, bf[0].C, acc[1][0], 0, 0, 0);             \
    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[1].C, bf[1].C, acc[1][1], 0, 0, 0);
        MSAT_STEP(x) MSAT_STEP(y) MSAT_STEP(z) MSAT_STEP(w)
#undef MSAT_STEP
    }
}

// C[M,N] (+)= A[M,K] @ op(B) + bias; A k-major; B o-major (B[K][N]) or k-major (B[N][K]).
// NST = 2: double buffer, slab s+1 lands while slab s is multiplied.  NST = 3: slabs s+1 and
// s+2 in flight; each wave waits (counted vmcnt) only for slab s.  Both retire the asm LDS-DMA
// with explicit vmcnt waits + an LDS-only barrier (common.h glds16_async).
template <int D, bool BK, int NST = 2>
__global__ void __launch_bounds__(kG2T, NST == 3 ? 3 : (D == 16 ? 4 : 2))
gemm2_kernel(const float *__restrict__ A, int lda, const float *__restrict__ B, int ldb, float *__restrict__ C,
             int ldc, const float *__restrict__ bias, int M, int N, int K, int accumulate, int ntn, int vec_out) {
    constexpr int IMG = kG2M * D;
    __shared__ __attribute__((aligned(16))) float lds[(NST == 3 ? 6 : 4) * IMG];  // [buf][A|B]
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int m0 = (id / ntn) * kG2M, n0 = (id % ntn) * kG2M;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wr = (w >> 1) * 64, wc = (w & 1) * 64;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    const int ns = K / D;
    auto fill = [&](int s, int buf) {
        float *Ai = lds + buf * 2 * IMG, *Bi = Ai + IMG;
        fill_kmajor<D>(Ai, A, lda, m0, M, s * D);
        if (BK) fill_kmajor<D>(Bi, B, ldb, n0, N, s * D);
        else fill_omajor<D>(Bi, B, ldb, n0, N, s * D, K);
    };
    if (NST == 3) {
        // glds per thread per slab: A image kG2M*D/1024 instructions per wave... (fill_* NI), both operands
        constexpr int G = 2 * (D / 8);
        fill(0, 0);
        if (ns > 1) fill(1, 1);
        for (int s = 0; s < ns; ++s) {
            __builtin_amdgcn_sched_barrier(0);  // slab s-1's MFMAs stay above the wait
            if (s + 1 < ns) wait_vmcnt<G>();  // slab s landed (this wave's part); slab s+1 may fly
            else wait_vmcnt<0>();
            barrier_lds();  // every wave's part of slab s landed; slab s-1 fully read
            if (s + 2 < ns) fill(s + 2, (s + 2) % 3);
            const float *Ai = lds + (s % 3) * 2 * IMG;
            mfma_slab<D, true, BK>(Ai, Ai + IMG, wr, wc, acc);
        }
        __syncthreads();  // last slab read by every wave before the epilogue reuses LDS
    } else {
        fill(0, 0);
        wait_vmcnt<0>();
        barrier_lds();
        for (int s = 0; s < ns; ++s) {
            const int buf = s & 1;
            if (s + 1 < ns) fill(s + 1, buf ^ 1);  // lands while slab s is multiplied
            const float *Ai = lds + buf * 2 * IMG;
            mfma_slab<D, true, BK>(Ai, Ai + IMG, wr, wc, acc);
            __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs above the wait (they hide the load)
            wait_vmcnt<0>();
            barrier_lds();  // next image landed (every wave) and this one fully read
        }
    }
    if (vec_out) {
        // LDS-staged epilogue: each wave's 32x64 half-tile goes through its own 8 KiB LDS region
        // and leaves as whole 256-byte rows of float4 stores (bias / accumulate in float4).
        float *stage = lds + w * 32 * 64;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int reg = 0; reg < 16; ++reg)
                    stage[((reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)) * 64 + 32 * j + (lane & 31)] = acc[i][j][reg];
            __syncthreads();
            const int col = n0 + wc + (lane & 15) * 4;
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (bias && col < N) bv = *reinterpret_cast<const float4 *>(bias + col);
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int r = it * 4 + (lane >> 4);
                const int row = m0 + wr + 32 * i + r;
                float4 v = *reinterpret_cast<const float4 *>(stage + r * 64 + (lane & 15) * 4);
                v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
                if (row < M && col < N) {
                    float4 *c = reinterpret_cast<float4 *>(C + (size_t)row * ldc + col);
                    if (accumulate) {
                        const float4 o = *c;
                        v.x = o.x + v.x; v.y = o.y + v.y; v.z = o.z + v.z; v.w = o.w + v.w;
                    }
                    *c = v;
                }
            }
            __syncthreads();
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = n0 + wc + 32 * j + (lane & 31);
            if (col >= N) continue;
            const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = m0 + wr + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
                if (row >= M) continue;
                float *c = C + (size_t)row * ldc + col;
                const float v = acc[i][j][reg] + bv;
                if (accumulate == 2) {
                    if (v != v) *c = v;
                    continue;
                }
                *c = accumulate ? *c + v : v;
            }
        }
}

// partial[s][k][n] = sum_{m in split s} A[m][k] G[m][n]: both operands o-major over the rows m.
template <int D>
__global__ void __launch_bounds__(kG2T, D == 16 ? 4 : 2)
wgrad2_kernel(const float *__restrict__ A, int lda, const float *__restrict__ G, int ldg, float *__restrict__ part,
              int M, int K, int N, int rows_per_split, int ntn, int tiles) {
    constexpr int IMG = kG2M * D;
    __shared__ __attribute__((aligned(16))) float lds[4 * IMG];
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int s = id / tiles, tile = id % tiles;
    const int k0 = (tile / ntn) * kG2M, n0 = (tile % ntn) * kG2M;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wr = (w >> 1) * 64, wc = (w & 1) * 64;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    const int rb = s * rows_per_split, re = min(M, rb + rows_per_split);
    const int ns = (re - rb + D - 1) / D;
    auto fill = [&](int sl, int buf) {
        float *Ai = lds + buf * 2 * IMG, *Gi = Ai + IMG;
        const int r0 = rb + sl * D;
        if (r0 + D <= re) {
            fill_omajor<D>(Ai, A, lda, k0, K, r0, re);
            fill_omajor<D>(Gi, G, ldg, n0, N, r0, re);
        } else {
            fill_omajor_zero<D>(Ai, A, lda, k0, K, r0, re);
            fill_omajor_zero<D>(Gi, G, ldg, n0, N, r0, re);
        }
    };
    if (ns > 0) {
        fill(0, 0);
        wait_vmcnt<0>();
        barrier_lds();
    }
    for (int sl = 0; sl < ns; ++sl) {
        const int buf = sl & 1;
        if (sl + 1 < ns) fill(sl + 1, buf ^ 1);  // lands while slab sl is multiplied
        const float *Ai = lds + buf * 2 * IMG;
        mfma_slab<D, false, false>(Ai, Ai + IMG, wr, wc, acc);
        __builtin_amdgcn_sched_barrier(0);
        wait_vmcnt<0>();
        barrier_lds();
    }
    float *P = part + (size_t)s * K * N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = n0 + wc + 32 * j + (lane & 31);
            if (col >= N) continue;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = k0 + wr + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
                if (row < K) P[(size_t)row * N + col] = acc[i][j][reg];
            }
        }
}

static bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace msat

using namespace msat;

// Fast-path predicates and launches (called from gemm.hip's C-ABI entry points).
// Slab depth 16 (32 KiB LDS, 3 workgroups per CU) and a double buffer: depth 32 and a third stage
// measured equal or slower in round 1.

bool msat_gemm2_ok(const float *A, int lda, const float *B, int ldb, int transB, int N, int K) {
    if (K % 32 || K == 0 || lda % 4 || ldb % 4 || !al16(A) || !al16(B)) return false;
    if (!transB && N % 4) return false;  // o-major B chunks are 4 columns wide
    return N >= 4;
}

int msat_gemm2_launch(const float *A, int lda, const float *B, int ldb, int transB, float *C, int ldc,
                      const float *bias, int M, int N, int K, int accumulate, hipStream_t s) {
    const int ntm = (M + kG2M - 1) / kG2M, ntn = (N + kG2M - 1) / kG2M;
    const dim3 grid(ntm * ntn), blk(kG2T);
    // float4 epilogue when whole 16-byte column chunks are addressable (else the scalar epilogue)
    const int vec = (N % 4 == 0 && ldc % 4 == 0 && al16(C) && (!bias || al16(bias))) ? 1 : 0;
    if (transB)
        hipLaunchKernelGGL((gemm2_kernel<16, true>), grid, blk, 0, s, A, lda, B, ldb, C, ldc, bias, M, N, K, accumulate,
                           ntn, vec);
    else
        hipLaunchKernelGGL((gemm2_kernel<16, false>), grid, blk, 0, s, A, lda, B, ldb, C, ldc, bias, M, N, K,
                           accumulate, ntn, vec);
    return check_launch("gemm2_kernel");
}

bool msat_wgrad2_ok(const float *A, int lda, const float *G, int ldg, int K, int N) {
    return K % 4 == 0 && N % 4 == 0 && K >= 4 && N >= 4 && lda % 4 == 0 && ldg % 4 == 0 && al16(A) && al16(G);
}

int msat_wgrad2_launch(const float *A, int lda, const float *G, int ldg, float *part, int M, int K, int N, int splits,
                       int rows_per_split, hipStream_t s) {
    const int ntk = (K + kG2M - 1) / kG2M, ntn = (N + kG2M - 1) / kG2M;
    const int tiles = ntk * ntn;
    hipLaunchKernelGGL((wgrad2_kernel<16>), dim3(tiles * splits), dim3(kG2T), 0, s, A, lda, G, ldg, part, M, K, N,
                       rows_per_split, ntn, tiles);
    return check_launch("wgrad2_kernel");
}
