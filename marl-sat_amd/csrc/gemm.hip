// fp32 GEMMs on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact fp32, a
// k-ordered fmaf chain per output -- the 1e-5 parity bar rules out bf16/xf32).
//
//   msat_gemm        C[M,N] (+)= A[M,K] @ op(B) (+ bias[N])      op(B) = B[K,N] or B[N,K]^T
//   msat_gemm_wgrad  W[K,N] (+)= A[M,K]^T @ G[M,N]                (weight gradients, M huge)
//
// One 256-thread workgroup computes a 128x128 output tile; wave w owns the 64x64
// quadrant (w>>1, w&1) as 2x2 MFMA 32x32 tiles (64 accumulator registers).  The
// reduction dimension is staged through LDS 16 deep, k-major on both operands
// ([red][out], rows padded to 132 words: conflict-free ds_read_b32 operand fetches),
// double-buffered with the next slab held in registers while the current one is
// consumed.  The weight-gradient GEMM splits M over `splits` workgroups per output
// tile, writes fp32 partial slabs and reduces them in a fixed order
// (bitwise reproducible, no float atomics).
#include <algorithm>
#include <stdlib.h>

#include <atomic>
#include <cstring>

#include "common.h"

namespace msat {

constexpr int kGT = 256;      // threads
constexpr int kTM = 128;      // output tile rows
constexpr int kTN = 128;      // output tile cols
constexpr int kKS = 16;       // reduction slab depth
constexpr int kLdsLd = 132;   // padded LDS row (words)

typedef float f32x16 __attribute__((ext_vector_type(16)));

// One operand slab: LDS[r][o] for r < 16 (reduction), o < 128 (output index).
// src(o, r) addressing is either "direct" (src[r][o], row-major over the reduction
// index) or "transposed" (src[o][r]).  Each thread moves 8 elements.
struct Slab {
    float v[8];
};

__device__ __forceinline__ void load_slab(Slab &s, const float *__restrict__ src, int ld, bool trans, int o0, int omax,
                                          int r0, int rmax, bool vec_ok) {
    const int t = threadIdx.x;
    if (!trans) {
        // direct: thread -> (r = t>>4, o = (t&15)*8 .. +8): 8 consecutive outputs of one reduction row
        const int r = r0 + (t >> 4), o = o0 + (t & 15) * 8;
        const float *p = src + (size_t)r * ld + o;
        if (r < rmax && vec_ok && o + 8 <= omax) {
            const float4 a = *reinterpret_cast<const float4 *>(p);
            const float4 b = *reinterpret_cast<const float4 *>(p + 4);
            s.v[0] = a.x; s.v[1] = a.y; s.v[2] = a.z; s.v[3] = a.w;
            s.v[4] = b.x; s.v[5] = b.y; s.v[6] = b.z; s.v[7] = b.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) s.v[j] = (r < rmax && o + j < omax) ? p[j] : 0.0f;
        }
    } else {
        // transposed: thread -> (o = t>>1, r = (t&1)*8 .. +8): 8 consecutive reduction elems of one output row
        const int o = o0 + (t >> 1), r = r0 + (t & 1) * 8;
        const float *p = src + (size_t)o * ld + r;
        if (o < omax && vec_ok && r + 8 <= rmax) {
            const float4 a = *reinterpret_cast<const float4 *>(p);
            const float4 b = *reinterpret_cast<const float4 *>(p + 4);
            s.v[0] = a.x; s.v[1] = a.y; s.v[2] = a.z; s.v[3] = a.w;
            s.v[4] = b.x; s.v[5] = b.y; s.v[6] = b.z; s.v[7] = b.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) s.v[j] = (o < omax && r + j < rmax) ? p[j] : 0.0f;
        }
    }
}

__device__ __forceinline__ void store_slab(const Slab &s, float *lds, bool trans) {
    const int t = threadIdx.x;
    if (!trans) {
        float *q = lds + (t >> 4) * kLdsLd + (t & 15) * 8;
        *reinterpret_cast<float4 *>(q) = make_float4(s.v[0], s.v[1], s.v[2], s.v[3]);
        *reinterpret_cast<float4 *>(q + 4) = make_float4(s.v[4], s.v[5], s.v[6], s.v[7]);
    } else {
        const int o = t >> 1, r = (t & 1) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) lds[(r + j) * kLdsLd + o] = s.v[j];
    }
}

// acc[i][j] += As[:, wr+32i ..] x Bs[:, wc+32j ..] over one 16-deep slab
__device__ __forceinline__ void mfma_slab(const float *As, const float *Bs, int wr, int wc, f32x16 (&acc)[2][2]) {
    const int lane = threadIdx.x & 63;
    const int li = lane & 31, lk = lane >> 5;
#pragma unroll
    for (int kk = 0; kk < kKS; kk += 2) {
        const float *a = As + (kk + lk) * kLdsLd + wr + li;
        const float *b = Bs + (kk + lk) * kLdsLd + wc + li;
        const float a0 = a[0], a1 = a[32], b0 = b[0], b1 = b[32];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
}

// Generic tile: out[o_a][o_b] = sum_r SA(o_a, r) * SB(o_b, r) for r in [rbeg, rend)
__device__ __forceinline__ void tile_accumulate(const float *__restrict__ A, int lda, bool transA, int oa0, int oamax,
                                                const float *__restrict__ B, int ldb, bool transB, int ob0, int obmax,
                                                int rbeg, int rend, bool vecA, bool vecB, f32x16 (&acc)[2][2],
                                                float *lds) {
    float *As[2] = {lds, lds + kKS * kLdsLd};
    float *Bs[2] = {lds + 2 * kKS * kLdsLd, lds + 3 * kKS * kLdsLd};
    const int w = threadIdx.x >> 6;
    const int wr = (w >> 1) * 64, wc = (w & 1) * 64;
    Slab sa, sb;
    if (rbeg >= rend) return;
    load_slab(sa, A, lda, transA, oa0, oamax, rbeg, rend, vecA);
    load_slab(sb, B, ldb, transB, ob0, obmax, rbeg, rend, vecB);
    store_slab(sa, As[0], transA);
    store_slab(sb, Bs[0], transB);
    __syncthreads();
    int buf = 0;
    for (int r = rbeg; r < rend; r += kKS) {
        const bool more = r + kKS < rend;
        if (more) {
            load_slab(sa, A, lda, transA, oa0, oamax, r + kKS, rend, vecA);
            load_slab(sb, B, ldb, transB, ob0, obmax, r + kKS, rend, vecB);
        }
        mfma_slab(As[buf], Bs[buf], wr, wc, acc);
        if (more) {
            store_slab(sa, As[buf ^ 1], transA);
            store_slab(sb, Bs[buf ^ 1], transB);
        }
        __syncthreads();
        buf ^= 1;
    }
}

// C[M,N] (+)= A[M,K] @ op(B) + bias   (A is "transposed" in slab terms: o = m, r = k)
__global__ void __launch_bounds__(kGT)
gemm_kernel(const float *__restrict__ A, int lda, const float *__restrict__ B, int ldb, int transB,
            float *__restrict__ C, int ldc, const float *__restrict__ bias, int M, int N, int K, int accumulate) {
    __shared__ __attribute__((aligned(16))) float lds[4 * kKS * kLdsLd];
    const int m0 = blockIdx.x * kTM, n0 = blockIdx.y * kTN;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    const bool vecA = (lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
    const bool vecB = (ldb % 4 == 0) && ((reinterpret_cast<uintptr_t>(B) & 15) == 0);
    // slab terms: A(o=m, r=k) is src[m][k] -> transposed; B(o=n, r=k): B[k][n] direct, B[n][k] transposed
    tile_accumulate(A, lda, true, m0, M, B, ldb, transB != 0, n0, N, 0, K, vecA, vecB, acc, lds);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wr = m0 + (w >> 1) * 64, wc = n0 + (w & 1) * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = wc + 32 * j + (lane & 31);
            if (col >= N) continue;
            const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = wr + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
                if (row >= M) continue;
                float *c = C + (size_t)row * ldc + col;
                const float v = acc[i][j][reg] + bv;
                *c = accumulate ? *c + v : v;
            }
        }
}

// partial[s][k][n] = sum_{m in split s} A[m][k] G[m][n]   (A(o=k, r=m) direct, G(o=n, r=m) direct)
__global__ void __launch_bounds__(kGT)
gemm_wgrad_kernel(const float *__restrict__ A, int lda, const float *__restrict__ G, int ldg, float *__restrict__ part,
                  int M, int K, int N, int rows_per_split) {
    __shared__ __attribute__((aligned(16))) float lds[4 * kKS * kLdsLd];
    const int k0 = blockIdx.x * kTM, n0 = blockIdx.y * kTN, s = blockIdx.z;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    const bool vecA = (lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
    const bool vecG = (ldg % 4 == 0) && ((reinterpret_cast<uintptr_t>(G) & 15) == 0);
    const int rb = s * rows_per_split, re = min(M, rb + rows_per_split);
    tile_accumulate(A, lda, false, k0, K, G, ldg, false, n0, N, rb, re, vecA, vecG, acc, lds);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wr = k0 + (w >> 1) * 64, wc = n0 + (w & 1) * 64;
    float *P = part + (size_t)s * K * N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = wc + 32 * j + (lane & 31);
            if (col >= N) continue;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = wr + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
                if (row < K) P[(size_t)row * N + col] = acc[i][j][reg];
            }
        }
}

// float4 form (N % 4 == 0, 16-byte aligned W rows): 8 independent loads in flight per thread
__global__ void wgrad_reduce4_kernel(const float4 *__restrict__ part, int splits, int K, int N4, float4 *__restrict__ W,
                                     int ldw4, int accumulate) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t KN4 = (size_t)K * N4;
    if (t >= (int)KN4) return;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    int i = 0;
    for (; i + 8 <= splits; i += 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(i + u) * KN4 + t];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
        }
    }
    for (; i < splits; ++i) {
        const float4 v = part[(size_t)i * KN4 + t];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    const int k = t / N4, n4 = t - k * N4;
    float4 *w = W + (size_t)k * ldw4 + n4;
    if (accumulate) {
        const float4 o = *w;
        a.x = o.x + a.x; a.y = o.y + a.y; a.z = o.z + a.z; a.w = o.w + a.w;
    }
    *w = a;
}

// Two wgrad_reduce4 launches in one (a GRU cell's dual weight gradient): blocks [0, nb0) reduce segment 0,
// the rest segment 1; per element the same adds in the same order as wgrad_reduce4_kernel.
struct Reduce4Seg {
    const float4 *part;
    float4 *W;
    int splits, K, N4, ldw4, accumulate, blocks;
};
__global__ void wgrad_reduce4_dual_kernel(Reduce4Seg s0, Reduce4Seg s1) {
    const bool second = (int)blockIdx.x >= s0.blocks;
    const Reduce4Seg &q = second ? s1 : s0;
    const int t = (blockIdx.x - (second ? s0.blocks : 0)) * blockDim.x + threadIdx.x;
    const size_t KN4 = (size_t)q.K * q.N4;
    if (t >= (int)KN4) return;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    int i = 0;
    for (; i + 8 <= q.splits; i += 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = q.part[(size_t)(i + u) * KN4 + t];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
        }
    }
    for (; i < q.splits; ++i) {
        const float4 v = q.part[(size_t)i * KN4 + t];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    const int k = t / q.N4, n4 = t - k * q.N4;
    float4 *w = q.W + (size_t)k * q.ldw4 + n4;
    if (q.accumulate) {
        const float4 o = *w;
        a.x = o.x + a.x; a.y = o.y + a.y; a.z = o.z + a.z; a.w = o.w + a.w;
    }
    *w = a;
}

// W[k][n] (+)= sum_s part[s][k][n]  (fixed split order -> reproducible)
__global__ void wgrad_reduce_kernel(const float *__restrict__ part, int splits, int K, int N, float *__restrict__ W,
                                    int ldw, int accumulate) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= K * N) return;
    float s = 0.0f;
    for (int i = 0; i < splits; ++i) s += part[(size_t)i * K * N + t];
    const int k = t / N, n = t - k * N;
    float *w = W + (size_t)k * ldw + n;
    *w = accumulate ? *w + s : s;
}

// Skinny weight gradient (K <= 8: input features, degree columns): a 128-row MFMA tile
// would multiply 32x more zeros than data, so this is a streaming reduction over G instead.
// Block (colblock, split): 16 column float4s x 16 row lanes; each thread keeps K float4
// accumulators over its rows (fixed order), the 16 row lanes combine through LDS in a fixed
// order, and part[split][k][n] is reduced by skinny_reduce4_kernel (fixed split order).
constexpr int kSkinnyK = 8;

template <bool AV>
__global__ void __launch_bounds__(256)
wgrad_skinny_kernel(const float *__restrict__ A, int lda, const float4 *__restrict__ G, int ldg4, int M, int K, int N4,
                    int rows_per, float4 *__restrict__ part) {
    constexpr int U = 4;  // rows in flight per thread (independent loads issued before use)
    __shared__ float4 red[16][16];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + tx;
    const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
    float4 acc[kSkinnyK];
#pragma unroll
    for (int k = 0; k < kSkinnyK; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < N4) {
        int r = r0 + ty;
        for (; r + 16 * (U - 1) < r1; r += 16 * U) {
            float4 g[U];
            float a[U][kSkinnyK];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int rr = r + 16 * u;
                g[u] = G[(size_t)rr * ldg4 + c];
                const float *ap = A + (size_t)rr * lda;
                if (AV) {
                    const float4 a0 = *reinterpret_cast<const float4 *>(ap);
                    a[u][0] = a0.x; a[u][1] = a0.y; a[u][2] = a0.z; a[u][3] = a0.w;
                    if (K > 4) {
                        const float4 a1 = *reinterpret_cast<const float4 *>(ap + 4);
                        a[u][4] = a1.x; a[u][5] = a1.y; a[u][6] = a1.z; a[u][7] = a1.w;
                    } else {
                        a[u][4] = a[u][5] = a[u][6] = a[u][7] = 0.0f;
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < kSkinnyK; ++k) a[u][k] = k < K ? ap[k] : 0.0f;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int k = 0; k < kSkinnyK; ++k) {
                    const float av = a[u][k];
                    acc[k].x += av * g[u].x; acc[k].y += av * g[u].y; acc[k].z += av * g[u].z; acc[k].w += av * g[u].w;
                }
        }
        for (; r < r1; r += 16) {
            const float4 g = G[(size_t)r * ldg4 + c];
            const float *ap = A + (size_t)r * lda;
#pragma unroll
            for (int k = 0; k < kSkinnyK; ++k)
                if (k < K) {
                    const float av = ap[k];
                    acc[k].x += av * g.x; acc[k].y += av * g.y; acc[k].z += av * g.z; acc[k].w += av * g.w;
                }
        }
    }
#pragma unroll
    for (int k = 0; k < kSkinnyK; ++k) {
        if (k >= K) break;
        red[ty][tx] = acc[k];
        __syncthreads();
        if (ty == 0 && c < N4) {
            float4 t = red[0][tx];
            for (int j = 1; j < 16; ++j) {
                const float4 v = red[j][tx];
                t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
            }
            part[((size_t)blockIdx.y * K + k) * N4 + c] = t;
        }
        __syncthreads();
    }
}

// W[k][n] (+)= sum_s part[s][k][n]: 16 output float4s x 16 split lanes per block, fixed order.
__global__ void __launch_bounds__(256)
skinny_reduce4_kernel(const float4 *__restrict__ part, int splits, int KN4, int N4, float4 *__restrict__ W, int ldw4,
                      int accumulate) {
    __shared__ float4 red[16][16];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + tx;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < KN4)
        for (int s = ty; s < splits; s += 16) {
            const float4 v = part[(size_t)s * KN4 + c];
            a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
    red[ty][tx] = a;
    __syncthreads();
    if (ty == 0 && c < KN4) {
        float4 t = red[0][tx];
        for (int j = 1; j < 16; ++j) {
            const float4 v = red[j][tx];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        const int k = c / N4, n4 = c - k * N4;
        float4 *w = W + (size_t)k * ldw4 + n4;
        if (accumulate) {
            const float4 o = *w;
            t.x = o.x + t.x; t.y = o.y + t.y; t.z = o.z + t.z; t.w = o.w + t.w;
        }
        *w = t;
    }
}

static int skinny_splits(int M, int N) {
    const int cb = std::max(1, (N / 4 + 15) / 16);
    return std::max(1, std::min((M + 63) / 64, std::max(1, 1024 / cb)));
}

static bool skinny_ok(const float *G, int ldg, const float *W, int ldw, int K, int N) {
    return K <= kSkinnyK && N % 4 == 0 && ldg % 4 == 0 && ldw % 4 == 0 &&
           (reinterpret_cast<uintptr_t>(G) & 15) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0;
}

// at most 768 workgroups (3 per CU: the x3 weight gradient's occupancy), >= ~1024 rows per split
static int wgrad_splits(int M, int K, int N) {
    constexpr int budget = 768;
    const int tiles = ((K + kTM - 1) / kTM) * ((N + kTN - 1) / kTN);
    return std::max(1, std::min(budget / std::max(tiles, 1), (M + 1023) / 1024));
}

}  // namespace msat

using namespace msat;

// LDS-DMA fast path (gemm2.hip); the register-staged kernels here take the shapes it cannot.
bool msat_gemm2_ok(const float *A, int lda, const float *B, int ldb, int transB, int N, int K);
int msat_gemm2_launch(const float *A, int lda, const float *B, int ldb, int transB, float *C, int ldc,
                      const float *bias, int M, int N, int K, int accumulate, hipStream_t s);
bool msat_wgrad2_ok(const float *A, int lda, const float *G, int ldg, int K, int N);
bool msat_wgrad_x3_ok(const float *A, int lda, const float *G, int ldg, int K, int N);
bool msat_wgrad_x3w_ok(const float *A, int lda, const float *G, int ldg, int K, int N);
int msat_wgrad_x3w_splits(int M, int K);
int msat_wgrad_x3w_launch(const float *A, int lda, const float *G, int ldg, float *part, int M, int K, int N, int rot,
                          int splits, hipStream_t s);
int msat_wgrad_dual_splits(int M, int K0, int K1);
int msat_wgrad_h2_dual_launch(const float *A0, int lda0, const float *G0, int ldg0, float *part0, int K0, int N0, int rot0,
                              const float *A1, int lda1, const float *G1, int ldg1, float *part1, int K1, int N1,
                              int rot1, const int *rexp, int M, int splits, int *flags, hipStream_t s);
int msat_wgrad_h2_dual_pl_launch(const float *A0, int lda0, const void *G0, int ldg0, float *part0, int K0, int N0,
                                 int rot0, const float *A1, int lda1, const void *G1, int ldg1, float *part1, int K1,
                                 int N1, int rot1, int plo, const int *rexp, int M, int splits, int *flags,
                                 hipStream_t s);
int msat_wgrad_h2w_launch(const float *A, int lda, const float *G, int ldg, const int *rexp, float *part, int M, int K,
                          int N, int rot, int splits, int *flags, hipStream_t s);
int msat_wgrad_x3_launch(const float *A, int lda, const float *G, int ldg, float *part, int M, int K, int N, int splits,
                         int rows_per_split, hipStream_t s);

// The arithmetic path (msat_set_precision): MSAT_PRECISION_FP32 (the accuracy reference path, README)
// keeps the weight gradients on fp32 MFMA; the other two run the fp32-accurate split kernels.  Until a
// host sets it, MARLSAT_PRECISION is read ONCE; an unknown value there is kept as an error state
// (kPrecisionBad), so every weight gradient fails loudly instead of silently picking a path.
constexpr int kPrecisionUnset = -100, kPrecisionBad = -101;
static std::atomic<int> g_precision{kPrecisionUnset};

static int precision_from_env() {
    const char *e = getenv("MARLSAT_PRECISION");
    if (!e || !*e || std::strcmp(e, "fp16x2") == 0) return MSAT_PRECISION_FP16X2;
    if (std::strcmp(e, "bf16x3") == 0) return MSAT_PRECISION_BF16X3;
    if (std::strcmp(e, "fp32") == 0) return MSAT_PRECISION_FP32;
    return kPrecisionBad;
}

static int precision_mode() {
    int p = g_precision.load(std::memory_order_relaxed);
    if (p == kPrecisionUnset) {
        int expect = kPrecisionUnset;
        g_precision.compare_exchange_strong(expect, precision_from_env());
        p = g_precision.load(std::memory_order_relaxed);
    }
    return p;
}

#define MSAT_REQUIRE_PRECISION(pm)                                                                             \
    MSAT_REQUIRE((pm) >= 0, "MARLSAT_PRECISION=%s: expected fp16x2, bf16x3 or fp32 (or msat_set_precision)", \
                 getenv("MARLSAT_PRECISION") ? getenv("MARLSAT_PRECISION") : "")
int msat_wgrad2_launch(const float *A, int lda, const float *G, int ldg, float *part, int M, int K, int N, int splits,
                       int rows_per_split, hipStream_t s);

// Small fp32 products accumulated in fp64 and rounded once (gnn.py phi folding: F = W Wi and its
// unfolding dW = dF Wi^T, dWi = W^T dF).  F multiplies every row of every message step, so a
// plain fp32 GEMM's rounding of F is a systematic weight perturbation that the 16 GRU + LayerNorm
// steps accumulate coherently (critic values ~4x the reference order's error at L = 16,
// tests/probe_value_error.py); rounded once from fp64, F is as accurate as the weights themselves.
// One thread per output element; the operands are at most a few hundred rows (microseconds).
__global__ void __launch_bounds__(256)
gemm_f64acc_kernel(const float *__restrict__ A, int lda, int transA, const float *__restrict__ B, int ldb, int transB,
                   float *__restrict__ C, int ldc, int M, int N, int K, int accumulate) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
    if (n >= N) return;
    double acc = accumulate ? (double)C[(size_t)m * ldc + n] : 0.0;
    for (int k = 0; k < K; ++k) {
        const double a = transA ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k];
        const double b = transB ? B[(size_t)n * ldb + k] : B[(size_t)k * ldb + n];
        acc = fma(a, b, acc);
    }
    C[(size_t)m * ldc + n] = (float)acc;
}

extern "C" int msat_gemm_f64acc(const float *A, int32_t lda, int32_t transA, const float *B, int32_t ldb,
                                int32_t transB, float *C, int32_t ldc, int32_t M, int32_t N, int32_t K,
                                int32_t accumulate, void *stream) {
    MSAT_REQUIRE(A && B && C, "NULL operand");
    MSAT_REQUIRE(M >= 0 && M <= 65535 && N >= 1 && K >= 0, "bad dims M=%d N=%d K=%d", M, N, K);
    MSAT_REQUIRE(lda >= (transA ? M : K) && ldb >= (transB ? K : N) && ldc >= N, "leading dims too small");
    if (M == 0) return MSAT_OK;
    hipLaunchKernelGGL(gemm_f64acc_kernel, dim3((N + 255) / 256, M), dim3(256), 0, (hipStream_t)stream, A, lda,
                       transA, B, ldb, transB, C, ldc, M, N, K, accumulate);
    return check_launch("gemm_f64acc_kernel");
}

extern "C" int msat_gemm(const float *A, int32_t lda, const float *B, int32_t ldb, int32_t transB, float *C,
                         int32_t ldc, const float *bias, int32_t M, int32_t N, int32_t K, int32_t accumulate,
                         void *stream) {
    MSAT_REQUIRE(A && B && C, "NULL operand");
    MSAT_REQUIRE(M >= 0 && N >= 1 && K >= 0, "bad dims M=%d N=%d K=%d", M, N, K);
    MSAT_REQUIRE(lda >= K && ldc >= N && ldb >= (transB ? K : N), "leading dims too small");
    if (M == 0) return MSAT_OK;
    if (msat_gemm2_ok(A, lda, B, ldb, transB, N, K))
        return msat_gemm2_launch(A, lda, B, ldb, transB, C, ldc, bias, M, N, K, accumulate, (hipStream_t)stream);
    dim3 grid((M + kTM - 1) / kTM, (N + kTN - 1) / kTN);
    hipLaunchKernelGGL(gemm_kernel, grid, dim3(kGT), 0, (hipStream_t)stream, A, lda, B, ldb, transB, C, ldc, bias, M,
                       N, K, accumulate);
    return check_launch("gemm_kernel");
}

constexpr size_t kWgradFlagBytes = 1024 * sizeof(int);  // >= 256 workgroups' flags

extern "C" size_t msat_gemm_wgrad_workspace_bytes(int32_t M, int32_t K, int32_t N) {
    const size_t sp = std::max({wgrad_splits(M, K, N), K <= kSkinnyK ? skinny_splits(M, N) : 0,
                                msat_wgrad_x3w_splits(M, K)});
    size_t floats = sp * K * N;
    // msat_gemm_wgrad_rot's tiled fallback runs two narrower products (N - rot and rot columns) in the
    // same workspace, and narrower products take more splits: size for the widest need of any width
    for (int n = 1; n < N; ++n) floats = std::max(floats, (size_t)wgrad_splits(M, K, n) * K * n);
    return floats * sizeof(float) + kWgradFlagBytes;  // + the fp16x2 kernel's workgroup flags
}

static int wgrad_reduce(const float *part, int splits, int K, int N, float *W, int ldw, int accumulate, hipStream_t s) {
    if (N % 4 == 0 && ldw % 4 == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(part) & 15) == 0) {
        const int n4 = N / 4;
        hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3((K * n4 + 255) / 256), dim3(256), 0, s,
                           (const float4 *)part, splits, K, n4, (float4 *)W, ldw / 4, accumulate);
        return check_launch("wgrad_reduce4_kernel");
    }
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((K * N + 255) / 256), dim3(256), 0, s, part, splits, K, N, W, ldw,
                       accumulate);
    return check_launch("wgrad_reduce_kernel");
}

extern "C" int msat_gemm_wgrad(const float *A, int32_t lda, const float *G, int32_t ldg, float *W, int32_t ldw,
                               int32_t M, int32_t K, int32_t N, int32_t accumulate, void *workspace, void *stream) {
    MSAT_REQUIRE(A && G && W && workspace, "NULL operand");
    MSAT_REQUIRE(M >= 0 && K >= 1 && N >= 1 && lda >= K && ldg >= N && ldw >= N, "bad dims");
    const int pm = precision_mode();
    MSAT_REQUIRE_PRECISION(pm);
    const bool x3 = pm != MSAT_PRECISION_FP32;
    hipStream_t s = (hipStream_t)stream;
    if (x3 && K > kSkinnyK && msat_wgrad_x3w_ok(A, lda, G, ldg, K, N)) {
        const int splits = msat_wgrad_x3w_splits(M, K);
        const int rc = msat_wgrad_x3w_launch(A, lda, G, ldg, (float *)workspace, M, K, N, 0, splits, s);
        if (rc) return rc;
        return wgrad_reduce((const float *)workspace, splits, K, N, W, ldw, accumulate, s);
    }
    if (skinny_ok(G, ldg, W, ldw, K, N) && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0) {
        const int sp = skinny_splits(M, N), rows_per = (M + sp - 1) / sp, N4 = N / 4;
        float4 *ws4 = reinterpret_cast<float4 *>(workspace);
        const bool av = lda % 4 == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0;
        if (av)
            hipLaunchKernelGGL((wgrad_skinny_kernel<true>), dim3((N4 + 15) / 16, sp), dim3(256), 0, s, A, lda,
                               reinterpret_cast<const float4 *>(G), ldg / 4, M, K, N4, rows_per, ws4);
        else
            hipLaunchKernelGGL((wgrad_skinny_kernel<false>), dim3((N4 + 15) / 16, sp), dim3(256), 0, s, A, lda,
                               reinterpret_cast<const float4 *>(G), ldg / 4, M, K, N4, rows_per, ws4);
        const int rc = check_launch("wgrad_skinny_kernel");
        if (rc) return rc;
        hipLaunchKernelGGL(skinny_reduce4_kernel, dim3((K * N4 + 15) / 16), dim3(256), 0, s, ws4, sp, K * N4, N4,
                           reinterpret_cast<float4 *>(W), ldw / 4, accumulate);
        return check_launch("skinny_reduce4_kernel");
    }
    const int splits = wgrad_splits(M, K, N);
    const int rows = (M + splits - 1) / splits;
    int rc;
    if (x3 && msat_wgrad_x3_ok(A, lda, G, ldg, K, N)) {
        const int rows16 = ((rows + 15) / 16) * 16;
        rc = msat_wgrad_x3_launch(A, lda, G, ldg, (float *)workspace, M, K, N, splits, rows16, s);
    } else if (msat_wgrad2_ok(A, lda, G, ldg, K, N)) {
        const int rows32 = ((rows + 31) / 32) * 32;
        rc = msat_wgrad2_launch(A, lda, G, ldg, (float *)workspace, M, K, N, splits, rows32, s);
    } else {
        const int rows16 = ((rows + kKS - 1) / kKS) * kKS;
        dim3 grid((K + kTM - 1) / kTM, (N + kTN - 1) / kTN, splits);
        hipLaunchKernelGGL(gemm_wgrad_kernel, grid, dim3(kGT), 0, s, A, lda, G, ldg, (float *)workspace, M, K, N,
                           rows16);
        rc = check_launch("gemm_wgrad_kernel");
    }
    if (rc) return rc;
    return wgrad_reduce((const float *)workspace, splits, K, N, W, ldw, accumulate, s);
}

// W[:, (n + rot) % N] (+)= (A^T G)[:, n]: the packed backward rows' gate blocks (n | r | z) into a
// weight stored (r | z | n).  The whole-row kernel rotates in its partial store; otherwise two
// column ranges of the plain product.
extern "C" int msat_gemm_wgrad_rot(const float *A, int32_t lda, const float *G, int32_t ldg, float *W, int32_t ldw,
                                   int32_t M, int32_t K, int32_t N, int32_t rot, int32_t accumulate, void *workspace,
                                   void *stream) {
    MSAT_REQUIRE(rot >= 0 && rot < N, "gemm_wgrad_rot: rot must be in [0, N)");
    if (rot == 0) return msat_gemm_wgrad(A, lda, G, ldg, W, ldw, M, K, N, accumulate, workspace, stream);
    MSAT_REQUIRE(A && G && W && workspace, "NULL operand");
    MSAT_REQUIRE(M >= 0 && K >= 1 && N >= 1 && lda >= K && ldg >= N && ldw >= N, "bad dims");
    const int pm = precision_mode();
    MSAT_REQUIRE_PRECISION(pm);
    hipStream_t s = (hipStream_t)stream;
    if (pm != MSAT_PRECISION_FP32 && K > kSkinnyK && rot % 4 == 0 && msat_wgrad_x3w_ok(A, lda, G, ldg, K, N)) {
        const int splits = msat_wgrad_x3w_splits(M, K);
        const int rc = msat_wgrad_x3w_launch(A, lda, G, ldg, (float *)workspace, M, K, N, rot, splits, s);
        if (rc) return rc;
        return wgrad_reduce((const float *)workspace, splits, K, N, W, ldw, accumulate, s);
    }
    const int rc = msat_gemm_wgrad(A, lda, G, ldg, W + rot, ldw, M, K, N - rot, accumulate, workspace, stream);
    if (rc) return rc;
    return msat_gemm_wgrad(A, lda, G + (N - rot), ldg, W, ldw, M, K, rot, accumulate, workspace, stream);
}

// fp16x2 whole-row weight gradient of a GRU backward's packed rows: G's rows carry scale exponents
// (rexp, msat_gru_ln_bwd_g4fe), A is range-checked (a workgroup that sees |a| >= 2^15 is recomputed
// in bf16x3).  Same product and rotation as msat_gemm_wgrad_rot.
extern "C" int msat_gemm_wgrad_h2(const float *A, int32_t lda, const float *G, int32_t ldg, const int32_t *rexp,
                                  float *W, int32_t ldw, int32_t M, int32_t K, int32_t N, int32_t rot,
                                  int32_t accumulate, void *workspace, void *stream) {
    MSAT_REQUIRE(A && G && W && rexp && workspace, "NULL operand");
    MSAT_REQUIRE(M >= 0 && K > kSkinnyK && N >= 1 && N <= 384 && lda >= K && ldg >= N && ldw >= N,
                 "gemm_wgrad_h2: bad dims (K > 8, N <= 384)");
    MSAT_REQUIRE(rot >= 0 && rot < N && rot % 4 == 0, "gemm_wgrad_h2: rot must be in [0, N), a multiple of 4");
    MSAT_REQUIRE(msat_wgrad_x3_ok(A, lda, G, ldg, K, N) && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0,
                 "gemm_wgrad_h2: K %% 4, N %% 4, ld %% 4 and 16-byte aligned operands required");
    hipStream_t s = (hipStream_t)stream;
    const int splits = msat_wgrad_x3w_splits(M, K);
    float *part = (float *)workspace;
    int *flags = reinterpret_cast<int *>(part + (size_t)splits * K * N);
    const int rc = msat_wgrad_h2w_launch(A, lda, G, ldg, rexp, part, M, K, N, rot, splits, flags, s);
    if (rc) return rc;
    return wgrad_reduce(part, splits, K, N, W, ldw, accumulate, s);
}

extern "C" size_t msat_gemm_wgrad_dual_workspace_bytes(int32_t M, int32_t K0, int32_t N0, int32_t K1, int32_t N1) {
    const size_t sp = msat_wgrad_dual_splits(M, K0, K1);
    return sp * ((size_t)K0 * N0 + (size_t)K1 * N1) * sizeof(float) + kWgradFlagBytes;
}

// W0 (+)= A0^T G0 and W1 (+)= A1^T G1 (each with its column rotation) over the same M rows of G's buffer,
// whose row exponents are rexp, in one fp16x2 launch (+ fixup) and two fixed-order reduces: a GRU cell's
// hidden and input weight gradients from its packed backward rows.  Conditions of msat_gemm_wgrad_h2.
// pl: G0 / G1 are fp16x2 planes (ldg in fp16 elements, lo plane plo elements after hi), else fp32 rows
static int wgrad_h2_dual_impl(const float *A0, int32_t lda0, const void *G0, int32_t ldg0, float *W0, int32_t ldw0,
                              int32_t K0, int32_t N0, int32_t rot0, const float *A1, int32_t lda1, const void *G1,
                              int32_t ldg1, float *W1, int32_t ldw1, int32_t K1, int32_t N1, int32_t rot1, int pl,
                              int32_t plo, const int32_t *rexp, int32_t M, int32_t accumulate, void *workspace,
                              void *stream) {
    MSAT_REQUIRE(A0 && G0 && W0 && A1 && G1 && W1 && rexp && workspace, "NULL operand");
    const int Ks[2] = {K0, K1}, Ns[2] = {N0, N1}, rots[2] = {rot0, rot1}, ldas[2] = {lda0, lda1},
              ldgs[2] = {ldg0, ldg1}, ldws[2] = {ldw0, ldw1};
    const float *As[2] = {A0, A1};
    const void *Gs[2] = {G0, G1};
    for (int i = 0; i < 2; ++i) {
        MSAT_REQUIRE(M >= 0 && Ks[i] > kSkinnyK && Ns[i] >= 1 && Ns[i] <= 384 && ldas[i] >= Ks[i] && ldgs[i] >= Ns[i] &&
                         ldws[i] >= Ns[i],
                     "gemm_wgrad_h2_dual: bad dims (K > 8, N <= 384)");
        MSAT_REQUIRE(rots[i] >= 0 && rots[i] < Ns[i] && rots[i] % 4 == 0, "gemm_wgrad_h2_dual: bad rot");
        if (pl)  // whole 16-byte chunks of both planes (the DMA pieces)
            MSAT_REQUIRE(Ks[i] % 4 == 0 && Ns[i] % 8 == 0 && ldas[i] % 4 == 0 && ldgs[i] % 8 == 0 && plo % 8 == 0 &&
                             plo >= Ns[i] && plo + Ns[i] <= ldgs[i] && (reinterpret_cast<uintptr_t>(As[i]) & 15) == 0 &&
                             (reinterpret_cast<uintptr_t>(Gs[i]) & 15) == 0,
                         "gemm_wgrad_h2_dual_planes: K %% 4, N %% 8, lda %% 4, ldg %% 8, plo %% 8 (>= N, plo + N <= "
                         "ldg) and 16-byte aligned operands required");
        else
            MSAT_REQUIRE(msat_wgrad_x3_ok(As[i], ldas[i], (const float *)Gs[i], ldgs[i], Ks[i], Ns[i]),
                         "gemm_wgrad_h2_dual: K %% 4, N %% 4, ld %% 4 and 16-byte aligned operands required");
    }
    MSAT_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "gemm_wgrad_h2_dual: workspace alignment");
    hipStream_t s = (hipStream_t)stream;
    const int splits = msat_wgrad_dual_splits(M, K0, K1);
    float *part0 = (float *)workspace, *part1 = part0 + (size_t)splits * K0 * N0;
    int *flags = reinterpret_cast<int *>(part1 + (size_t)splits * K1 * N1);
    int rc = pl ? msat_wgrad_h2_dual_pl_launch(A0, lda0, G0, ldg0, part0, K0, N0, rot0, A1, lda1, G1, ldg1, part1, K1,
                                               N1, rot1, plo, rexp, M, splits, flags, s)
                : msat_wgrad_h2_dual_launch(A0, lda0, (const float *)G0, ldg0, part0, K0, N0, rot0, A1, lda1,
                                            (const float *)G1, ldg1, part1, K1, N1, rot1, rexp, M, splits, flags, s);
    if (rc) return rc;
    const bool v0 = N0 % 4 == 0 && ldw0 % 4 == 0 && (reinterpret_cast<uintptr_t>(W0) & 15) == 0;
    const bool v1 = N1 % 4 == 0 && ldw1 % 4 == 0 && (reinterpret_cast<uintptr_t>(W1) & 15) == 0;
    if (v0 && v1) {  // both reduces in one launch (one kernel boundary fewer per GRU cell)
        Reduce4Seg q[2];
        const float *parts[2] = {part0, part1};
        float *Ws[2] = {W0, W1};
        for (int i = 0; i < 2; ++i) {
            q[i].part = reinterpret_cast<const float4 *>(parts[i]);
            q[i].W = reinterpret_cast<float4 *>(Ws[i]);
            q[i].splits = splits;
            q[i].K = Ks[i];
            q[i].N4 = Ns[i] / 4;
            q[i].ldw4 = ldws[i] / 4;
            q[i].accumulate = accumulate;
            q[i].blocks = (int)(((size_t)Ks[i] * (Ns[i] / 4) + 255) / 256);
        }
        hipLaunchKernelGGL(wgrad_reduce4_dual_kernel, dim3(q[0].blocks + q[1].blocks), dim3(256), 0, s, q[0], q[1]);
        return check_launch("wgrad_reduce4_dual_kernel");
    }
    rc = wgrad_reduce(part0, splits, K0, N0, W0, ldw0, accumulate, s);
    if (rc) return rc;
    return wgrad_reduce(part1, splits, K1, N1, W1, ldw1, accumulate, s);
}

extern "C" int msat_gemm_wgrad_h2_dual(const float *A0, int32_t lda0, const float *G0, int32_t ldg0, float *W0,
                                       int32_t ldw0, int32_t K0, int32_t N0, int32_t rot0, const float *A1,
                                       int32_t lda1, const float *G1, int32_t ldg1, float *W1, int32_t ldw1,
                                       int32_t K1, int32_t N1, int32_t rot1, const int32_t *rexp, int32_t M,
                                       int32_t accumulate, void *workspace, void *stream) {
    return wgrad_h2_dual_impl(A0, lda0, G0, ldg0, W0, ldw0, K0, N0, rot0, A1, lda1, G1, ldg1, W1, ldw1, K1, N1, rot1, 0,
                              0, rexp, M, accumulate, workspace, stream);
}

// Same products with G0 / G1 the GRU backward's packed rows as fp16x2 planes (msat_gru_ln_bwd_g4fe, flags bit
// 3): ldg in fp16 elements (% 8), the lo plane plo elements after the hi plane, N % 8 == 0.  Workspace as
// msat_gemm_wgrad_dual_workspace_bytes.
extern "C" int msat_gemm_wgrad_h2_dual_planes(const float *A0, int32_t lda0, const void *G0, int32_t ldg0, float *W0,
                                              int32_t ldw0, int32_t K0, int32_t N0, int32_t rot0, const float *A1,
                                              int32_t lda1, const void *G1, int32_t ldg1, float *W1, int32_t ldw1,
                                              int32_t K1, int32_t N1, int32_t rot1, int32_t plo, const int32_t *rexp,
                                              int32_t M, int32_t accumulate, void *workspace, void *stream) {
    return wgrad_h2_dual_impl(A0, lda0, G0, ldg0, W0, ldw0, K0, N0, rot0, A1, lda1, G1, ldg1, W1, ldw1, K1, N1, rot1, 1,
                              plo, rexp, M, accumulate, workspace, stream);
}

extern "C" int msat_set_precision(int32_t mode) {
    MSAT_REQUIRE(mode == MSAT_PRECISION_FP16X2 || mode == MSAT_PRECISION_BF16X3 || mode == MSAT_PRECISION_FP32,
                 "msat_set_precision: unknown mode %d (0 fp16x2, 1 bf16x3, 2 fp32)", mode);
    g_precision.store(mode, std::memory_order_relaxed);
    return MSAT_OK;
}

extern "C" int msat_get_precision(void) {
    const int pm = precision_mode();
    MSAT_REQUIRE_PRECISION(pm);
    return pm;
}
