// fp32 GEMM on the bf16 matrix cores by three-way operand splitting ("bf16x3").
//
// An fp32 value x is split exactly into three bf16 parts x = x1 + x2 + x3 + O(2^-24 |x|)
// (x1 = bf16(x), x2 = bf16(x - x1), x3 = bf16(x - x1 - x2); each difference is exact in fp32).
// A product a*b then keeps every term above the fp32 rounding level:
//     a b ~= a1 b1 + (a1 b2 + a2 b1) + (a1 b3 + a2 b2 + a3 b1)          (dropped terms <= 3 * 2^-24 |a b|)
// and bf16 x bf16 products are exact in fp32, so six v_mfma_f32_32x32x16_bf16 per 16-deep k step
// reproduce the fp32 dot product to fp32 rounding (the 1e-5 parity bar holds with margin; see
// tests/test_gemm_gpu.py).  Six bf16 MFMAs (32 cycles each per SIMD) replace eight f32 32x32x2
// MFMAs (64 cycles each): 2.67x fewer matrix-core cycles for the same fp32 result.
//
// msat_gemm_x3: C[M,N] (+)= A[M,K] @ W^T (+ bias) with W [N][K] given as pre-split bf16 planes
// (msat_split_bf16x3, once per weight update).  The activation operand A is split while it is
// staged: global fp32 -> registers -> three bf16 planes in LDS; the weight planes arrive by
// LDS-DMA.  128x128 tile per 256-thread workgroup (wave = 64x64 = 2x2 MFMA tiles), 16-deep slabs,
// double-buffered in LDS, A prefetched two slabs ahead in registers (the six bf16 MFMAs of a slab
// are too short to cover an HBM load issued one slab ahead).

#include <algorithm>
#include <type_traits>

#include "common.h"
#include "split3.h"

namespace msat {

typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kX3T = 256;
constexpr int kX3M = 128;  // tile rows / cols
constexpr int kX3D = 16;   // slab depth (one bf16 MFMA k step)
// LDS plane: 128 rows x 16 k bf16 = 4 KiB = 256 uint4 (row r, k-half h at uint4 index 2r + h)
constexpr int kX3Plane = kX3M * kX3D / 8;
constexpr int kW3Plane = 16 * kX3M;  // bf16 elements per weight-gradient plane (16 rows x 128 cols)

__device__ __forceinline__ int xcd_remap_x3(int orig, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__global__ void split_bf16x3_kernel(const float *__restrict__ W, int rows, int cols, int ldw, int rot,
                                    __bf16 *__restrict__ out) {
    const size_t n = (size_t)rows * cols;
    const size_t plane = n;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / cols, c = i - r * cols;
        const size_t cs = c + rot < (size_t)cols ? c + rot : c + rot - cols;
        const float x = W[r * ldw + cs];
        const __bf16 a = (__bf16)x;
        const float res = x - (float)a;
        const __bf16 b = (__bf16)res;
        out[i] = a;
        out[plane + i] = b;
        out[2 * plane + i] = (__bf16)(res - (float)b);
    }
}

// C[M,N] (+)= A[M,K] @ W^T + bias, W planes [3][N][K] bf16.  K % 16 == 0, lda % 4 == 0, A 16-B aligned.
// The LDS-staged form, for K % 32 != 0 (the register-A kernel below takes K % 32 == 0).
// TI = 32-row MFMA tiles per wave: the workgroup tile is (64 TI) x 128 (2 x 2 waves); launched with
// TI = 2 (TI = 4, 256-row tiles, measured 8 % slower on the 407 K-row shape in round 1).
template <int TI>
__global__ void __launch_bounds__(kX3T, TI == 2 ? 3 : 2)
gemm_x3_kernel(const float *__restrict__ A, int lda, const __bf16 *__restrict__ Wp, float *__restrict__ C, int ldc,
               const float *__restrict__ bias, int M, int N, int K, int accumulate, int ntn, int vec_out) {
    constexpr int MT = 64 * TI, APL = MT * 2, SR = TI / 2;  // tile rows; A plane uint4s; staging rows per thread
    __shared__ uint4 lds_raw[2 * 3 * (APL + kX3Plane)];  // [buf][A planes] then [buf][W planes]
    uint4 (*lds_a)[3][APL] = reinterpret_cast<uint4 (*)[3][APL]>(lds_raw);
    uint4 (*lds_w)[3][kX3Plane] = reinterpret_cast<uint4 (*)[3][kX3Plane]>(lds_raw + 2 * 3 * APL);
    const int id = xcd_remap_x3(blockIdx.x, gridDim.x);
    const int m0 = (id / ntn) * MT, n0 = (id % ntn) * kX3M;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int wr = (w >> 1) * 32 * TI, wc = (w & 1) * 64;
    const int srow = t >> 1, shalf = t & 1;  // staging: row-halves (8 k values) srow + 128 j
    const float *arow[SR];
#pragma unroll
    for (int j = 0; j < SR; ++j) arow[j] = A + (size_t)min(m0 + srow + 128 * j, M - 1) * lda + 8 * shalf;
    const size_t NK = (size_t)N * K;
    // LDS images: row r's 16-byte k-halves h at uint4 2 r + (h ^ ((r >> 3) & 1)) -- the XOR makes the
    // ds_read_b128 fragment reads (32-byte row stride) conflict-free in every 16-lane group
    const __bf16 *wrow = Wp + (size_t)min(n0 + srow, N - 1) * K + 8 * (shalf ^ ((srow >> 3) & 1));
    f32x16v acc[TI][2];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16v{};
    const int ns = K / kX3D;
    // A is prefetched two slabs ahead in registers (slots R0 / R1 by slab parity), the weight planes
    // one slab ahead by LDS-DMA.  Per slab s: issue W(s+1), then load A(s+2) (so waiting for W(s+1)
    // never waits for A(s+2): vector-memory counts retire in issue order), multiply slab s, split
    // and store A(s+1), barrier.
    float4 R0[SR][2], R1[SR][2];
    auto loadA = [&](int s, float4 (&r)[SR][2]) {
#pragma unroll
        for (int j = 0; j < SR; ++j) {
            const float4 *p = reinterpret_cast<const float4 *>(arow[j] + s * kX3D);
            r[j][0] = p[0];
            r[j][1] = p[1];
        }
    };
    auto storeA = [&](const float4 (&r)[SR][2], int buf) {
#pragma unroll
        for (int j = 0; j < SR; ++j) {
            const Split8 sp = split8(r[j][0], r[j][1]);
#pragma unroll
            for (int q = 0; q < 3; ++q) lds_a[buf][q][2 * (srow + 128 * j) + (shalf ^ ((srow >> 3) & 1))] = sp.p[q];
        }
    };
    auto issueW = [&](int s, int buf) {
#pragma unroll
        for (int q = 0; q < 3; ++q) glds16_async(wrow + q * NK + s * kX3D, &lds_w[buf][q][w * 64]);
    };
    const int li = lane & 31, h = lane >> 5;
    auto slab = [&](int buf) {
        bf16x8 fa[TI][3], fb[2][3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
#pragma unroll
            for (int i = 0; i < TI; ++i)
                fa[i][q] = __builtin_bit_cast(bf16x8, lds_a[buf][q][(wr + 32 * i + li) * 2 + (h ^ ((li >> 3) & 1))]);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                fb[j][q] = __builtin_bit_cast(bf16x8, lds_w[buf][q][(wc + 32 * j + li) * 2 + (h ^ ((li >> 3) & 1))]);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x16v c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
                acc[i][j] = c;
            }
    };
    loadA(0, R0);
    if (ns > 1) loadA(1, R1);
    issueW(0, 0);
    storeA(R0, 0);
    wait_vmcnt<0>();
    barrier_lds();
    if (ns > 2) loadA(2, R0);
    constexpr int NL = 2 * SR;  // A loads per slab per thread
    // Rn holds A(s+1); Rf is free and receives A(s+2)
    auto iter = [&](int s, float4 (&Rn)[SR][2], float4 (&Rf)[SR][2]) {
        const int buf = s & 1;
        const bool more = s + 1 < ns;
        if (more) issueW(s + 1, buf ^ 1);
        if (s >= 1 && s + 2 < ns) loadA(s + 2, Rf);  // s = 0: A(2) was issued in the prologue
        slab(buf);
        __builtin_amdgcn_sched_barrier(0);
        if (more) storeA(Rn, buf ^ 1);
        // W(s+1) and A(s+1) landed; A(s+2) (issued after W(s+1) for s >= 1) may fly.  At s = 0,
        // A(2) precedes W(1) in issue order, so the wait drains everything.
        if (s >= 1 && s + 2 < ns) wait_vmcnt<NL>();
        else wait_vmcnt<0>();
        barrier_lds();
    };
    for (int s = 0; s < ns; s += 2) {
        iter(s, R1, R0);
        if (s + 1 < ns) iter(s + 1, R0, R1);
    }
    float *ldsf = reinterpret_cast<float *>(lds_raw);  // >= 48 KiB: four 8 KiB epilogue stages
    if (vec_out) {
        // LDS-staged epilogue: each wave's 32x64 half-tile leaves as whole 256-byte rows of float4
        float *stage = ldsf + w * 32 * 64;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
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
    for (int i = 0; i < TI; ++i)
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
                *c = accumulate ? *c + v : v;
            }
        }
}

// ---------------------------------------------------------------------------------------------
// The register-A kernel on v_mfma_f32_16x16x32_bf16: one MFMA k step covers the whole 32-deep
// double slab (lane l holds A[l & 15][8 (l >> 4) + j], i.e. 32 contiguous bytes of its row), the
// wave tile is 2 x 8 tiles of 16 x 16.  Same MFMA work and LDS reads as the 32x32x16 form; the
// 16x16 loop holds a higher clock under load (MI355X_MICROARCH.md, DVFS item 7).  Weight chunk c of
// row n sits at slot c ^ f((n >> 2) & 3), f = {0, 2, 3, 1}: conflict-free for this lane map.
__device__ __forceinline__ int x3swz16(int b) { return (0x78 >> (2 * b)) & 3; }  // {0, 2, 3, 1}

template <int RT>  // 16-row tiles per wave: the workgroup tile is 64 RT rows x 128 columns
__global__ void __launch_bounds__(kX3T, RT == 2 ? 3 : 2)
gemm_x3r16_kernel(const float *__restrict__ A, int lda, const __bf16 *__restrict__ Wp, float *__restrict__ C, int ldc,
                  const float *__restrict__ bias, int M, int N, int K, int accumulate, int ntn, int vec_out) {
    constexpr int WPL = kX3M * 4;
    __shared__ uint4 lds_w[2][3][WPL];  // 48 KiB
    const int id = xcd_remap_x3(blockIdx.x, gridDim.x);
    const int m0 = (id / ntn) * 64 * RT, n0 = (id % ntn) * kX3M;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63, l16 = lane & 15, g = lane >> 4;
    const int wr = w * 16 * RT;
    const float *arow[RT];
#pragma unroll
    for (int i = 0; i < RT; ++i) arow[i] = A + (size_t)min(m0 + wr + 16 * i + l16, M - 1) * lda + 8 * g;
    unsigned voff[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) {
        const int x = 6 * w + e, q = x >> 3, p = x & 7, row = 16 * p + (lane >> 2);
        const int ch = (lane & 3) ^ x3swz16((row >> 2) & 3);
        voff[e] = (unsigned)(((size_t)q * N * K + (size_t)min(n0 + row, N - 1) * K + 8 * ch) * 2);
    }
    auto issueW = [&](int d, int buf) {
        const char *base = reinterpret_cast<const char *>(Wp) + (size_t)d * 64;
#pragma unroll
        for (int e = 0; e < 6; ++e) {
            const int x = 6 * w + e;
            glds16_async_s(base, voff[e], &lds_w[buf][x >> 3][64 * (x & 7)]);
        }
    };
    f32x4 acc[RT][8];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};
    float4 ra[RT][2];  // the next double slab's raw A: [row tile][half]
    auto loadA = [&](int d) {
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int e = 0; e < 2; ++e) ra[i][e] = *reinterpret_cast<const float4 *>(arow[i] + 32 * d + 4 * e);
    };
    const int slot = g ^ x3swz16((l16 >> 2) & 3);
    const int nd = K / 32;
    loadA(0);
    issueW(0, 0);
    wait_vmcnt<0>();
    barrier_lds();
    // per double slab d: split A(d), issue W(d+1) and A(d+1), MFMAs of d, wait for W(d+1) (vector-
    // memory counts retire in issue order, so A(d+1) may still fly), barrier
    for (int d = 0; d < nd; ++d) {
        const int buf = d & 1;
        bf16x8 fa[RT][3];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const Split8 sp = split8(ra[i][0], ra[i][1]);
#pragma unroll
            for (int q = 0; q < 3; ++q) fa[i][q] = __builtin_bit_cast(bf16x8, sp.p[q]);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bool more = d + 1 < nd;
        if (more) issueW(d + 1, buf ^ 1);
        if (more) loadA(d + 1);
        __builtin_amdgcn_sched_barrier(0);
        {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                bf16x8 fb[3];
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    fb[q] = __builtin_bit_cast(bf16x8, lds_w[buf][q][(16 * j + l16) * 4 + slot]);
#pragma unroll
                for (int i = 0; i < RT; ++i) {
                    f32x4 c = acc[i][j];
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[0], c, 0, 0, 0);
                    acc[i][j] = c;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (more) wait_vmcnt<2 * RT>();
        else wait_vmcnt<0>();
        barrier_lds();
    }
    // C/D map: col = lane & 15, row = 4 (lane >> 4) + reg.  The stage is wave-private (32 rows x 64
    // columns per wave).
    float *stage = reinterpret_cast<float *>(&lds_w[0][0][0]) + w * 32 * 64;
    if (vec_out) {
        // (the main loop's last barrier already ordered every wave's weight reads before the stage)
        // accumulating calls order only the wave's own LDS operations (a workgroup barrier's release
        // fence would drain the stores issued so far, and with them the next rows' old-C loads);
        // overwriting calls measured faster with the barrier (275 vs 290 us, var dh)
        auto stage_sync = [&] {
            if (accumulate) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            else __syncthreads();
        };
#pragma unroll
        for (int i0 = 0; i0 < RT; i0 += 2) {  // 32 rows at a time
            // accumulate: the old C values of these 32 rows are all loaded before any of their stores
            // (a load issued after a store waits for it: vector-memory counts retire in issue order)
            float4 o[2][8];
#pragma unroll
            for (int hc = 0; hc < 2; ++hc) {
                const int col = n0 + 64 * hc + l16 * 4;
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int row = m0 + wr + 16 * i0 + it * 4 + g;
                    if (accumulate && row < M && col < N)
                        o[hc][it] = *reinterpret_cast<const float4 *>(C + (size_t)row * ldc + col);
                }
            }
#pragma unroll
            for (int hc = 0; hc < 2; ++hc) {  // columns 64 hc .. 64 hc + 63
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                        for (int reg = 0; reg < 4; ++reg)
                            stage[(16 * i + 4 * g + reg) * 64 + 16 * jj + l16] = acc[i0 + i][4 * hc + jj][reg];
                stage_sync();
                const int col = n0 + 64 * hc + l16 * 4;
                float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (bias && col < N) bv = *reinterpret_cast<const float4 *>(bias + col);
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int rr = it * 4 + g;
                    const int row = m0 + wr + 16 * i0 + rr;
                    float4 v = *reinterpret_cast<const float4 *>(stage + rr * 64 + l16 * 4);
                    v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
                    if (accumulate) {
                        const float4 &ov = o[hc][it];
                        v.x = ov.x + v.x; v.y = ov.y + v.y; v.z = ov.z + v.z; v.w = ov.w + v.w;
                    }
                    if (row < M && col < N) *reinterpret_cast<float4 *>(C + (size_t)row * ldc + col) = v;
                }
                stage_sync();
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int col = n0 + 16 * j + l16;
            if (col >= N) continue;
            const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int row = m0 + wr + 16 * i + 4 * g + reg;
                if (row >= M) continue;
                float *c = C + (size_t)row * ldc + col;
                const float v = acc[i][j][reg] + bv;
                *c = accumulate ? *c + v : v;
            }
        }
}

// ---------------------------------------------------------------------------------------------
// fp16x2 form of the register-A data gradient (msat_gemm_h2): C[M,N] (+)= A[M,K] @ W^T for A = a GRU
// backward's packed rows, whose row scale exponents rexp (written by that backward, split3.h
// f16x2_row_exp) put every scaled row inside fp16's range with its largest elements at full
// precision.  Each lane's activation rows are fixed (register-A: lane l holds row l & 15 of each 16-row
// tile), so a row's scale is one load per tile, the split is x 2^e -> (h, l) in registers, and the
// epilogue rescales each output row by 2^-(e + kDgW) (exact).  Weights: [2][N][K] fp16x2 planes of
// 2^kDgW W (msat_split_f16x2_rot), two LDS images per slab instead of three.  Three fp16 MFMAs per
// 16x16x32 block instead of six bf16.  If the weight split overflowed (*wbad), the kernel runs the
// bf16x3 body on the bf16x3 planes instead (same grid and LDS).
constexpr int kDgW = 10;  // weight scale 2^10: |W| < 32 fits

// PL: A is the GRU backward's packed rows as fp16x2 planes (gnn_kernels.hip, flags bit 3): row r at
// A + r lda fp16 elements, hi there and lo plo elements further, both already at the row exponent -- the
// fp16x2 body takes them as its MFMA operands as loaded (bit for bit the split it makes of fp32 rows);
// the bf16x3 body rebuilds each element as (hi + lo) 2^-e (22 significant bits) before its split.
template <int RT, int NP, int NWV = 4, bool PL = false>
__device__ __forceinline__ void gemm_r16_body(const void *__restrict__ Av, int lda, const int *__restrict__ rexp,
                                              const uint16_t *__restrict__ Wp, float *__restrict__ C, int ldc,
                                              const float *__restrict__ bias, int M, int N, int K, int accumulate,
                                              int m0, int n0, int vec_out, uint4 (*lds_w)[3][kX3M * 4], int kr = 0,
                                              int plo = 0) {
    typedef _Float16 f16x8v __attribute__((ext_vector_type(8)));
    const int t = threadIdx.x, w = t >> 6, lane = t & 63, l16 = lane & 15, g = lane >> 4;
    const int wr = w * 16 * RT;
    constexpr int ESZ = PL ? 2 : 4;  // bytes per A element
    const char *arow[RT];
    int ea[RT];  // fp16x2 / planes: the scale exponent of this lane's activation row in each tile
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int r = min(m0 + wr + 16 * i + l16, M - 1);
        arow[i] = reinterpret_cast<const char *>(Av) + ((size_t)r * lda + 8 * g) * ESZ;
        if constexpr (NP == 2 || PL) {
            const int e = rexp[r];
            ea[i] = e == kExpZero ? 0 : e;
        }
    }
    // weight DMA: 8 NP wave-instructions (1 KiB = 16 rows x 4 chunks) per double slab, 2 NP per wave at
    // NWV = 4 (NWV waves: ceil(8 NP / NWV), the last waves' surplus slots idle)
    constexpr int PW = (8 * NP + NWV - 1) / NWV;
    unsigned voff[PW];
#pragma unroll
    for (int e = 0; e < PW; ++e) {
        const int x = min(PW * w + e, 8 * NP - 1), q = x >> 3, p = x & 7, row = 16 * p + (lane >> 2);
        const int ch = (lane & 3) ^ x3swz16((row >> 2) & 3);
        voff[e] = (unsigned)(((size_t)q * N * K + (size_t)min(n0 + row, N - 1) * K + 8 * ch) * 2);
    }
    auto issueW = [&](int d, int buf) {
        const char *base = reinterpret_cast<const char *>(Wp) + (size_t)d * 64;
#pragma unroll
        for (int e = 0; e < PW; ++e) {
            const int x = PW * w + e;
            if (8 * NP % NWV == 0 || x < 8 * NP) glds16_async_s(base, voff[e], &lds_w[buf][x >> 3][64 * (x & 7)]);
        }
    };
    f32x4 acc[RT][8];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};
    // activations two double slabs ahead in two register sets (plain loads: hipcc tracks them and
    // waits for A(d) just before its split; its count ignores the asm weight DMAs, which only makes
    // that wait stricter, and W(d) has landed by then anyway)
    // the bf16x3 body keeps one set (its split needs the registers)
    constexpr int PF = (NP == 2 && RT <= 2) ? 2 : 1;  // 256-row tiles: twice the MFMAs per step, one set ahead
    float4 ras[PF][RT][2];
    auto loadA = [&](int d, float4 (&ra)[RT][2]) {  // PL: [0] = 8 hi, [1] = 8 lo fp16 (bits)
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int e = 0; e < 2; ++e)
                ra[i][e] = *reinterpret_cast<const float4 *>(arow[i] + (PL ? (e * plo + 32 * d) * 2 : (32 * d + 4 * e) * 4));
    };
    const int slot = g ^ x3swz16((l16 >> 2) & 3);
    const int nd = K / 32;
    // the k walk starts at double slab kr (0 <= kr < nd) and wraps: the dual launch aligns its two
    // products' walks over the packed rows they share, so sibling workgroups read the same columns of a
    // row at the same time and the second read hits L2 (msat_gemm_h2_dual)
    auto sl = [&](int d) { const int x = d + kr; return x >= nd ? x - nd : x; };
    loadA(sl(0), ras[0]);
    if (PF == 2 && nd > 1) loadA(sl(1), ras[PF - 1]);
    issueW(sl(0), 0);
    wait_vmcnt<0>();
    barrier_lds();
    auto step = [&](int d, float4 (&ra)[RT][2]) {
        const int buf = d & 1;
        uint4 fa[RT][NP];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            if constexpr (NP == 3 && PL) {
                const f16x8v hv = __builtin_bit_cast(f16x8v, ra[i][0]), lv = __builtin_bit_cast(f16x8v, ra[i][1]);
                float x[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = ldexpf((float)hv[j] + (float)lv[j], -ea[i]);
                const Split8 sp = split8(make_float4(x[0], x[1], x[2], x[3]), make_float4(x[4], x[5], x[6], x[7]));
#pragma unroll
                for (int q = 0; q < 3; ++q) fa[i][q] = sp.p[q];
            } else if constexpr (NP == 3) {
                const Split8 sp = split8(ra[i][0], ra[i][1]);
#pragma unroll
                for (int q = 0; q < 3; ++q) fa[i][q] = sp.p[q];
            } else if constexpr (PL) {
                fa[i][0] = __builtin_bit_cast(uint4, ra[i][0]);
                fa[i][1] = __builtin_bit_cast(uint4, ra[i][1]);
            } else {
                const float4 u = ra[i][0], v = ra[i][1];
                const int e = ea[i];
                const SplitH4 s0 = splith4(make_float4(ldexpf(u.x, e), ldexpf(u.y, e), ldexpf(u.z, e), ldexpf(u.w, e)));
                const SplitH4 s1 = splith4(make_float4(ldexpf(v.x, e), ldexpf(v.y, e), ldexpf(v.z, e), ldexpf(v.w, e)));
                fa[i][0] = make_uint4(s0.p[0].x, s0.p[0].y, s1.p[0].x, s1.p[0].y);
                fa[i][1] = make_uint4(s0.p[1].x, s0.p[1].y, s1.p[1].x, s1.p[1].y);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        const bool more = d + 1 < nd;
        if (more) issueW(sl(d + 1), buf ^ 1);
        if (d + PF < nd) loadA(sl(d + PF), ra);  // this set was just split
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint4 fb[NP];
#pragma unroll
            for (int q = 0; q < NP; ++q) fb[q] = lds_w[buf][q][(16 * j + l16) * 4 + slot];
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                f32x4 c = acc[i][j];
                if constexpr (NP == 3) {
                    auto m = [](const uint4 &a, const uint4 &b, const f32x4 &c) {
                        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                                       __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
                    };
                    c = m(fa[i][2], fb[0], c);
                    c = m(fa[i][1], fb[1], c);
                    c = m(fa[i][0], fb[2], c);
                    c = m(fa[i][1], fb[0], c);
                    c = m(fa[i][0], fb[1], c);
                    c = m(fa[i][0], fb[0], c);
                } else {
                    auto m = [](const uint4 &a, const uint4 &b, const f32x4 &c) {
                        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8v, a),
                                                                      __builtin_bit_cast(f16x8v, b), c, 0, 0, 0);
                    };
                    c = m(fa[i][0], fb[1], c);  // h l
                    c = m(fa[i][1], fb[0], c);  // l h
                    c = m(fa[i][0], fb[0], c);  // h h
                }
                acc[i][j] = c;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // W(d + 1) landed; A(d + PF), issued after it, may fly
        if (d + PF < nd) wait_vmcnt<2 * RT>();
        else wait_vmcnt<0>();
        barrier_lds();
    };
    if constexpr (PF == 2) {
        int d = 0;
        for (; d + 1 < nd; d += 2) {
            step(d, ras[0]);
            step(d + 1, ras[PF - 1]);
        }
        if (d < nd) step(d, ras[0]);
    } else {
        for (int d = 0; d < nd; ++d) step(d, ras[0]);
    }
    // fp16x2: rescale each output row (C/D map: row 4 (lane >> 4) + reg of the tile) by 2^-(e + kDgW)
    if constexpr (NP == 2) {
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int e = rexp[min(m0 + wr + 16 * i + 4 * g + reg, M - 1)];
                const int sh = -((e == kExpZero ? 0 : e) + kDgW);
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[i][j][reg] = ldexpf(acc[i][j][reg], sh);
            }
    }
    float *stage = reinterpret_cast<float *>(&lds_w[0][0][0]) + w * 32 * 64;
    if (vec_out) {
        auto stage_sync = [&] {
            if (accumulate) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            else __syncthreads();
        };
#pragma unroll
        for (int i0 = 0; i0 < RT; i0 += 2) {
            float4 o[2][8];
#pragma unroll
            for (int hc = 0; hc < 2; ++hc) {
                const int col = n0 + 64 * hc + l16 * 4;
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int row = m0 + wr + 16 * i0 + it * 4 + g;
                    if (accumulate && row < M && col < N)
                        o[hc][it] = *reinterpret_cast<const float4 *>(C + (size_t)row * ldc + col);
                }
            }
#pragma unroll
            for (int hc = 0; hc < 2; ++hc) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                        for (int reg = 0; reg < 4; ++reg)
                            stage[(16 * i + 4 * g + reg) * 64 + 16 * jj + l16] = acc[i0 + i][4 * hc + jj][reg];
                stage_sync();
                const int col = n0 + 64 * hc + l16 * 4;
                float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (bias && col < N) bv = *reinterpret_cast<const float4 *>(bias + col);
#pragma unroll
                for (int it = 0; it < 8; ++it) {
                    const int rr = it * 4 + g;
                    const int row = m0 + wr + 16 * i0 + rr;
                    float4 v = *reinterpret_cast<const float4 *>(stage + rr * 64 + l16 * 4);
                    v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
                    if (accumulate) {
                        const float4 &ov = o[hc][it];
                        v.x = ov.x + v.x; v.y = ov.y + v.y; v.z = ov.z + v.z; v.w = ov.w + v.w;
                    }
                    if (row < M && col < N) *reinterpret_cast<float4 *>(C + (size_t)row * ldc + col) = v;
                }
                stage_sync();
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int col = n0 + 16 * j + l16;
            if (col >= N) continue;
            const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int row = m0 + wr + 16 * i + 4 * g + reg;
                if (row >= M) continue;
                float *c = C + (size_t)row * ldc + col;
                const float v = acc[i][j][reg] + bv;
                *c = accumulate ? *c + v : v;
            }
        }
}

template <int RT>
__global__ void __launch_bounds__(kX3T, RT == 2 ? 3 : 2)
gemm_h2r16_kernel(const float *__restrict__ A, int lda, const int *__restrict__ rexp, const uint16_t *__restrict__ Wh2,
                  const uint16_t *__restrict__ Wx3, const int *__restrict__ wbad, float *__restrict__ C, int ldc,
                  const float *__restrict__ bias, int M, int N, int K, int accumulate, int ntn, int vec_out) {
    __shared__ uint4 lds_w[2][3][kX3M * 4];  // 48 KiB (the fp16x2 body uses two of the three images)
    const int id = xcd_remap_x3(blockIdx.x, gridDim.x);
    const int m0 = (id / ntn) * 64 * RT, n0 = (id % ntn) * kX3M;
    if (*wbad)
        gemm_r16_body<RT, 3>(A, lda, nullptr, Wx3, C, ldc, bias, M, N, K, accumulate, m0, n0, vec_out, lds_w);
    else
        gemm_r16_body<RT, 2>(A, lda, rexp, Wh2, C, ldc, bias, M, N, K, accumulate, m0, n0, vec_out, lds_w);
}

// Two data gradients of the same packed rows in one launch (a GRU cell's dh and d(input)): for each
// 128-row block the n tiles of both products are consecutive workgroup ids, so the workgroups that read
// the same rows of the packed buffer run together on one XCD and all but the first read them from L2.
struct DgradProblem {
    const void *A;  // fp32 rows, or (planes launches) fp16x2 planes with the lo plane plo elements after hi
    int lda, plo;
    const uint16_t *Wh2, *Wx3;
    const int *wbad;
    float *C;
    int ldc, N, accumulate, vec_out, ntn;
    int kr;  // first double slab of the k walk (aligns the two products' reads of the shared rows)
};

template <int RT, int NWV = 4, bool PL = false>
__global__ void __launch_bounds__(64 * NWV, NWV == 4 ? (RT == 2 ? 3 : 2) : 1)
gemm_h2r16_dual_kernel(DgradProblem p0, DgradProblem p1, const int *__restrict__ rexp, int M, int K) {
    // the weight buffers, and the epilogue's per-wave stage (8 KiB per wave) in the same memory
    constexpr int LDSU = (NWV * 8192 > 2 * 3 * kX3M * 4 * 16 ? NWV * 8192 : 2 * 3 * kX3M * 4 * 16) / 16;
    __shared__ uint4 lds_raw[LDSU];
    uint4 (*lds_w)[3][kX3M * 4] = reinterpret_cast<uint4 (*)[3][kX3M * 4]>(lds_raw);
    const int id = xcd_remap_x3(blockIdx.x, gridDim.x);
    const int T = p0.ntn + p1.ntn, sub = id % T;
    const int m0 = (id / T) * 16 * NWV * RT;
    const bool first = sub < p0.ntn;
    const DgradProblem &p = first ? p0 : p1;
    const int n0 = (first ? sub : sub - p0.ntn) * kX3M;
    if (*p.wbad)
        gemm_r16_body<RT, 3, NWV, PL>(p.A, p.lda, PL ? rexp : nullptr, p.Wx3, p.C, p.ldc, nullptr, M, p.N, K,
                                      p.accumulate, m0, n0, p.vec_out, lds_w, p.kr, p.plo);
    else
        gemm_r16_body<RT, 2, NWV, PL>(p.A, p.lda, rexp, p.Wh2, p.C, p.ldc, nullptr, M, p.N, K, p.accumulate, m0, n0,
                                      p.vec_out, lds_w, p.kr, p.plo);
}

// planes[q][r][c] = part q of 2^kDgW W[r][(c + rot) % cols] (fp16x2, q = 0, 1); *bad = 1 if a scaled
// weight is outside (-2^15, 2^15) or not finite (msat_gemm_h2 then runs its bf16x3 body)
__global__ void split_f16x2_rot_kernel(const float *__restrict__ W, int rows, int cols, int ldw, int rot,
                                       _Float16 *__restrict__ out, int *__restrict__ bad) {
    const size_t n = (size_t)rows * cols;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / cols, c = i - r * cols;
        const size_t cs = c + rot < (size_t)cols ? c + rot : c + rot - cols;
        const float x = W[r * ldw + cs] * (float)(1 << kDgW);
        const _Float16 p = (_Float16)x;
        out[i] = p;
        out[n + i] = (_Float16)(x - (float)p);
        if (!(fabsf(x) < 32768.0f)) *bad = 1;
    }
}

// ---------------------------------------------------------------------------------------------
// Weight gradient on the same split: part[s][k][n] = sum_{m in split s} A[m][k] G[m][n].
// The MFMA reduction runs over the rows m, so both fragments are 8-row column strips.  Both
// operands are staged row-major as three bf16 planes [16 rows][128 cols] (256-byte rows, chunks
// XOR-swizzled for conflict-free transposed reads) and read with ds_read_b64_tr_b16: each
// 16-lane group gets 4 rows x 16 columns delivered column-major, two reads per fragment.
__global__ void __launch_bounds__(kX3T, 3)
wgrad_x3_kernel(const float *__restrict__ A, int lda, const float *__restrict__ G, int ldg, float *__restrict__ part,
                int M, int K, int N, int rows_per_split, int ntn, int tiles) {
    __shared__ __attribute__((aligned(16))) unsigned short lds[2][6][kW3Plane];  // [buf][A planes | G planes]
    const int id = xcd_remap_x3(blockIdx.x, gridDim.x);
    const int sp = id / tiles, tile = id % tiles;
    const int k0 = (tile / ntn) * kX3M, n0 = (tile % ntn) * kX3M;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int wr = (w >> 1) * 64, wc = (w & 1) * 64;
    f32x16v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16v{};
    const int rb = sp * rows_per_split, re = min(M, rb + rows_per_split);
    const int ns = (re - rb + 15) / 16;
    // staging: thread t -> row t >> 4 of the slab, columns 4 (t & 15) and 4 (t & 15) + 64.
    // Loads run two slabs ahead in registers (sets R0 / R1 by slab parity) and are always issued
    // (clamped row / columns; out-of-range values are zeroed when stored, after they landed), so
    // hipcc's counted wait before a store leaves the next set's loads in flight.
    const int srow = t >> 4, sc = (t & 15) * 4;
    struct Stage {
        float4 a[2], g[2];
    };
    bool kok[2], nok[2];
    const float *pa[2];
    const float *pg[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int kc = k0 + sc + 64 * u, nc = n0 + sc + 64 * u;
        kok[u] = kc < K;
        nok[u] = nc < N;
        pa[u] = A + (kok[u] ? kc : 0);
        pg[u] = G + (nok[u] ? nc : 0);
    }
    auto load = [&](int s, Stage &r) {
        const int m = rb + s * 16 + srow;
        const size_t mc = m < re ? m : re - 1;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            r.a[u] = *reinterpret_cast<const float4 *>(pa[u] + mc * lda);
            r.g[u] = *reinterpret_cast<const float4 *>(pg[u] + mc * ldg);
        }
    };
    auto store = [&](int s, Stage r, int buf) {
        const bool mok = rb + s * 16 + srow < re;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (!(mok && kok[u])) r.a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!(mok && nok[u])) r.g[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            const int col = sc + 64 * u;
            const int off = w3off(srow, col >> 3) + 8 * ((col >> 2) & 1);
            const Split4 xa = split4(r.a[u]), xg = split4(r.g[u]);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(lds[buf][q]) + off) = xa.p[q];
                *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(lds[buf][3 + q]) + off) = xg.p[q];
            }
        }
    };
    const int h = lane >> 5, g = (lane >> 4) & 1;
    auto slab = [&](int buf) {
        bf16x8 fa[2][3], fb[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                fa[i][q] = tr_frag(lds[buf][q], 8 * h, (wr + 32 * i + 16 * g) >> 3, lane);
                fb[i][q] = tr_frag(lds[buf][3 + q], 8 * h, (wc + 32 * i + 16 * g) >> 3, lane);
            }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x16v c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
                acc[i][j] = c;
            }
    };
    if (ns > 0) {
        Stage R0, R1;
        load(0, R0);
        load(1 < ns ? 1 : 0, R1);
        store(0, R0, 0);
        __syncthreads();
        // Rn holds slab s + 1, Rf receives slab s + 2 (past the end: a repeated, never stored load)
        auto iter = [&](int s, const Stage &Rn, Stage &Rf) {
            const int buf = s & 1;
            load(s + 2 < ns ? s + 2 : ns - 1, Rf);
            __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMAs
            slab(buf);
            __builtin_amdgcn_sched_barrier(0);
            // unconditional (past the end it fills the unused buffer): a store in its own basic
            // block lets hipcc sink the slab s + 2 loads into it, right before their use
            store(s + 1, Rn, buf ^ 1);
            __syncthreads();
        };
        int s = 0;
        for (; s + 1 < ns; s += 2) {
            iter(s, R1, R0);
            iter(s + 1, R0, R1);
        }
        if (s < ns) iter(s, R1, R0);
    }
    float *P = part + (size_t)sp * K * N;
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

// ---------------------------------------------------------------------------------------------
// Whole-row weight gradient: part[s][k][(n + rot) % N] = sum_{m in split s} A[m][k] G[m][n] for one
// 128-row k tile and ALL N <= 384 columns per workgroup.  Every A element is loaded by exactly one
// workgroup and every G element by ceil(K / 128), so the kernel streams A and G from HBM once
// (the 128 x 128 tiles of wgrad_x3_kernel re-read each operand per tile of the other, from L2 at
// best).  512 threads, 8 waves at two per SIMD, one workgroup per CU; wave w owns k rows
// 64 (w & 1) .. +63 x columns 96 (w >> 1) .. +95 as 2 x 3 tiles of 32x32 (96 accumulator registers).
// Staging as wgrad_x3_kernel: 16-row slabs loaded two ahead in registers, split into NP planes of
// [16 rows][128 cols] images (G: three column blocks), transposed fragment reads, one barrier per
// slab.  rot rotates the output columns (the packed backward rows' gate blocks are (n | r | z), the
// weights' (r | z | n)); rot % 4 == 0.
//
// NP = 3: bf16x3 (six bf16 MFMAs per tile and slab).  With `flags` it is the fixup launch of the
// fp16x2 kernel: it computes only the workgroups flagged there.
// NP = 2: fp16x2 (three fp16 MFMAs).  G is scaled by 2^e with e the smallest row exponent of the
// split (rexp, written by the GRU backward that produced G: every scaled row below 2^15, the
// largest at full precision) and the partial by 2^-e (exact).  A is range-checked (|a| < 2^15): a
// workgroup that loads anything outside sets flags[id] and stores nothing; G needs no check (a
// non-finite G row stays non-finite through the fp16 products, as it would in fp32).
//
// IL: the split and LDS store of slab s + 1 are interleaved with slab s's MFMAs by scheduling groups
// (one MFMA, then a few vector instructions; an LDS store every few MFMAs), so the split fills the
// MFMA issue gaps instead of running as its own phase between the MFMA phase and the barrier.

constexpr int kWWT = 512;
constexpr int kWWN = 384;  // widest N

typedef unsigned short WwLds[2][12][kW3Plane];  // [buf][A planes | G planes]: 96 KiB

// one workgroup's share: split sp (rows sp * rows_per_split ..), k tile k0; flag: this workgroup's
// range flag (fp16x2), lds: the kernel's WwLds
// PLG (the fixup of the planes launch, NP = 3 only): G is fp16x2 planes at the row exponents (ldg in fp16
// elements, lo plane plo elements after hi), rebuilt per element as (hi + lo) 2^-e (22 significant bits).
template <int NP, bool IL, bool PLG = false>
__device__ __forceinline__ void wgrad_w_body(const float *__restrict__ A, int lda, const void *__restrict__ Gv, int ldg,
                                             const int *__restrict__ rexp, float *__restrict__ part, int M, int K,
                                             int N, int rot, int rows_per_split, int sp, int k0, int *flag,
                                             WwLds &ldsr, int plo = 0) {
    static_assert(!PLG || NP == 3, "planes G: the bf16x3 fixup only");
    // [buf][A planes 0 .. NP-1 | G plane q, column block u at NP + 3 q + u]
    unsigned short (*lds)[4 * NP][kW3Plane] = reinterpret_cast<unsigned short (*)[4 * NP][kW3Plane]>(&ldsr[0][0][0]);
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int wk = (w & 1) * 64, wn = __builtin_amdgcn_readfirstlane((w >> 1) * 96);
    const int rb = sp * rows_per_split, re = min(M, rb + rows_per_split);
    const int ns = (re - rb + 15) / 16;
    int ge = 0;  // fp16x2: G scale exponent of this split
    if constexpr (NP == 2) {
        int *red = reinterpret_cast<int *>(&ldsr[1][11][0]);  // the last image: free until the first store
        int mn = kExpZero;
        for (int r = rb + t; r < re; r += kWWT) mn = min(mn, rexp[r]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mn = min(mn, __shfl_xor(mn, o, 64));
        if (lane == 0) red[w] = mn;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kWWT / 64; ++i) mn = min(mn, red[i]);
        ge = mn == kExpZero ? 0 : mn;
    }
    f32x16v acc[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = f32x16v{};
    // staging: thread t -> slab row t >> 5, columns sc .. sc + 3 of the A tile and of each G block
    const int srow = t >> 5, sc = (t & 31) * 4;
    const bool kok = k0 + sc < K;
    bool nok[3];
    const float *pa = A + (kok ? k0 + sc : 0);
    constexpr int GSZ = PLG ? 2 : 4;  // bytes per G element
    const char *pg[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        nok[u] = sc + 128 * u < N;
        pg[u] = reinterpret_cast<const char *>(Gv) + (nok[u] ? sc + 128 * u : 0) * GSZ;
    }
    struct Stage {
        float4 a, g[3];
    };
    auto load = [&](int s, Stage &r) {
        const int m = rb + s * 16 + srow;
        const size_t mc = m < re ? m : re - 1;
        r.a = *reinterpret_cast<const float4 *>(pa + mc * lda);
        if constexpr (PLG) {
            typedef _Float16 f16x4g __attribute__((ext_vector_type(4)));
            const int e = rexp[mc], es = e == kExpZero ? 0 : e;
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const f16x4g hv = *reinterpret_cast<const f16x4g *>(pg[u] + mc * ldg * 2);
                const f16x4g lv = *reinterpret_cast<const f16x4g *>(pg[u] + (mc * ldg + plo) * 2);
                r.g[u] = make_float4(ldexpf((float)hv[0] + (float)lv[0], -es), ldexpf((float)hv[1] + (float)lv[1], -es),
                                     ldexpf((float)hv[2] + (float)lv[2], -es), ldexpf((float)hv[3] + (float)lv[3], -es));
            }
        } else {
#pragma unroll
            for (int u = 0; u < 3; ++u) r.g[u] = *reinterpret_cast<const float4 *>(pg[u] + mc * ldg * 4);
        }
    };
    float amax = 0.f;  // fp16x2: largest |operand| staged by this thread (range check)
    const int off = w3off(srow, sc >> 3) + 8 * ((sc >> 2) & 1);
    auto put = [&](int buf, int plane, const uint2 &v) {
        *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(lds[buf][plane]) + off) = v;
    };
    auto store = [&](int s, Stage r, int buf) {
        const bool mok = rb + s * 16 + srow < re;
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (NP == 2) {
            // rows past the split: zero A only (the product of a zero row is zero whatever G holds);
            // columns past K or N read clamped, finite data and land in dW rows / columns that are
            // never stored, so they need no zeroing; G is in fp16 range by construction (ge is the
            // split's smallest row exponent), so only A is range-checked.  -4.7 % on the dual launch
            // (profiles/r02_ab_wgrad_lean.log); the split by v_fma_mix{lo,hi}_f16 (two instructions per
            // element pair instead of four) measured +0.3 % on top (r02_ab_wgrad_mix.log, not kept)
            if (!mok) r.a = z;
        } else {
            if (!(mok && kok)) r.a = z;
#pragma unroll
            for (int u = 0; u < 3; ++u)
                if (!(mok && nok[u])) r.g[u] = z;
        }
        if constexpr (NP == 3) {
            const Split4 xa = split4(r.a);
#pragma unroll
            for (int q = 0; q < 3; ++q) put(buf, q, xa.p[q]);
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const Split4 xg = split4(r.g[u]);
#pragma unroll
                for (int q = 0; q < 3; ++q) put(buf, 3 + 3 * q + u, xg.p[q]);
            }
        } else {
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(r.a.x), fabsf(r.a.y)), fmaxf(fabsf(r.a.z), fabsf(r.a.w))));
            const SplitH4 xa = splith4(r.a);
            put(buf, 0, xa.p[0]);
            put(buf, 1, xa.p[1]);
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const float4 v = make_float4(ldexpf(r.g[u].x, ge), ldexpf(r.g[u].y, ge), ldexpf(r.g[u].z, ge),
                                             ldexpf(r.g[u].w, ge));
                const SplitH4 xg = splith4(v);
                put(buf, 2 + u, xg.p[0]);
                put(buf, 5 + u, xg.p[1]);
            }
        }
    };
    const int h = lane >> 5, g = (lane >> 4) & 1;
    auto slab = [&](int buf) {
        bf16x8 fa[2][NP], fb[3][NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i][q] = tr_frag(lds[buf][q], 8 * h, (wk + 32 * i + 16 * g) >> 3, lane);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int n = wn + 32 * j;
                fb[j][q] = tr_frag(lds[buf][NP + 3 * q + (n >> 7)], 8 * h, ((n & 127) + 16 * g) >> 3, lane);
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                f32x16v c = acc[i][j];
                if constexpr (NP == 3) {
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
                } else {
                    typedef _Float16 f16x8w __attribute__((ext_vector_type(8)));
                    const f16x8w a0 = __builtin_bit_cast(f16x8w, fa[i][0]), a1 = __builtin_bit_cast(f16x8w, fa[i][1]);
                    const f16x8w b0 = __builtin_bit_cast(f16x8w, fb[j][0]), b1 = __builtin_bit_cast(f16x8w, fb[j][1]);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, c, 0, 0, 0);  // h l
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, c, 0, 0, 0);  // l h
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, c, 0, 0, 0);  // h h
                }
                acc[i][j] = c;
            }
    };
    if (ns > 0) {
        // NPF register sets of raw slabs: at iteration s they hold slabs s + 1 .. s + NPF - 1 (in flight or
        // landed) and the set of slab s (stored at the end of iteration s - 1) receives slab s + NPF.
        // Two sets (three or four, 96-128 KiB in flight per CU, measured 1 % slower for the fp16x2 form:
        // the kernel is not latency-bound on its loads).
        constexpr int NPF = 2;
        Stage R[NPF];
#pragma unroll
        for (int k = 0; k < NPF; ++k) load(k < ns ? k : ns - 1, R[k]);
        store(0, R[0], 0);
        __syncthreads();
        // Rn holds slab s + 1, Rf receives slab s + NPF (past the end: a repeated, never stored load)
        // (a stagger of SIMD partners -- waves 4..7 issuing their loads after the slab's MFMAs --
        // measured 5 % slower on the dual launch, profiles/r02_ab_wgrad_stg.log)
        auto iter = [&](int s, const Stage &Rn, Stage &Rf) {
            const int buf = s & 1;
            load(s + NPF < ns ? s + NPF : ns - 1, Rf);
            __builtin_amdgcn_sched_barrier(0);
            slab(buf);
            if constexpr (IL) {
                store(s + 1, Rn, buf ^ 1);
                constexpr int NM = 6 * NP;  // MFMAs per wave and slab
                __builtin_amdgcn_sched_group_barrier(0x100, 10 * NP, 0);  // the fragment reads first
#pragma unroll
                for (int k = 0; k < NM; ++k) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);               // one MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, NP == 3 ? 4 : 5, 0);  // vector ALU
                    if (k % (NP == 3 ? 3 : 2) == 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // LDS store
                }
            } else {
                __builtin_amdgcn_sched_barrier(0);
                store(s + 1, Rn, buf ^ 1);
            }
            __syncthreads();
        };
        int s = 0;
        for (; s + NPF - 1 < ns; s += NPF) {
#pragma unroll
            for (int k = 0; k < NPF; ++k) iter(s + k, R[(k + 1) % NPF], R[k]);
        }
#pragma unroll
        for (int k = 0; k < NPF - 1; ++k)
            if (s + k < ns) iter(s + k, R[(k + 1) % NPF], R[k]);
    }
    if constexpr (NP == 2) {
        const int bad = __syncthreads_or(!(amax < 32768.0f));
        if (t == 0) *flag = bad;
        if (bad) return;
    }
    float *P = part + (size_t)sp * K * N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int n = wn + 32 * j + (lane & 31);
            if (n >= N) continue;
            const int oc = n + rot < N ? n + rot : n + rot - N;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = k0 + wk + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                if (row < K) P[(size_t)row * N + oc] = NP == 2 ? ldexpf(acc[i][j][reg], -ge) : acc[i][j][reg];
            }
        }
}

template <int NP, bool IL>
__global__ void __launch_bounds__(kWWT, 1)
wgrad_w_kernel(const float *__restrict__ A, int lda, const float *__restrict__ G, int ldg, const int *__restrict__ rexp,
               float *__restrict__ part, int M, int K, int N, int rot, int rows_per_split, int ktiles,
               int *__restrict__ flags) {
    __shared__ __attribute__((aligned(16))) WwLds lds;
    const int id = xcd_remap_x3(blockIdx.x, gridDim.x);
    if (NP == 3 && flags && flags[id] == 0) return;  // fixup launch: only the flagged workgroups
    wgrad_w_body<NP, IL>(A, lda, G, ldg, rexp, part, M, K, N, rot, rows_per_split, id / ktiles, (id % ktiles) * kX3M,
                         flags ? flags + id : nullptr, lds);
}

// Two weight gradients over the same rows of G's buffer in one launch (a GRU cell's dWh = h^T dGh and
// dF = x^T dGi, both from the packed backward rows): the k tiles of both products for one row split
// are consecutive workgroup ids, so they stream the same rows together (L2 hits for all but one).
struct WgradProblem {
    const float *A;
    int lda;
    const void *G;  // fp32 rows, or (planes launches) fp16x2 planes, ldg in fp16 elements
    int ldg;
    float *part;
    int K, N, rot, ktiles;
};

template <int NP, bool PLG = false>
__global__ void __launch_bounds__(kWWT, 1)
wgrad_w_dual_kernel(WgradProblem p0, WgradProblem p1, const int *__restrict__ rexp, int M, int rows_per_split,
                    int *__restrict__ flags, int plo = 0) {
    __shared__ __attribute__((aligned(16))) WwLds lds;
    const int id = xcd_remap_x3(blockIdx.x, gridDim.x);
    if (NP == 3 && flags[id] == 0) return;  // fixup launch: only the flagged workgroups
    const int T = p0.ktiles + p1.ktiles, sub = id % T, sp = id / T;
    const bool first = sub < p0.ktiles;
    const WgradProblem &p = first ? p0 : p1;
    const int k0 = (first ? sub : sub - p0.ktiles) * kX3M;
    wgrad_w_body<NP, true, PLG>(p.A, p.lda, p.G, p.ldg, rexp, p.part, M, p.K, p.N, p.rot, rows_per_split, sp, k0,
                                flags + id, lds, plo);
}

// ---------------------------------------------------------------------------------------------
// Planes weight gradient (msat_gemm_wgrad_h2_dual_planes): the same two products as wgrad_w_dual_kernel<2>
// with G the GRU backward's packed rows as fp16x2 planes, each row already split at its own exponent e_r.
// G is therefore staged with no vector work at all: LDS-DMA (global_load_lds_dwordx4) writes the planes
// straight into the swizzled [16 rows][128 cols] images the transposed fragment reads expect (lane l of a
// 1 KiB piece fetches the source chunk that w3off maps to position l).  The split-wide scale moves to A:
// with ge the split's smallest row exponent, a' = a 2^(kPlA + ge - e_r) (range-checked as before) and
// sum_r a'_r g'_r = 2^(ge + kPlA) sum_r a_r g_r, rescaled on store.  A's raw fp32 slabs and the slab's row
// exponents arrive by LDS-DMA too; each thread splits its 4 A elements from LDS into the A images.  Every global
// access in the k walk is an asm DMA, so its counted waits (5 per wave and slab: 3 G pieces, 1 A piece, 1 row-
// exponent piece) are exact.  Per slab and wave: 18 MFMAs, ~45 vector instructions (the A split and the DMA
// offsets), against ~100 in wgrad_w_body<2> (A and G split per k tile).  Each slab's fragments are read one
// iteration ahead into registers, so its MFMAs start right after the barrier and the next slab's LDS reads run
// under them; three DMA groups (96 KiB) are in flight per CU (the ring discipline is at `iter` below).
//
// A's headroom exponent kPlA: with G at full scale in every row, a row whose G is 2^d below the split's largest
// carries a' = a 2^(kPlA - d); once a' is an fp16 subnormal its absolute error (2^-25) multiplies a full-scale g
// (2^14): relative to the split's dominant term |a_0| 2^14 that is 2^-(25 + kPlA) / |a_0| per such row (the
// fp32-row form's G-side scale: 2^-39 |a_r / a_0|).  kPlA = 0 failed the 4e-6 bound at |a_0| < 2^-7 on rows
// spread over 43 binades (tests/test_planes_gpu.py); kPlA = 8 moves that to |a_0| < 2^-15.  The price: the range
// check flags |a| >= 2^(15 - kPlA) = 128 in the split's largest rows (a flagged workgroup is recomputed in bf16x3,
// correct either way).  Shifts are capped at 63 (with |a'| < 2^15 a larger one leaves a' below fp16's smallest
// subnormal either way); an all-zero G row (kExpZero) leaves its a unscaled (the product is zero).
constexpr int kPlA = 8;
// Ablation builds only (make ab AB_FLAGS=-DMSAT_WGRAD_ABL=n, timing diagnostics, wrong results): bit 0 drops the
// MFMAs, bit 1 the fragment reads, bit 2 the DMAs, bit 3 the A split, bit 4 the k walk's barriers (with bits
// 1-3 only).  0 in every product build.
#ifndef MSAT_WGRAD_ABL
#define MSAT_WGRAD_ABL 0
#endif
constexpr int kPlSlots = 4;  // G / raw A / row-exponent ring depth: 3 groups in flight + the slab being read

struct WpLds {
    unsigned short a[2][2][kW3Plane];         // A images (hi, lo) by slab parity: 16 KiB
    unsigned short g[kPlSlots][6][kW3Plane];  // G images [slot][q * 3 + u] (q: hi / lo, u: 128-column block): 96 KiB
    float raw[kPlSlots][16 * kX3M];           // raw fp32 A slabs: 32 KiB
    int rx[kPlSlots][8][64];                  // per wave: its two rows' exponents, lane l -> row 2 w + (l & 1)
    int red[8];
};

// One DMA group of a wave: its three G pieces (consecutive 1 KiB of one G slot), its raw A piece and its row-
// exponent piece (4 B per lane), M0 saved and restored once for the five.
__device__ __forceinline__ void pl_group_dma(const void *gbase, unsigned gv0, unsigned gv1, unsigned gv2, unsigned gdst,
                                             const void *abase, unsigned av, unsigned adst, const void *xbase,
                                             unsigned xv, unsigned xdst) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %7\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %7\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %7\n\t"
        "s_mov_b32 m0, %8\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %9\n\t"
        "s_mov_b32 m0, %10\n\ts_nop 0\n\tglobal_load_lds_dword %5, %11\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gv0), "v"(gv1), "v"(gv2), "v"(av), "v"(xv), "s"(gdst), "s"(gbase), "s"(adst), "s"(abase), "s"(xdst),
          "s"(xbase)
        : "memory");
}

__device__ __forceinline__ float vsub_f32(float a, float b) {  // one v_sub_f32 (not SLP-packed beside the MFMAs)
    float r;
    asm volatile("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ void wgrad_pl_body(const float *__restrict__ A, int lda, const _Float16 *__restrict__ G,
                                              int ldg, int plo, const int *__restrict__ rexp, float *__restrict__ part,
                                              int M, int K, int N, int rot, int rows_per_split, int sp, int k0,
                                              int *flag, WpLds &L) {
    const int t = threadIdx.x, w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int wk = (w & 1) * 64, wn = (w >> 1) * 96;
    const int rb = sp * rows_per_split, re = min(M, rb + rows_per_split), nr = re - rb;
    const int ns = (nr + 15) / 16;
    // the split's smallest row exponent
    int mn = kExpZero;
    for (int r = rb + t; r < re; r += kWWT) mn = min(mn, rexp[r]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mn = min(mn, __shfl_xor(mn, o, 64));
    if (lane == 0) L.red[w] = mn;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kWWT / 64; ++i) mn = min(mn, L.red[i]);
    const int ge = mn == kExpZero ? 0 : mn;
    f32x16v acc[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = f32x16v{};
    // per-lane DMA pieces: G piece x = 3 w + e (plane block x >> 2 = q * 3 + u, rows 4 (x & 3) ..; the three are
    // consecutive 1 KiB of a G slot), raw A rows 2 w, 2 w + 1, row exponents of rows 2 w + (lane & 1)
    int grow[3];
    unsigned goff[3], gcb[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const int x = 3 * w + e, pb = x >> 2, row = 4 * (x & 3) + (lane >> 4);
        const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
        const int col = 128 * (pb % 3) + 8 * ch;
        const int gco = (pb / 3) * plo + (col < N ? col : 0);
        grow[e] = row;
        goff[e] = (unsigned)((row * ldg + gco) * 2);  // the last slab clamps: min(off(row), off(lim))
        gcb[e] = (unsigned)(gco * 2);
    }
    const int arow = 2 * w + (lane >> 5), kc = k0 + 4 * (lane & 31), aco = kc < K ? kc : 0;
    const unsigned aoff = (unsigned)((arow * lda + aco) * 4), acb = (unsigned)(aco * 4);
    const int xrow = 2 * w + (lane & 1);
    const unsigned xoff = (unsigned)(xrow * 4);
    const char *gsplit = reinterpret_cast<const char *>(G + (size_t)rb * ldg);  // slab kk at + kk * 16 rows
    const char *asplit = reinterpret_cast<const char *>(A + (size_t)rb * lda);
    const char *xsplit = reinterpret_cast<const char *>(rexp + rb);
    const int gstep = 32 * ldg, astep = 64 * lda;  // bytes per 16-row slab
    // slots are compile-time: the k walk is unrolled by four (kPlSlots, a multiple of the two A images)
    // group k: G(k) -> g[RG], raw A(k + 1) + its row exponents -> slot (RG + 1) % 4; RG == k % 4.  CL: the group
    // may reach the split's last, partial slab or past it (rows clamped); the main walk runs without
    auto issue = [&](int k, auto RG, auto CL) {
        constexpr int rg = decltype(RG)::value, ra = (rg + 1) % kPlSlots;
        if constexpr ((MSAT_WGRAD_ABL & 4) != 0) return;
        const int kg = decltype(CL)::value ? min(k, ns - 1) : k, ka = decltype(CL)::value ? min(k + 1, ns - 1) : k + 1;
        unsigned gv[3], av = aoff, xv = xoff;
#pragma unroll
        for (int e = 0; e < 3; ++e) gv[e] = goff[e];
        if constexpr (decltype(CL)::value) {
            const int limg = nr - 1 - 16 * kg, lima = nr - 1 - 16 * ka;
            const unsigned lb = (unsigned)(limg * ldg * 2);
#pragma unroll
            for (int e = 0; e < 3; ++e) {
                MSAT_DCHECK(rb + 16 * kg + min(grow[e], limg), M);  // debug: the clamped source row
                gv[e] = min(goff[e], lb + gcb[e]);
            }
            MSAT_DCHECK(rb + 16 * ka + min(arow, lima), M);
            av = min(aoff, (unsigned)(lima * lda * 4) + acb);
            xv = (unsigned)(min(xrow, lima) * 4);
        }
        const unsigned gdst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)&L.g[rg][0][0] + 3072u * w);
        const unsigned adst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)&L.raw[ra][w * 256]);
        const unsigned xdst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)&L.rx[ra][w][0]);
        pl_group_dma(gsplit + (size_t)kg * gstep, gv[0], gv[1], gv[2], gdst, asplit + (size_t)ka * astep, av, adst,
                     xsplit + (size_t)ka * 64, xv, xdst);
    };
    auto issue_a0 = [&]() {  // raw A(0) + row exponents -> slot 0 (the prologue)
        if constexpr ((MSAT_WGRAD_ABL & 4) != 0) return;
        const int lim = nr - 1;
        glds16_async_s(asplit, min(aoff, (unsigned)(lim * lda * 4) + acb), &L.raw[0][w * 256]);
        glds4_async_s(xsplit, (unsigned)(min(xrow, lim) * 4), &L.rx[0][w][0]);
    };
    const int srow = t >> 5, sc = (t & 31) * 4;
    const int off = w3off(srow, sc >> 3) + 8 * ((sc >> 2) & 1);
    // the split of raw A(k) (slot RK == k % 4) into image k & 1 in two halves: its LDS reads (issued ahead of the
    // iteration's fragment reads, so waiting for them never waits for those) and the vector work + image store.
    // a' = ldexp(a, sh), fp16 hi by v_cvt_pk_f16_f32 (RNE, as (_Float16)), lo = fp16(a' - hi) (v_sub_f32 kept
    // unpacked: packed f32 beside MFMAs costs issue cycles).
    struct SplitIn {
        float4 v;
        int e;
    };
    auto split_load = [&](auto RK) {
        constexpr int rk = decltype(RK)::value;
        SplitIn r;
        r.v = *reinterpret_cast<const float4 *>(&L.raw[rk][srow * kX3M + sc]);
        r.e = L.rx[rk][w][srow & 1];
        return r;
    };
    float4 cmx = make_float4(0.f, 0.f, 0.f, 0.f);  // largest |a'| of this thread's four columns (small-column check)
    auto split_store = [&](const SplitIn &in, int k, auto RK, auto CL) {
        constexpr int rk = decltype(RK)::value;
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        typedef float f2 __attribute__((ext_vector_type(2)));
        int sh = in.e == kExpZero ? 0 : kPlA - min(in.e - ge, 63);  // in [-55, 8]
        // CL: rows past the split -> 2^-200 (0 for every finite a; a non-finite one stays non-finite and flags)
        if constexpr (decltype(CL)::value) sh = 16 * k + srow < nr ? sh : -200;
        const f2 x01 = {ldexpf(in.v.x, sh), ldexpf(in.v.y, sh)}, x23 = {ldexpf(in.v.z, sh), ldexpf(in.v.w, sh)};
        cmx.x = fmaxf(cmx.x, fabsf(x01[0]));
        cmx.y = fmaxf(cmx.y, fabsf(x01[1]));
        cmx.z = fmaxf(cmx.z, fabsf(x23[0]));
        cmx.w = fmaxf(cmx.w, fabsf(x23[1]));
        const h2 h01 = __builtin_convertvector(x01, h2), h23 = __builtin_convertvector(x23, h2);
        const f2 b01 = __builtin_convertvector(h01, f2), b23 = __builtin_convertvector(h23, f2);
        const f2 r01 = {vsub_f32(x01[0], b01[0]), vsub_f32(x01[1], b01[1])};
        const f2 r23 = {vsub_f32(x23[0], b23[0]), vsub_f32(x23[1], b23[1])};
        const h2 l01 = __builtin_convertvector(r01, h2), l23 = __builtin_convertvector(r23, h2);
        *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(L.a[rk & 1][0]) + off) =
            make_uint2(__builtin_bit_cast(unsigned, h01), __builtin_bit_cast(unsigned, h23));
        *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(L.a[rk & 1][1]) + off) =
            make_uint2(__builtin_bit_cast(unsigned, l01), __builtin_bit_cast(unsigned, l23));
    };
    auto split_a = [&](int k, auto RK) {  // raw[k % 4] -> a[k & 1]; RK == k % 4 (the prologue)
        if constexpr ((MSAT_WGRAD_ABL & 8) != 0) return;
        split_store(split_load(RK), k, RK, std::true_type{});
    };
    const int h = lane >> 5, g = (lane >> 4) & 1;
    struct Frags {
        bf16x8 fa[2][2], fb[3][2];  // [tile][hi, lo]
    };
    auto read_frags = [&](Frags &F, auto RS, bool first = false) {  // the slab's A image and G slot, RS == slab % 4
        constexpr int rs = decltype(RS)::value;
        if ((MSAT_WGRAD_ABL & 2) != 0 && !first) return;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int i = 0; i < 2; ++i) F.fa[i][q] = tr_frag(L.a[rs & 1][q], 8 * h, (wk + 32 * i + 16 * g) >> 3, lane);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int n = wn + 32 * j;
                F.fb[j][q] = tr_frag(L.g[rs][3 * q + (n >> 7)], 8 * h, ((n & 127) + 16 * g) >> 3, lane);
            }
        }
    };
    auto mfmas = [&](const Frags &F) {
        if constexpr ((MSAT_WGRAD_ABL & 1) != 0) {  // keep the fragment reads alive: one add per fragment
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int q = 0; q < 2; ++q) acc[i][0][q] += __builtin_bit_cast(float4, F.fa[i][q]).x;
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int q = 0; q < 2; ++q) acc[1][j][4 + q] += __builtin_bit_cast(float4, F.fb[j][q]).x;
            return;
        }
        // pass-major (an accumulator's three products six MFMAs apart; measured the same as accumulator-major)
        typedef _Float16 f16x8w __attribute__((ext_vector_type(8)));
#pragma unroll
        for (int pass = 0; pass < 3; ++pass)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    // h l, l h, h h (each element's order of accumulation)
                    const f16x8w a = __builtin_bit_cast(f16x8w, F.fa[i][pass == 1 ? 1 : 0]);
                    const f16x8w b = __builtin_bit_cast(f16x8w, F.fb[j][pass == 0 ? 1 : 0]);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[i][j], 0, 0, 0);
                }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    // Iteration s (RS == s % 4): slab s's fragments are already in registers (Fc, read during iteration s - 1), so
    // its MFMAs start at once; slab s + 1's fragment reads (Fn) run under them, as does the split of raw A(s + 2)
    // into image (s + 2) & 1 == s & 1 (slab s's image, read out during s - 1).  DMA group s + 4 (5 per wave) goes
    // into G slot s % 4 (read out during s - 1) and raw / exponent slot (s + 5) % 4 (split during s - 1).  The end
    // waits for group s + 2 (vmcnt 10: groups s + 3 and s + 4 may fly) and a barrier: iteration s + 1 reads slab
    // s + 2's fragments from G(s + 2) and the image written here, and splits raw A(s + 3) (group s + 2).
    auto iter = [&](int s, auto RS, const Frags &Fc, Frags &Fn, auto CL) {
        constexpr int rs = decltype(RS)::value;
        using RK = std::integral_constant<int, (rs + 2) % kPlSlots>;
        issue(s + 4, RS, CL);
        __builtin_amdgcn_sched_barrier(0);
        // unconditional split (straight-line code): near the end it splits clamped slabs into the unused image,
        // every row of them past the split (zeros)
        SplitIn si{};
        if constexpr ((MSAT_WGRAD_ABL & 8) == 0) si = split_load(RK{});
        mfmas(Fc);
        read_frags(Fn, std::integral_constant<int, (rs + 1) % kPlSlots>{});
        if constexpr ((MSAT_WGRAD_ABL & 8) == 0) split_store(si, s + 2, RK{}, CL);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // the split's reads first
#pragma unroll
        for (int k = 0; k < 18; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            if (k < 10) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // fragment reads
            __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // vector ALU
            if (k == 13) __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);  // A image store
        }
        wait_vmcnt<10>();  // group s + 2
        if constexpr ((MSAT_WGRAD_ABL & 16) == 0) barrier_lds();
    };
    if (ns > 0) {
        Frags F0, F1;
        using T1 = std::true_type;
        using F_ = std::false_type;
        issue_a0();
        issue(0, I0{}, T1{});
        issue(1, I1{}, T1{});
        issue(2, I2{}, T1{});
        wait_vmcnt<15>();  // raw A(0) + exponents (this wave's own rows)
        split_a(0, I0{});
        // this wave's reads of slot 0 are done before group 3 refills it with raw A(4) (each wave reads only the
        // rows its own DMA pieces write)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(3, I3{}, T1{});
        wait_vmcnt<15>();  // group 0: G(0), raw A(1)
        split_a(1, I1{});
        wait_vmcnt<10>();  // group 1: G(1), raw A(2)
        barrier_lds();
        read_frags(F0, I0{}, true);
        if ((MSAT_WGRAD_ABL & 2) != 0) F1 = F0;
        barrier_lds();  // every wave's slab-0 reads are done before group 4 refills G slot 0
        // main walk: every group it issues (k <= s + 7, raw A k + 1 <= s + 8) and every slab it splits (<= s + 5)
        // is a full slab of the split (nfull of them), so no row is clamped or masked
        const int nfull = nr / 16;
        int s = 0;
        for (; s + 9 <= nfull; s += 4) {
            iter(s, I0{}, F0, F1, F_{});
            iter(s + 1, I1{}, F1, F0, F_{});
            iter(s + 2, I2{}, F0, F1, F_{});
            iter(s + 3, I3{}, F1, F0, F_{});
        }
        for (; s + 4 <= ns; s += 4) {
            iter(s, I0{}, F0, F1, T1{});
            iter(s + 1, I1{}, F1, F0, T1{});
            iter(s + 2, I2{}, F0, F1, T1{});
            iter(s + 3, I3{}, F1, F0, T1{});
        }
        if (s < ns) iter(s, I0{}, F0, F1, T1{});
        if (s + 1 < ns) iter(s + 1, I1{}, F1, F0, T1{});
        if (s + 2 < ns) iter(s + 2, I2{}, F0, F1, T1{});
        wait_vmcnt<0>();  // the last (clamped, unused) groups land before the workgroup's LDS is released
    }
    // Range: an A element whose scaled value overflows fp16 (|a'| >= 65520) or any non-finite input leaves a
    // non-finite accumulator (Inf hi, Inf * 0 = NaN), so a workgroup with one is recomputed by the bf16x3 fixup --
    // which also reproduces a genuine Inf / NaN of the fp32 product.  Below that the split is exact to 2^-22
    // (|a' - hi| <= 16 is exact in fp32 and its fp16 keeps 11 bits).
    bool nonfin = false;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) nonfin |= !(fabsf(acc[i][j][reg]) <= 3.402823466e38f);
    if (MSAT_WGRAD_ABL) nonfin = false;  // ablation builds: never the fixup (its time is not the kernel's)
    // Small columns: a column of A whose largest |a'| over the split is below 2^-7 but not zero (a
    // collapsed LayerNorm unit, say) keeps only fp16-subnormal precision in a' (absolute 2^-25, i.e. > 2^-18 of
    // its own terms): the workgroup goes to the bf16x3 fixup, whose operands keep fp32's exponent range.  The 16
    // threads of a column group pool their maxima in the (now free) raw-A slots.
    __syncthreads();  // every wave is past its last split and fragment reads
    float *cm = L.raw[0];
    *reinterpret_cast<float4 *>(&cm[srow * kX3M + sc]) = cmx;
    __syncthreads();
    bool small = false;
    if (t < kX3M && k0 + t < K) {
        float m = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) m = fmaxf(m, cm[r * kX3M + t]);
        small = m > 0.f && m < 0.0078125f;
    }
    if (MSAT_WGRAD_ABL) small = false;
    const int bad = __syncthreads_or(nonfin || small);
    if (t == 0) *flag = bad;
    if (bad) return;
    float *P = part + (size_t)sp * K * N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int n = wn + 32 * j + (lane & 31);
            if (n >= N) continue;
            const int oc = n + rot < N ? n + rot : n + rot - N;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = k0 + wk + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                if (row < K) P[(size_t)row * N + oc] = ldexpf(acc[i][j][reg], -(ge + kPlA));
            }
        }
}

__global__ void __launch_bounds__(kWWT, 1)
wgrad_w_dual_pl_kernel(WgradProblem p0, WgradProblem p1, int plo, const int *__restrict__ rexp, int M,
                       int rows_per_split, int *__restrict__ flags) {
    __shared__ __attribute__((aligned(16))) WpLds lds;
    const int id = xcd_remap_x3(blockIdx.x, gridDim.x);
    const int T = p0.ktiles + p1.ktiles, sub = id % T, sp = id / T;
    const bool first = sub < p0.ktiles;
    const WgradProblem &p = first ? p0 : p1;
    const int k0 = (first ? sub : sub - p0.ktiles) * kX3M;
    wgrad_pl_body(p.A, p.lda, reinterpret_cast<const _Float16 *>(p.G), p.ldg, plo, rexp, p.part, M, p.K, p.N, p.rot,
                  rows_per_split, sp, k0, flags + id, lds);
}

static bool a16x3(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace msat

using namespace msat;

extern "C" int msat_split_bf16x3_rot(const float *W, int32_t rows, int32_t cols, int32_t ldw, int32_t rot,
                                     void *planes, void *stream) {
    if (rows == 0 || cols == 0) return MSAT_OK;
    MSAT_REQUIRE(W && planes && rows > 0 && cols > 0 && ldw >= cols && rot >= 0 && rot < cols,
                 "bad split_bf16x3 args");
    const size_t n = (size_t)rows * cols;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(split_bf16x3_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, W, rows, cols, ldw, rot,
                       reinterpret_cast<__bf16 *>(planes));
    return check_launch("split_bf16x3_kernel");
}

extern "C" int msat_split_bf16x3(const float *W, int32_t rows, int32_t cols, int32_t ldw, void *planes, void *stream) {
    return msat_split_bf16x3_rot(W, rows, cols, ldw, 0, planes, stream);
}

extern "C" int msat_gemm_x3(const float *A, int32_t lda, const void *Wplanes, float *C, int32_t ldc, const float *bias,
                            int32_t M, int32_t N, int32_t K, int32_t accumulate, void *stream) {
    if (M == 0) return MSAT_OK;
    MSAT_REQUIRE(A && Wplanes && C && M > 0 && N > 0 && K > 0, "bad gemm_x3 args");
    MSAT_REQUIRE(K % kX3D == 0 && lda % 4 == 0 && lda >= K && ldc >= N && a16x3(A) && a16x3(Wplanes) &&
                     (K * 2) % 16 == 0,
                 "gemm_x3: K %% 16, lda %% 4 and 16-byte aligned operands required");
    const int ntn = (N + kX3M - 1) / kX3M;
    const int vec = (N % 4 == 0 && ldc % 4 == 0 && a16x3(C) && (!bias || a16x3(bias))) ? 1 : 0;
    const __bf16 *Wb = reinterpret_cast<const __bf16 *>(Wplanes);
    const int ntm = (M + 127) / 128;
    if (K % 32 == 0) {  // register-A kernel on 16x16x32 MFMAs, 128-row tiles
        hipLaunchKernelGGL((gemm_x3r16_kernel<2>), dim3(ntm * ntn), dim3(kX3T), 0, (hipStream_t)stream, A, lda, Wb, C,
                           ldc, bias, M, N, K, accumulate, ntn, vec);
        return check_launch("gemm_x3r16_kernel");
    }
    hipLaunchKernelGGL((gemm_x3_kernel<2>), dim3(ntm * ntn), dim3(kX3T), 0, (hipStream_t)stream, A, lda, Wb, C, ldc,
                       bias, M, N, K, accumulate, ntn, vec);
    return check_launch("gemm_x3_kernel");
}

// Launch of the split weight gradient (called from gemm.hip's msat_gemm_wgrad): K % 4, N % 4,
// 16-byte aligned rows.  part >= splits * K * N floats.
bool msat_wgrad_x3_ok(const float *A, int lda, const float *G, int ldg, int K, int N) {
    return K % 4 == 0 && N % 4 == 0 && K >= 16 && lda % 4 == 0 && ldg % 4 == 0 && a16x3(A) && a16x3(G);
}

int msat_wgrad_x3_launch(const float *A, int lda, const float *G, int ldg, float *part, int M, int K, int N, int splits,
                         int rows_per_split, hipStream_t s) {
    const int ntk = (K + kX3M - 1) / kX3M, ntn = (N + kX3M - 1) / kX3M, tiles = ntk * ntn;
    hipLaunchKernelGGL(wgrad_x3_kernel, dim3(tiles * splits), dim3(kX3T), 0, s, A, lda, G, ldg, part, M, K, N,
                       rows_per_split, ntn, tiles);
    return check_launch("wgrad_x3_kernel");
}

// Whole-row weight gradient (wgrad_w_kernel): N <= 384 besides the x3 conditions.
bool msat_wgrad_x3w_ok(const float *A, int lda, const float *G, int ldg, int K, int N) {
    return N <= kWWN && msat_wgrad_x3_ok(A, lda, G, ldg, K, N);
}

// one workgroup per CU: 256 workgroups over the k tiles and row splits, >= 512 rows per split
int msat_wgrad_x3w_splits(int M, int K) {
    const int ktiles = (K + kX3M - 1) / kX3M;
    return std::max(1, std::min(256 / ktiles, (M + 511) / 512));
}

int msat_wgrad_x3w_launch(const float *A, int lda, const float *G, int ldg, float *part, int M, int K, int N, int rot,
                          int splits, hipStream_t s) {
    const int ktiles = (K + kX3M - 1) / kX3M;
    const int rows = (M + splits - 1) / splits, rows16 = ((rows + 15) / 16) * 16;
    hipLaunchKernelGGL((wgrad_w_kernel<3, true>), dim3(ktiles * splits), dim3(kWWT), 0, s, A, lda, G, ldg, nullptr,
                       part, M, K, N, rot, rows16, ktiles, nullptr);
    return check_launch("wgrad_w_kernel<3> (bf16x3)");
}

int msat_wgrad_dual_splits(int M, int K0, int K1) {
    const int T = (K0 + kX3M - 1) / kX3M + (K1 + kX3M - 1) / kX3M;
    return std::max(1, std::min(std::max(1, 256 / T), (M + 511) / 512));
}

// the planes form (wgrad_w_dual_pl_kernel) + its bf16x3 fixup over the flagged workgroups; G0 / G1 fp16x2
// planes (ldg in fp16 elements, lo plane plo elements after hi)
int msat_wgrad_h2_dual_pl_launch(const float *A0, int lda0, const void *G0, int ldg0, float *part0, int K0, int N0,
                                 int rot0, const float *A1, int lda1, const void *G1, int ldg1, float *part1, int K1,
                                 int N1, int rot1, int plo, const int *rexp, int M, int splits, int *flags,
                                 hipStream_t s) {
    WgradProblem p0 = {A0, lda0, G0, ldg0, part0, K0, N0, rot0, (K0 + kX3M - 1) / kX3M};
    WgradProblem p1 = {A1, lda1, G1, ldg1, part1, K1, N1, rot1, (K1 + kX3M - 1) / kX3M};
    const int rows = (M + splits - 1) / splits, rows16 = ((rows + 15) / 16) * 16;
    const dim3 grid(splits * (p0.ktiles + p1.ktiles));
    hipLaunchKernelGGL(wgrad_w_dual_pl_kernel, grid, dim3(kWWT), 0, s, p0, p1, plo, rexp, M, rows16, flags);
    const int rc = check_launch("wgrad_w_dual_pl_kernel (fp16x2 planes)");
    if (rc) return rc;
    hipLaunchKernelGGL((wgrad_w_dual_kernel<3, true>), grid, dim3(kWWT), 0, s, p0, p1, rexp, M, rows16, flags, plo);
    return check_launch("wgrad_w_dual_kernel<3> (planes fixup)");
}

// both products of a cell (wgrad_w_dual_kernel, fp16x2) + the bf16x3 fixup over the flagged workgroups
int msat_wgrad_h2_dual_launch(const float *A0, int lda0, const float *G0, int ldg0, float *part0, int K0, int N0, int rot0,
                              const float *A1, int lda1, const float *G1, int ldg1, float *part1, int K1, int N1,
                              int rot1, const int *rexp, int M, int splits, int *flags, hipStream_t s) {
    WgradProblem p0 = {A0, lda0, G0, ldg0, part0, K0, N0, rot0, (K0 + kX3M - 1) / kX3M};
    WgradProblem p1 = {A1, lda1, G1, ldg1, part1, K1, N1, rot1, (K1 + kX3M - 1) / kX3M};
    const int rows = (M + splits - 1) / splits, rows16 = ((rows + 15) / 16) * 16;
    const dim3 grid(splits * (p0.ktiles + p1.ktiles));
    hipLaunchKernelGGL(wgrad_w_dual_kernel<2>, grid, dim3(kWWT), 0, s, p0, p1, rexp, M, rows16, flags);
    const int rc = check_launch("wgrad_w_dual_kernel<2> (fp16x2)");
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_w_dual_kernel<3>, grid, dim3(kWWT), 0, s, p0, p1, rexp, M, rows16, flags);
    return check_launch("wgrad_w_dual_kernel<3> (fixup)");
}

// fp16x2 form + its bf16x3 fixup launch over the workgroups it flagged (flags: ktiles * splits ints)
int msat_wgrad_h2w_launch(const float *A, int lda, const float *G, int ldg, const int *rexp, float *part, int M, int K,
                          int N, int rot, int splits, int *flags, hipStream_t s) {
    const int ktiles = (K + kX3M - 1) / kX3M;
    const int rows = (M + splits - 1) / splits, rows16 = ((rows + 15) / 16) * 16;
    hipLaunchKernelGGL((wgrad_w_kernel<2, true>), dim3(ktiles * splits), dim3(kWWT), 0, s, A, lda, G, ldg, rexp, part,
                       M, K, N, rot, rows16, ktiles, flags);
    int rc = check_launch("wgrad_w_kernel<2> (fp16x2)");
    if (rc) return rc;
    hipLaunchKernelGGL((wgrad_w_kernel<3, true>), dim3(ktiles * splits), dim3(kWWT), 0, s, A, lda, G, ldg, nullptr,
                       part, M, K, N, rot, rows16, ktiles, flags);
    return check_launch("wgrad_w_kernel<3> (fixup)");
}

extern "C" int msat_split_f16x2_rot(const float *W, int32_t rows, int32_t cols, int32_t ldw, int32_t rot, void *planes,
                                    int32_t *bad, void *stream) {
    MSAT_REQUIRE(W && planes && bad && rows > 0 && cols > 0 && ldw >= cols && rot >= 0 && rot < cols,
                 "bad split_f16x2_rot args");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(bad, 0, sizeof(int32_t), s) != hipSuccess) return check_launch("split_f16x2_rot memset");
    const size_t n = (size_t)rows * cols;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(split_f16x2_rot_kernel, dim3(grid), dim3(256), 0, s, W, rows, cols, ldw, rot,
                       reinterpret_cast<_Float16 *>(planes), bad);
    return check_launch("split_f16x2_rot_kernel");
}

extern "C" int msat_gemm_h2(const float *A, int32_t lda, const int32_t *rexp, const void *Wplanes_h2,
                            const void *Wplanes_x3, const int32_t *wbad, float *C, int32_t ldc, const float *bias,
                            int32_t M, int32_t N, int32_t K, int32_t accumulate, void *stream) {
    if (M == 0) return MSAT_OK;
    MSAT_REQUIRE(A && rexp && Wplanes_h2 && Wplanes_x3 && wbad && C && M > 0 && N > 0 && K > 0, "bad gemm_h2 args");
    MSAT_REQUIRE(K % 32 == 0 && lda % 4 == 0 && lda >= K && ldc >= N && a16x3(A) && a16x3(Wplanes_h2) &&
                     a16x3(Wplanes_x3),
                 "gemm_h2: K %% 32, lda %% 4 and 16-byte aligned operands required");
    const int ntn = (N + kX3M - 1) / kX3M, ntm = (M + 127) / 128;
    const int vec = (N % 4 == 0 && ldc % 4 == 0 && a16x3(C) && (!bias || a16x3(bias))) ? 1 : 0;
    hipLaunchKernelGGL((gemm_h2r16_kernel<2>), dim3(ntm * ntn), dim3(kX3T), 0, (hipStream_t)stream, A, lda, rexp,
                       reinterpret_cast<const uint16_t *>(Wplanes_h2), reinterpret_cast<const uint16_t *>(Wplanes_x3),
                       wbad, C, ldc, bias, M, N, K, accumulate, ntn, vec);
    return check_launch("gemm_h2r16_kernel");
}

// C0 (+)= A0 @ W0^T and C1 (+)= A1 @ W1^T over the same M rows (one row-exponent array), in one launch
// (gemm_h2r16_dual_kernel).  Conditions of msat_gemm_h2 for each product; no bias.
// pl: A0 / A1 are fp16x2 planes (element size 2, lo plane plo elements after hi), else fp32 rows
static int gemm_h2_dual_impl(const void *A0, int32_t lda0, const void *W0_h2, const void *W0_x3,
                             const int32_t *wbad0, float *C0, int32_t ldc0, int32_t N0, int32_t acc0,
                             const void *A1, int32_t lda1, const void *W1_h2, const void *W1_x3,
                             const int32_t *wbad1, float *C1, int32_t ldc1, int32_t N1, int32_t acc1, int pl,
                             int32_t plo, const int32_t *rexp, int32_t M, int32_t K, void *stream) {
    if (M == 0) return MSAT_OK;
    MSAT_REQUIRE(A0 && A1 && W0_h2 && W0_x3 && W1_h2 && W1_x3 && wbad0 && wbad1 && C0 && C1 && rexp && M > 0 &&
                     N0 > 0 && N1 > 0 && K > 0,
                 "bad gemm_h2_dual args");
    const int la = pl ? 8 : 4;  // elements per 16 bytes
    MSAT_REQUIRE(K % 32 == 0 && lda0 % la == 0 && lda1 % la == 0 && lda0 >= K && lda1 >= K && ldc0 >= N0 &&
                     ldc1 >= N1 && a16x3(A0) && a16x3(A1) && a16x3(W0_h2) && a16x3(W0_x3) && a16x3(W1_h2) &&
                     a16x3(W1_x3),
                 "gemm_h2_dual: K %% 32, lda %% 4 (planes: %% 8) and 16-byte aligned operands required");
    // the lo plane of a row's K columns lies inside the row: plo + K <= lda (a layout whose column offset pushes it
    // further is the caller's to rule out; the learner's rows are [hi 4H | lo 4H] with K <= 3H at offsets <= H)
    MSAT_REQUIRE(!pl || (plo % 8 == 0 && plo >= K && plo + K <= lda0 && plo + K <= lda1),
                 "gemm_h2_dual_planes: plo %% 8, plo >= K and plo + K <= lda required");
    DgradProblem p[2];
    const void *As[2] = {A0, A1};
    const int ldas[2] = {lda0, lda1}, ldcs[2] = {ldc0, ldc1}, Ns[2] = {N0, N1}, accs[2] = {acc0, acc1};
    const void *W2[2] = {W0_h2, W1_h2}, *W3[2] = {W0_x3, W1_x3};
    const int32_t *wb[2] = {wbad0, wbad1};
    float *Cs[2] = {C0, C1};
    for (int i = 0; i < 2; ++i) {
        p[i].A = As[i];
        p[i].lda = ldas[i];
        p[i].plo = pl ? plo : 0;
        p[i].Wh2 = reinterpret_cast<const uint16_t *>(W2[i]);
        p[i].Wx3 = reinterpret_cast<const uint16_t *>(W3[i]);
        p[i].wbad = wb[i];
        p[i].C = Cs[i];
        p[i].ldc = ldcs[i];
        p[i].N = Ns[i];
        p[i].accumulate = accs[i];
        p[i].vec_out = (Ns[i] % 4 == 0 && ldcs[i] % 4 == 0 && a16x3(Cs[i])) ? 1 : 0;
        p[i].ntn = (Ns[i] + kX3M - 1) / kX3M;
        p[i].kr = 0;
    }
    // A GRU cell's packed rows D = [dan | dar | daz | dan r]: dh reads D[:, H:4H] (A0 = D + H), the input
    // gradient D[:, 0:3H] (A1 = D).  Started H / 32 double slabs in, the input gradient's walk reads the
    // columns the dh walk reads at the same step for the first 3H - H of its K, so the workgroups of a
    // row block fetch those bytes from HBM once (their walks are otherwise offset by H columns, which at
    // 96 resident workgroups per XCD and 2 KiB rows is enough to lose the L2 copy: 1.33x fetch, round 2).
    {
        const long diff = (long)((const char *)A0 - (const char *)A1);
        const long off = diff / (pl ? 2 : 4);  // in elements
        if (lda0 == lda1 && diff % (pl ? 2 : 4) == 0 && off > 0 && off % 32 == 0 && off / 32 < K / 32)
            p[1].kr = (int)(off / 32);
    }
    // 384-row workgroups of 12 waves (one per CU, three per SIMD as before): each weight slab fetched into
    // LDS serves 384 rows instead of 128, a third of the weight DMA pieces per output; bitwise the same
    // result as 128-row workgroups, 1-2 % faster (profiles/r04w_ab_dgrad_waves.log)
    const int ntm = (M + 383) / 384;
    if (pl)
        hipLaunchKernelGGL((gemm_h2r16_dual_kernel<2, 12, true>), dim3(ntm * (p[0].ntn + p[1].ntn)), dim3(768), 0,
                           (hipStream_t)stream, p[0], p[1], rexp, M, K);
    else
        hipLaunchKernelGGL((gemm_h2r16_dual_kernel<2, 12>), dim3(ntm * (p[0].ntn + p[1].ntn)), dim3(768), 0,
                           (hipStream_t)stream, p[0], p[1], rexp, M, K);
    return check_launch(pl ? "gemm_h2r16_dual_kernel (planes)" : "gemm_h2r16_dual_kernel");
}

extern "C" int msat_gemm_h2_dual(const float *A0, int32_t lda0, const void *W0_h2, const void *W0_x3,
                                 const int32_t *wbad0, float *C0, int32_t ldc0, int32_t N0, int32_t acc0,
                                 const float *A1, int32_t lda1, const void *W1_h2, const void *W1_x3,
                                 const int32_t *wbad1, float *C1, int32_t ldc1, int32_t N1, int32_t acc1,
                                 const int32_t *rexp, int32_t M, int32_t K, void *stream) {
    return gemm_h2_dual_impl(A0, lda0, W0_h2, W0_x3, wbad0, C0, ldc0, N0, acc0, A1, lda1, W1_h2, W1_x3, wbad1, C1, ldc1,
                             N1, acc1, 0, 0, rexp, M, K, stream);
}

// Same products with A0 / A1 the GRU backward's packed rows as fp16x2 planes (msat_gru_ln_bwd_g4fe, flags bit
// 3): lda in fp16 elements (% 8), the lo plane plo elements after the hi plane, rows already at rexp's scale.
extern "C" int msat_gemm_h2_dual_planes(const void *A0, int32_t lda0, const void *W0_h2, const void *W0_x3,
                                        const int32_t *wbad0, float *C0, int32_t ldc0, int32_t N0, int32_t acc0,
                                        const void *A1, int32_t lda1, const void *W1_h2, const void *W1_x3,
                                        const int32_t *wbad1, float *C1, int32_t ldc1, int32_t N1, int32_t acc1,
                                        int32_t plo, const int32_t *rexp, int32_t M, int32_t K, void *stream) {
    return gemm_h2_dual_impl(A0, lda0, W0_h2, W0_x3, wbad0, C0, ldc0, N0, acc0, A1, lda1, W1_h2, W1_x3, wbad1, C1, ldc1,
                             N1, acc1, 1, plo, rexp, M, K, stream);
}
