// Fused GRU cell + LayerNorm forward on the gfx950 matrix cores.
//
// One kernel per encoder GRU call (learner:68-80: update_c / update_v_pos / update_v_neg
// followed by a fresh nn.LayerNorm) computes, for a 64-row tile,
//     [r_pre | z_pre | gin | ghn] = [h | x] @ [[Wh_r Wh_z 0 Wh_n], [Wi_r Wi_z Wi_n 0]] + biases
// on fp32 MFMA 32x32x2 (exact f32), then the flax GRUCell gate algebra and the
// LayerNorm (eps 1e-6, E[x^2]-E[x]^2 variance) in the epilogue, writing only h'.
// It replaces two GEMMs (N = 3H), the gate round trips through HBM and the separate
// GRU/LN row kernel.
//
// Reduction order: k runs over the hidden state first (H rows of Wh, slab-aligned), then
// over the input segments x = [seg0 | seg1 | seg2] (the rows of Wi).  The third gate
// tile therefore accumulates ghn in the hidden slabs and gin in the input slabs; the
// structurally-zero blocks of the stacked weight are never multiplied.
//
// Tile: 64 rows x 4H gate columns per workgroup of H/32 waves.  Wave w owns hidden units
// [32w, 32w+32) of all four gates for all 64 rows (2 x 4 MFMA tiles, 128 accumulators),
// so the gate algebra is lane-local; the LayerNorm row sums are reduced across the 32
// lanes of a half-wave and then across waves through LDS in a fixed order.
// Operand slabs (16 deep) are staged in LDS, register double-buffered.
//
// training: `g4` (nullable) receives the pre-activations [r_pre | z_pre | gin | ghn]
// (R x 4H) that gru_ln_bwd (G4 form) consumes.
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "split3.h"

namespace msat {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kFR = 64;     // rows per workgroup
constexpr int kFK = 16;     // slab depth
constexpr int kFAP = 66;    // A slab row stride (words): conflict-free transposed ds_write_b32

struct GruFwdArgs {
    const float *seg[3];
    int seg_ld[3];
    int seg_w[3];
    const float *hp;
    int ldp;
    const float *wi, *bi, *wh, *bh, *ln_scale, *ln_bias;
    const __bf16 *wip, *whp;  // bf16x3 weight planes [3][kxp][3H] / [3][H][3H] (x3 kernel)
    int kxp;
    float *out;
    int ldo;
    float *g4;
    int ldg;
    int R, Kx;
};

__device__ __forceinline__ float fsig(float x) { return 1.0f / (1.0f + __expf(-x)); }

// GRU gate algebra + LayerNorm on the accumulators of a 64-row tile (shared by both kernels):
// acc[rt][0..3] = [r_pre | z_pre | gin | ghn] (biases not yet added) for rows wrow + 32 rt + ...
template <int NW, int RS, int ROWS = kFR>
__device__ __forceinline__ void gru_ln_epilogue(const GruFwdArgs &a, f32x16 (&acc)[ROWS / 32 / RS][4], float *red_lds,
                                                int row0, int wu, int wrow, int li, int lk) {
    constexpr int H = 32 * NW, RT = ROWS / 32 / RS;
    const int u = 32 * wu + li;
    const float br = a.bi[u] + a.bh[u], bz = a.bi[H + u] + a.bh[H + u];
    const float bni = a.bi[2 * H + u], bnh = a.bh[2 * H + u];
    float2 *red = reinterpret_cast<float2 *>(red_lds);  // [NW][64]
    // h of every row first, all loads in flight together (clamped rows; the value of a row
    // past R is never stored)
    float hvs[RT][16];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = row0 + wrow + rt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * lk;
            hvs[rt][reg] = a.hp[(size_t)(row < a.R ? row : a.R - 1) * a.ldp + u];
        }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int lr = wrow + rt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * lk;
            const int row = row0 + lr;
            const float rp = acc[rt][0][reg] + br, zp = acc[rt][1][reg] + bz;
            const float gi = acc[rt][2][reg] + bni, gh = acc[rt][3][reg] + bnh;
            const float hv = hvs[rt][reg];
            if (row < a.R) {
                if (a.g4) {
                    float *q = a.g4 + (size_t)row * a.ldg + u;
                    q[0] = rp;
                    q[H] = zp;
                    q[2 * H] = gi;
                    q[3 * H] = gh;
                }
            }
            const float rg = fsig(rp), zg = fsig(zp);
            const float ng = tanhf(gi + rg * gh);
            const float hn = (1.0f - zg) * ng + zg * hv;
            acc[rt][0][reg] = hn;
            float s1 = hn, s2 = hn * hn;
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                s1 += __shfl_xor(s1, o, 64);
                s2 += __shfl_xor(s2, o, 64);
            }
            if (li == 0) red[wu * ROWS + lr] = make_float2(s1, s2);
        }
    __syncthreads();
    const float sc = a.ln_scale[u], lb = a.ln_bias[u];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int lr = wrow + rt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * lk;
            const int row = row0 + lr;
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int v = 0; v < NW; ++v) {
                const float2 p = red[v * ROWS + lr];
                s1 += p.x;
                s2 += p.y;
            }
            const float mean = s1 / (float)H;
            const float var = fmaxf(s2 / (float)H - mean * mean, 0.0f);
            const float rs = rsqrtf(var + 1e-6f);
            if (row < a.R) a.out[(size_t)row * a.ldo + u] = (acc[rt][0][reg] - mean) * (rs * sc) + lb;
        }
}

// NW = H / 32 unit groups; RS = waves per unit group (row split of the 64-row tile): wave w
// owns units [32 (w % NW), +32) of all four gates for rows [(w / NW) * 64 / RS, +64 / RS).
template <int NW, int RS>
__global__ void __launch_bounds__(64 * NW * RS, 2)
gru_ln_fused_fwd_kernel(GruFwdArgs a) {
    constexpr int H = 32 * NW, T = 64 * NW * RS, BW = 3 * H, RT = 2 / RS;
    constexpr int AN = (kFR * kFK / 4 + T - 1) / T;  // float4 A loads per thread
    constexpr int BN = (kFK * BW / 4) / T;           // float4 B loads per thread (= 6)
    static_assert((kFK * BW / 4) % T == 0, "B slab split");
    __shared__ __attribute__((aligned(16))) float As[2][kFK * kFAP];
    __shared__ __attribute__((aligned(16))) float Bs[2][kFK * BW];

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wu = w % NW, wrow = (w / NW) * (kFR / RS);
    const int row0 = blockIdx.x * kFR;
    const int nsh = H / kFK;
    const int ns = nsh + (a.Kx + kFK - 1) / kFK;

    // A (activations): register-staged, stored k-major (transposed) into LDS.
    // B (weights, L2-resident): global_load_lds_dwordx4 straight into a lane-linear LDS image
    // (rows of Wi / Wh are contiguous, ld = 3H), no VGPRs.  Rows past Kx are clamped to the
    // last valid row; the matching A columns are zero, so they contribute exact zeros.
    float4 ra[AN];
    auto loadA = [&](int s) {
        const bool hid = s < nsh;
#pragma unroll
        for (int i = 0; i < AN; ++i) {
            const int idx = t + i * T;
            ra[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (idx < kFR * kFK / 4) {
                const int r = row0 + (idx >> 2), kq = (idx & 3) * 4;
                if (r < a.R) {
                    const float *p = nullptr;
                    if (hid) {
                        p = a.hp + (size_t)r * a.ldp + s * kFK + kq;
                    } else {
                        int k = (s - nsh) * kFK + kq;
#pragma unroll
                        for (int g = 0; g < 3; ++g) {
                            if (!p && k < a.seg_w[g]) p = a.seg[g] + (size_t)r * a.seg_ld[g] + k;
                            k -= a.seg_w[g];
                        }
                    }
                    if (p) ra[i] = *reinterpret_cast<const float4 *>(p);
                }
            }
        }
    };
    auto issueB = [&](int s, int buf) {
        const bool hid = s < nsh;
        const float *W = hid ? a.wh : a.wi;
        const int kb = hid ? s * kFK : (s - nsh) * kFK;
        const int klast = (hid ? H : a.Kx) - 1;
#pragma unroll
        for (int i = 0; i < BN; ++i) {
            const int f = i * T + t;  // float4 index in the slab image
            const int r = f / (BW / 4), c4 = f - r * (BW / 4);
            const float *src = W + (size_t)min(kb + r, klast) * BW + 4 * c4;
            float *dst = Bs[buf] + 4 * (i * T + 64 * w);  // wave-uniform base; lane l lands at +16 l bytes
            glds16_async(src, dst);  // retired by the explicit vmcnt wait before the slab barrier
        }
    };
    auto storeA = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AN; ++i) {
            const int idx = t + i * T;
            if (idx < kFR * kFK / 4) {
                const int r = idx >> 2, kq = (idx & 3) * 4;
                float *q = As[buf] + kq * kFAP + r;
                q[0] = ra[i].x;
                q[kFAP] = ra[i].y;
                q[2 * kFAP] = ra[i].z;
                q[3 * kFAP] = ra[i].w;
            }
        }
    };

    f32x16 acc[RT][4];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[i][g] = f32x16{};

    const int li = lane & 31, lk = lane >> 5;
    // hid: third gate tile accumulates ghn (hidden slabs) or gin (input slabs)
    auto slab = [&](int buf, bool hid) {
        const float *A_ = As[buf] + wrow + li, *B_ = Bs[buf] + 32 * wu + li;
#pragma unroll
        for (int kk = 0; kk < kFK; kk += 2) {
            const int kr = kk + lk;
            const float *bp = B_ + kr * BW;
            const float b0 = bp[0], b1 = bp[H], b2 = bp[2 * H];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const float av = A_[kr * kFAP + 32 * rt];
                acc[rt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b0, acc[rt][0], 0, 0, 0);
                acc[rt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b1, acc[rt][1], 0, 0, 0);
                if (hid) acc[rt][3] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b2, acc[rt][3], 0, 0, 0);
                else acc[rt][2] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b2, acc[rt][2], 0, 0, 0);
            }
        }
    };

    issueB(0, 0);
    loadA(0);
    storeA(0);
    wait_vmcnt<0>();
    barrier_lds();
    // two loops (hidden slabs, then input slabs) so each carries one accumulator subset.  Slab
    // s+1 (B by LDS-DMA, A into registers) is in flight while slab s is multiplied; the
    // scheduling barriers keep the MFMAs ahead of the waits that retire it.
    int buf = 0;
    for (int s = 0; s < nsh; ++s) {
        issueB(s + 1, buf ^ 1);  // ns > nsh: there is always a next slab here
        loadA(s + 1);
        slab(buf, true);
        __builtin_amdgcn_sched_barrier(0);
        storeA(buf ^ 1);
        wait_vmcnt<0>();
        barrier_lds();  // B image and A stores of slab s+1 complete; slab s fully read
        buf ^= 1;
    }
    for (int s = nsh; s < ns; ++s) {
        const bool more = s + 1 < ns;
        if (more) {
            issueB(s + 1, buf ^ 1);
            loadA(s + 1);
        }
        slab(buf, false);
        __builtin_amdgcn_sched_barrier(0);
        if (more) storeA(buf ^ 1);
        wait_vmcnt<0>();
        barrier_lds();
        buf ^= 1;
    }

    // ---------------------------------------------------------------- epilogue --
    gru_ln_epilogue<NW, RS>(a, acc, &As[0][0], row0, wu, wrow, li, lk);  // As is free after the last sync
}

// ---------------------------------------------------------------------------------------------
// Transposed-weight form (msat_gru_ln_fused_fwd_t): the weights arrive as W^T [3H][Kp] (k
// contiguous, zero-padded to a multiple of 16), so both operand slabs are k-major 16-deep images
// [o][16] with the 16-byte chunk c of row o at slot c ^ ((o >> 2) & 3) (conflict-free
// ds_read_b128).  A lane's float4 then covers four MFMA k steps (step 4q + r takes k = 8q + r on
// lanes 0-31 and 8q + 4 + r on lanes 32-63, the same permutation on both operands), so a wave
// reads each slab with (RT + 3) x 2 ds_read_b128 instead of 4 ds_read_b32 per k step.
__device__ __forceinline__ int gswz(int o) { return (o >> 2) & 3; }

template <int NW, int RS>
__global__ void __launch_bounds__(64 * NW * RS, 2)
gru_ln_fused_fwd_t_kernel(GruFwdArgs a) {
    constexpr int H = 32 * NW, T = 64 * NW * RS, BW = 3 * H, RT = 2 / RS;
    constexpr int AN = (kFR * kFK / 4 + T - 1) / T;  // float4 A chunks per thread
    constexpr int BN = (BW * kFK / 4) / T;           // float4 B chunks per thread
    static_assert((BW * kFK / 4) % T == 0, "B slab split");
    __shared__ __attribute__((aligned(16))) float As[2][kFR * kFK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BW * kFK];

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wu = w % NW, wrow = (w / NW) * (kFR / RS);
    const int row0 = blockIdx.x * kFR;
    const int nsh = H / kFK;
    const int ns = nsh + (a.Kx + kFK - 1) / kFK;
    const int kxp = (a.Kx + kFK - 1) / kFK * kFK;

    float4 ra[AN];
    auto loadA = [&](int s) {
        const bool hid = s < nsh;
#pragma unroll
        for (int i = 0; i < AN; ++i) {
            const int idx = t + i * T;
            ra[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (idx < kFR * kFK / 4) {
                const int r = row0 + (idx >> 2), kq = (idx & 3) * 4;
                if (r < a.R) {
                    const float *p = nullptr;
                    if (hid) {
                        p = a.hp + (size_t)r * a.ldp + s * kFK + kq;
                    } else {
                        int k = (s - nsh) * kFK + kq;
#pragma unroll
                        for (int g = 0; g < 3; ++g) {
                            if (!p && k < a.seg_w[g]) p = a.seg[g] + (size_t)r * a.seg_ld[g] + k;
                            k -= a.seg_w[g];
                        }
                    }
                    if (p) ra[i] = *reinterpret_cast<const float4 *>(p);
                }
            }
        }
    };
    auto storeA = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AN; ++i) {
            const int idx = t + i * T;
            if (idx < kFR * kFK / 4) {
                const int r = idx >> 2, c = idx & 3;
                *reinterpret_cast<float4 *>(As[buf] + r * kFK + 4 * (c ^ gswz(r))) = ra[i];
            }
        }
    };
    auto issueB = [&](int s, int buf) {
        const bool hid = s < nsh;
        const float *W = hid ? a.wh : a.wi;  // transposed: [3H][H] / [3H][kxp]
        const int ldk = hid ? H : kxp;
        const int kb = hid ? s * kFK : (s - nsh) * kFK;
#pragma unroll
        for (int i = 0; i < BN; ++i) {
            const int f = i * T + t;  // float4 slot of the image: row o = f >> 2, slot f & 3
            const int o = f >> 2, c = (f & 3) ^ gswz(o);
            glds16_async(W + (size_t)o * ldk + kb + 4 * c, Bs[buf] + 4 * (i * T + 64 * w));
        }
    };

    f32x16 acc[RT][4];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[i][g] = f32x16{};

    const int li = lane & 31, lk = lane >> 5;
    auto slab = [&](int buf, bool hid) {
        float4 af[2][RT], bf[2][3];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const int r = wrow + 32 * rt + li;
                af[q][rt] = *reinterpret_cast<const float4 *>(As[buf] + r * kFK + 4 * ((2 * q + lk) ^ gswz(r)));
            }
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const int o = g * H + 32 * wu + li;
                bf[q][g] = *reinterpret_cast<const float4 *>(Bs[buf] + o * kFK + 4 * ((2 * q + lk) ^ gswz(o)));
            }
        }
#define MSAT_GSTEP(Q, C)                                                                                      \
    for (int rt = 0; rt < RT; ++rt) {                                                                         \
        acc[rt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[Q][rt].C, bf[Q][0].C, acc[rt][0], 0, 0, 0);      \
        acc[rt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[Q][rt].C, bf[Q][1].C, acc[rt][1], 0, 0, 0);      \
        if (hid) acc[rt][3] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[Q][rt].C, bf[Q][2].C, acc[rt][3], 0, 0, 0); \
        else acc[rt][2] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[Q][rt].C, bf[Q][2].C, acc[rt][2], 0, 0, 0);     \
    }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (q == 0) {
                MSAT_GSTEP(0, x) MSAT_GSTEP(0, y) MSAT_GSTEP(0, z) MSAT_GSTEP(0, w)
            } else {
                MSAT_GSTEP(1, x) MSAT_GSTEP(1, y) MSAT_GSTEP(1, z) MSAT_GSTEP(1, w)
            }
        }
#undef MSAT_GSTEP
    };

    issueB(0, 0);
    loadA(0);
    storeA(0);
    wait_vmcnt<0>();
    barrier_lds();
    int buf = 0;
    for (int s = 0; s < nsh; ++s) {
        issueB(s + 1, buf ^ 1);
        loadA(s + 1);
        slab(buf, true);
        __builtin_amdgcn_sched_barrier(0);
        storeA(buf ^ 1);
        wait_vmcnt<0>();
        barrier_lds();
        buf ^= 1;
    }
    for (int s = nsh; s < ns; ++s) {
        const bool more = s + 1 < ns;
        if (more) {
            issueB(s + 1, buf ^ 1);
            loadA(s + 1);
        }
        slab(buf, false);
        __builtin_amdgcn_sched_barrier(0);
        if (more) storeA(buf ^ 1);
        wait_vmcnt<0>();
        barrier_lds();
        buf ^= 1;
    }
    gru_ln_epilogue<NW, RS>(a, acc, &As[0][0], row0, wu, wrow, li, lk);
}

// out[c][k] = k < K ? W[k][c] : 0 for c < N, k < Kp (weights -> transposed, zero-padded)
__global__ void transpose_pad_kernel(const float *__restrict__ W, int K, int N, int ldw, float *__restrict__ out,
                                     int Kp) {
    __shared__ float tile[32][33];
    const int k0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
    for (int j = ty; j < 32; j += 8) {
        const int k = k0 + j, c = c0 + tx;
        tile[j][tx] = (k < K && c < N) ? W[(size_t)k * ldw + c] : 0.0f;
    }
    __syncthreads();
    for (int j = ty; j < 32; j += 8) {
        const int c = c0 + j, k = k0 + tx;
        if (c < N && k < Kp) out[(size_t)c * Kp + k] = tile[tx][j];
    }
}

// Fast gate nonlinearities for the x3 epilogue: v_exp + v_rcp (<= 2 ulp each), no IEEE division.
__device__ __forceinline__ float fsig_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float ftanh_fast(float x) {  // 2 sigma(2x) - 1, saturates cleanly at +-1
    return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f;
}

// x3 epilogue (128-row tile, 16 waves, wave = 32 rows x 32 units of all four gates): the gate
// algebra per accumulator, h' staged to LDS as [row][unit] (row stride 132 floats: conflict-free
// for both the column writes and the row reads), then one row per 8 threads: 16 units each,
// LayerNorm sums over 8 lanes, float4 output rows.  hv = h of each accumulator's (row, unit).
template <int NW>
__device__ __forceinline__ void gru_ln_epilogue_x3(const GruFwdArgs &a, f32x16 (&acc)[1][4], const float (&hv)[16],
                                                   float *stage, int row0, int wu, int wrow, int li, int lk, int t) {
    constexpr int H = 32 * NW, HP = H + 4;
    const int u = 32 * wu + li;
    const float br = a.bi[u] + a.bh[u], bz = a.bi[H + u] + a.bh[H + u];
    const float bni = a.bi[2 * H + u], bnh = a.bh[2 * H + u];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int lr = wrow + (reg & 3) + 8 * (reg >> 2) + 4 * lk;
        const int row = row0 + lr;
        const float rp = acc[0][0][reg] + br, zp = acc[0][1][reg] + bz;
        const float gi = acc[0][2][reg] + bni, gh = acc[0][3][reg] + bnh;
        if (a.g4 && row < a.R) {
            float *q = a.g4 + (size_t)row * a.ldg + u;
            q[0] = rp;
            q[H] = zp;
            q[2 * H] = gi;
            q[3 * H] = gh;
        }
        const float rg = fsig_fast(rp), zg = fsig_fast(zp);
        const float ng = ftanh_fast(gi + rg * gh);
        stage[lr * HP + u] = (1.0f - zg) * ng + zg * hv[reg];
    }
    __syncthreads();
    const int r = t >> 3, c0 = (t & 7) * (H / 8);
    float4 v[H / 32];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < H / 32; ++j) {
        v[j] = *reinterpret_cast<const float4 *>(stage + r * HP + c0 + 4 * j);
        s1 += (v[j].x + v[j].y) + (v[j].z + v[j].w);
        s2 += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        s1 += __shfl_xor(s1, o, 8);
        s2 += __shfl_xor(s2, o, 8);
    }
    const float mean = s1 / (float)H;
    const float var = fmaxf(s2 / (float)H - mean * mean, 0.0f);
    const float rs = rsqrtf(var + 1e-6f);
    const int row = row0 + r;
    if (row < a.R) {
#pragma unroll
        for (int j = 0; j < H / 32; ++j) {
            const float4 sc = *reinterpret_cast<const float4 *>(a.ln_scale + c0 + 4 * j);
            const float4 lb = *reinterpret_cast<const float4 *>(a.ln_bias + c0 + 4 * j);
            float4 o;
            o.x = (v[j].x - mean) * (rs * sc.x) + lb.x;
            o.y = (v[j].y - mean) * (rs * sc.y) + lb.y;
            o.z = (v[j].z - mean) * (rs * sc.z) + lb.z;
            o.w = (v[j].w - mean) * (rs * sc.w) + lb.w;
            *reinterpret_cast<float4 *>(a.out + (size_t)row * a.ldo + c0 + 4 * j) = o;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// bf16x3 form (msat_gru_ln_fused_fwd_x3, H = 128): the same cell on the bf16 matrix cores with the
// exact three-way operand split of gemm_x3.hip (six bf16 MFMAs per 16-deep k step, fp32-accurate).
// 128-row tiles, 16 waves (4 unit groups x 4 row groups of 32).  Per 16-deep slab:
//   A (h, then x) is split while staged: fp32 -> registers -> three bf16 planes [128 rows][16 k]
//   (32-byte rows, chunk slot h ^ ((row >> 3) & 1)), read with ds_read_b128;
//   the weights arrive pre-split ([3 planes][K][3H] bf16, msat_split_bf16x3) by LDS-DMA as
//   [plane][gate][16 k][128 cols] images (256-byte rows, w3off swizzle applied on the source
//   side), read as 8-row column fragments with ds_read_b64_tr_b16.
constexpr int kXR = 128;  // rows per workgroup (x3 kernel)
// diagnostic ablations of the x3 kernel's pipeline (timing only, wrong results; never set in the
// product build): bit 0 no weight DMA after slab 0, 1 no activation DMA after the prologue,
// 2 no split after the prologue, 3 no MFMAs, 4 no epilogue
#ifndef MSAT_GRU_ABL
#define MSAT_GRU_ABL 0
#endif
// 16 waves x 32 rows (RS = 4, RT = 1).
//
// Pipeline: every global read of the loop is an LDS-DMA issued from asm (glds16_async*), so the
// compiler inserts no vector-memory waits and one counted wait per slab is exact.  In step s
// (planes buffer s & 1):
//   issue the weight DMA of slab s + 1 (Bs[(s + 1) & 1]) and the raw fp32 activation DMA of
//   slab s + 3 (raw ring slot (s + 3) % 3);
//   MFMAs of slab s;
//   split the raw activations of slab s + 1 (landed one step ago) into the bf16 planes (s + 1) & 1;
//   wait for all but the youngest DMA (slab s + 3's activations) and barrier.
// The hidden-state slabs and the input slabs run as two loops with the gate index of the third
// accumulator fixed at compile time.  Raw activation rows past R are clamped (and zeroed when
// split), k past Kx reads a valid address (zeroed when split).
template <int NW, int RS>
__global__ void __launch_bounds__(64 * NW * RS, 1)
gru_ln_fused_fwd_x3_kernel(GruFwdArgs a) {
    constexpr int H = 32 * NW, T = 64 * NW * RS, BW = 3 * H, RT = 4 / RS;
    static_assert(H == 128, "x3 GRU: one 128-column image per gate");
    static_assert(T == 1024, "x3 GRU: 16 waves");
    constexpr int APL = kXR * kFK;            // bf16 per A plane (128 rows x 16 k)
    constexpr int BPL = kFK * H;              // bf16 per (plane, gate) image (16 k x 128 cols)
    constexpr int BCH = 3 * 3 * BPL / 8;      // 16-byte chunks of a B slab (2304)
    constexpr int BN = (BCH + T - 1) / T;     // glds per thread (3, the last on waves 0..3)
    constexpr int RAWW = kXR * kFK * 4 / 1024;  // waves issuing the raw A DMA (8)
    __shared__ __attribute__((aligned(16))) unsigned short As[2][3][APL];
    __shared__ __attribute__((aligned(16))) unsigned short Bs[2][3 * 3 * BPL];
    __shared__ __attribute__((aligned(16))) float Raw[3][kXR * kFK];

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wv = __builtin_amdgcn_readfirstlane(w);  // wave index, provably uniform
    const int wu = w % NW, wrow = (w / NW) * 32 * RT;
    const int row0 = blockIdx.x * kXR;
    constexpr int nsh = H / kFK;
    const int ns = nsh + a.kxp / kFK;

    // raw A DMA: waves 0..7, lane -> row 16 wv + (lane >> 2), k quad lane & 3 (16 B each);
    // Raw[slot] is row-major [128][16] fp32
    const bool rawer = wv < RAWW;
    const int rrow = (wv & (RAWW - 1)) * 16 + (lane >> 2), rk = (lane & 3) * 4;
    const int rr = row0 + rrow;
    const int rrc = rr < a.R ? rr : a.R - 1;
    const int w0 = a.seg_w[0], w01 = a.seg_w[0] + a.seg_w[1], kx_end = a.Kx;
    // segment bases / strides as scalars (a per-lane select between struct members is otherwise
    // turned into a per-lane load of the kernel argument block)
    const float *const hp = a.hp, *const sg0 = a.seg[0], *const sg1 = a.seg[1], *const sg2 = a.seg[2];
    const int ldp = a.ldp, ld0 = a.seg_ld[0], ld1 = a.seg_ld[1], ld2 = a.seg_ld[2];
    auto issueA = [&](int s) {
        if (!rawer) return;
        const float *p;
        if (s < nsh) {  // uniform branch
            p = hp + ((size_t)rrc * ldp + s * kFK + rk);
        } else {  // per-lane segment select, branch-free
            const int kx = (s - nsh) * kFK + rk;
            const float *q0 = sg0 + ((size_t)rrc * ld0 + (kx < w0 ? kx : 0));
            const float *q1 = sg1 + ((size_t)rrc * ld1 + (kx - w0));
            const float *q2 = sg2 + ((size_t)rrc * ld2 + (kx - w01));
            p = (kx >= w01 && kx < kx_end) ? q2 : ((kx >= w0 && kx < w01) ? q1 : q0);
        }
        glds16_async(p, reinterpret_cast<char *>(Raw[s % 3]) + 1024 * (wv & (RAWW - 1)));
    };
    // split: thread -> row t >> 3, k pair 2 (t & 7) of the raw slab into the three bf16 planes
    // (32-byte rows, chunk slot h ^ ((row >> 3) & 1))
    const int arow = t >> 3, ak = (t & 7) * 2;
    const bool arow_ok = row0 + arow < a.R;
    const int aoff = arow * 32 + 16 * ((ak >> 3) ^ ((arow >> 3) & 1)) + 2 * (ak & 7);
    auto splitA = [&](int s) {
        float2 v = *reinterpret_cast<const float2 *>(&Raw[s % 3][arow * kFK + ak]);
        if (!arow_ok || (s >= nsh && (s - nsh) * kFK + ak >= kx_end)) v = make_float2(0.f, 0.f);
        const Split2 sp = split2(v);
#pragma unroll
        for (int q = 0; q < 3; ++q)
            *reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(As[s & 1][q]) + aoff) = sp.p[q];
    };
    // B chunk idx = i * T + t of [plane][gate][k row][16 slots]: plane / gate are wave-uniform,
    // the per-lane part (k row, swizzled slot) is one 32-bit offset
    const unsigned boff = 2u * (((t >> 4) & 15) * BW + 8 * ((t & 15) ^ ((((t >> 4) & 3) << 2) | ((t >> 6) & 3))));
    auto issueB = [&](int s) {
        const bool hid = s < nsh;
        const __bf16 *W = hid ? a.whp : a.wip;
        const int krows = hid ? H : a.kxp;
        const int kb = hid ? s * kFK : (s - nsh) * kFK;
#pragma unroll
        for (int i = 0; i < BN; ++i) {
            if (i * T + 64 * wv < BCH) {  // whole waves (BCH % 64 == 0)
                const int pg = i * (T / 256) + (wv >> 2);  // plane * 3 + gate
                const int q = pg / 3, g = pg - 3 * q;
                glds16_async_s(W + ((size_t)q * krows + kb) * BW + g * H, boff,
                               reinterpret_cast<char *>(Bs[s & 1]) + 16 * (i * T + 64 * wv));
            }
        }
    };

    f32x16 acc[RT][4];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[i][g] = f32x16{};
    const int li = lane & 31, lk = lane >> 5, gl = (lane >> 4) & 1;
    auto slab = [&](int buf, auto hidc) {
        constexpr bool hid = decltype(hidc)::value;
        bf16x8 fa[RT][3];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const int r = wrow + 32 * i + li;
#pragma unroll
            for (int q = 0; q < 3; ++q)
                fa[i][q] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4 *>(
                                                          reinterpret_cast<const char *>(As[buf][q]) + r * 32 +
                                                          16 * (lk ^ ((r >> 3) & 1))));
        }
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            bf16x8 fb[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) fb[q] = tr_frag(Bs[buf] + (q * 3 + g) * BPL, 8 * lk, (32 * wu + 16 * gl) >> 3, lane);
            constexpr int ai3 = hid ? 3 : 2;
            const int ai = g < 2 ? g : ai3;
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                f32x16 c = acc[i][ai];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[0], c, 0, 0, 0);
                acc[i][ai] = c;
            }
        }
    };

    // prologue: weights of slab 0, raw activations of slabs 0..2 (ns >= 9 > 3)
    issueB(0);
    issueA(0);
    issueA(1);
    issueA(2);
    wait_vmcnt<0>();
    barrier_lds();
    splitA(0);
    barrier_lds();
    auto step = [&](int s, auto hidc) {
        if (s + 1 < ns) {
            if (!(MSAT_GRU_ABL & 1)) issueB(s + 1);
            if (!(MSAT_GRU_ABL & 2) && s + 3 < ns) issueA(s + 3);
        }
        if (!(MSAT_GRU_ABL & 8)) slab(s & 1, hidc);
        __builtin_amdgcn_sched_barrier(0);
        if (!(MSAT_GRU_ABL & 4) && s + 1 < ns) splitA(s + 1);
        // all but this wave's youngest DMA (slab s + 3's activations, raw waves only)
        if (rawer && s + 3 < ns) wait_vmcnt<1>();
        else wait_vmcnt<0>();
        barrier_lds();
    };
#pragma unroll 1
    for (int s = 0; s < nsh; ++s) step(s, std::true_type{});
#pragma unroll 1
    for (int s = nsh; s < ns - 1; ++s) step(s, std::false_type{});
    // last slab: nothing left to fetch; the epilogue's h values load under its MFMAs
    float hv[16];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = row0 + wrow + (reg & 3) + 8 * (reg >> 2) + 4 * lk;
        hv[reg] = hp[(size_t)(row < a.R ? row : a.R - 1) * ldp + 32 * wu + li];
    }
    if (!(MSAT_GRU_ABL & 8)) slab((ns - 1) & 1, std::false_type{});
    barrier_lds();  // every wave is done with the slab buffers before the epilogue reuses them
    if (MSAT_GRU_ABL & 16) {  // keep the accumulators live, store one value per lane
        if (row0 + wrow + li < a.R) a.out[(size_t)(row0 + wrow + li) * a.ldo + 32 * wu + lk] = acc[0][0][0] + acc[0][1][1] + acc[0][2][2] + acc[0][3][3] + hv[0];
        return;
    }
    gru_ln_epilogue_x3<NW>(a, acc, hv, reinterpret_cast<float *>(&Bs[0][0]), row0, wu, wrow, li, lk, t);
}

// ---------------------------------------------------------------------------------------------
// Register-A GRU forward, fp16x2 operands on v_mfma_f32_16x16x32_f16 (msat_gru_ln_fused_fwd_h2r,
// H = 128).  The structure of the bf16x3 register-A kernel below (gru_ln_fused_fwd_x3r_kernel): 128-row
// tile, 8 waves; wave w owns rows 16 w .. 16 w + 15 and ALL 128 units of all four gates (acc[gate][8
// column tiles of 16], 128 accumulator registers), so its activation rows are private and go straight
// from HBM to registers, split there; only the weights go through LDS, transposed planes
// W^T [2][3H][Kp] (Kp % 32 == 0) by LDS-DMA as per-(plane, gate) images [128 units][4 chunks of 8 k]
// (64-byte rows, chunk c at slot c ^ f((u >> 2) & 3), f = {0, 2, 3, 1}), double-buffered.
//
// Operands: x = x1 + x2, x1 = fp16(x), x2 = fp16(x - x1) (22 significant bits, x - x1 exact); the
// weights are scaled by 2^kH2Shift before their split (msat_split_f16x2_t) and the sums by 2^-kH2Shift
// after (both exact).  Three MFMAs per (gate, column tile) block, a1b2 a2b1 a1b1; the dropped a2b2 and
// the representation residuals are <= 3 * 2^-22 |ab| per product, under the fp32 accumulation error of
// a 288..416-deep dot product (tests/test_gnn_gpu.py at L = 16 bounds the network against the fp32 CPU
// oracle).  Against bf16x3: half the MFMAs (3 vs 6), 48 instead of 72 KiB of weights per step.
// fp16's range is checked, not assumed: a tile that loads an activation with |a| >= 2^15, or whose
// weights overflowed at the split (wbad), writes flags[tile] = 1 and no output, and the bf16x3 kernel,
// launched next with the same flags, recomputes exactly the flagged tiles.
constexpr int kH2Shift = 10;  // weight scale 2^10: |W| < 32 fits, |W| >= 2^-24 keeps 11 bits


__device__ __forceinline__ int gswz16(int b) { return (0x78 >> (2 * b)) & 3; }  // {0, 2, 3, 1}

struct GruX3rArgs {
    const float *seg[3];
    int seg_ld[3];
    int seg_w[3];
    const float *hp;
    int ldp;
    const float *bi, *bh, *ln_scale, *ln_bias;
    const uint16_t *wiT, *whT;  // [planes][3H][kxp] / [planes][3H][H] (bf16 x3 or fp16 x2 bits)
    int kxp;                    // multiple of 32
    float *out;
    int ldo;
    float *g4;
    int ldg;
    int R, Kx;
    int *flags;        // h2r: per-tile overflow flag (written); x3r: tiles to recompute (nullptr: all)
    const int *wbad;   // h2r: weight-split overflow flags [2] (wi, wh)
};

typedef float f32x4g __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct SplitH8 {
    uint4 p[2];
};

__device__ __forceinline__ SplitH8 splith8(const float4 &u, const float4 &v) {
    const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const _Float16 a = (_Float16)x[j];
        h[j] = a;
        l[j] = (_Float16)(x[j] - (float)a);
    }
    SplitH8 s;
    s.p[0] = __builtin_bit_cast(uint4, h);
    s.p[1] = __builtin_bit_cast(uint4, l);
    return s;
}

__device__ __forceinline__ f32x4g h2mma(const uint4 &a, const uint4 &b, const f32x4g &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
}

// ST = true: the activations go through LDS as well.  Each step's [128 rows][32 k] fp32 tile (16 KiB) is
// fetched by LDS-DMA three steps ahead into one of three slots ([row][8 chunks of 16 B], chunk c of row
// r at slot c ^ ((r >> 1) & 5): conflict-free ds_read_b128 for the register-A lane map), and split from
// LDS in the middle of the step before its use.  With no registers in flight across steps, the step end
// waits only for the next step's weights and the activations of step s + 2 (vmcnt(2)): the activation
// fetches get 2.5 steps of lead instead of one.  ST = false: activations loaded to registers by asm one
// step ahead and drained at every step end (see the note at the wait).  LDS: 96 KiB of weights + 48 KiB.
// diagnostic ablations of the staged form (timing only, wrong results; never set in the product build):
// bit 0 no weight DMA after the prologue, 1 no activation DMA after it, 2 no MFMAs, 3 no weight
// fragment reads (registers reused), 4 no split, 5 no step-end barrier, 6 no step-end vmcnt wait,
// 7 no epilogue, 8 one k step (prologue and epilogue alone)
#ifndef MSAT_GRU_ABL
#define MSAT_GRU_ABL 0
#endif
// NW waves (16 rows each) per workgroup, WB weight buffers.  <ST, 8, 2>: 128-row tiles, one workgroup
// per CU (147 KiB of LDS).  <true, 4, 1> ("ping-pong"): 64-row tiles, weights single-buffered, 72 KiB,
// two workgroups per CU, so one's DMA waits, barriers and epilogue run beside the other's MFMAs; its
// range flags go to the 128-row tile the x3r fixup launch indexes (pre-zeroed, written only on overflow).
#ifndef MSAT_GRU_LA2
#define MSAT_GRU_LA2 1
#endif
#ifndef MSAT_GRU_STG
#define MSAT_GRU_STG 2
#endif
#ifndef MSAT_GRU_DMA0
#define MSAT_GRU_DMA0 -1
#endif
#ifndef MSAT_GRU_DMA1
#define MSAT_GRU_DMA1 8
#endif
#ifndef MSAT_GRU_PKE
#define MSAT_GRU_PKE 1
#endif
#ifndef MSAT_GRU_HVE
#define MSAT_GRU_HVE 1
#endif
template <bool ST, int NW = 8, int WB = 2>
__device__ __forceinline__ void gru_h2r_tile(const GruX3rArgs &a, int tile) {
    constexpr int H = 128, IMG = H * 4;  // uint4 per (plane, gate) image: 128 units x 4 chunks = 8 KiB
    constexpr int NI = 6;                // (plane, gate) images per step
    constexpr int NIW = 8 * NI / NW;     // weight DMA instructions per wave and step
    constexpr int TR = 16 * NW;          // tile rows
    static_assert(WB == 2 || ST, "single-buffered weights need the LDS-staged activations");
    __shared__ uint4 Bs[WB * NI * IMG];  // 48 KiB per buffer
    constexpr int ASL = TR * 8;          // uint4 per activation slot (128 B per row)
    __shared__ uint4 As[ST ? 3 * ASL : 1];
    const int t = threadIdx.x, lane = t & 63, l16 = lane & 15, g = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int row0 = tile * TR, wr = 16 * w;
    int *const flag = a.flags + (NW == 8 ? tile : tile >> 1);
    if (a.wbad[0] | a.wbad[1]) {  // weights out of fp16 range: the bf16x3 launch does every tile
        if (t == 0) *flag = 1;
        return;
    }
    const int arow = row0 + wr + l16, arc = arow < a.R ? arow : a.R - 1;
    constexpr int nsh = H / 32;
    // ablation bit 8: one step instead of ns (prologue + epilogue cost)
    const int ns = (ST && (MSAT_GRU_ABL & 256)) ? 1 : nsh + a.kxp / 32;
    const float *const hp = a.hp, *const sg0 = a.seg[0], *const sg1 = a.seg[1], *const sg2 = a.seg[2];
    const int w0 = a.seg_w[0], w01 = a.seg_w[0] + a.seg_w[1], kx_end = a.Kx;
    const unsigned ro0 = (unsigned)arc * (unsigned)a.seg_ld[0], ro1 = (unsigned)arc * (unsigned)a.seg_ld[1],
                   ro2 = (unsigned)arc * (unsigned)a.seg_ld[2];
    const float *const hrow = hp + (size_t)arc * a.ldp + 8 * g;
    // weight DMA: 8 NI wave-instructions (1 KiB = 16 units x 4 chunks) per step, NI per wave;
    // instruction e of wave w fills image x = (NI w + e) / 8 (plane * 3 + gate), units 16 p .. 16 p + 15
    // (p = (NI w + e) % 8).  Lane -> unit 16 p + (lane >> 2), LDS chunk lane & 3 = source chunk
    // (lane & 3) ^ f((lane >> 4) & 3).
    const unsigned lpart = (unsigned)(lane >> 2) * 2u, chb = 16u * ((lane & 3) ^ gswz16((lane >> 4) & 3));
    auto issueW = [&](int s, int buf) {
        const bool hid = s < nsh;
        const uint16_t *W = hid ? a.whT : a.wiT;
        const int Kp = hid ? H : a.kxp;
        const int k0 = hid ? 32 * s : 32 * (s - nsh);
        const unsigned voff = lpart * (unsigned)Kp + chb;
#pragma unroll
        for (int e = 0; e < NIW; ++e) {
            const int x = NIW * w + e, img = x >> 3, p = x & 7, q = img / 3, gt = img - 3 * q;
            const uint16_t *base = W + ((size_t)q * 3 * H + gt * H + 16 * p) * Kp + k0;
            glds16_async_s(base, voff, &Bs[(buf * NI + img) * IMG + 64 * p]);
        }
    };
    f32x4g acc[4][8];
#pragma unroll
    for (int G = 0; G < 4; ++G)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[G][j] = f32x4g{};
    const int slot = g ^ gswz16((l16 >> 2) & 3);
    float amax = 0.f;  // largest |activation| this lane split (range check)
    // Activation loads one or two steps ahead into alternating register sets (plain loads, tracked by
    // hipcc); the split of step s + 1 runs among step s's MFMAs; one vmcnt(0) + barrier per step.
    // These were asm loads once: hipcc treats an asm output as ready at the asm and may copy or move
    // its registers before the data lands (it did once the x3r body was inlined into a second kernel:
    // rows of garbage), so register loads stay visible to the compiler; only LDS-DMA is asm.
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v ras[2][2];  // [set = step & 1][half]
    auto aptr = [&](int st, int e) -> const float * {
        if (st < nsh) return hrow + 32 * st + 4 * e;
        const int kx = (st - nsh) * 32 + 8 * g + 4 * e;
        const float *q0 = sg0 + (ro0 + (unsigned)(kx < w0 ? kx : 0));
        const float *q1 = sg1 + (ro1 + (unsigned)(kx - w0));
        const float *q2 = sg2 + (ro2 + (unsigned)(kx - w01));
        return (kx >= w01 && kx < kx_end) ? q2 : ((kx >= w0 && kx < w01) ? q1 : q0);
    };
    auto aload = [&](int st, f4v (&r)[2]) {
#pragma unroll
        for (int e = 0; e < 2; ++e) r[e] = *reinterpret_cast<const f4v *>(aptr(st, e));
    };
    // all vector memory of this wave (the weight DMA, which hipcc cannot see, and the activation loads)
    auto await0 = [&](f4v (&)[2]) { wait_vmcnt<0>(); };
    auto asplit = [&](int st, const f4v (&r)[2], uint4 (&f)[2]) {  // branch-free (selects)
        const int kx = (st - nsh) * 32 + 8 * g;
        const bool z0 = st >= nsh && kx >= kx_end, z1 = st >= nsh && kx + 4 >= kx_end;
        const f4v zero = {0.f, 0.f, 0.f, 0.f};
        const float4 v0 = __builtin_bit_cast(float4, z0 ? zero : r[0]);
        const float4 v1 = __builtin_bit_cast(float4, z1 ? zero : r[1]);
        const float m0 = fmaxf(fmaxf(fabsf(v0.x), fabsf(v0.y)), fmaxf(fabsf(v0.z), fabsf(v0.w)));
        const float m1 = fmaxf(fmaxf(fabsf(v1.x), fabsf(v1.y)), fmaxf(fabsf(v1.z), fabsf(v1.w)));
        amax = fmaxf(amax, fmaxf(m0, m1));
        const SplitH8 sp = splith8(v0, v1);
        f[0] = sp.p[0];
        f[1] = sp.p[1];
    };
    uint4 fas[2][2];  // split activations of step s in fas[s & 1]
    // ST: activation DMA, 16 wave-instructions (1 KiB = 8 rows x 8 chunks) per step, 2 per wave;
    // instruction e of wave w: rows 8 x .. 8 x + 7 (x = 2 w + e), lane -> row 8 x + (lane >> 3), LDS slot
    // lane & 7 holding chunk (lane & 7) ^ ((row >> 1) & 5).  Rows past R read row R - 1; k past Kx read
    // a valid address (zeroed at the split).
    const float *dsrc[2];  // per instruction: this lane's source row base, set per step below
    int dchunk[2], drow[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int r = 8 * (2 * w + e) + (lane >> 3);
        drow[e] = r;
        dchunk[e] = (lane & 7) ^ ((r >> 1) & 5);
        dsrc[e] = nullptr;
    }
    auto issueA = [&](int st) {
        if constexpr (ST) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int rr = row0 + drow[e], rc = rr < a.R ? rr : a.R - 1;
                const float *src;
                if (st < nsh) {
                    src = hp + (size_t)rc * a.ldp + 32 * st + 4 * dchunk[e];
                } else {
                    const int kx = (st - nsh) * 32 + 4 * dchunk[e];
                    if (kx < w0) src = sg0 + (size_t)rc * a.seg_ld[0] + kx;
                    else if (kx < w01) src = sg1 + (size_t)rc * a.seg_ld[1] + (kx - w0);
                    else if (kx < kx_end) src = sg2 + (size_t)rc * a.seg_ld[2] + (kx - w01);
                    else src = hp + (size_t)rc * a.ldp;  // padding k: any valid row, zeroed at the split
                }
                glds16_async(src, &As[(st % 3) * ASL + 64 * (2 * w + e)]);
            }
        }
    };
    auto lsplit = [&](int st, uint4 (&f)[2]) {  // ST: split step st's activations from its LDS slot
        const int r = wr + l16, sw = (r >> 1) & 5;
        const uint4 *row = &As[(st % 3) * ASL + 8 * r];
        f4v v[2];
        v[0] = __builtin_bit_cast(f4v, row[(2 * g) ^ sw]);
        v[1] = __builtin_bit_cast(f4v, row[(2 * g + 1) ^ sw]);
        asplit(st, v, f);
    };
    if constexpr (ST) {
        issueA(0);
        if (ns > 1) issueA(1);
        if (ns > 2) issueA(2);
        issueW(0, 0);
        wait_vmcnt<0>();
        barrier_lds();
        lsplit(0, fas[0]);
    } else {
        aload(0, ras[0]);
        if (ns > 1) aload(1, ras[1]);
        issueW(0, 0);
        await0(ras[0]);
        await0(ras[1]);
        asplit(0, ras[0], fas[0]);
        barrier_lds();
    }
    // HVE: the h values of the epilogue (h of each accumulator's (row, unit)) are fetched by LDS-DMA at
    // the start of the last step, so their HBM latency runs under its MFMAs instead of at the epilogue
    // (the rows' h passed through the activation slots in steps 0..3 and are long evicted).  In the last
    // step the three activation slots and the other weight buffer are free: waves 0..5 put their 16 rows
    // (8 KiB, [row][128]) in the slots, waves 6 and 7 in that buffer.
    constexpr bool HVE = MSAT_GRU_HVE && ST && WB == 2 && NW == 8;
    auto hbase = [&](int fb) -> float * {
        return w < 6 ? reinterpret_cast<float *>(&As[512 * w]) : reinterpret_cast<float *>(&Bs[fb * NI * IMG + 512 * (w - 6)]);
    };
    auto issueH = [&](int fb, int z) {  // z = 0, passed from the step so nothing is hoisted into the loop
        const uint4 *dst = reinterpret_cast<const uint4 *>(hbase(fb));
        const float *sb = hp + (size_t)row0 * a.ldp;  // wave-uniform base, per-lane 32-bit offsets
        const int rmax = a.R - 1 - row0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // rows wr + 2 e + (lane >> 5), float4 (lane & 31)
            const int rr = wr + 2 * e + (lane >> 5) + z, rc = rr < rmax ? rr : rmax;
            glds16_async_s(sb, 4u * ((unsigned)rc * (unsigned)a.ldp + 4u * (unsigned)(lane & 31)), dst + 64 * e);
        }
    };
    auto pstep = [&](int st, auto hidc, auto parc) {
        constexpr bool hid = decltype(hidc)::value;
        constexpr int PB = decltype(parc)::value;  // st & 1
        const int buf = WB == 2 ? PB : 0;
        if (HVE && st + 1 == ns) issueH(buf ^ 1, ns - 1 - st);
        // STG (stagger of SIMD partners: waves w and w + 4 share a SIMD): bit 0 moves waves 4..7's split
        // to block 19, bit 1 (default) their DMA issue to before block MSAT_GRU_DMA1 = 8, so partners'
        // DMA bursts do not coincide.  Measured (profiles/ab_gru_dma.sh, tape on): DMA at block 8 -2.9 %
        // clause / -1.1 % var; blocks 4, 6, 10, 12, 16 -1..-2.5 %; delaying waves 0..3 too (4 / 16,
        // 6 / 18) +2 %; the split stagger 0 .. +0.5 %.
        constexpr bool stg_split = ST && WB == 2 && NW == 8 && (MSAT_GRU_STG & 1);
        constexpr bool stg_dma = ST && WB == 2 && NW == 8;
        // the block before which waves 0..3 / 4..7 issue the step's DMA (-1: at the step start)
        constexpr int dma_n0 = MSAT_GRU_DMA0, dma_n1 = (MSAT_GRU_STG & 2) ? MSAT_GRU_DMA1 : MSAT_GRU_DMA0;
        const bool late = w >= 4;
        auto dma = [&]() {
            if (WB == 2 && !(ST && (MSAT_GRU_ABL & 1)) && st + 1 < ns) issueW(st + 1, buf ^ 1);
            if constexpr (ST) {
                if (WB == 2 && !(MSAT_GRU_ABL & 2) && st + 3 < ns) issueA(st + 3);
            }
        };
        if (!stg_dma || (late ? dma_n1 : dma_n0) < 0) dma();
        if constexpr (!ST) {
            if (st + 2 < ns) aload(st + 2, ras[PB]);
        }
        // weight fragments carried across the 24 (gate, column tile) blocks: each plane is re-read
        // for the next block as soon as its last MFMA here has issued, so the reads fly under the
        // MFMAs instead of each block waiting for its own reads (at 255 VGPRs the compiler had
        // issued every block's reads just before its MFMAs and waited on them).
        auto bfrag = [&](int n, int q) {
            const int gt = n >> 3, j = n & 7;
            return Bs[(buf * NI + q * 3 + gt) * IMG + (16 * j + l16) * 4 + slot];
        };
        uint4 (&fa)[2] = fas[PB];
        {
            // ST: fragments LA = MSAT_GRU_LA2 + 1 blocks ahead in LA rotating register sets (block n uses
            // set n % LA; each plane's register is refilled for block n + LA right after its last MFMA in
            // block n); otherwise one block ahead in one set
            constexpr int LA = (ST && MSAT_GRU_LA2) ? MSAT_GRU_LA2 + 1 : 1;
            uint4 bb[LA][2];
#pragma unroll
            for (int q = 0; q < LA; ++q) {  // blocks 0 .. LA - 1
                bb[q][0] = bfrag(q, 0);
                bb[q][1] = bfrag(q, 1);
            }
#pragma unroll
            for (int n = 0; n < 24; ++n) {
                const int gt = n >> 3, j = n & 7;
                const int G = gt < 2 ? gt : (hid ? 3 : 2);
                uint4 &b0 = bb[n % LA][0], &b1 = bb[n % LA][1];
                f32x4g c = acc[G][j];
                constexpr bool nomma = ST && (MSAT_GRU_ABL & 4), noread = ST && (MSAT_GRU_ABL & 8);
                if (!nomma) c = h2mma(fa[0], b1, c);  // a1 b2
                if (!noread && n + LA < 24) b1 = bfrag(n + LA, 1);
                if (!nomma) c = h2mma(fa[1], b0, c);  // a2 b1
                if (!nomma) c = h2mma(fa[0], b0, c);  // a1 b1
                if (nomma) c += __builtin_bit_cast(f32x4g, b0 ^ b1);
                if (!noread && n + LA < 24) b0 = bfrag(n + LA, 0);
                acc[G][j] = c;
                if constexpr (ST) {
                    if ((n == 7 && !(stg_split && late)) || (stg_split && n == 19 && late))
                        if (!(MSAT_GRU_ABL & 16) && st + 1 < ns) lsplit(st + 1, fas[PB ^ 1]);
                } else if (n == 7) {
                    asplit(st + 1, ras[PB ^ 1], fas[PB ^ 1]);
                }
                if (stg_dma && n + 1 < 24 && n + 1 == (late ? dma_n1 : dma_n0)) dma();
                __builtin_amdgcn_sched_barrier(0);  // keep the blocks in order (the reads lead by one)
            }
        }
        if constexpr (ST && WB == 1) {
            // single weight buffer: every wave is done with W(st) before W(st + 1) overwrites it
            barrier_lds();
            if (st + 1 < ns) issueW(st + 1, 0);
            if (st + 3 < ns) issueA(st + 3);
        }
        if constexpr (ST) {
            // W(st + 1) and A(st + 2) landed (A(st + 3), issued last, may fly); no registers in flight
            if (!(MSAT_GRU_ABL & 64)) {
                if (st + 3 < ns) wait_vmcnt<2>();
                else wait_vmcnt<0>();
            }
        } else {
            // Every asm load must complete within the step that issued it: hipcc treats an asm output as
            // ready at the asm and reuses or moves its registers at the loop back-edge (leaving the
            // step-s+2 activations in flight across it, vmcnt(2) here, faulted: the late data landed in
            // registers the latch block had reassigned to index arithmetic).
            await0(ras[PB]);
        }
        if (!(ST && (MSAT_GRU_ABL & 32))) barrier_lds();
    };
    {
        int st = 0;
#pragma unroll 1
        for (; st + 1 < nsh; st += 2) {
            pstep(st, std::true_type{}, std::integral_constant<int, 0>{});
            pstep(st + 1, std::true_type{}, std::integral_constant<int, 1>{});
        }
        // nsh = 4 is even: the input steps start at parity 0
#pragma unroll 1
        for (; st + 1 < ns; st += 2) {
            pstep(st, std::false_type{}, std::integral_constant<int, 0>{});
            pstep(st + 1, std::false_type{}, std::integral_constant<int, 1>{});
        }
        if (st < ns) pstep(st, std::false_type{}, std::integral_constant<int, 0>{});
    }
    {  // range check: |a| < 2^15 keeps a1 = fp16(a) finite with margin.  A ballot per wave and an
       // LDS-only barrier: __syncthreads_or's fence would also wait for the h DMA in flight.
        __shared__ int wbadl[NW];
        const bool wb = __ballot(!(amax < 32768.0f)) != 0;
        if (lane == 0) wbadl[w] = wb;
        barrier_lds();
        int bad = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) bad |= wbadl[q];
        if (t == 0 && (NW == 8 || bad)) *flag = bad;
        if (bad) {
            wait_vmcnt<0>();  // no LDS-DMA may land after the workgroup's LDS is released
            return;
        }
    }

    if (ST && (MSAT_GRU_ABL & 128)) {  // ablation bit 7: no epilogue (accumulators kept live)
        if constexpr (HVE) wait_vmcnt<0>();
        float v = 0.f;
#pragma unroll
        for (int G = 0; G < 4; ++G)
#pragma unroll
            for (int j = 0; j < 8; ++j) v += acc[G][j][0] + acc[G][j][1] + acc[G][j][2] + acc[G][j][3];
        if (arow < a.R) a.out[(size_t)arow * a.ldo + lane] = v;
        return;
    }
    // ---- epilogue.  C/D map: unit u = 16 j + l16, row wr + 4 g + reg.
    float *stage = reinterpret_cast<float *>(Bs) + w * 16 * 132;  // [16 rows][132] per wave
    const bool tape = a.g4 != nullptr;
    float hv[8][4];
    if constexpr (HVE) {
        wait_vmcnt<0>();  // this wave's own h rows have landed
        const float *hl = hbase(((ns - 1) & 1) ^ 1);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) hv[j][r] = hl[(4 * g + r) * H + 16 * j + l16];
        barrier_lds();  // every wave has read its h before any wave's stage (over Bs) is written
    } else {
        // loaded before the tape stores (vector-memory counts retire in issue order, so a load issued
        // after them would wait for them)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = row0 + wr + 4 * g + r;
                hv[j][r] = hp[(size_t)(row < a.R ? row : a.R - 1) * a.ldp + 16 * j + l16];
            }
    }
    constexpr float sc = 1.0f / (float)(1 << kH2Shift);  // exact power of two
#if MSAT_GRU_PKE
    // packed fp32 (v_pk_mul / v_pk_add on row pairs): no MFMAs run here, so the packed forms halve the
    // epilogue's vector issue instead of competing with matrix work
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int u = 16 * j + l16;
        const float br = a.bi[u] + a.bh[u], bz = a.bi[H + u] + a.bh[H + u];
        const float bni = a.bi[2 * H + u], bnh = a.bh[2 * H + u];
        const f32x4g s4 = {sc, sc, sc, sc};
        acc[0][j] = acc[0][j] * s4 + f32x4g{br, br, br, br};
        acc[1][j] = acc[1][j] * s4 + f32x4g{bz, bz, bz, bz};
        acc[2][j] = acc[2][j] * s4 + f32x4g{bni, bni, bni, bni};
        acc[3][j] = acc[3][j] * s4 + f32x4g{bnh, bnh, bnh, bnh};
    }
#else
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int u = 16 * j + l16;
        const float br = a.bi[u] + a.bh[u], bz = a.bi[H + u] + a.bh[H + u];
        const float bni = a.bi[2 * H + u], bnh = a.bh[2 * H + u];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            acc[0][j][r] = acc[0][j][r] * sc + br;
            acc[1][j][r] = acc[1][j][r] * sc + bz;
            acc[2][j][r] = acc[2][j][r] * sc + bni;
            acc[3][j][r] = acc[3][j][r] * sc + bnh;
        }
    }
#endif
    // float4 rows of the wave's [16][128] stage -> dst (row stride ld), rows < R only.  The stage is
    // wave-private and a wave's LDS operations complete in issue order, so waiting for its own stage
    // writes (lgkmcnt) is the only ordering needed: no workgroup barrier, whose release fence would
    // also drain the wave's global stores.
    auto flush = [&](float *dst, int ld) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int rr = 2 * it + (lane >> 5), c4 = lane & 31;
            const float4 v = *reinterpret_cast<const float4 *>(stage + rr * 132 + 4 * c4);
            const int row = row0 + wr + rr;
            if (row < a.R) *reinterpret_cast<float4 *>(dst + (size_t)row * ld + 4 * c4) = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    if (tape) {
        // pre-activations straight from the accumulators (16 lanes x 4 B per row segment; staging them
        // through LDS as float4 rows measured 0-4 % slower, float4 rows by a DPP 4 x 4 transpose inside
        // each lane quad 5 % slower: profiles/r02_ab_gru_tq.log; non-temporal stores +1.3 % clause / -1.3 % var,
        // r02_ab_gru_nt.log)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = row0 + wr + 4 * g + r;
            if (row < a.R) {
                float *q = a.g4 + (size_t)row * a.ldg + l16;
#pragma unroll
                for (int G = 0; G < 4; ++G)
#pragma unroll
                    for (int j = 0; j < 8; ++j) q[G * H + 16 * j] = acc[G][j][r];
            }
        }
    }
#if MSAT_GRU_PKE
    typedef float f2 __attribute__((ext_vector_type(2)));
    constexpr float kL2E = 1.4426950408889634f;  // exp(x) = 2^(x log2 e), as __expf
    auto exp2v = [](f2 x) { return f2{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; };
    auto rcpv = [](f2 x) { return f2{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)}; };
    const f2 one = {1.f, 1.f}, ml2e = {-kL2E, -kL2E}, m2l2e = {-2.f * kL2E, -2.f * kL2E}, two = {2.f, 2.f};
    f2 s1v[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}}, s2v[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int p = 0; p < 2; ++p) {  // rows 2p, 2p + 1
            const f2 rp = {acc[0][j][2 * p], acc[0][j][2 * p + 1]}, zp = {acc[1][j][2 * p], acc[1][j][2 * p + 1]};
            const f2 gi = {acc[2][j][2 * p], acc[2][j][2 * p + 1]}, gh = {acc[3][j][2 * p], acc[3][j][2 * p + 1]};
            const f2 h = {hv[j][2 * p], hv[j][2 * p + 1]};
            const f2 rg = rcpv(one + exp2v(rp * ml2e)), zg = rcpv(one + exp2v(zp * ml2e));
            const f2 ng = two * rcpv(one + exp2v((gi + rg * gh) * m2l2e)) - one;  // tanh = 2 sigma(2x) - 1
            const f2 hn = (one - zg) * ng + zg * h;
            acc[0][j][2 * p] = hn.x;
            acc[0][j][2 * p + 1] = hn.y;
            s1v[p] += hn;
            s2v[p] += hn * hn;
        }
    // sums over the 16 lanes of a row group: the xor butterfly of __shfl_xor(v, 1 / 2 / 4 / 8, 16) (same
    // association, so bit-identical sums) by DPP instead of LDS permutes -- quad swaps for 1 and 2,
    // row shifts selected by the lane's bit for 4 and 8
    auto row16 = [lane](float v) {
        auto dpp = [](float x, auto ctl) {
            return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), decltype(ctl)::value,
                                                                      0xF, 0xF, true));
        };
        v += dpp(v, std::integral_constant<int, 0xB1>{});  // quad_perm [1,0,3,2]: lane ^ 1
        v += dpp(v, std::integral_constant<int, 0x4E>{});  // quad_perm [2,3,0,1]: lane ^ 2
        {
            const float up = dpp(v, std::integral_constant<int, 0x104>{});  // row_shl:4: lane + 4
            const float dn = dpp(v, std::integral_constant<int, 0x114>{});  // row_shr:4: lane - 4
            v += (lane & 4) ? dn : up;
        }
        {
            const float up = dpp(v, std::integral_constant<int, 0x108>{});  // row_shl:8
            const float dn = dpp(v, std::integral_constant<int, 0x118>{});  // row_shr:8
            v += (lane & 8) ? dn : up;
        }
        return v;
    };
    float mean[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float t1 = row16(r & 1 ? s1v[r >> 1].y : s1v[r >> 1].x);
        const float t2 = row16(r & 1 ? s2v[r >> 1].y : s2v[r >> 1].x);
        mean[r] = t1 / (float)H;
        const float var = fmaxf(t2 / (float)H - mean[r] * mean[r], 0.0f);
        rs[r] = rsqrtf(var + 1e-6f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int u = 16 * j + l16;
        const float scl = a.ln_scale[u], lb = a.ln_bias[u];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const f2 hn = {acc[0][j][2 * p], acc[0][j][2 * p + 1]};
            const f2 y = (hn - f2{mean[2 * p], mean[2 * p + 1]}) * (f2{rs[2 * p], rs[2 * p + 1]} * f2{scl, scl}) +
                         f2{lb, lb};
            stage[(4 * g + 2 * p) * 132 + u] = y.x;
            stage[(4 * g + 2 * p + 1) * 132 + u] = y.y;
        }
    }
#else
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float rg = fsig_fast(acc[0][j][r]), zg = fsig_fast(acc[1][j][r]);
            const float ng = ftanh_fast(acc[2][j][r] + rg * acc[3][j][r]);
            const float hn = (1.0f - zg) * ng + zg * hv[j][r];
            acc[0][j][r] = hn;
            s1[r] += hn;
            s2[r] += hn * hn;
        }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            s1[r] += __shfl_xor(s1[r], o, 16);
            s2[r] += __shfl_xor(s2[r], o, 16);
        }
    float mean[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        mean[r] = s1[r] / (float)H;
        const float var = fmaxf(s2[r] / (float)H - mean[r] * mean[r], 0.0f);
        rs[r] = rsqrtf(var + 1e-6f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int u = 16 * j + l16;
        const float scl = a.ln_scale[u], lb = a.ln_bias[u];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            stage[(4 * g + r) * 132 + u] = (acc[0][j][r] - mean[r]) * (rs[r] * scl) + lb;
    }
#endif
    flush(a.out, a.ldo);
}

__global__ void __launch_bounds__(512, 1) gru_ln_fused_fwd_h2r_kernel(GruX3rArgs a) {
    gru_h2r_tile<false>(a, blockIdx.x);
}

__global__ void __launch_bounds__(512, 1) gru_ln_fused_fwd_h2s_kernel(GruX3rArgs a) {
    gru_h2r_tile<true>(a, blockIdx.x);
}

__global__ void __launch_bounds__(256, 2) gru_ln_fused_fwd_h2p_kernel(GruX3rArgs a) {
    gru_h2r_tile<true, 4, 1>(a, blockIdx.x);
}


// bf16x3 register-A kernel (the template above is fp16x2-only: instantiated for bf16x3 it computed
// wrong results; this is the round-1 kernel, unchanged).  Pipeline switches: activations loaded two
// steps ahead by asm, weight fragments carried across column blocks, tape stored from the accumulators.
#define MSAT_GRU_X3R_BPIPE 1
#define MSAT_GRU_X3R_PIPE 1
#define MSAT_GRU_TAPE_DIRECT 1
__device__ __forceinline__ void gru_x3r_tile(const GruX3rArgs &a, int tile) {
    constexpr int H = 128, IMG = H * 4;  // uint4 per (plane, gate) image: 128 units x 4 chunks = 8 KiB
    __shared__ uint4 Bs[2][9][IMG];      // [buf][plane * 3 + gate], 144 KiB
    const int t = threadIdx.x, lane = t & 63, l16 = lane & 15, g = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int row0 = tile * 128, wr = 16 * w;
    const int arow = row0 + wr + l16, arc = arow < a.R ? arow : a.R - 1;
    constexpr int nsh = H / 32;
    const int ns = nsh + a.kxp / 32;
    const float *const hp = a.hp, *const sg0 = a.seg[0], *const sg1 = a.seg[1], *const sg2 = a.seg[2];
    const int w0 = a.seg_w[0], w01 = a.seg_w[0] + a.seg_w[1], kx_end = a.Kx;
    const unsigned ro0 = (unsigned)arc * (unsigned)a.seg_ld[0], ro1 = (unsigned)arc * (unsigned)a.seg_ld[1],
                   ro2 = (unsigned)arc * (unsigned)a.seg_ld[2];
    const float *const hrow = hp + (size_t)arc * a.ldp + 8 * g;
    // raw A of step s: two float4 (k = k0 + 8 g + 4 e); input steps select the segment per float4
    float4 ra[2];
    auto loadA = [&](int s) {
        if (s < nsh) {
#pragma unroll
            for (int e = 0; e < 2; ++e) ra[e] = *reinterpret_cast<const float4 *>(hrow + 32 * s + 4 * e);
        } else {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int kx = (s - nsh) * 32 + 8 * g + 4 * e;
                const float *q0 = sg0 + (ro0 + (unsigned)(kx < w0 ? kx : 0));
                const float *q1 = sg1 + (ro1 + (unsigned)(kx - w0));
                const float *q2 = sg2 + (ro2 + (unsigned)(kx - w01));
                const float *pp = (kx >= w01 && kx < kx_end) ? q2 : ((kx >= w0 && kx < w01) ? q1 : q0);
                ra[e] = *reinterpret_cast<const float4 *>(pp);
            }
        }
    };
    // weight DMA: 72 wave-instructions (1 KiB = 16 units x 4 chunks) per step, 9 per wave; instruction
    // e of wave w fills image x = (9 w + e) / 8 (plane * 3 + gate), units 16 p .. 16 p + 15 (p = (9 w + e) % 8).
    // Lane -> unit 16 p + (lane >> 2), LDS chunk lane & 3 = source chunk (lane & 3) ^ f((lane >> 4) & 3).
    const unsigned lpart = (unsigned)(lane >> 2) * 2u, chb = 16u * ((lane & 3) ^ gswz16((lane >> 4) & 3));
    auto issueW = [&](int s, int buf) {
        const bool hid = s < nsh;
        const __bf16 *W = reinterpret_cast<const __bf16 *>(hid ? a.whT : a.wiT);
        const int Kp = hid ? H : a.kxp;
        const int k0 = hid ? 32 * s : 32 * (s - nsh);
        const unsigned voff = lpart * (unsigned)Kp + chb;
#pragma unroll
        for (int e = 0; e < 9; ++e) {
            const int x = 9 * w + e, img = x >> 3, p = x & 7, q = img / 3, gt = img - 3 * q;
            const __bf16 *base = W + ((size_t)q * 3 * H + gt * H + 16 * p) * Kp + k0;
            glds16_async_s(base, voff, &Bs[buf][img][64 * p]);
        }
    };
    f32x4g acc[4][8];
#pragma unroll
    for (int G = 0; G < 4; ++G)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[G][j] = f32x4g{};
    const int slot = g ^ gswz16((l16 >> 2) & 3);
    [[maybe_unused]] auto step = [&](int s, auto hidc) {  // the MSAT_GRU_X3R_PIPE = 0 form
        constexpr bool hid = decltype(hidc)::value;
        const int buf = s & 1;
        float4 v0 = ra[0], v1 = ra[1];
        if (!hid) {  // zero k >= Kx (padded weight rows are zero, the activations there are not)
            const int kx = (s - nsh) * 32 + 8 * g;
            if (kx >= kx_end) v0 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (kx + 4 >= kx_end) v1 = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        bf16x8 fa[3];
        {
            const Split8 sp = split8(v0, v1);
#pragma unroll
            for (int q = 0; q < 3; ++q) fa[q] = __builtin_bit_cast(bf16x8, sp.p[q]);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bool more = s + 1 < ns;
        if (more) {
            if (!(MSAT_GRU_ABL & 1)) issueW(s + 1, buf ^ 1);
            if (!(MSAT_GRU_ABL & 2)) loadA(s + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int gt = 0; gt < (MSAT_GRU_ABL & 8 ? 0 : 3); ++gt) {
            const int G = gt < 2 ? gt : (hid ? 3 : 2);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                bf16x8 fb[3];
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    fb[q] = __builtin_bit_cast(bf16x8, Bs[buf][q * 3 + gt][(16 * j + l16) * 4 + slot]);
                f32x4g c = acc[G][j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[0], c, 0, 0, 0);
                acc[G][j] = c;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (more && !(MSAT_GRU_ABL & 2)) wait_vmcnt<2>();  // W(s+1) landed; A(s+1), issued after it, may fly
        else wait_vmcnt<0>();
        barrier_lds();
    };
#if MSAT_GRU_X3R_PIPE
    // Pipelined form: activation loads two steps ahead into alternating register sets (plain loads,
    // tracked by hipcc: see the note in gru_h2r_tile); the split of step s + 1 runs among step s's
    // MFMAs; one vmcnt(0) + barrier per step (the weights of s + 1 and the activations of s + 2, both
    // issued at the start of step s, have landed).
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v ras[2][2];  // [set = step & 1][half]
    auto aptr = [&](int st, int e) -> const float * {
        if (st < nsh) return hrow + 32 * st + 4 * e;
        const int kx = (st - nsh) * 32 + 8 * g + 4 * e;
        const float *q0 = sg0 + (ro0 + (unsigned)(kx < w0 ? kx : 0));
        const float *q1 = sg1 + (ro1 + (unsigned)(kx - w0));
        const float *q2 = sg2 + (ro2 + (unsigned)(kx - w01));
        return (kx >= w01 && kx < kx_end) ? q2 : ((kx >= w0 && kx < w01) ? q1 : q0);
    };
    auto aload = [&](int st, f4v (&r)[2]) {
#pragma unroll
        for (int e = 0; e < 2; ++e) r[e] = *reinterpret_cast<const f4v *>(aptr(st, e));
    };
    // all vector memory of this wave (the weight DMA, which hipcc cannot see, and the activation loads)
    auto await0 = [&](f4v (&)[2]) { wait_vmcnt<0>(); };
    auto asplit = [&](int st, const f4v (&r)[2], bf16x8 (&f)[3]) {  // branch-free (selects)
        const int kx = (st - nsh) * 32 + 8 * g;
        const bool z0 = st >= nsh && kx >= kx_end, z1 = st >= nsh && kx + 4 >= kx_end;
        const f4v zero = {0.f, 0.f, 0.f, 0.f};
        const float4 v0 = __builtin_bit_cast(float4, z0 ? zero : r[0]);
        const float4 v1 = __builtin_bit_cast(float4, z1 ? zero : r[1]);
        const Split8 sp = split8(v0, v1);
#pragma unroll
        for (int q = 0; q < 3; ++q) f[q] = __builtin_bit_cast(bf16x8, sp.p[q]);
    };
    bf16x8 fas[2][3];  // split activations of step s in fas[s & 1]
    aload(0, ras[0]);
    if (ns > 1) aload(1, ras[1]);
    issueW(0, 0);
    await0(ras[0]);
    await0(ras[1]);
    asplit(0, ras[0], fas[0]);
    barrier_lds();
    auto pstep = [&](int st, auto hidc, auto parc) {
        constexpr bool hid = decltype(hidc)::value;
        constexpr int P = decltype(parc)::value;  // st & 1
        const int buf = P;
        if (st + 1 < ns) issueW(st + 1, buf ^ 1);
        if (st + 2 < ns) aload(st + 2, ras[P]);
#if MSAT_GRU_X3R_BPIPE
        // weight fragments carried across the 24 (gate, column tile) blocks: each plane is re-read
        // for the next block as soon as its last MFMA here has issued (w3 after the 1st, w2 after
        // the 3rd, w1 after the 6th), so the reads fly under the MFMAs instead of each block
        // waiting for its own three reads.  Term order a1w3, a2w2, a1w2, a3w1, a2w1, a1w1.
        auto bfrag = [&](int n, int q) {
            const int gt = n >> 3, j = n & 7;
            return __builtin_bit_cast(bf16x8, Bs[buf][q * 3 + gt][(16 * j + l16) * 4 + slot]);
        };
        bf16x8 b0 = bfrag(0, 0), b1 = bfrag(0, 1), b2 = bfrag(0, 2);
#pragma unroll
        for (int n = 0; n < 24; ++n) {
            const int gt = n >> 3, j = n & 7;
            const int G = gt < 2 ? gt : (hid ? 3 : 2);
            f32x4g c = acc[G][j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][0], b2, c, 0, 0, 0);
            if (n + 1 < 24) b2 = bfrag(n + 1, 2);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][1], b1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][0], b1, c, 0, 0, 0);
            if (n + 1 < 24) b1 = bfrag(n + 1, 1);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][2], b0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][1], b0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][0], b0, c, 0, 0, 0);
            if (n + 1 < 24) b0 = bfrag(n + 1, 0);
            acc[G][j] = c;
            if (n == 7) asplit(st + 1, ras[P ^ 1], fas[P ^ 1]);
            __builtin_amdgcn_sched_barrier(0);  // keep the blocks in order (the reads lead by one)
        }
#else
#pragma unroll
        for (int gt = 0; gt < 3; ++gt) {
            const int G = gt < 2 ? gt : (hid ? 3 : 2);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                bf16x8 fb[3];
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    fb[q] = __builtin_bit_cast(bf16x8, Bs[buf][q * 3 + gt][(16 * j + l16) * 4 + slot]);
                f32x4g c = acc[G][j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][2], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][1], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][0], fb[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][1], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][0], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fas[P][0], fb[0], c, 0, 0, 0);
                acc[G][j] = c;
            }
            // among the MFMAs; unconditional (after the last step it splits stale registers, unused)
            if (gt == 0) asplit(st + 1, ras[P ^ 1], fas[P ^ 1]);
        }
#endif
        await0(ras[P]);
        barrier_lds();
    };
    {
        int st = 0;
#pragma unroll 1
        for (; st + 1 < nsh; st += 2) {
            pstep(st, std::true_type{}, std::integral_constant<int, 0>{});
            pstep(st + 1, std::true_type{}, std::integral_constant<int, 1>{});
        }
        // nsh = 4 is even: the input steps start at parity 0
#pragma unroll 1
        for (; st + 1 < ns; st += 2) {
            pstep(st, std::false_type{}, std::integral_constant<int, 0>{});
            pstep(st + 1, std::false_type{}, std::integral_constant<int, 1>{});
        }
        if (st < ns) pstep(st, std::false_type{}, std::integral_constant<int, 0>{});
    }
#else
    loadA(0);
    issueW(0, 0);
    wait_vmcnt<0>();
    barrier_lds();
#pragma unroll 1
    for (int s = 0; s < nsh; ++s) step(s, std::true_type{});
#pragma unroll 1
    for (int s = nsh; s < ns; ++s) step(s, std::false_type{});
#endif

    if (MSAT_GRU_ABL & 16) {  // keep the accumulators live, store one value per lane
        float v = 0.f;
#pragma unroll
        for (int G = 0; G < 4; ++G)
#pragma unroll
            for (int j = 0; j < 8; ++j) v += acc[G][j][j & 3];
        if (arow < a.R) a.out[(size_t)arow * a.ldo + lane] = v;
        return;
    }
    // ---- epilogue.  C/D map: unit u = 16 j + l16, row wr + 4 g + reg.
    float *stage = reinterpret_cast<float *>(&Bs[0][0][0]) + w * 16 * 132;  // [16 rows][132] per wave
    const bool tape = a.g4 != nullptr;
    // h of each accumulator's (row, unit), loaded before the tape stores (vector-memory counts retire
    // in issue order, so a load issued after them would wait for them)
    float hv[8][4];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = row0 + wr + 4 * g + r;
            hv[j][r] = hp[(size_t)(row < a.R ? row : a.R - 1) * a.ldp + 16 * j + l16];
        }

#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int u = 16 * j + l16;
        const float br = a.bi[u] + a.bh[u], bz = a.bi[H + u] + a.bh[H + u];
        const float bni = a.bi[2 * H + u], bnh = a.bh[2 * H + u];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            acc[0][j][r] += br;
            acc[1][j][r] += bz;
            acc[2][j][r] += bni;
            acc[3][j][r] += bnh;
        }
    }
    // float4 rows of the wave's [16][128] stage -> dst (row stride ld), rows < R only.  The stage is
    // wave-private and a wave's LDS operations complete in issue order, so waiting for its own stage
    // writes (lgkmcnt) is the only ordering needed: no workgroup barrier, whose release fence would
    // also drain the wave's global stores.  (Storing the ghn tape columns right after the hidden
    // steps, under the input steps' MFMAs, measured 2-4 % slower: each step's vmcnt(0) waits for them.)
    auto flush = [&](float *dst, int ld) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int rr = 2 * it + (lane >> 5), c4 = lane & 31;
            const float4 v = *reinterpret_cast<const float4 *>(stage + rr * 132 + 4 * c4);
            const int row = row0 + wr + rr;
            if (row < a.R) *reinterpret_cast<float4 *>(dst + (size_t)row * ld + 4 * c4) = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    if (tape) {
#if MSAT_GRU_TAPE_DIRECT
        // pre-activations straight from the accumulators (16 lanes x 4 B per row segment)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = row0 + wr + 4 * g + r;
            if (row < a.R) {
                float *q = a.g4 + (size_t)row * a.ldg + l16;
#pragma unroll
                for (int G = 0; G < 4; ++G)
#pragma unroll
                    for (int j = 0; j < 8; ++j) q[G * H + 16 * j] = acc[G][j][r];
            }
        }
#else
#pragma unroll
        for (int G = 0; G < 4; ++G) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) stage[(4 * g + r) * 132 + 16 * j + l16] = acc[G][j][r];
            flush(a.g4 + (size_t)G * H, a.ldg);
        }
#endif
    }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float rg = fsig_fast(acc[0][j][r]), zg = fsig_fast(acc[1][j][r]);
            const float ng = ftanh_fast(acc[2][j][r] + rg * acc[3][j][r]);
            const float hn = (1.0f - zg) * ng + zg * hv[j][r];
            acc[0][j][r] = hn;
            s1[r] += hn;
            s2[r] += hn * hn;
        }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            s1[r] += __shfl_xor(s1[r], o, 16);
            s2[r] += __shfl_xor(s2[r], o, 16);
        }
    float mean[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        mean[r] = s1[r] / (float)H;
        const float var = fmaxf(s2[r] / (float)H - mean[r] * mean[r], 0.0f);
        rs[r] = rsqrtf(var + 1e-6f);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int u = 16 * j + l16;
        const float sc = a.ln_scale[u], lb = a.ln_bias[u];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            stage[(4 * g + r) * 132 + u] = (acc[0][j][r] - mean[r]) * (rs[r] * sc) + lb;
    }
    flush(a.out, a.ldo);
}

__global__ void __launch_bounds__(512, 1) gru_ln_fused_fwd_x3r_kernel(GruX3rArgs a) { gru_x3r_tile(a, blockIdx.x); }

// The bf16x3 fixup after an fp16x2 launch: recompute the tiles it flagged.  A few workgroups (one per
// CU at most) scan the flags 64 tiles per load (lane i reads tile c0 + i * grid) and loop over the
// flagged ones, instead of one workgroup per tile that reads its flag and exits (~17 us of dispatch
// per launch when nothing is flagged, which is nearly always).  The mask is the same in every wave of
// the workgroup, so the barrier between tiles is uniform.
__global__ void __launch_bounds__(512, 1) gru_ln_fused_fwd_x3r_fix_kernel(GruX3rArgs a, int ntiles) {
    const int lane = threadIdx.x & 63;
    for (int c0 = blockIdx.x; c0 < ntiles; c0 += 64 * gridDim.x) {
        const int tl = c0 + lane * gridDim.x;
        uint64_t m = __ballot(tl < ntiles && a.flags[tl] != 0);
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            gru_x3r_tile(a, c0 + b * gridDim.x);
            __syncthreads();  // the next tile's DMA reuses the LDS the last one's epilogue read
        }
    }
}

// planes[q][n][k] = part q of (k < K ? W[k][n] : 0), n < N, k < Kp: the transposed, zero-padded
// bf16x3 split of a [K][N] weight (the x3r GRU kernel's W^T planes)
__global__ void split_bf16x3_t_kernel(const float *__restrict__ W, int K, int N, int ldw, int Kp,
                                      __bf16 *__restrict__ out) {
    const size_t n = (size_t)N * Kp;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t c = i / Kp, k = i - c * Kp;
        const float x = k < (size_t)K ? W[k * ldw + c] : 0.0f;
        const __bf16 p = (__bf16)x;
        const float res = x - (float)p;
        const __bf16 m = (__bf16)res;
        out[i] = p;
        out[n + i] = m;
        out[2 * n + i] = (__bf16)(res - (float)m);
    }
}

// planes[q][n][k] = part q of 2^kH2Shift (k < K ? W[k][n] : 0): the transposed, zero-padded fp16x2 split
// (x1 = fp16(x), x2 = fp16(x - x1)) for the h2r GRU kernel; *bad = 1 if a scaled weight is outside
// (-2^15, 2^15) (or not finite): the GRU launch then recomputes every tile in bf16x3.
__global__ void split_f16x2_t_kernel(const float *__restrict__ W, int K, int N, int ldw, int Kp,
                                     _Float16 *__restrict__ out, int *__restrict__ bad) {
    const size_t n = (size_t)N * Kp;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t c = i / Kp, k = i - c * Kp;
        const float x = k < (size_t)K ? W[k * ldw + c] * (float)(1 << kH2Shift) : 0.0f;
        const _Float16 p = (_Float16)x;
        out[i] = p;
        out[n + i] = (_Float16)(x - (float)p);
        if (!(fabsf(x) < 32768.0f)) *bad = 1;
    }
}

static bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace msat

using namespace msat;

extern "C" int msat_gru_ln_fused_fwd(const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1,
                                     int32_t w1, const float *x2, int32_t ld2, int32_t w2, const float *hprev,
                                     int32_t ldp, const float *wi, const float *bi, const float *wh, const float *bh,
                                     const float *ln_scale, const float *ln_bias, float *out, int32_t ldo, float *g4,
                                     int32_t ldg, int32_t R, int32_t H, void *stream) {
    MSAT_REQUIRE(H == 64 || H == 128 || H == 256, "gru_ln_fused: H must be 64, 128 or 256 (got %d)", H);
    MSAT_REQUIRE(R >= 0, "gru_ln_fused: R < 0");
    if (R == 0) return MSAT_OK;  // empty batches may carry NULL row pointers
    MSAT_REQUIRE(x0 && hprev && wi && bi && wh && bh && ln_scale && ln_bias && out, "NULL pointer");
    MSAT_REQUIRE(R >= 0 && ldo >= H && ldp >= H && (!g4 || ldg >= 4 * H), "gru_ln_fused: bad dims");
    const float *seg[3] = {x0, x1, x2};
    const int lds_[3] = {ld0, ld1, ld2}, ws[3] = {w0, w1, w2};
    int Kx = 0;
    for (int g = 0; g < 3; ++g) {
        MSAT_REQUIRE(ws[g] >= 0 && ws[g] % 4 == 0, "gru_ln_fused: segment %d width %d must be a multiple of 4", g,
                     ws[g]);
        if (ws[g] == 0) continue;
        MSAT_REQUIRE(seg[g] && aligned16(seg[g]) && lds_[g] % 4 == 0 && lds_[g] >= ws[g],
                     "gru_ln_fused: segment %d must be 16-byte aligned with ld %% 4 == 0", g);
        Kx += ws[g];
    }
    MSAT_REQUIRE(Kx > 0 && w0 > 0, "gru_ln_fused: empty input");
    MSAT_REQUIRE(aligned16(hprev) && ldp % 4 == 0 && aligned16(wi) && aligned16(wh),
                 "gru_ln_fused: hprev / weights must be 16-byte aligned");
    GruFwdArgs a;
    for (int g = 0; g < 3; ++g) {
        a.seg[g] = ws[g] ? seg[g] : nullptr;
        a.seg_ld[g] = lds_[g];
        a.seg_w[g] = ws[g];
    }
    a.hp = hprev;
    a.ldp = ldp;
    a.wi = wi;
    a.bi = bi;
    a.wh = wh;
    a.bh = bh;
    a.ln_scale = ln_scale;
    a.ln_bias = ln_bias;
    a.out = out;
    a.ldo = ldo;
    a.g4 = g4;
    a.ldg = ldg;
    a.R = R;
    a.Kx = Kx;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((R + kFR - 1) / kFR);
    const char *e = getenv("MARLSAT_GRU_RS");  // row split (1 or 2 waves per unit group), A/B measurements
    const int rs = (e && atoi(e) == 1) ? 1 : 2;
    if (H == 64) {
        if (rs == 2) hipLaunchKernelGGL((gru_ln_fused_fwd_kernel<2, 2>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((gru_ln_fused_fwd_kernel<2, 1>), grid, dim3(128), 0, s, a);
    } else if (H == 128) {
        if (rs == 2) hipLaunchKernelGGL((gru_ln_fused_fwd_kernel<4, 2>), grid, dim3(512), 0, s, a);
        else hipLaunchKernelGGL((gru_ln_fused_fwd_kernel<4, 1>), grid, dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL((gru_ln_fused_fwd_kernel<8, 1>), grid, dim3(512), 0, s, a);
    }
    return check_launch("gru_ln_fused_fwd_kernel");
}

extern "C" int msat_transpose_pad(const float *W, int32_t K, int32_t N, int32_t ldw, float *out, int32_t Kp,
                                  void *stream) {
    if (K == 0 || N == 0) return MSAT_OK;
    MSAT_REQUIRE(W && out && K > 0 && N > 0 && ldw >= N && Kp >= K, "bad transpose_pad args");
    const dim3 grid((Kp + 31) / 32, (N + 31) / 32);
    hipLaunchKernelGGL(transpose_pad_kernel, grid, dim3(256), 0, (hipStream_t)stream, W, K, N, ldw, out, Kp);
    return check_launch("transpose_pad_kernel");
}

extern "C" int msat_gru_ln_fused_fwd_t(const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1,
                                       int32_t w1, const float *x2, int32_t ld2, int32_t w2, const float *hprev,
                                       int32_t ldp, const float *wiT, const float *bi, const float *whT,
                                       const float *bh, const float *ln_scale, const float *ln_bias, float *out,
                                       int32_t ldo, float *g4, int32_t ldg, int32_t R, int32_t H, void *stream) {
    MSAT_REQUIRE(H == 64 || H == 128, "gru_ln_fused_fwd_t: H must be 64 or 128 (got %d)", H);
    MSAT_REQUIRE(R >= 0, "gru_ln_fused_fwd_t: R < 0");
    if (R == 0) return MSAT_OK;
    MSAT_REQUIRE(x0 && hprev && wiT && bi && whT && bh && ln_scale && ln_bias && out, "NULL pointer");
    MSAT_REQUIRE(ldo >= H && ldp >= H && (!g4 || ldg >= 4 * H), "gru_ln_fused_fwd_t: bad dims");
    const float *seg[3] = {x0, x1, x2};
    const int lds_[3] = {ld0, ld1, ld2}, ws[3] = {w0, w1, w2};
    int Kx = 0;
    for (int g = 0; g < 3; ++g) {
        MSAT_REQUIRE(ws[g] >= 0 && ws[g] % 4 == 0, "gru_ln_fused_fwd_t: segment %d width %d must be a multiple of 4",
                     g, ws[g]);
        if (ws[g] == 0) continue;
        MSAT_REQUIRE(seg[g] && aligned16(seg[g]) && lds_[g] % 4 == 0 && lds_[g] >= ws[g],
                     "gru_ln_fused_fwd_t: segment %d must be 16-byte aligned with ld %% 4 == 0", g);
        Kx += ws[g];
    }
    MSAT_REQUIRE(Kx > 0 && w0 > 0, "gru_ln_fused_fwd_t: empty input");
    MSAT_REQUIRE(aligned16(hprev) && ldp % 4 == 0 && aligned16(wiT) && aligned16(whT),
                 "gru_ln_fused_fwd_t: hprev / weights must be 16-byte aligned");
    GruFwdArgs a;
    for (int g = 0; g < 3; ++g) {
        a.seg[g] = ws[g] ? seg[g] : nullptr;
        a.seg_ld[g] = lds_[g];
        a.seg_w[g] = ws[g];
    }
    a.hp = hprev;
    a.ldp = ldp;
    a.wi = wiT;
    a.bi = bi;
    a.wh = whT;
    a.bh = bh;
    a.ln_scale = ln_scale;
    a.ln_bias = ln_bias;
    a.out = out;
    a.ldo = ldo;
    a.g4 = g4;
    a.ldg = ldg;
    a.R = R;
    a.Kx = Kx;
    const dim3 grid((R + kFR - 1) / kFR);
    hipStream_t s = (hipStream_t)stream;
    if (H == 64) hipLaunchKernelGGL((gru_ln_fused_fwd_t_kernel<2, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((gru_ln_fused_fwd_t_kernel<4, 2>), grid, dim3(512), 0, s, a);
    return check_launch("gru_ln_fused_fwd_t_kernel");
}

extern "C" int msat_gru_ln_fused_fwd_x3(const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1,
                                        int32_t w1, const float *x2, int32_t ld2, int32_t w2, const float *hprev,
                                        int32_t ldp, const void *wi_planes, int32_t kxp, const float *bi,
                                        const void *wh_planes, const float *bh, const float *ln_scale,
                                        const float *ln_bias, float *out, int32_t ldo, float *g4, int32_t ldg,
                                        int32_t R, int32_t H, void *stream) {
    MSAT_REQUIRE(H == 128, "gru_ln_fused_fwd_x3: H must be 128 (got %d)", H);
    MSAT_REQUIRE(R >= 0, "gru_ln_fused_fwd_x3: R < 0");
    if (R == 0) return MSAT_OK;
    MSAT_REQUIRE(x0 && hprev && wi_planes && bi && wh_planes && bh && ln_scale && ln_bias && out, "NULL pointer");
    MSAT_REQUIRE(ldo >= H && ldp >= H && (!g4 || ldg >= 4 * H), "gru_ln_fused_fwd_x3: bad dims");
    const float *seg[3] = {x0, x1, x2};
    const int lds_[3] = {ld0, ld1, ld2}, ws[3] = {w0, w1, w2};
    int Kx = 0;
    for (int g = 0; g < 3; ++g) {
        MSAT_REQUIRE(ws[g] >= 0 && ws[g] % 4 == 0, "gru_ln_fused_fwd_x3: segment %d width %d must be a multiple of 4",
                     g, ws[g]);
        if (ws[g] == 0) continue;
        MSAT_REQUIRE(seg[g] && aligned16(seg[g]) && lds_[g] % 4 == 0 && lds_[g] >= ws[g],
                     "gru_ln_fused_fwd_x3: segment %d must be 16-byte aligned with ld %% 4 == 0", g);
        Kx += ws[g];
    }
    MSAT_REQUIRE(Kx > 0 && w0 > 0, "gru_ln_fused_fwd_x3: empty input");
    MSAT_REQUIRE(kxp % kFK == 0 && kxp >= Kx, "gru_ln_fused_fwd_x3: kxp must be >= Kx and a multiple of 16");
    MSAT_REQUIRE(aligned16(hprev) && ldp % 4 == 0 && aligned16(wi_planes) && aligned16(wh_planes),
                 "gru_ln_fused_fwd_x3: hprev / weight planes must be 16-byte aligned");
    MSAT_REQUIRE(aligned16(out) && ldo % 4 == 0 && aligned16(ln_scale) && aligned16(ln_bias),
                 "gru_ln_fused_fwd_x3: out (ld %% 4 == 0) and the LayerNorm rows must be 16-byte aligned");
    GruFwdArgs a = {};
    for (int g = 0; g < 3; ++g) {
        a.seg[g] = ws[g] ? seg[g] : nullptr;
        a.seg_ld[g] = lds_[g];
        a.seg_w[g] = ws[g];
    }
    a.hp = hprev;
    a.ldp = ldp;
    a.wip = reinterpret_cast<const __bf16 *>(wi_planes);
    a.whp = reinterpret_cast<const __bf16 *>(wh_planes);
    a.kxp = kxp;
    a.bi = bi;
    a.bh = bh;
    a.ln_scale = ln_scale;
    a.ln_bias = ln_bias;
    a.out = out;
    a.ldo = ldo;
    a.g4 = g4;
    a.ldg = ldg;
    a.R = R;
    a.Kx = Kx;
    // 16 waves x 32 rows; 8 waves x 64 rows (RS = 2, half the transposed reads per MFMA but half the
    // waves) measured 3-12 % slower (profiles/gru_bench.py)
    hipLaunchKernelGGL((gru_ln_fused_fwd_x3_kernel<4, 4>), dim3((R + kXR - 1) / kXR), dim3(1024), 0,
                       (hipStream_t)stream, a);
    return check_launch("gru_ln_fused_fwd_x3_kernel");
}

extern "C" int msat_split_bf16x3_t(const float *W, int32_t K, int32_t N, int32_t ldw, int32_t Kp, void *planes,
                                   void *stream) {
    if (K == 0 || N == 0) return MSAT_OK;
    MSAT_REQUIRE(W && planes && K > 0 && N > 0 && ldw >= N && Kp >= K, "bad split_bf16x3_t args");
    const size_t n = (size_t)N * Kp;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(split_bf16x3_t_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, W, K, N, ldw, Kp,
                       reinterpret_cast<__bf16 *>(planes));
    return check_launch("split_bf16x3_t_kernel");
}

static int gru_r_args(GruX3rArgs &a, const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1, int32_t w1,
                      const float *x2, int32_t ld2, int32_t w2, const float *hprev, int32_t ldp, const void *wiT,
                      int32_t kxp, const float *bi, const void *whT, const float *bh, const float *ln_scale,
                      const float *ln_bias, float *out, int32_t ldo, float *g4, int32_t ldg, int32_t R, int32_t H) {
    MSAT_REQUIRE(H == 128, "gru_ln_fused_fwd_x3r/h2r: H must be 128 (got %d)", H);
    MSAT_REQUIRE(R > 0, "gru_ln_fused_fwd_x3r/h2r: R <= 0");
    MSAT_REQUIRE(x0 && hprev && wiT && bi && whT && bh && ln_scale && ln_bias && out, "NULL pointer");
    MSAT_REQUIRE(ldo >= H && ldp >= H && (!g4 || ldg >= 4 * H), "gru_ln_fused_fwd_x3r/h2r: bad dims");
    const float *seg[3] = {x0, x1, x2};
    const int lds_[3] = {ld0, ld1, ld2}, ws[3] = {w0, w1, w2};
    int Kx = 0;
    for (int g = 0; g < 3; ++g) {
        MSAT_REQUIRE(ws[g] >= 0 && ws[g] % 4 == 0,
                     "gru_ln_fused_fwd_x3r/h2r: segment %d width %d must be a multiple of 4", g, ws[g]);
        if (ws[g] == 0) continue;
        MSAT_REQUIRE(seg[g] && aligned16(seg[g]) && lds_[g] % 4 == 0 && lds_[g] >= ws[g],
                     "gru_ln_fused_fwd_x3r/h2r: segment %d must be 16-byte aligned with ld %% 4 == 0", g);
        Kx += ws[g];
    }
    MSAT_REQUIRE(Kx > 0 && w0 > 0, "gru_ln_fused_fwd_x3r/h2r: empty input");
    MSAT_REQUIRE(kxp % 32 == 0 && kxp >= Kx, "gru_ln_fused_fwd_x3r/h2r: kxp must be >= Kx and a multiple of 32");
    MSAT_REQUIRE(aligned16(hprev) && ldp % 4 == 0 && aligned16(wiT) && aligned16(whT),
                 "gru_ln_fused_fwd_x3r/h2r: hprev / weight planes must be 16-byte aligned");
    MSAT_REQUIRE(aligned16(out) && ldo % 4 == 0 && (!g4 || (aligned16(g4) && ldg % 4 == 0)),
                 "gru_ln_fused_fwd_x3r/h2r: out / g4 rows must be 16-byte aligned");
    a = GruX3rArgs{};
    for (int g = 0; g < 3; ++g) {
        a.seg[g] = ws[g] ? seg[g] : nullptr;
        a.seg_ld[g] = lds_[g];
        a.seg_w[g] = ws[g];
    }
    a.hp = hprev;
    a.ldp = ldp;
    a.wiT = reinterpret_cast<const uint16_t *>(wiT);
    a.whT = reinterpret_cast<const uint16_t *>(whT);
    a.kxp = kxp;
    a.bi = bi;
    a.bh = bh;
    a.ln_scale = ln_scale;
    a.ln_bias = ln_bias;
    a.out = out;
    a.ldo = ldo;
    a.g4 = g4;
    a.ldg = ldg;
    a.R = R;
    a.Kx = Kx;
    return MSAT_OK;
}

extern "C" int msat_gru_ln_fused_fwd_x3r(const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1,
                                         int32_t w1, const float *x2, int32_t ld2, int32_t w2, const float *hprev,
                                         int32_t ldp, const void *wiT_planes, int32_t kxp, const float *bi,
                                         const void *whT_planes, const float *bh, const float *ln_scale,
                                         const float *ln_bias, float *out, int32_t ldo, float *g4, int32_t ldg,
                                         int32_t R, int32_t H, void *stream) {
    MSAT_REQUIRE(R >= 0, "gru_ln_fused_fwd_x3r: R < 0");
    if (R == 0) return MSAT_OK;
    GruX3rArgs a;
    const int rc = gru_r_args(a, x0, ld0, w0, x1, ld1, w1, x2, ld2, w2, hprev, ldp, wiT_planes, kxp, bi, whT_planes,
                              bh, ln_scale, ln_bias, out, ldo, g4, ldg, R, H);
    if (rc) return rc;
    hipLaunchKernelGGL(gru_ln_fused_fwd_x3r_kernel, dim3((R + 127) / 128), dim3(512), 0, (hipStream_t)stream, a);
    return check_launch("gru_ln_fused_fwd_x3r_kernel");
}

extern "C" int msat_split_f16x2_t(const float *W, int32_t K, int32_t N, int32_t ldw, int32_t Kp, void *planes,
                                  int32_t *bad, void *stream) {
    MSAT_REQUIRE(W && planes && bad && K > 0 && N > 0 && ldw >= N && Kp >= K, "bad split_f16x2_t args");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(bad, 0, sizeof(int32_t), s) != hipSuccess) return check_launch("split_f16x2_t memset");
    const size_t n = (size_t)N * Kp;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(split_f16x2_t_kernel, dim3(grid), dim3(256), 0, s, W, K, N, ldw, Kp,
                       reinterpret_cast<_Float16 *>(planes), bad);
    return check_launch("split_f16x2_t_kernel");
}

extern "C" int msat_gru_ln_fused_fwd_h2r(const float *x0, int32_t ld0, int32_t w0, const float *x1, int32_t ld1,
                                         int32_t w1, const float *x2, int32_t ld2, int32_t w2, const float *hprev,
                                         int32_t ldp, const void *wiT_h2, const void *whT_h2, const void *wiT_x3,
                                         const void *whT_x3, int32_t kxp, const float *bi, const float *bh,
                                         const float *ln_scale, const float *ln_bias, float *out, int32_t ldo,
                                         float *g4, int32_t ldg, int32_t R, int32_t H, int32_t *tile_flags,
                                         const int32_t *wbad, void *stream) {
    MSAT_REQUIRE(R >= 0, "gru_ln_fused_fwd_h2r: R < 0");
    if (R == 0) return MSAT_OK;
    MSAT_REQUIRE(tile_flags && wbad, "gru_ln_fused_fwd_h2r: NULL flags");
    GruX3rArgs a;
    int rc = gru_r_args(a, x0, ld0, w0, x1, ld1, w1, x2, ld2, w2, hprev, ldp, wiT_h2, kxp, bi, whT_h2, bh, ln_scale,
                        ln_bias, out, ldo, g4, ldg, R, H);
    if (rc) return rc;
    MSAT_REQUIRE(wiT_x3 && whT_x3 && aligned16(wiT_x3) && aligned16(whT_x3), "gru_ln_fused_fwd_h2r: bf16x3 planes");
    a.flags = tile_flags;
    a.wbad = wbad;
    const int tiles = (R + 127) / 128;
    const char *e = getenv("MARLSAT_GRU_H2S");  // 0: activations to registers (round-1 form), A/B
    const char *pp = getenv("MARLSAT_GRU_H2P");  // 1: 64-row ping-pong tiles (two workgroups per CU)
    if (pp && pp[0] == '1') {
        if (hipMemsetAsync(tile_flags, 0, sizeof(int32_t) * tiles, (hipStream_t)stream) != hipSuccess)
            return check_launch("gru h2p flags memset");
        hipLaunchKernelGGL(gru_ln_fused_fwd_h2p_kernel, dim3((R + 63) / 64), dim3(256), 0, (hipStream_t)stream, a);
        rc = check_launch("gru_ln_fused_fwd_h2p_kernel");
    } else if (e && e[0] == '0') {
        hipLaunchKernelGGL(gru_ln_fused_fwd_h2r_kernel, dim3(tiles), dim3(512), 0, (hipStream_t)stream, a);
        rc = check_launch("gru_ln_fused_fwd_h2r_kernel");
    } else {
        hipLaunchKernelGGL(gru_ln_fused_fwd_h2s_kernel, dim3(tiles), dim3(512), 0, (hipStream_t)stream, a);
        rc = check_launch("gru_ln_fused_fwd_h2s_kernel");
    }
    if (rc) return rc;
    a.wiT = reinterpret_cast<const uint16_t *>(wiT_x3);
    a.whT = reinterpret_cast<const uint16_t *>(whT_x3);
    a.wbad = nullptr;
    hipLaunchKernelGGL(gru_ln_fused_fwd_x3r_fix_kernel, dim3(std::min(tiles, 256)), dim3(512), 0, (hipStream_t)stream,
                       a, tiles);
    return check_launch("gru_ln_fused_fwd_x3r_fix_kernel (fixup)");
}
