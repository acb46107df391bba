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
// Fast gate nonlinearities for the register-A epilogues: v_exp + v_rcp (<= 2 ulp each), no IEEE division.
__device__ __forceinline__ float fsig_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// tanh to ~1.3 ulp relative everywhere.  2 sigma(2x) - 1 alone cancels for small |x| (absolute error ~1e-7
// where tanh is ~x): in the L = 16 encoder that absolute error, divided by a LayerNorm row's small standard
// deviation step after step, moved one uf100 critic value by 1e-5 (5e-4 relative) where the fp32 oracle
// stays at 1e-7 (profiles/r05/r05d_*, r05e_*).  |x| < 0.625: odd minimax polynomial x + x u P(u), u = x^2
// (degree 4 in u, fitted on the relative error, max 1.3 ulp); above: 2 sigma(2|x|) - 1 >= 0.55 (no
// cancellation) with the sign of x.  Both branches evaluated, one selected (no divergence).
constexpr float kTh1 = -0.33333277702331543f, kTh2 = 0.13331381976604462f, kTh3 = -0.05373896285891533f,
                kTh4 = 0.020646216347813606f, kTh5 = -0.005720897577702999f, kThCut = 0.625f;
__device__ __forceinline__ float ftanh_fast(float x) {
    const float u = x * x;
    float p = fmaf(u, kTh5, kTh4);
    p = fmaf(u, p, kTh3);
    p = fmaf(u, p, kTh2);
    p = fmaf(u, p, kTh1);
    const float small = fmaf(x, u * p, x);
    const float big = 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * fabsf(x))) - 1.0f;
    return fabsf(x) < kThCut ? small : copysignf(big, x);
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
// Operands: x = x1 + x2, x1 = fp16(x), x2 = fp16(x - x1) (x - x1 exact; 22 significant bits while x2
// stays in fp16's normal range, i.e. |x| >~ 2^-3, below that the representation error is absolute,
// <= 2^-25); the activations are scaled by 2^kH2AShift and the weights by 2^kH2Shift before their splits
// (msat_split_f16x2_t), the sums by 2^-(kH2Shift + kH2AShift) after (all exact).  Three MFMAs per (gate,
// column tile) block, a1b2 a2b1 a1b1; the dropped a2b2 and the representation residuals are <= 3 * 2^-22 |ab|
// per product, under the fp32 accumulation error of a 288..416-deep dot product.
// Why the activations are scaled (round 6): unscaled, every activation below 2^-3 (LayerNorm outputs near
// zero, small message sums) kept only an absolute 2^-25; in the L = 16 train cycle that error, applied to
// every row, moved the var-negative cell's n-gate bias gradients by up to 10x the fp32 oracle's own error at
// fixed parameters (profiles/parity_attrib.py + parity_orderings.py).  2^7 keeps 22 bits
// down to |x| ~ 1e-3 and leaves |x| < 256 inside the range check below.
// Against bf16x3: half the MFMAs (3 vs 6), 48 instead of 72 KiB of weights per step.
// fp16's range is checked, not assumed: a tile that loads an activation with |a| 2^kH2AShift >= 2^15 (|a| >=
// 256), or whose weights overflowed at the split (wbad), writes flags[tile] = 1 and no output, and the
// bf16x3 kernel, launched next with the same flags, recomputes exactly the flagged tiles.
constexpr int kH2Shift = 10;  // weight scale 2^10: |W| < 32 fits, |W| >= 2^-24 keeps 11 bits
constexpr int kH2AShift = 7;  // activation scale 2^7: |a| < 256 fits, |a| >= 2^-10 keeps 22 bits


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

// The activations go through LDS as well.  Each step's [128 rows][32 k] fp32 tile (16 KiB) is fetched by
// LDS-DMA three steps ahead into one of four slots ([row][8 chunks of 16 B], chunk c of row r at slot
// c ^ ((r >> 1) & 5): conflict-free ds_read_b128 for the register-A lane map), and split from LDS in the
// middle of the step before its use.  With no registers in flight across steps, the step end waits only
// for the next step's weights and the activations of step s + 2 (vmcnt(2)): the activation fetches get
// 2.5 steps of lead.  The input steps run first and h's four quarters last, so at the epilogue the four
// slots still hold h: the gate algebra reads it there instead of fetching the rows again (512 B per
// row).  128-row tiles of 8 waves (16 rows each), one workgroup per CU: 96 KiB of double-buffered
// weights + 64 KiB of activation slots, the whole LDS.
//
// Measured and not kept: activations to registers instead of LDS (-0.5..-1 %),
// 64-row "ping-pong" tiles at two workgroups per CU (5-7 % slower), 16-wave tiles (5-9 % slower),
// deeper fragment lookahead (+-0.5 %), a split stagger of SIMD partners (0..+0.5 %).
constexpr int kDmaLate = 8;  // waves 4..7 issue the step's DMA before this block (SIMD-partner stagger)
// (A persistent form -- one workgroup per CU walking tiles, each prefetching the next tile's prologue from its
// epilogue -- measured 1-7 % slower in round 4; its source is profiles/archive_r04/gru_persistent.patch.)
__device__ __forceinline__ void gru_h2s_tile(const GruX3rArgs &a, int tile) {
    constexpr int NW = 8;                // waves (16 rows each)
    constexpr int H = 128, IMG = H * 4;  // uint4 per (plane, gate) image: 128 units x 4 chunks = 8 KiB
    constexpr int NI = 6;                // (plane, gate) images per step
    constexpr int NIW = 8 * NI / NW;     // weight DMA instructions per wave and step
    constexpr int TR = 16 * NW;          // tile rows
    __shared__ uint4 Bs[2 * NI * IMG];   // 48 KiB per buffer
    constexpr int ASL = TR * 8;          // uint4 per activation slot (128 B per row)
    __shared__ uint4 As[4 * ASL];        // four activation slots: step s in slot s & 3
    const int t = threadIdx.x;
    const int lane = t & 63, l16 = lane & 15, g = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int row0 = tile * TR, wr = 16 * w;
    int *const flag = a.flags + tile;
    // weights out of fp16 range: the bf16x3 launch does every tile
    if (a.wbad[0] | a.wbad[1]) {
        if (t == 0) *flag = 1;
        return;
    }
    // step order: the input steps 0 .. nin - 1 first, then the hidden steps (h's four 32-column quarters),
    // whose activation slots still hold all of h at the epilogue (no refetch of h)
    constexpr int nsh = H / 32;
    const int nin = a.kxp / 32, ns = nin + nsh;
    const float *const hp = a.hp, *const sg0 = a.seg[0], *const sg1 = a.seg[1], *const sg2 = a.seg[2];
    const int w0 = a.seg_w[0], w01 = a.seg_w[0] + a.seg_w[1], kx_end = a.Kx;
    // weight DMA: 8 NI wave-instructions (1 KiB = 16 units x 4 chunks) per step, NI per wave;
    // instruction e of wave w fills image x = (NI w + e) / 8 (plane * 3 + gate), units 16 p .. 16 p + 15
    // (p = (NI w + e) % 8).  Lane -> unit 16 p + (lane >> 2), LDS chunk lane & 3 = source chunk
    // (lane & 3) ^ f((lane >> 4) & 3).
    const unsigned lpart = (unsigned)(lane >> 2) * 2u, chb = 16u * ((lane & 3) ^ gswz16((lane >> 4) & 3));
    // piece x = NIW w + e covers W^T rows 16 x .. 16 x + 15 and LDS bytes [1 KiB x, +1 KiB) of the buffer:
    // both linear in x, so the pieces go in pairs with one M0 setup and no per-piece index arithmetic
    auto issueW = [&](int s, int buf) {
        const bool hid = s >= nin;
        const int Kp = hid ? H : a.kxp;
        const uint16_t *bw = (hid ? a.whT + 32 * (s - nin) : a.wiT + 32 * s) + (size_t)(16 * NIW * w) * Kp;
        const unsigned voff = lpart * (unsigned)Kp + chb;
#pragma unroll
        for (int e = 0; e < NIW; e += 2)
            glds16_async_s2<1024>(bw + (size_t)(16 * e) * Kp, bw + (size_t)(16 * e + 16) * Kp, voff,
                                  &Bs[buf * NI * IMG + 64 * (NIW * w + e)]);
    };
    f32x4g acc[4][8];
#pragma unroll
    for (int G = 0; G < 4; ++G)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[G][j] = f32x4g{};
    const int slot = g ^ gswz16((l16 >> 2) & 3);
    float amax = 0.f;  // largest |activation| this lane split (range check)
    typedef float f4v __attribute__((ext_vector_type(4)));
    auto asplit = [&](int st, const f4v (&r)[2], uint4 (&f)[2]) {  // branch-free (selects)
        const int kx = st * 32 + 8 * g;
        const bool z0 = st < nin && kx >= kx_end, z1 = st < nin && kx + 4 >= kx_end;
        const f4v zero = {0.f, 0.f, 0.f, 0.f};
        const f4v as = {(float)(1 << kH2AShift), (float)(1 << kH2AShift), (float)(1 << kH2AShift),
                        (float)(1 << kH2AShift)};  // exact power of two
        const float4 v0 = __builtin_bit_cast(float4, z0 ? zero : r[0] * as);
        const float4 v1 = __builtin_bit_cast(float4, z1 ? zero : r[1] * as);
        const float m0 = fmaxf(fmaxf(fabsf(v0.x), fabsf(v0.y)), fmaxf(fabsf(v0.z), fabsf(v0.w)));
        const float m1 = fmaxf(fmaxf(fabsf(v1.x), fabsf(v1.y)), fmaxf(fabsf(v1.z), fabsf(v1.w)));
        amax = fmaxf(amax, fmaxf(m0, m1));
        const SplitH8 sp = splith8(v0, v1);
        f[0] = sp.p[0];
        f[1] = sp.p[1];
    };
    uint4 fas[1][2], fnx[2];  // split activations of this step / the next (moved over at the step end)
    // activation DMA, 16 wave-instructions (1 KiB = 8 rows x 8 chunks) per step, 2 per wave;
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
    // full tiles whose step lies inside one segment: a wave-uniform base and per-lane 32-bit offsets
    // (precomputed per source leading dimension); the last tile and a step straddling segments take the
    // per-lane form below (r0: the tile's first row)
    auto issueA = [&](int st, int r0) {
        const int k = st * 32;
        const bool full = r0 + TR <= a.R;
        if (full && (st >= nin || k + 32 <= w0)) {
            const bool h = st >= nin;
            const int ld = h ? a.ldp : a.seg_ld[0];
            const float *b = (h ? hp + 32 * (st - nin) : sg0 + k) + (size_t)r0 * ld;
            uint4 *dst = &As[(st & 3) * ASL + 64 * 2 * w];
#pragma unroll
            for (int e = 0; e < 2; ++e)
                glds16_async_s(b, (unsigned)(drow[e] * ld + 4 * dchunk[e]) * 4u, dst + 64 * e);
            return;
        }
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int rr = r0 + drow[e], rc = rr < a.R ? rr : a.R - 1;
            const float *src;
            if (st >= nin) {
                src = hp + (size_t)rc * a.ldp + 32 * (st - nin) + 4 * dchunk[e];
            } else {
                const int kx = st * 32 + 4 * dchunk[e];
                if (kx < w0) src = sg0 + (size_t)rc * a.seg_ld[0] + kx;
                else if (kx < w01) src = sg1 + (size_t)rc * a.seg_ld[1] + (kx - w0);
                else if (kx < kx_end) src = sg2 + (size_t)rc * a.seg_ld[2] + (kx - w01);
                else src = hp;  // padding k: one fixed valid line (L2-resident: no HBM bytes), zeroed at the split
            }
            glds16_async(src, &As[(st & 3) * ASL + 64 * (2 * w + e)]);
        }
    };
    auto lsplit = [&](int st, uint4 (&f)[2]) {  // split step st's activations from its LDS slot
        const int r = wr + l16, sw = (r >> 1) & 5;
        const uint4 *row = &As[(st & 3) * ASL + 8 * r];
        f4v v[2];
        v[0] = __builtin_bit_cast(f4v, row[(2 * g) ^ sw]);
        v[1] = __builtin_bit_cast(f4v, row[(2 * g + 1) ^ sw]);
        asplit(st, v, f);
    };
    auto prologue = [&](int r0) {  // step 0's weights and activation steps 0..2 of the tile at row r0
        issueA(0, r0);
        if (ns > 1) issueA(1, r0);
        if (ns > 2) issueA(2, r0);
        issueW(0, 0);
    };
    prologue(row0);
    wait_vmcnt<0>();
    barrier_lds();
    lsplit(0, fas[0]);
    // one 32-k step; two static copies (input, hidden): the weight buffer's parity is a runtime offset and
    // the next step's split activations are moved into place at the step end, so the accumulators keep
    // one register assignment through the whole loop (a copy per parity and step kind spilled them)
    auto pstep = [&](int st, auto hidc) {
        constexpr bool hid = decltype(hidc)::value;
        const int buf = st & 1;
        // Stagger of SIMD partners (waves w and w + 4 share a SIMD): waves 4..7 issue the step's DMA
        // before block kDmaLate, so partners' DMA bursts do not coincide (profiles/ab_gru_dma.sh, tape
        // on: -2.9 % clause / -1.1 % var; blocks 4..16 -1..-2.5 %; delaying waves 0..3 too +2 %).
        const bool late = w >= 4;
        auto dma = [&]() {
            if (st + 1 < ns) issueW(st + 1, buf ^ 1);
            if (st + 3 < ns) issueA(st + 3, row0);
        };
        if (!late) dma();
        // weight fragments carried across the 24 (gate, column tile) blocks: each plane is re-read
        // for the next block as soon as its last MFMA here has issued, so the reads fly under the
        // MFMAs instead of each block waiting for its own reads (at 255 VGPRs the compiler had
        // issued every block's reads just before its MFMAs and waited on them).
        auto bfrag = [&](int n, int q) {
            const int gt = n >> 3, j = n & 7;
            return Bs[(buf * NI + q * 3 + gt) * IMG + (16 * j + l16) * 4 + slot];
        };
        uint4 (&fa)[2] = fas[0];
        {
            // fragments LA = 2 blocks ahead in LA rotating register sets (block n uses set n % LA; each
            // plane's register is refilled for block n + LA right after its last MFMA in block n)
            constexpr int LA = 2;
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
                c = h2mma(fa[0], b1, c);  // a1 b2
                if (n + LA < 24) b1 = bfrag(n + LA, 1);
                c = h2mma(fa[1], b0, c);  // a2 b1
                c = h2mma(fa[0], b0, c);  // a1 b1
                if (n + LA < 24) b0 = bfrag(n + LA, 0);
                acc[G][j] = c;
                if (n == 7 && st + 1 < ns) lsplit(st + 1, fnx);
                if (late && n + 1 == kDmaLate) dma();
                __builtin_amdgcn_sched_barrier(0);  // keep the blocks in order (the reads lead by one)
            }
        }
        // W(st + 1) and A(st + 2) landed (A(st + 3), issued last, may fly); no registers in flight
        if (st + 3 < ns) wait_vmcnt<2>();
        else wait_vmcnt<0>();
        fas[0][0] = fnx[0];
        fas[0][1] = fnx[1];
        barrier_lds();
    };
    {
        int st = 0;
#pragma unroll 1
        for (; st < nin; ++st) pstep(st, std::false_type{});
#pragma unroll 1
        for (; st < ns; ++st) pstep(st, std::true_type{});
    }
    {  // range check: |a 2^kH2AShift| < 2^15 keeps a1 = fp16(a 2^kH2AShift) finite with margin.  A ballot per wave and an
       // LDS-only barrier: __syncthreads_or's fence would also wait for the h DMA in flight.
        // the weight buffers are free past the last step's barrier: the flags sit in Bs's last 32 bytes,
        // beyond the epilogue's stage (LDS is full: 96 KiB of weights + 64 KiB of activation slots)
        int *const wbadl = reinterpret_cast<int *>(&Bs[2 * NI * IMG]) - NW;
        const bool wb = __ballot(!(amax < 32768.0f)) != 0;
        if (lane == 0) wbadl[w] = wb;
        barrier_lds();
        int bad = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) bad |= wbadl[q];
        if (t == 0) *flag = bad;
        if (bad) {
            wait_vmcnt<0>();  // no LDS-DMA may land after the workgroup's LDS is released
            return;
        }
    }

    // ---- epilogue.  C/D map: unit u = 16 j + l16, row wr + 4 g + reg.
    // stage: [16 rows][132] per wave in weight buffer 0
    constexpr int SW = 132;
    float *stage = reinterpret_cast<float *>(Bs) + w * 16 * SW;
    const bool tape = a.g4 != nullptr;
    // h of each accumulator's (row, unit) from the hidden steps' slots: quarter q (units 32 q ..) is step
    // nin + q in slot (nin + q) & 3, [row][8 chunks], chunk c of row r at c ^ ((r >> 1) & 5).  All four
    // landed before the last step's barrier; the stage below lives in Bs, not in the slots.
    float hv[8][4];
    {
        const float *Af = reinterpret_cast<const float *>(As);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int kq = 16 * (j & 1) + l16, sb = ((nin + (j >> 1)) & 3) * ASL;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int R = wr + 4 * g + r;
                hv[j][r] = Af[4 * (sb + 8 * R + ((kq >> 2) ^ ((R >> 1) & 5))) + (kq & 3)];
            }
        }
    }
    constexpr float sc = 1.0f / (float)(1 << (kH2Shift + kH2AShift));  // exact power of two
    // packed fp32 (v_pk_mul / v_pk_add on row pairs): no MFMAs run here, so the packed forms halve the
    // epilogue's vector issue instead of competing with matrix work
    // LayerNorm scale / bias, loaded with the gate biases
    float lsc[8], lbs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int u = 16 * j + l16;
        const float br = a.bi[u] + a.bh[u], bz = a.bi[H + u] + a.bh[H + u];
        const float bni = a.bi[2 * H + u], bnh = a.bh[2 * H + u];
        lsc[j] = a.ln_scale[u];
        lbs[j] = a.ln_bias[u];
        const f32x4g s4 = {sc, sc, sc, sc};
        acc[0][j] = acc[0][j] * s4 + f32x4g{br, br, br, br};
        acc[1][j] = acc[1][j] * s4 + f32x4g{bz, bz, bz, bz};
        acc[2][j] = acc[2][j] * s4 + f32x4g{bni, bni, bni, bni};
        acc[3][j] = acc[3][j] * s4 + f32x4g{bnh, bnh, bnh, bnh};
    }
    // float4 rows of the wave's [16][128] stage -> dst (row stride ld), rows < R only.  The stage is
    // wave-private and a wave's LDS operations complete in issue order, so waiting for its own stage
    // writes (lgkmcnt) is the only ordering needed: no workgroup barrier, whose release fence would
    // also drain the wave's global stores.
    auto flush = [&](float *dst, int ld) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int rr = 2 * it + (lane >> 5), c4 = lane & 31;
            const float4 v = *reinterpret_cast<const float4 *>(stage + rr * SW + 4 * c4);
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
    typedef float f2 __attribute__((ext_vector_type(2)));
    constexpr float kL2E = 1.4426950408889634f;  // exp(x) = 2^(x log2 e), as __expf
    auto exp2v = [](f2 x) { return f2{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; };
    auto rcpv = [](f2 x) { return f2{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)}; };
    const f2 one = {1.f, 1.f}, ml2e = {-kL2E, -kL2E}, m2l2e = {-2.f * kL2E, -2.f * kL2E}, two = {2.f, 2.f};
    // ftanh_fast on a row pair (packed FMAs for the polynomial branch)
    auto tanhv = [&](f2 x) {
        const f2 u = x * x;
        auto fm = [](f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); };
        f2 p = fm(u, f2{kTh5, kTh5}, f2{kTh4, kTh4});
        p = fm(u, p, f2{kTh3, kTh3});
        p = fm(u, p, f2{kTh2, kTh2});
        p = fm(u, p, f2{kTh1, kTh1});
        const f2 small = fm(x, u * p, x);
        const f2 ax = {fabsf(x.x), fabsf(x.y)};
        const f2 big = two * rcpv(one + exp2v(ax * m2l2e)) - one;
        return f2{ax.x < kThCut ? small.x : copysignf(big.x, x.x), ax.y < kThCut ? small.y : copysignf(big.y, x.y)};
    };
    f2 s1v[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}}, s2v[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int p = 0; p < 2; ++p) {  // rows 2p, 2p + 1
            const f2 rp = {acc[0][j][2 * p], acc[0][j][2 * p + 1]}, zp = {acc[1][j][2 * p], acc[1][j][2 * p + 1]};
            const f2 gi = {acc[2][j][2 * p], acc[2][j][2 * p + 1]}, gh = {acc[3][j][2 * p], acc[3][j][2 * p + 1]};
            const f2 h = {hv[j][2 * p], hv[j][2 * p + 1]};
            const f2 rg = rcpv(one + exp2v(rp * ml2e)), zg = rcpv(one + exp2v(zp * ml2e));
            const f2 ng = tanhv(gi + rg * gh);
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
        const float scl = lsc[j], lb = lbs[j];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const f2 hn = {acc[0][j][2 * p], acc[0][j][2 * p + 1]};
            const f2 y = (hn - f2{mean[2 * p], mean[2 * p + 1]}) * (f2{rs[2 * p], rs[2 * p + 1]} * f2{scl, scl}) +
                         f2{lb, lb};
            stage[(4 * g + 2 * p) * SW + u] = y.x;
            stage[(4 * g + 2 * p + 1) * SW + u] = y.y;
        }
    }
    flush(a.out, a.ldo);
}

__global__ void __launch_bounds__(512, 1) gru_ln_fused_fwd_h2s_kernel(GruX3rArgs a) { gru_h2s_tile(a, blockIdx.x); }

// bf16x3 register-A kernel (the fp16x2 kernel above is fp16x2-only: instantiated for bf16x3 it computed
// wrong results; this is the round-1 kernel).  Activations loaded two steps ahead into registers, weight
// fragments carried across column blocks, tape stored from the accumulators.
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
    // Pipelined form: activation loads two steps ahead into alternating register sets (plain loads,
    // tracked by hipcc, which may move an asm load's output registers before the data lands); the
    // split of step s + 1 runs among step s's
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
    // two waves per unit group (row split of the 64-row tile; one wave measured slower in round 1)
    if (H == 64) {
        hipLaunchKernelGGL((gru_ln_fused_fwd_kernel<2, 2>), grid, dim3(256), 0, s, a);
    } else if (H == 128) {
        hipLaunchKernelGGL((gru_ln_fused_fwd_kernel<4, 2>), grid, dim3(512), 0, s, a);
    } else {
        hipLaunchKernelGGL((gru_ln_fused_fwd_kernel<8, 1>), grid, dim3(512), 0, s, a);
    }
    return check_launch("gru_ln_fused_fwd_kernel");
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
    hipLaunchKernelGGL(gru_ln_fused_fwd_h2s_kernel, dim3(tiles), dim3(512), 0, (hipStream_t)stream, a);
    rc = check_launch("gru_ln_fused_fwd_h2s_kernel");
    if (rc) return rc;
    a.wiT = reinterpret_cast<const uint16_t *>(wiT_x3);
    a.whT = reinterpret_cast<const uint16_t *>(whT_x3);
    a.wbad = nullptr;
    hipLaunchKernelGGL(gru_ln_fused_fwd_x3r_fix_kernel, dim3(std::min(tiles, 256)), dim3(512), 0, (hipStream_t)stream,
                       a, tiles);
    return check_launch("gru_ln_fused_fwd_x3r_fix_kernel (fixup)");
}
