// bf16x3 split helpers shared by gemm_x3.hip and gru_fused.hip.
//
// split: x = x1 + x2 + x3 (+ O(2^-24 |x|)) with x1 = bf16(x), x2 = bf16(x - x1), x3 = bf16(x - x1 - x2);
// each difference is exact in fp32.  tr_frag: a 32x32x16 bf16 MFMA fragment (8 consecutive rows of
// one column per lane) read with ds_read_b64_tr_b16 from a [rows][128 cols] bf16 image with
// 256-byte rows whose 16-byte chunks are XOR-swizzled by w3off (conflict-free transposed reads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msat {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct Split8 {
    uint4 p[3];
};

__device__ __forceinline__ Split8 split8(const float4 &u, const float4 &v) {
    const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
    bf16x8 h, m, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 a = (__bf16)x[j];
        const float r = x[j] - (float)a;
        const __bf16 b = (__bf16)r;
        const float r2 = r - (float)b;
        h[j] = a;
        m[j] = b;
        l[j] = (__bf16)r2;
    }
    Split8 s;
    s.p[0] = __builtin_bit_cast(uint4, h);
    s.p[1] = __builtin_bit_cast(uint4, m);
    s.p[2] = __builtin_bit_cast(uint4, l);
    return s;
}

// planes[q][r][c] = part q of W[r][(c + rot) % cols]  (rot: a column rotation of the gate blocks)
struct Split4 {
    uint2 p[3];
};

__device__ __forceinline__ Split4 split4(const float4 &u) {
    const float x[4] = {u.x, u.y, u.z, u.w};
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 h, m, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const __bf16 a = (__bf16)x[j];
        const float r = x[j] - (float)a;
        const __bf16 b = (__bf16)r;
        h[j] = a;
        m[j] = b;
        l[j] = (__bf16)(r - (float)b);
    }
    Split4 s;
    s.p[0] = __builtin_bit_cast(uint2, h);
    s.p[1] = __builtin_bit_cast(uint2, m);
    s.p[2] = __builtin_bit_cast(uint2, l);
    return s;
}

struct Split2 {
    uint32_t p[3];
};

__device__ __forceinline__ Split2 split2(const float2 &u) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const float x[2] = {u.x, u.y};
    bf16x2 h, m, l;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const __bf16 a = (__bf16)x[j];
        const float r = x[j] - (float)a;
        const __bf16 b = (__bf16)r;
        h[j] = a;
        m[j] = b;
        l[j] = (__bf16)(r - (float)b);
    }
    Split2 s;
    s.p[0] = __builtin_bit_cast(uint32_t, h);
    s.p[1] = __builtin_bit_cast(uint32_t, m);
    s.p[2] = __builtin_bit_cast(uint32_t, l);
    return s;
}

// fp16x2 split: x = h + l, h = fp16(x), l = fp16(x - h) (x - h exact; 22 significant bits while x and
// l stay in fp16's normal range).  Three fp16 MFMAs per product (h h, h l, l h) keep every term above
// 3 * 2^-22 |a b|.  fp16's range is the caller's business: operands are scaled by exact powers of
// two (f16x2_row_exp) or range-checked.
struct SplitH4 {
    uint2 p[2];
};

__device__ __forceinline__ SplitH4 splith4(const float4 &u) {
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    const float x[4] = {u.x, u.y, u.z, u.w};
    f16x4 h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const _Float16 a = (_Float16)x[j];
        h[j] = a;
        l[j] = (_Float16)(x[j] - (float)a);
    }
    SplitH4 s;
    s.p[0] = __builtin_bit_cast(uint2, h);
    s.p[1] = __builtin_bit_cast(uint2, l);
    return s;
}

// Scale exponent of a row whose largest |x| is m, for the fp16x2 split: m * 2^e in [2^14, 2^15), so the
// scaled row is inside fp16's range with its largest elements at full precision.  kExpZero marks an
// all-zero row (no constraint); a non-finite m gives 0 (the Inf / NaN then propagates as in fp32).
constexpr int kExpZero = 0x3fff;
__device__ __forceinline__ int f16x2_row_exp(float m) {
    if (!(m <= 3.402823466e38f)) return 0;
    if (m == 0.0f) return kExpZero;
    int E;
    (void)frexpf(m, &E);  // m = f 2^E, f in [0.5, 1)
    return 15 - E;
}

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int w3off(int row, int ch) {  // byte offset of 16-byte chunk ch of row
    return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ bf16x8 tr_frag(const unsigned short *plane, int r0, int c0, int lane) {
    // lanes 16g..16g+15 of a half: rows r0..r0+3 then r0+4..r0+7, columns 8 c0 + 16 g' .. (see the map)
    const int i = lane & 15, q = i >> 2, p = i & 3;
    const char *b = reinterpret_cast<const char *>(plane);
    typedef __attribute__((address_space(3))) s16x4 *lp;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(b + w3off(r0 + q, c0 + (p >> 1)) + 8 * (p & 1)));
    const s16x4 hi =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(b + w3off(r0 + 4 + q, c0 + (p >> 1)) + 8 * (p & 1)));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}


}  // namespace msat
