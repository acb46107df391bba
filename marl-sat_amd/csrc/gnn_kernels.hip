// GNN encoder / actor-critic building blocks for the MAPPO update (gfx950).
//
// The reference's encoder (src/learners/mappo_gnn_sat_learner.py:19-82) multiplies
// DENSE V x C adjacency matrices; a 3-SAT clause has <= 3 literals, so here both
// message directions are signed gathers over the literal incidence of a ragged
// batch of graphs (each sample contributes its critic graph plus one local graph
// per agent, see marlsat/learners/graphs.py):
//   clause side  m_c = [sum_{pos lits} src_v[:H], sum_{neg lits} src_v[H:]]   (A^T M)
//   var side     n_v = [sum_{pos occ} src_c[:H], sum_{neg occ} src_c[H:]]     (A M)
// and each is the other's transpose, so the backward pass reuses them.
// GRU + LayerNorm (flax nn.GRUCell / nn.LayerNorm semantics) are fused row kernels
// (one wave per row) on top of the fp32 MFMA GEMMs of gemm.hip.
#include "common.h"
#include "split3.h"

namespace msat {

constexpr int kRowThreads = 256;  // 4 waves -> 4 rows per block iteration

// Debug builds (MSAT_DCHECK): elements from each buffer's pointer to the end of its allocation (dbg_extent):
// the sources, the destinations and the index array (slots / inc) and ptr; zeros in product builds.
struct GatherDbg {
    long long src_pos, src_neg, dst_pos, dst_neg, idx, ptr;
};
static GatherDbg gather_dbg(const void *sp, const void *sn, const void *dp, const void *dn, const void *idx,
                            const void *ptr) {
    return GatherDbg{dbg_extent(sp, 4), dbg_extent(sn, 4), dbg_extent(dp, 4), dbg_extent(dn, 4), dbg_extent(idx, 4),
                     dbg_extent(ptr, 4)};
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// ------------------------------------------------------------------ gathers --
// slots: (Nc, 3) int32, (var_row << 1) | neg, or -1.  One wave per clause row.
// Positive literals read src_pos rows, negative ones src_neg rows (both H wide, ld_src).
//   split  (merged = 0): dst[c] (+)= [sum_{pos} src_pos[v] | sum_{neg} src_neg[v]]   (2H wide)
//   merged (merged = 1): dst[c] (+)= sum_{pos} src_pos[v] + sum_{neg} src_neg[v]      (H wide)
// The merged form is the transpose of var_gather with one shared source (the backward of
// the gather-first var messages); per output the slots are summed in slot order.
__global__ void __launch_bounds__(kRowThreads)
clause_gather_kernel(const float *__restrict__ src_pos, const float *__restrict__ src_neg, int lds_,
                     const int *__restrict__ slots, float *__restrict__ dst, int ldd, int Nc, int H, int merged,
                     int accumulate, GatherDbg dbg) {
    const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
    const int W = merged ? H : 2 * H;
    // two clause rows per wave, one per 32-lane half: twice the independent slot -> row load chains in
    // flight per wave (the gather is latency-bound at full occupancy), and the merged form (W = H) keeps
    // every lane busy
    for (int c0 = 2 * (blockIdx.x * 4 + (threadIdx.x >> 6)); c0 < Nc; c0 += gridDim.x * 8) {
        const int c = c0 + half;
        if (c >= Nc) continue;
        MSAT_DCHECK(3 * (long long)c + 2, dbg.idx);
        const int s0 = slots[3 * (size_t)c], s1 = slots[3 * (size_t)c + 1], s2 = slots[3 * (size_t)c + 2];
        for (int j = l32 * 4; j < W; j += 128) {
            const int want = j < H ? 0 : 1;  // split: first half positive literals, second negative
            const int col = j < H ? j : j - H;
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            // all three slot loads in flight before the (slot-ordered) adds
            const int sl[3] = {s0, s1, s2};
            bool ok[3];
            float4 x[3];
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const int S = sl[u];
                ok[u] = S >= 0 && (merged || (S & 1) == want);
                const float *src = (S & 1) ? src_neg : src_pos;
                x[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (ok[u]) {
                    MSAT_DCHECK((long long)(S >> 1) * lds_ + col + 3, (S & 1) ? dbg.src_neg : dbg.src_pos);
                    x[u] = *reinterpret_cast<const float4 *>(src + (size_t)(S >> 1) * lds_ + col);
                }
            }
#pragma unroll
            for (int u = 0; u < 3; ++u)
                if (ok[u]) {
                    acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w;
                }
            MSAT_DCHECK((long long)c * ldd + j + 3, dbg.dst_pos);
            float4 *d = reinterpret_cast<float4 *>(dst + (size_t)c * ldd + j);
            if (accumulate) {
                const float4 o = *d;
                acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
            }
            *d = acc;
        }
    }
}

// Two var rows per wave (H % 128 == 0), one per 32-lane half: each half walks its row's whole entry
// list in ascending order, eight entry rows in flight, and adds each into the positive or the negative
// accumulator by the entry's sign bit -- per output the same adds in the same order as the kernel below
// (bitwise equal), with twice the rows and the load chains of a wave in flight.
__global__ void __launch_bounds__(kRowThreads)
var_gather_hw_kernel(const float *__restrict__ src_pos, const float *__restrict__ src_neg, int lds_,
                     const int *__restrict__ ptr, const int *__restrict__ inc, float *__restrict__ dst_pos,
                     float *__restrict__ dst_neg, int ldd, int Nv, int H, int accumulate, GatherDbg dbg) {
    __shared__ int s_idx[4][64];  // per wave: each half's current chunk of 32 entries
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
    for (int v0 = 2 * (blockIdx.x * 4 + wv); v0 < Nv; v0 += gridDim.x * 8) {  // wave-uniform trip count
        const int v = v0 + half;
        const bool ok = v < Nv;
        if (ok) MSAT_DCHECK(v + 1, dbg.ptr);
        const int e0 = ok ? ptr[v] : 0, ne = ok ? ptr[v + 1] - e0 : 0;
        const int nmax = max(__builtin_amdgcn_readlane(ne, 0), __builtin_amdgcn_readlane(ne, 32));
        for (int col = l32 * 4; col < H; col += 128) {
            float4 ap = make_float4(0.f, 0.f, 0.f, 0.f), an = ap;
            for (int cb = 0; cb < nmax; cb += 32) {
                const int n = min(32, ne - cb);  // this half's entries in the chunk (<= 0: none)
                if (l32 < n) MSAT_DCHECK((long long)e0 + cb + l32, dbg.idx);
                s_idx[wv][lane] = l32 < n ? inc[e0 + cb + l32] : 0;
                const int nm = min(32, nmax - cb);
                for (int k = 0; k < nm; k += 8) {
                    float4 x[8];
                    int sg[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int kk = k + u;
                        const int sl = s_idx[wv][32 * half + (kk < 32 ? kk : 31)];
                        sg[u] = kk < n ? (sl & 1) : -1;  // -1: no entry
                        const float *src = (sl & 1) ? src_neg : src_pos;
                        if (sg[u] >= 0)
                            MSAT_DCHECK((long long)(sl >> 1) * lds_ + col + 3, (sl & 1) ? dbg.src_neg : dbg.src_pos);
                        x[u] = sg[u] >= 0 ? *reinterpret_cast<const float4 *>(src + (size_t)(sl >> 1) * lds_ + col)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (sg[u] == 0) {
                            ap.x += x[u].x; ap.y += x[u].y; ap.z += x[u].z; ap.w += x[u].w;
                        } else if (sg[u] == 1) {
                            an.x += x[u].x; an.y += x[u].y; an.z += x[u].z; an.w += x[u].w;
                        }
                    }
                }
            }
            if (ok) {
                MSAT_DCHECK((long long)v * ldd + col + 3, dbg.dst_pos);
                MSAT_DCHECK((long long)v * ldd + col + 3, dbg.dst_neg);
                float4 *dp = reinterpret_cast<float4 *>(dst_pos + (size_t)v * ldd + col);
                float4 *dn = reinterpret_cast<float4 *>(dst_neg + (size_t)v * ldd + col);
                if (accumulate) {
                    const float4 o = *dp, q = *dn;
                    ap.x += o.x; ap.y += o.y; ap.z += o.z; ap.w += o.w;
                    an.x += q.x; an.y += q.y; an.z += q.z; an.w += q.w;
                }
                *dp = ap;
                *dn = an;
            }
        }
    }
}

// CSR over var rows: entries (clause_row << 1) | neg.  One wave per var row:
//   dst_pos[v] (+)= sum_{pos entries} src_pos[c],  dst_neg[v] (+)= sum_{neg entries} src_neg[c]
// (src_pos == src_neg: both halves gather the same H-wide clause rows).
__global__ void __launch_bounds__(kRowThreads)
var_gather_kernel(const float *__restrict__ src_pos, const float *__restrict__ src_neg, int lds_,
                  const int *__restrict__ ptr, const int *__restrict__ inc, float *__restrict__ dst_pos,
                  float *__restrict__ dst_neg, int ldd, int Nv, int H, int accumulate, GatherDbg dbg) {
    __shared__ int s_idx[4][64];  // per wave: one chunk of the var row's entry list
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int v = blockIdx.x * 4 + (threadIdx.x >> 6); v < Nv; v += gridDim.x * 4) {
        MSAT_DCHECK(v + 1, dbg.ptr);
        const int e0 = ptr[v], e1 = ptr[v + 1];
        if (e1 > e0) MSAT_DCHECK((long long)e1 - 1, dbg.idx);
        for (int j = lane * 4; j < 2 * H; j += 256) {
            const int want = j < H ? 0 : 1;
            const int col = j < H ? j : j - H;
            const float *src = want ? src_neg : src_pos;
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            if (H % 128) {  // H = 64: half the wave idle in this loop, plain walk
                for (int e = e0; e < e1; ++e) {
                    const int s = inc[e];
                    if ((s & 1) != want) continue;
                    MSAT_DCHECK((long long)(s >> 1) * lds_ + col + 3, want ? dbg.src_neg : dbg.src_pos);
                    const float4 x = *reinterpret_cast<const float4 *>(src + (size_t)(s >> 1) * lds_ + col);
                    acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
                }
            }
            // H % 128 == 0 (every lane active here): the entry list is fetched lane-parallel (64 per
            // load) and split by sign with ballots; each half-wave walks its entries in ascending order
            // (the same summation order as the plain walk), four row loads in flight
            for (int cb = e0; H % 128 == 0 && cb < e1; cb += 64) {
                const int n = min(64, e1 - cb);
                const int my = lane < n ? inc[cb + lane] : 0;
                const uint64_t negm = __ballot(lane < n && (my & 1));
                const uint64_t posm = __ballot(lane < n && !(my & 1));
                s_idx[wv][lane] = my;  // read back below by the (diverged) half-waves: no cross-lane ops there
                uint64_t m = want ? negm : posm;
                while (m) {
                    int k[4];
                    bool ok[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        ok[u] = m != 0;
                        k[u] = ok[u] ? __builtin_ctzll(m) : 0;
                        m &= m - 1;
                    }
                    float4 x[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int s = s_idx[wv][k[u]];
                        if (ok[u]) MSAT_DCHECK((long long)(s >> 1) * lds_ + col + 3, want ? dbg.src_neg : dbg.src_pos);
                        x[u] = ok[u] ? *reinterpret_cast<const float4 *>(src + (size_t)(s >> 1) * lds_ + col)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (ok[u]) {
                            acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w;
                        }
                }
            }
            MSAT_DCHECK((long long)v * ldd + col + 3, want ? dbg.dst_neg : dbg.dst_pos);
            float4 *d = reinterpret_cast<float4 *>((want ? dst_neg : dst_pos) + (size_t)v * ldd + col);
            if (accumulate) {
                const float4 o = *d;
                acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
            }
            *d = acc;
        }
    }
}

// ------------------------------------------------------------- GRU + LN fwd --
// Gi = x Wi + bi ([r|z|n], 3H), Gh = h Wh + bh ([r|z|n], bh = [0,0,b_hn]).
// h' = (1-z) n + z h,  r = s(Gi_r+Gh_r), z = s(Gi_z+Gh_z), n = tanh(Gi_n + r Gh_n)
// y = (h' - mean) * (rsqrt(var + 1e-6) * scale) + bias,  var = E[h'^2] - mean^2.
template <int PER>
__global__ void __launch_bounds__(kRowThreads)
gru_ln_fwd_kernel(const float *__restrict__ Gi, int ldi, const float *__restrict__ Gh, int ldh,
                  const float *__restrict__ hp, int ldp, const float *__restrict__ scale,
                  const float *__restrict__ bias, float *__restrict__ out, int ldo, int R, int H) {
    const int lane = threadIdx.x & 63;
    for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < R; r += gridDim.x * 4) {
        const float *gi = Gi + (size_t)r * ldi, *gh = Gh + (size_t)r * ldh, *h = hp + (size_t)r * ldp;
        float hn[PER];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = lane + 64 * u;
            const float rg = sigmoidf_(gi[j] + gh[j]);
            const float zg = sigmoidf_(gi[H + j] + gh[H + j]);
            const float ng = tanhf(gi[2 * H + j] + rg * gh[2 * H + j]);
            hn[u] = (1.0f - zg) * ng + zg * h[j];
            s1 += hn[u];
            s2 += hn[u] * hn[u];
        }
        s1 = wave_sum_f32(s1);
        s2 = wave_sum_f32(s2);
        const float mean = s1 / (float)H;
        const float var = fmaxf(s2 / (float)H - mean * mean, 0.0f);
        const float rs = rsqrtf(var + 1e-6f);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = lane + 64 * u;
            out[(size_t)r * ldo + j] = (hn[u] - mean) * (rs * scale[j]) + bias[j];
        }
    }
}

// ------------------------------------------------------------- GRU + LN bwd --
// dy -> dGi, dGh (3H each), dh (+=), and per-block partial sums of dscale / dbias
// (part[block][0:H] = sum dy*xhat, part[block][H:2H] = sum dy), reduced later in a
// fixed order.
// G4 = true: Gi is the fused forward's pre-activation tape [r_pre | z_pre | gin | ghn]
// (gru_fused.hip) and Gh is unused.
// NQ = 6: the partials also carry the gate-bias gradients, part[block] =
// [dscale | dbias | d b_ir | d b_iz | d b_in | d b_hn] (H each), so no column-sum pass
// over dGi / dGh is needed.
// NF > 0: the partials also carry feature-weighted gate sums for the input-matrix rows of NF
// per-row features (feat, ld ldf): part[block][NQ + 3k + g] = sum_rows feat[r][k] * dG_g[r]
// (g = r, z, n gate) -- the weight gradient of those input rows without another pass over dGi.
// VEC (the var cell, NF = 6, PER >= 2): a lane owns PER adjacent columns (PER * lane + u), loaded and
// stored as one PER-wide vector access, instead of columns lane + 64 u (one dword access each).  The
// per-column partials keep their row order; only the row sums behind the LayerNorm statistics change
// order.  Measured -0.3..-2 % on the var cell and +16 % on the clause cell, which keeps the scalar
// layout.
template <int N>
__device__ __forceinline__ void ldv(const float *__restrict__ p, float *o) {
    if constexpr (N == 1) {
        o[0] = *p;
    } else {
        typedef float v __attribute__((ext_vector_type(N)));
        const v t = *reinterpret_cast<const v *>(p);
#pragma unroll
        for (int u = 0; u < N; ++u) o[u] = t[u];
    }
}
template <int N>
__device__ __forceinline__ void stv(float *__restrict__ p, const float *o) {
    if constexpr (N == 1) {
        *p = o[0];
    } else {
        typedef float v __attribute__((ext_vector_type(N)));
        v t;
#pragma unroll
        for (int u = 0; u < N; ++u) t[u] = o[u];
        *reinterpret_cast<v *>(p) = t;
    }
}

// PL (flags bit 3): the packed row [dan | dar | daz | dan r] is written as fp16x2 planes at its row exponent
// e (f16x2_row_exp; kExpZero -> 0): the row's 4H floats of buffer hold [hi (4H fp16) | lo (4H fp16)],
// hi = fp16(x 2^e), lo = fp16(x 2^e - hi) -- bit for bit the split the fp16x2 data gradient makes of the fp32
// row (gemm_x3.hip gemm_r16_body), done once here instead of once per consumer and k tile.  The weight
// gradient then stages G with LDS-DMA and no vector work (wgrad_pl_body).
__device__ __forceinline__ void put_h2(_Float16 *__restrict__ ph, int c, float v, int es, int lo_off) {
    const float x = ldexpf(v, es);
    const _Float16 h = (_Float16)x;
    ph[c] = h;
    ph[lo_off + c] = (_Float16)(x - (float)h);
}

template <int N>
__device__ __forceinline__ void put_h2v(_Float16 *__restrict__ ph, int c, const float *v, int es, int lo_off) {
    typedef _Float16 hv __attribute__((ext_vector_type(N)));
    hv h, l;
#pragma unroll
    for (int u = 0; u < N; ++u) {
        const float x = ldexpf(v[u], es);
        h[u] = (_Float16)x;
        l[u] = (_Float16)(x - (float)h[u]);
    }
    *reinterpret_cast<hv *>(ph + c) = h;
    *reinterpret_cast<hv *>(ph + lo_off + c) = l;
}

// One row of the backward in the vector column layout (columns PER * lane + u); same arithmetic per
// element as the scalar body of gru_ln_bwd_kernel below.  Row means multiply by 1 / H (exact: H is a
// power of two, so x * 2^-k == x / 2^k bit for bit) instead of an IEEE division each: var cell -3..-8 %,
// clause cell -2..-3 % (profiles/r03_ab_gru_bwd_recip.log; profiles/r03_ab_gru_bwd_modes.log, mode 0).  Measured there and not kept: the
// forward's v_exp / v_rcp gate forms (clause cell +5 %: the transcendental unit, not the division
// sequence, is the contended resource) and DPP wave reductions instead of the shuffles (neutral).
template <int PER, int NQ, int NF, int NQT, bool PL>
__device__ __forceinline__ void bwd_row_vec(const float *__restrict__ gi, const float *__restrict__ h,
                                            const float *__restrict__ g, const float *__restrict__ scale,
                                            float *__restrict__ di, float *__restrict__ dhh, float *__restrict__ dhp,
                                            int H, int dh_assign, int packed, const float *__restrict__ feat,
                                            int *__restrict__ rexp_r, int lane, float (&pq)[NQT][PER]) {
    const int j0 = PER * lane;
    float fw[NF > 0 ? NF : 1];
#pragma unroll
    for (int k = 0; k < NF; ++k) {
        fw[k] = feat[k];
        MSAT_DCHECK(isfinite(fw[k]) ? 0 : -1, 1);  // debug: an unwritten (NaN-poisoned) feature row
    }
    float rp[PER], zp[PER], np_[PER], ghn[PER], hv[PER], dyv[PER], sc[PER];
    ldv<PER>(gi + j0, rp);
    ldv<PER>(gi + H + j0, zp);
    ldv<PER>(gi + 2 * H + j0, np_);
    ldv<PER>(gi + 3 * H + j0, ghn);
    ldv<PER>(h + j0, hv);
    ldv<PER>(g + j0, dyv);
    ldv<PER>(scale + j0, sc);
    float old_dh[PER];
    if (!dh_assign) ldv<PER>(dhp + j0, old_dh);
    float rg[PER], zg[PER], ng[PER], hn[PER];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        rg[u] = sigmoidf_(rp[u]);
        zg[u] = sigmoidf_(zp[u]);
        ng[u] = tanhf(np_[u] + rg[u] * ghn[u]);
        hn[u] = (1.0f - zg[u]) * ng[u] + zg[u] * hv[u];
        s1 += hn[u];
        s2 += hn[u] * hn[u];
    }
    s1 = wave_sum_f32(s1);
    s2 = wave_sum_f32(s2);
    const float mean = s1 * (1.0f / (float)H);
    const float var = fmaxf(s2 * (1.0f / (float)H) - mean * mean, 0.0f);
    const float rs = rsqrtf(var + 1e-6f);
    float xh[PER], dxh[PER];
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        xh[u] = (hn[u] - mean) * rs;
        dxh[u] = dyv[u] * sc[u];
        a1 += dxh[u];
        a2 += dxh[u] * xh[u];
        pq[0][u] += dyv[u] * xh[u];
        pq[1][u] += dyv[u];
    }
    a1 = wave_sum_f32(a1) * (1.0f / (float)H);
    a2 = wave_sum_f32(a2) * (1.0f / (float)H);
    float rmax = 0.f;
    float o_an[PER], o_ar[PER], o_az[PER], o_anr[PER], o_dh[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const float dhn = rs * (dxh[u] - a1 - xh[u] * a2);
        const float dn = dhn * (1.0f - zg[u]);
        const float dz = dhn * (hv[u] - ng[u]);
        const float dan = dn * (1.0f - ng[u] * ng[u]);
        const float dr = dan * ghn[u];
        const float dar = dr * rg[u] * (1.0f - rg[u]);
        const float daz = dz * zg[u] * (1.0f - zg[u]);
        o_an[u] = dan;
        o_ar[u] = dar;
        o_az[u] = daz;
        o_anr[u] = dan * rg[u];
        o_dh[u] = dh_assign ? dhn * zg[u] : old_dh[u] + dhn * zg[u];
        if (rexp_r) rmax = fmaxf(rmax, fmaxf(fmaxf(fabsf(dan), fabsf(dar)), fmaxf(fabsf(daz), fabsf(o_anr[u]))));
        if constexpr (NQ == 6) {
            pq[2][u] += dar;
            pq[3][u] += daz;
            pq[4][u] += dan;
            pq[5][u] += o_anr[u];
        }
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            pq[NQ + 3 * k][u] += fw[k] * dar;
            pq[NQ + 3 * k + 1][u] += fw[k] * daz;
            pq[NQ + 3 * k + 2][u] += fw[k] * dan;
        }
    }
    if constexpr (PL) {
        // stored below, once the row exponent is known
    } else if (packed) {  // [dan | dar | daz | dan r]
        stv<PER>(di + j0, o_an);
        stv<PER>(di + H + j0, o_ar);
        stv<PER>(di + 2 * H + j0, o_az);
        stv<PER>(di + 3 * H + j0, o_anr);
    } else {
        stv<PER>(di + j0, o_ar);
        stv<PER>(di + H + j0, o_az);
        stv<PER>(di + 2 * H + j0, o_an);
        stv<PER>(dhh + j0, o_ar);
        stv<PER>(dhh + H + j0, o_az);
        stv<PER>(dhh + 2 * H + j0, o_anr);
    }
    stv<PER>(dhp + j0, o_dh);
    if (rexp_r) {
        rmax = wave_max_f32(rmax);
        const int e = f16x2_row_exp(rmax);
        if (lane == 0) *rexp_r = e;
        if constexpr (PL) {
            const int es = e == kExpZero ? 0 : e;
            _Float16 *ph = reinterpret_cast<_Float16 *>(di);
            put_h2v<PER>(ph, j0, o_an, es, 4 * H);
            put_h2v<PER>(ph, H + j0, o_ar, es, 4 * H);
            put_h2v<PER>(ph, 2 * H + j0, o_az, es, 4 * H);
            put_h2v<PER>(ph, 3 * H + j0, o_anr, es, 4 * H);
        }
    }
}

template <int PER, bool G4, int NQ = 2, int NF = 0, bool VEC = false, bool PL = false>
__global__ void __launch_bounds__(kRowThreads, 1)
gru_ln_bwd_kernel(const float *__restrict__ dy, int ldy, const float *__restrict__ Gi, int ldi,
                  const float *__restrict__ Gh, int ldh, const float *__restrict__ hp, int ldp,
                  const float *__restrict__ scale, float *__restrict__ dGi, int lddi, float *__restrict__ dGh, int lddh,
                  float *__restrict__ dh, int lddh_prev, float *__restrict__ part, int R, int H, int dh_assign,
                  int packed, const float *__restrict__ feat, int ldf, int *__restrict__ rexp, long long part_cap) {
    constexpr int NQT = NQ + 3 * NF, QC = NQ;  // partial rows; LDS reduction in chunks of QC rows
    __shared__ float s_part[4][QC * 64 * PER];
    // w through readfirstlane: the row index r is then wave-uniform to the compiler, so every per-row base
    // address (tape, h, dy, outputs, the features) is scalar arithmetic and the features scalar loads
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float pq[NQT][PER];
#pragma unroll
    for (int q = 0; q < NQT; ++q)
#pragma unroll
        for (int u = 0; u < PER; ++u) pq[q][u] = 0.f;
    for (int r = blockIdx.x * 4 + w; r < R; r += gridDim.x * 4) {
        const float *gi = Gi + (size_t)r * ldi, *gh = G4 ? gi : Gh + (size_t)r * ldh, *h = hp + (size_t)r * ldp;
        const float *g = dy + (size_t)r * ldy;
        if constexpr (VEC) {
            static_assert(G4, "vector form reads the packed tape");
            bwd_row_vec<PER, NQ, NF, NQT, PL>(gi, h, g, scale, dGi + (size_t)r * lddi, dGh + (size_t)r * lddh,
                                          dh + (size_t)r * lddh_prev, H, dh_assign, packed, feat + (size_t)r * ldf,
                                          rexp ? rexp + r : nullptr, lane, pq);
            continue;
        }
        float fw[NF > 0 ? NF : 1];
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            fw[k] = feat[(size_t)r * ldf + k];
            // debug: an unwritten feature row (the debug path poisons cdeg / vfeat with NaN before assembly)
            // reports index -1 - r
            MSAT_DCHECK(isfinite(fw[k]) ? r : -1 - r, R);
        }
        float rg[PER], zg[PER], ng[PER], hn[PER], hv[PER], ghn[PER], dyv[PER];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = lane + 64 * u;
            if (G4) {
                rg[u] = sigmoidf_(gi[j]);
                zg[u] = sigmoidf_(gi[H + j]);
                ghn[u] = gi[3 * H + j];
            } else {
                rg[u] = sigmoidf_(gi[j] + gh[j]);
                zg[u] = sigmoidf_(gi[H + j] + gh[H + j]);
                ghn[u] = gh[2 * H + j];
            }
            ng[u] = tanhf(gi[2 * H + j] + rg[u] * ghn[u]);
            hv[u] = h[j];
            hn[u] = (1.0f - zg[u]) * ng[u] + zg[u] * hv[u];
            dyv[u] = g[j];
            s1 += hn[u];
            s2 += hn[u] * hn[u];
        }
        s1 = wave_sum_f32(s1);
        s2 = wave_sum_f32(s2);
        const float mean = s1 * (1.0f / (float)H);
        const float var = fmaxf(s2 * (1.0f / (float)H) - mean * mean, 0.0f);
        const float rs = rsqrtf(var + 1e-6f);
        float xh[PER], dxh[PER];
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = lane + 64 * u;
            xh[u] = (hn[u] - mean) * rs;
            dxh[u] = dyv[u] * scale[j];
            a1 += dxh[u];
            a2 += dxh[u] * xh[u];
            pq[0][u] += dyv[u] * xh[u];
            pq[1][u] += dyv[u];
        }
        a1 = wave_sum_f32(a1) * (1.0f / (float)H);
        a2 = wave_sum_f32(a2) * (1.0f / (float)H);
        float rmax = 0.f;  // largest |dG| of the row (rexp)
        float o_an[PL ? PER : 1], o_ar[PL ? PER : 1], o_az[PL ? PER : 1], o_anr[PL ? PER : 1];  // PL: held
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = lane + 64 * u;
            const float dhn = rs * (dxh[u] - a1 - xh[u] * a2);
            const float dn = dhn * (1.0f - zg[u]);
            const float dz = dhn * (hv[u] - ng[u]);
            const float dan = dn * (1.0f - ng[u] * ng[u]);
            const float dr = dan * ghn[u];
            const float dar = dr * rg[u] * (1.0f - rg[u]);
            const float daz = dz * zg[u] * (1.0f - zg[u]);
            float *di = dGi + (size_t)r * lddi, *dhh = dGh + (size_t)r * lddh;
            if constexpr (PL) {
                o_an[u] = dan;
                o_ar[u] = dar;
                o_az[u] = daz;
                o_anr[u] = dan * rg[u];
            } else if (packed) {  // one row [dan | dar | daz | dan r]: dGi = cols 0..3H (gate order n, r, z), dGh = cols H..4H
                di[j] = dan;
                di[H + j] = dar;
                di[2 * H + j] = daz;
                di[3 * H + j] = dan * rg[u];
            } else {
                di[j] = dar;
                di[H + j] = daz;
                di[2 * H + j] = dan;
                dhh[j] = dar;
                dhh[H + j] = daz;
                dhh[2 * H + j] = dan * rg[u];
            }
            if (rexp) rmax = fmaxf(rmax, fmaxf(fmaxf(fabsf(dan), fabsf(dar)), fmaxf(fabsf(daz), fabsf(dan * rg[u]))));
            float *dhp = dh + (size_t)r * lddh_prev + j;
            *dhp = dh_assign ? dhn * zg[u] : *dhp + dhn * zg[u];
            if constexpr (NQ == 6) {
                pq[2][u] += dar;
                pq[3][u] += daz;
                pq[4][u] += dan;
                pq[5][u] += dan * rg[u];
            }
#pragma unroll
            for (int k = 0; k < NF; ++k) {
                pq[NQ + 3 * k][u] += fw[k] * dar;
                pq[NQ + 3 * k + 1][u] += fw[k] * daz;
                pq[NQ + 3 * k + 2][u] += fw[k] * dan;
            }
        }
        if (rexp) {
            rmax = wave_max_f32(rmax);
            const int e = f16x2_row_exp(rmax);
            if (lane == 0) rexp[r] = e;
            if constexpr (PL) {
                const int es = e == kExpZero ? 0 : e;
                _Float16 *ph = reinterpret_cast<_Float16 *>(dGi + (size_t)r * lddi);
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const int j = lane + 64 * u;
                    put_h2(ph, j, o_an[u], es, 4 * H);
                    put_h2(ph, H + j, o_ar[u], es, 4 * H);
                    put_h2(ph, 2 * H + j, o_az[u], es, 4 * H);
                    put_h2(ph, 3 * H + j, o_anr[u], es, 4 * H);
                }
            }
        }
    }
#pragma unroll
    for (int q0 = 0; q0 < NQT; q0 += QC) {
        if (q0) __syncthreads();
#pragma unroll
        for (int q = 0; q < QC; ++q)
#pragma unroll
            for (int u = 0; u < PER; ++u) s_part[w][q * 64 * PER + (VEC ? PER * lane + u : lane + 64 * u)] = pq[q0 + q][u];
        __syncthreads();
        for (int j = threadIdx.x; j < QC * 64 * PER; j += kRowThreads) {
            const float v = (s_part[0][j] + s_part[1][j]) + (s_part[2][j] + s_part[3][j]);
            const int q = j / (64 * PER), jj = j - q * 64 * PER;
            if (jj < H) {
                const size_t o = (size_t)blockIdx.x * NQT * H + (q0 + q) * H + jj;
                // debug: inside the block partials (below the reduction workspace) and the caller's allocation
                MSAT_DCHECK(o, (long long)gridDim.x * NQT * H);
                MSAT_DCHECK(o, part_cap);
                part[o] = v;
            }
        }
    }
}

// dst[j] (+)= sum_b part[b][j]: block per 64 columns, 4 waves stride the partial rows, fixed-order
// combine (bitwise reproducible).
__global__ void __launch_bounds__(256)
partial_reduce_kernel(const float *__restrict__ part, int nblocks, int width, float *__restrict__ dst, int accumulate,
                      int ld) {
    __shared__ float red[4][64];
    const int j = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
    float s = 0.f;
    if (j < width)
        for (int b = w; b < nblocks; b += 4) s += part[(size_t)b * ld + j];
    red[w][threadIdx.x & 63] = s;
    __syncthreads();
    if (w == 0 && j < width) {
        const float t = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
        dst[j] = accumulate ? dst[j] + t : t;
    }
}

// Up to four partial_reduce4 launches in one (the GRU backward's LN / gate-bias / feature gradients): block b
// serves segment i while b < ends[i]; per column the same adds in the same order as partial_reduce4_kernel.
struct PartialSeg4 {
    const float4 *src[4];
    float4 *dst[4];
    int N4[4], accumulate[4], ends[4];
    int nseg, nrows, ld4;
    long long esrc[4], edst[4];  // debug builds: float4s to the end of each buffer's allocation
};
__global__ void __launch_bounds__(256)
partial_reduce4_multi_kernel(PartialSeg4 p) {
    __shared__ float4 red[16][16];
    int i = 0, b0 = 0;
    while (i + 1 < p.nseg && (int)blockIdx.x >= p.ends[i]) b0 = p.ends[i++];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int c = ((int)blockIdx.x - b0) * 16 + tx;
    const int N4 = p.N4[i];
    const float4 *part = p.src[i];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < N4)
        for (int r = ty; r < p.nrows; r += 16) {
            MSAT_DCHECK((long long)r * p.ld4 + c, p.esrc[i]);
            const float4 v = part[(size_t)r * p.ld4 + c];
            a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
    red[ty][tx] = a;
    __syncthreads();
    if (ty == 0 && c < N4) {
        float4 t = red[0][tx];
        for (int k = 1; k < 16; ++k) {
            const float4 v = red[k][tx];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        float4 *dst = p.dst[i];
        MSAT_DCHECK(c, p.edst[i]);
        if (p.accumulate[i]) {
            const float4 o = dst[c];
            t.x = o.x + t.x; t.y = o.y + t.y; t.z = o.z + t.z; t.w = o.w + t.w;
        }
        dst[c] = t;
    }
}

// Column sums of G (M x N): block (column chunk of 256, row split) partials, then partial_reduce.
__global__ void __launch_bounds__(256)
colsum_partial_kernel(const float *__restrict__ G, int ldg, int M, int N, int rows_per, float *__restrict__ part) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= N) return;
    const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
    float s = 0.f;
    for (int r = r0; r < r1; ++r) s += G[(size_t)r * ldg + j];
    part[(size_t)blockIdx.y * N + j] = s;
}

// float4 forms of the two reduction stages (16 column-float4 lanes x 16 row lanes per block,
// rows strided over the row lanes, combined through LDS in a fixed order -> deterministic).
// part[split][:] = column sums of G rows [split*rows_per, +rows_per).
__global__ void __launch_bounds__(256)
colsum4_kernel(const float4 *__restrict__ G, int ldg4, int M, int N4, int rows_per, float4 *__restrict__ part,
               long long eg, long long ep) {  // eg / ep: debug builds' extents of G and part, in float4s
    __shared__ float4 red[16][16];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + tx;
    const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < N4)
        for (int r = r0 + ty; r < r1; r += 16) {
            MSAT_DCHECK((long long)r * ldg4 + c, eg);
            const float4 v = G[(size_t)r * ldg4 + c];
            a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
    red[ty][tx] = a;
    __syncthreads();
    if (ty == 0 && c < N4) {
        float4 t = red[0][tx];
        for (int k = 1; k < 16; ++k) {
            const float4 v = red[k][tx];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        MSAT_DCHECK((long long)blockIdx.y * N4 + c, ep);
        part[(size_t)blockIdx.y * N4 + c] = t;
    }
}

// dst[c] (+)= sum over the nrows rows of part (row stride ld4 float4s).
__global__ void __launch_bounds__(256)
partial_reduce4_kernel(const float4 *__restrict__ part, int nrows, int N4, int ld4, float4 *__restrict__ dst,
                       int accumulate, long long ep, long long ed) {  // ep / ed: debug extents, float4s
    __shared__ float4 red[16][16];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + tx;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < N4)
        for (int r = ty; r < nrows; r += 16) {
            MSAT_DCHECK((long long)r * ld4 + c, ep);
            const float4 v = part[(size_t)r * ld4 + c];
            a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
    red[ty][tx] = a;
    __syncthreads();
    if (ty == 0 && c < N4) {
        float4 t = red[0][tx];
        for (int k = 1; k < 16; ++k) {
            const float4 v = red[k][tx];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        MSAT_DCHECK(c, ed);
        if (accumulate) {
            const float4 o = dst[c];
            t.x = o.x + t.x; t.y = o.y + t.y; t.z = o.z + t.z; t.w = o.w + t.w;
        }
        dst[c] = t;
    }
}

// ------------------------------------------------------------ elementwise --
__global__ void relu_fwd_kernel(float *__restrict__ x, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = fmaxf(x[i], 0.0f);
}

// dx = dy * (y > 0), in place on dy
__global__ void relu_bwd_kernel(float *__restrict__ dy, const float *__restrict__ y, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && !(y[i] > 0.0f)) dy[i] = 0.0f;
}

// ---------------------------------------------------------- batch assembly --
// Block per sample: instantiate the instance's graph templates at the sample's row
// bases and compute its node features from the sample's assignment.
// Debug builds: element extents of every buffer the kernel indexes (dbg_extent), checked at each access.
struct AsmDbg {
    long long x, svf, pool, t_vgid, t_cgid, t_slots, t_ptr, t_inc, vfeat, cfeat, cdeg, slots, ptr, inc, g_vbase, g_nv,
        g_cbase, g_nc;
};
__global__ void __launch_bounds__(256)
assemble_graph_batch_kernel(int S, int G, int A, int V, int C, const int *__restrict__ inst,
                            const uint8_t *__restrict__ x, const float *__restrict__ svf,
                            const uint64_t *__restrict__ pool, const int *__restrict__ sb,
                            const int *__restrict__ t_vgid, const int *__restrict__ t_cgid,
                            const int *__restrict__ t_slots, const int *__restrict__ t_ptr,
                            const int *__restrict__ t_inc, const int *__restrict__ voff, const int *__restrict__ coff,
                            const int *__restrict__ eoff, const int *__restrict__ poff, const int *__restrict__ gv,
                            const int *__restrict__ gc, float *__restrict__ vfeat, float *__restrict__ cfeat,
                            float *__restrict__ cdeg, int *__restrict__ slots, int *__restrict__ ptr, int *__restrict__ inc,
                            int *__restrict__ g_vbase, int *__restrict__ g_nv, int *__restrict__ g_cbase,
                            int *__restrict__ g_nc, int Nv, int nnz, AsmDbg dbg) {
    const int s = blockIdx.x;
    const int n = inst[s];
    const int vr0 = sb[3 * s], cr0 = sb[3 * s + 1], e0 = sb[3 * s + 2];
    const int tv0 = voff[n], tc0 = coff[n], te0 = eoff[n], tp0 = poff[n];
    const int *gvn = gv + (size_t)n * (A + 2), *gcn = gc + (size_t)n * (A + 2);
    const int nvr = gvn[G], ncr = gcn[G];
    const int ne = t_ptr[tp0 + nvr];
    const uint8_t *xs = x + (size_t)s * V;
    if (threadIdx.x == 0) {
        MSAT_DCHECK((long long)(s + 1) * V - 1, dbg.x);
        MSAT_DCHECK((long long)tp0 + nvr, dbg.t_ptr);
    }
    for (int t = threadIdx.x; t < nvr; t += blockDim.x) {
        MSAT_DCHECK((long long)tv0 + t, dbg.t_vgid);
        const int gid = t_vgid[tv0 + t];
        MSAT_DCHECK(gid, V);
        MSAT_DCHECK((long long)(vr0 + t) * 8 + 7, dbg.vfeat);
        MSAT_DCHECK(((long long)n * V + gid) * 3 + 2, dbg.svf);
        float *f = vfeat + (size_t)(vr0 + t) * 8;
        const float *sv = svf + ((size_t)n * V + gid) * 3;
        const int pb = t_ptr[tp0 + t], pe = t_ptr[tp0 + t + 1];
        if (pe > pb) MSAT_DCHECK((long long)te0 + pe - 1, dbg.t_inc);
        MSAT_DCHECK((long long)vr0 + t, dbg.ptr);
        int nneg = 0;
        for (int e = pb; e < pe; ++e) nneg += t_inc[te0 + e] & 1;
        f[0] = (float)(xs[gid] & 1u);
        f[1] = sv[0];
        f[2] = sv[1];
        f[3] = sv[2];
        f[4] = (float)(pe - pb - nneg);  // incidences of the var row in its graph: positive, negative
        f[5] = (float)nneg;
        f[6] = 0.0f;
        f[7] = 0.0f;
        ptr[vr0 + t] = e0 + pb;
    }
    for (int e = threadIdx.x; e < ne; e += blockDim.x) {
        MSAT_DCHECK((long long)te0 + e, dbg.t_inc);
        MSAT_DCHECK((long long)e0 + e, dbg.inc);
        const int ent = t_inc[te0 + e];
        inc[e0 + e] = ((cr0 + (ent >> 1)) << 1) | (ent & 1);
    }
    for (int t = threadIdx.x; t < ncr; t += blockDim.x) {
        MSAT_DCHECK((long long)tc0 + t, dbg.t_cgid);
        MSAT_DCHECK((long long)(tc0 + t) * 3 + 2, dbg.t_slots);
        MSAT_DCHECK((long long)(cr0 + t) * 3 + 2, dbg.slots);
        MSAT_DCHECK((long long)(cr0 + t) * 3 + 2, dbg.cfeat);
        if (cdeg) MSAT_DCHECK((long long)(cr0 + t) * 4 + 3, dbg.cdeg);
        const int gcid = t_cgid[tc0 + t];
        MSAT_DCHECK(gcid, C);
        MSAT_DCHECK((long long)n * C + gcid, dbg.pool);
        int npos = 0, nneg = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int sl = t_slots[(size_t)(tc0 + t) * 3 + j];
            slots[(size_t)(cr0 + t) * 3 + j] = sl < 0 ? -1 : (((vr0 + (sl >> 1)) << 1) | (sl & 1));
            npos += sl >= 0 && !(sl & 1);
            nneg += sl >= 0 && (sl & 1);
        }
        if (cdeg) {
            float *d = cdeg + (size_t)(cr0 + t) * 4;
            d[0] = (float)npos;
            d[1] = (float)nneg;
            d[2] = 0.0f;
            d[3] = 0.0f;
        }
        const uint64_t w = pool[(size_t)n * C + gcid];
        int ntrue = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint32_t lit = (uint32_t)(w >> (16 * j)) & 0xFFFFu;
            if (lit < MSAT_LIT_ABSENT) ntrue += (int)(((xs[lit >> 1] & 1u) ^ lit) & 1u);
        }
        float *f = cfeat + (size_t)(cr0 + t) * 3;
        f[0] = ntrue > 0 ? 1.0f : 0.0f;
        f[1] = (float)ntrue / 3.0f;
        f[2] = 1.0f;
    }
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        MSAT_DCHECK((long long)s * G + g, dbg.g_vbase);
        MSAT_DCHECK((long long)s * G + g, dbg.g_nv);
        MSAT_DCHECK((long long)s * G + g, dbg.g_cbase);
        MSAT_DCHECK((long long)s * G + g, dbg.g_nc);
        g_vbase[s * G + g] = vr0 + gvn[g];
        g_nv[s * G + g] = gvn[g + 1] - gvn[g];
        g_cbase[s * G + g] = cr0 + gcn[g];
        g_nc[s * G + g] = gcn[g + 1] - gcn[g];
    }
    if (s == 0 && threadIdx.x == 0) {
        MSAT_DCHECK(Nv, dbg.ptr);
        ptr[Nv] = nnz;
    }
}

}  // namespace msat

using namespace msat;

static int grid_rows(long rows) { return (int)std::min<long>((rows + 3) / 4, 8192); }
// GRU/LN backward: at most 1024 blocks (16 waves per CU), so its per-block LN partials stay small
constexpr long kBwdMaxBlocks = 1024;  // GRU backward grid cap (partial-sum rows = blocks)
static int bwd_blocks(long rows) { return (int)std::min<long>((rows + 3) / 4, kBwdMaxBlocks); }
constexpr int kPartRows = 16;  // rows per first-stage block when reducing LN partials


static bool a16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// float4 column-sum plan: ~1024 blocks, >= 64 rows per split
static int colsum4_splits(int M, int N) {
    const int cb = std::max(1, (N / 4 + 15) / 16);
    return std::max(1, std::min((M + 63) / 64, std::max(1, 1024 / cb)));
}
static int colsum_splits(int M, int N) {
    const int colblocks = (N + 255) / 256;
    return std::max(1, std::min((M + 255) / 256, 1024 / colblocks));
}

extern "C" size_t msat_colsum_workspace_floats(int32_t M, int32_t N) {
    return (size_t)std::max(colsum_splits(M, N), colsum4_splits(M, N)) * N;
}

// out (+)= column sums of G (M x N) in two fixed-order stages; float4 form when every row and
// the output are 16-byte addressable.  ws >= msat_colsum_workspace_floats(M, N).
static int colsum_det(const float *G, int ldg, int M, int N, float *out, int accumulate, float *ws, hipStream_t s) {
    if (N % 4 == 0 && ldg % 4 == 0 && a16(G) && a16(out) && a16(ws)) {
        const int sp = colsum4_splits(M, N), rows_per = (M + sp - 1) / sp, N4 = N / 4;
        hipLaunchKernelGGL(colsum4_kernel, dim3((N4 + 15) / 16, sp), dim3(256), 0, s,
                           reinterpret_cast<const float4 *>(G), ldg / 4, M, N4, rows_per, reinterpret_cast<float4 *>(ws),
                           dbg_extent(G, 16), dbg_extent(ws, 16));
        int rc = check_launch("colsum4_kernel");
        if (rc) return rc;
        hipLaunchKernelGGL(partial_reduce4_kernel, dim3((N4 + 15) / 16), dim3(256), 0, s,
                           reinterpret_cast<const float4 *>(ws), sp, N4, N4, reinterpret_cast<float4 *>(out), accumulate,
                           dbg_extent(ws, 16), dbg_extent(out, 16));
        return check_launch("partial_reduce4_kernel");
    }
    const int sp = colsum_splits(M, N);
    const int rows_per = (M + sp - 1) / sp;
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((N + 255) / 256, sp), dim3(256), 0, s, G, ldg, M, N, rows_per, ws);
    int rc = check_launch("colsum_partial_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(partial_reduce_kernel, dim3((N + 63) / 64), dim3(256), 0, s, ws, sp, N, out, accumulate, N);
    return check_launch("partial_reduce_kernel");
}

static int reduce_partials(const float *part, int nrows, int width, float *dst, int accumulate, float *ws,
                           hipStream_t s) {
    return colsum_det(part, width, nrows, width, dst, accumulate, ws, s);
}

extern "C" int msat_colsum(const float *G, int32_t ldg, int32_t M, int32_t N, float *out, int32_t accumulate,
                           float *workspace, void *stream) {
    MSAT_REQUIRE((G || M == 0) && out && workspace && N >= 1 && M >= 0 && ldg >= N, "bad colsum args");
    return colsum_det(G, ldg, M, N, out, accumulate, workspace, (hipStream_t)stream);
}

extern "C" int msat_clause_gather2(const float *src_pos, const float *src_neg, int32_t ld_src, const int32_t *slots,
                                   float *dst, int32_t ld_dst, int32_t num_clause_rows, int32_t H, int32_t merged,
                                   int32_t accumulate, void *stream) {
    if (num_clause_rows == 0) return MSAT_OK;
    MSAT_REQUIRE(src_pos && src_neg && slots && dst && H % 32 == 0 && ld_src % 4 == 0 && ld_dst % 4 == 0 &&
                     a16(src_pos) && a16(src_neg) && a16(dst) && ld_src >= H && ld_dst >= (merged ? H : 2 * H),
                 "bad clause_gather args");
    hipLaunchKernelGGL(clause_gather_kernel, dim3(grid_rows(num_clause_rows)), dim3(kRowThreads), 0,
                       (hipStream_t)stream, src_pos, src_neg, ld_src, slots, dst, ld_dst, num_clause_rows, H,
                       merged ? 1 : 0, accumulate, gather_dbg(src_pos, src_neg, dst, dst, slots, nullptr));
    return check_launch("clause_gather_kernel");
}

extern "C" int msat_clause_gather(const float *src, int32_t ld_src, const int32_t *slots, float *dst, int32_t ld_dst,
                                  int32_t num_clause_rows, int32_t H, int32_t accumulate, void *stream) {
    MSAT_REQUIRE(src || num_clause_rows == 0, "bad clause_gather args");
    return msat_clause_gather2(src, src ? src + H : nullptr, ld_src, slots, dst, ld_dst, num_clause_rows, H, 0,
                               accumulate, stream);
}

extern "C" int msat_var_gather2(const float *src_pos, const float *src_neg, int32_t ld_src, const int32_t *ptr,
                                const int32_t *inc, float *dst_pos, float *dst_neg, int32_t ld_dst,
                                int32_t num_var_rows, int32_t H, int32_t accumulate, void *stream) {
    if (num_var_rows == 0) return MSAT_OK;
    MSAT_REQUIRE(src_pos && src_neg && ptr && inc && dst_pos && dst_neg && H % 32 == 0 && ld_src % 4 == 0 &&
                     ld_dst % 4 == 0 && a16(src_pos) && a16(src_neg) && a16(dst_pos) && a16(dst_neg) &&
                     ld_src >= H && ld_dst >= H,
                 "bad var_gather args");
    // two rows per wave where a half-wave spans a row (profiles/r03_ab_var_gather_halfwave.log: forward
    // 401 -> 359 us on the uf100 training batch shape, the backward's accumulating form unchanged)
    if (H % 128 == 0) {
        hipLaunchKernelGGL(var_gather_hw_kernel, dim3(grid_rows(num_var_rows)), dim3(kRowThreads), 0,
                           (hipStream_t)stream, src_pos, src_neg, ld_src, ptr, inc, dst_pos, dst_neg, ld_dst,
                           num_var_rows, H, accumulate, gather_dbg(src_pos, src_neg, dst_pos, dst_neg, inc, ptr));
        return check_launch("var_gather_hw_kernel");
    }
    hipLaunchKernelGGL(var_gather_kernel, dim3(grid_rows(num_var_rows)), dim3(kRowThreads), 0, (hipStream_t)stream,
                       src_pos, src_neg, ld_src, ptr, inc, dst_pos, dst_neg, ld_dst, num_var_rows, H, accumulate,
                       gather_dbg(src_pos, src_neg, dst_pos, dst_neg, inc, ptr));
    return check_launch("var_gather_kernel");
}

extern "C" int msat_var_gather(const float *src, int32_t ld_src, const int32_t *ptr, const int32_t *inc, float *dst,
                               int32_t ld_dst, int32_t num_var_rows, int32_t H, int32_t accumulate, void *stream) {
    MSAT_REQUIRE((src && dst) || num_var_rows == 0, "bad var_gather args");
    return msat_var_gather2(src, src ? src + H : nullptr, ld_src, ptr, inc, dst, dst ? dst + H : nullptr, ld_dst,
                            num_var_rows, H, accumulate, stream);
}

extern "C" int msat_gru_ln_fwd(const float *Gi, int32_t ldi, const float *Gh, int32_t ldh, const float *hprev,
                               int32_t ldp, const float *ln_scale, const float *ln_bias, float *out, int32_t ldo,
                               int32_t R, int32_t H, void *stream) {
    MSAT_REQUIRE(Gi && Gh && hprev && ln_scale && ln_bias && out, "NULL pointer");
    MSAT_REQUIRE(H == 64 || H == 128 || H == 256, "gru_ln: H must be 64, 128 or 256 (got %d)", H);
    if (R == 0) return MSAT_OK;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g(grid_rows(R)), b(kRowThreads);
    if (H == 64) hipLaunchKernelGGL(gru_ln_fwd_kernel<1>, g, b, 0, s, Gi, ldi, Gh, ldh, hprev, ldp, ln_scale, ln_bias, out, ldo, R, H);
    else if (H == 128) hipLaunchKernelGGL(gru_ln_fwd_kernel<2>, g, b, 0, s, Gi, ldi, Gh, ldh, hprev, ldp, ln_scale, ln_bias, out, ldo, R, H);
    else hipLaunchKernelGGL(gru_ln_fwd_kernel<4>, g, b, 0, s, Gi, ldi, Gh, ldh, hprev, ldp, ln_scale, ln_bias, out, ldo, R, H);
    return check_launch("gru_ln_fwd_kernel");
}

extern "C" size_t msat_gru_ln_bwd_partial_floats(int32_t R, int32_t H) {
    const size_t nb = bwd_blocks(R), q = 6 + 3 * 6;  // LN + gate biases + up to six feature rows
    return nb * q * H + (nb + kPartRows - 1) / kPartRows * q * H;  // block partials + reduction workspace
}

extern "C" int msat_gru_ln_bwd(const float *dy, int32_t ldy, const float *Gi, int32_t ldi, const float *Gh, int32_t ldh,
                               const float *hprev, int32_t ldp, const float *ln_scale, float *dGi, int32_t lddi,
                               float *dGh, int32_t lddh, float *dhprev, int32_t lddp, float *dln_scale,
                               float *dln_bias, float *partial, int32_t R, int32_t H, int32_t accumulate_ln,
                               void *stream) {
    MSAT_REQUIRE(dy && Gi && Gh && hprev && ln_scale && dGi && dGh && dhprev && dln_scale && dln_bias && partial,
                 "NULL pointer");
    MSAT_REQUIRE(H == 64 || H == 128 || H == 256, "gru_ln: H must be 64, 128 or 256 (got %d)", H);
    MSAT_REQUIRE(dln_bias == dln_scale + H, "dln_bias must follow dln_scale (contiguous [scale|bias] grads)");
    if (R == 0) return MSAT_OK;
    hipStream_t s = (hipStream_t)stream;
    const int nb = bwd_blocks(R);
    const dim3 g(nb), b(kRowThreads);
    const long long cap = (long long)msat_gru_ln_bwd_partial_floats(R, H);
    if (H == 64) hipLaunchKernelGGL((gru_ln_bwd_kernel<1, false>), g, b, 0, s, dy, ldy, Gi, ldi, Gh, ldh, hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, partial, R, H, 0, 0, nullptr, 0, nullptr, cap);
    else if (H == 128) hipLaunchKernelGGL((gru_ln_bwd_kernel<2, false>), g, b, 0, s, dy, ldy, Gi, ldi, Gh, ldh, hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, partial, R, H, 0, 0, nullptr, 0, nullptr, cap);
    else hipLaunchKernelGGL((gru_ln_bwd_kernel<4, false>), g, b, 0, s, dy, ldy, Gi, ldi, Gh, ldh, hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, partial, R, H, 0, 0, nullptr, 0, nullptr, cap);
    int rc = check_launch("gru_ln_bwd_kernel");
    if (rc) return rc;
    return reduce_partials(partial, nb, 2 * H, dln_scale, accumulate_ln, partial + (size_t)nb * 2 * H, s);
}

static int gru_ln_bwd_g4_impl(const float *dy, int32_t ldy, const float *g4, int32_t ldg, const float *hprev,
                              int32_t ldp, const float *ln_scale, float *dGi, int32_t lddi, float *dGh, int32_t lddh,
                              float *dhprev, int32_t lddp, float *dln_scale, float *dln_bias, float *dbi,
                              float *dbh_n, const float *feat, int32_t ldf, int32_t nfeat, float *dfeat,
                              float *partial, int32_t R, int32_t H, int32_t accumulate_ln, int32_t *rexp,
                              void *stream) {
    MSAT_REQUIRE(H == 64 || H == 128 || H == 256, "gru_ln: H must be 64, 128 or 256 (got %d)", H);
    MSAT_REQUIRE(ldg >= 4 * H, "gru_ln_bwd_g4: ldg must be >= 4H");
    MSAT_REQUIRE(dln_bias == dln_scale + H, "dln_bias must follow dln_scale (contiguous [scale|bias] grads)");
    MSAT_REQUIRE((dbi == nullptr) == (dbh_n == nullptr), "gru_ln_bwd_g4: dbi and dbh_n go together");
    MSAT_REQUIRE(nfeat == 0 || ((nfeat == 2 || nfeat == 6) && feat && dfeat && dbi && ldf >= nfeat),
                 "gru_ln_bwd_g4f: nfeat must be 0, 2 or 6 (with feat, dfeat and the bias outputs)");
    if (R == 0) return MSAT_OK;
    MSAT_REQUIRE(dy && g4 && hprev && ln_scale && dGi && dGh && dhprev && dln_scale && partial, "NULL pointer");
    hipStream_t s = (hipStream_t)stream;
    const int nb = bwd_blocks(R);
    const dim3 g(nb), b(kRowThreads);
    const bool bias = dbi != nullptr;
    const long long cap = (long long)msat_gru_ln_bwd_partial_floats(R, H);
    if (MSAT_DEBUG_BUILD) {  // the partial buffer lies inside one device allocation of at least `cap` floats
        hipDeviceptr_t base = nullptr;
        size_t bytes = 0;
        MSAT_REQUIRE(hipMemGetAddressRange(&base, &bytes, (hipDeviceptr_t)partial) == hipSuccess &&
                         (const char *)partial + cap * sizeof(float) <= (const char *)base + bytes,
                     "MSAT_DEBUG: gru_ln_bwd partial buffer smaller than msat_gru_ln_bwd_partial_floats(%d, %d)", R,
                     H);
    }
    const int dh_assign = (accumulate_ln >> 1) & 1;  // bit 1: dhprev = ..., else dhprev += ...
    const int packed = (accumulate_ln >> 2) & 1;     // bit 2: packed [dan | dar | daz | dan r] rows
    const int planes = (accumulate_ln >> 3) & 1;     // bit 3: ... as fp16x2 planes at the row exponent
    accumulate_ln &= 1;
    MSAT_REQUIRE(!packed || (dGh == dGi + H && lddi == lddh && lddi >= 4 * H),
                 "gru_ln_bwd_g4: packed rows need dGh = dGi + H and a shared ld >= 4H");
    MSAT_REQUIRE(!planes || (packed && rexp && bias && (nfeat == 2 || nfeat == 6)),
                 "gru_ln_bwd_g4: fp16x2 planes (flags bit 3) need the packed rows, rexp, the bias outputs and 2 or 6 "
                 "features");
    const int NQ = (bias ? 6 : 2) + 3 * nfeat;
    // vector column layout for the var cell (nfeat = 6) when every row start is PER-float aligned (H = 64
    // has PER = 1: same layout).  Measured on the uf50 training shapes (profiles/r02y_ab_bwd_vec.log):
    // var cell 503-506 vs 510-517 us; the clause cell (nfeat = 2) ran 1310-1341 vs 1132-1135 us in this
    // layout, so it and the bias-less / feature-less forms keep the scalar layout.
    const int vper = H / 64, va = 4 * vper;
    const bool vec = nfeat == 6 && vper >= 2 && ((uintptr_t)dy | (uintptr_t)g4 | (uintptr_t)hprev |
                                                   (uintptr_t)ln_scale | (uintptr_t)dGi | (uintptr_t)dGh |
                                                   (uintptr_t)dhprev) % va == 0 &&
                     (ldy | ldg | ldp | lddi | lddh | lddp) % vper == 0;
#define MSAT_BWD1(PER, Q, F)                                                                                      \
    if (planes && vec)                                                                                            \
        hipLaunchKernelGGL((gru_ln_bwd_kernel<PER, true, Q, F, PER >= 2 && F == 6, (Q == 6 && F > 0)>), g, b, 0, s,  \
                           dy, ldy, g4, ldg, g4, ldg, hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp,       \
                           partial, R, H, dh_assign, packed, feat, ldf, rexp, cap);                                   \
    else if (planes)                                                                                              \
        hipLaunchKernelGGL((gru_ln_bwd_kernel<PER, true, Q, F, false, (Q == 6 && F > 0)>), g, b, 0, s, dy, ldy, g4,  \
                           ldg, g4, ldg, hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, partial, R, H,     \
                           dh_assign, packed, feat, ldf, rexp, cap);                                                  \
    else if (vec)                                                                                                 \
        hipLaunchKernelGGL((gru_ln_bwd_kernel<PER, true, Q, F, PER >= 2 && F == 6>), g, b, 0, s, dy, ldy, g4, ldg, g4, ldg, \
                           hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, partial, R, H, dh_assign,    \
                           packed, feat, ldf, rexp, cap);                                                              \
    else                                                                                                          \
        hipLaunchKernelGGL((gru_ln_bwd_kernel<PER, true, Q, F>), g, b, 0, s, dy, ldy, g4, ldg, g4, ldg, hprev,   \
                           ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, partial, R, H, dh_assign, packed,   \
                           feat, ldf, rexp, cap)
#define MSAT_BWD(PER)                                                                                             \
    if (!bias) { MSAT_BWD1(PER, 2, 0); }                                                                           \
    else if (nfeat == 0) { MSAT_BWD1(PER, 6, 0); }                                                                 \
    else if (nfeat == 2) { MSAT_BWD1(PER, 6, 2); }                                                                 \
    else { MSAT_BWD1(PER, 6, 6); }
    if (H == 64) { MSAT_BWD(1) }
    else if (H == 128) { MSAT_BWD(2) }
    else { MSAT_BWD(4) }
#undef MSAT_BWD
#undef MSAT_BWD1
    int rc = check_launch("gru_ln_bwd_kernel");
    if (rc) return rc;
    // stage 1: 16-row float4 sums of the block partials; stage 2: fixed-order reduce of each column segment
    float *ws = partial + (size_t)nb * NQ * H;
    const int sp = (nb + kPartRows - 1) / kPartRows, width = NQ * H, W4 = width / 4;
    // the reduction workspace follows the block partials without overlap and ends inside the allocation plan
    MSAT_REQUIRE((long long)nb * NQ * H + (long long)sp * NQ * H <= cap, "gru_ln_bwd: partial plan overflow");
    MSAT_REQUIRE(a16(partial) && a16(dln_scale) && (!bias || (a16(dbi) && a16(dbh_n))) && (!nfeat || a16(dfeat)),
                 "gru_ln_bwd_g4: partial / gradient outputs must be 16-byte aligned");
    hipLaunchKernelGGL(colsum4_kernel, dim3((W4 + 15) / 16, sp), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(partial), W4, nb, W4, kPartRows, reinterpret_cast<float4 *>(ws),
                       dbg_extent(partial, 16), dbg_extent(ws, 16));
    rc = check_launch("colsum4_kernel");
    if (rc) return rc;
    // stage 2: the segments [dln (2H) | dbi (3H) | dbh_n (H) | dfeat (3 nfeat H, the input matrix's feature rows,
    // accumulated)] of the reduced row, in ONE launch (partial_reduce4_multi_kernel)
    const float4 *ws4 = reinterpret_cast<const float4 *>(ws);
    PartialSeg4 ps{};
    ps.nrows = sp;
    ps.ld4 = W4;
    auto add_seg = [&](int off4, int n4, float *dst, int acc) {
        const int i = ps.nseg++;
        ps.src[i] = ws4 + off4;
        ps.dst[i] = reinterpret_cast<float4 *>(dst);
        ps.N4[i] = n4;
        ps.accumulate[i] = acc;
        ps.ends[i] = (i ? ps.ends[i - 1] : 0) + (n4 + 15) / 16;
        ps.esrc[i] = dbg_extent(ps.src[i], 16);
        ps.edst[i] = dbg_extent(dst, 16);
    };
    add_seg(0, 2 * H / 4, dln_scale, accumulate_ln);
    if (bias) {
        add_seg(2 * H / 4, 3 * H / 4, dbi, 1);
        add_seg(5 * H / 4, H / 4, dbh_n, 1);
    }
    if (nfeat) add_seg(6 * H / 4, 3 * nfeat * H / 4, dfeat, 1);
    hipLaunchKernelGGL(partial_reduce4_multi_kernel, dim3(ps.ends[ps.nseg - 1]), dim3(256), 0, s, ps);
    return check_launch("partial_reduce4_multi_kernel");
}

extern "C" int msat_gru_ln_bwd_g4f(const float *dy, int32_t ldy, const float *g4, int32_t ldg, const float *hprev,
                                   int32_t ldp, const float *ln_scale, float *dGi, int32_t lddi, float *dGh,
                                   int32_t lddh, float *dhprev, int32_t lddp, float *dln_scale, float *dln_bias,
                                   float *dbi, float *dbh_n, const float *feat, int32_t ldf, int32_t nfeat,
                                   float *dfeat, float *partial, int32_t R, int32_t H, int32_t accumulate_ln,
                                   void *stream) {
    return gru_ln_bwd_g4_impl(dy, ldy, g4, ldg, hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, dln_scale,
                              dln_bias, dbi, dbh_n, feat, ldf, nfeat, dfeat, partial, R, H, accumulate_ln, nullptr,
                              stream);
}

extern "C" int msat_gru_ln_bwd_g4fe(const float *dy, int32_t ldy, const float *g4, int32_t ldg, const float *hprev,
                                    int32_t ldp, const float *ln_scale, float *dGi, int32_t lddi, float *dGh,
                                    int32_t lddh, float *dhprev, int32_t lddp, float *dln_scale, float *dln_bias,
                                    float *dbi, float *dbh_n, const float *feat, int32_t ldf, int32_t nfeat,
                                    float *dfeat, float *partial, int32_t R, int32_t H, int32_t accumulate_ln,
                                    int32_t *rexp, void *stream) {
    MSAT_REQUIRE(rexp, "gru_ln_bwd_g4fe: NULL rexp");
    MSAT_REQUIRE((accumulate_ln >> 2) & 1, "gru_ln_bwd_g4fe: row exponents need the packed rows (flags bit 2)");
    return gru_ln_bwd_g4_impl(dy, ldy, g4, ldg, hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, dln_scale,
                              dln_bias, dbi, dbh_n, feat, ldf, nfeat, dfeat, partial, R, H, accumulate_ln, rexp, stream);
}

extern "C" int msat_gru_ln_bwd_g4(const float *dy, int32_t ldy, const float *g4, int32_t ldg, const float *hprev,
                                  int32_t ldp, const float *ln_scale, float *dGi, int32_t lddi, float *dGh, int32_t lddh,
                                  float *dhprev, int32_t lddp, float *dln_scale, float *dln_bias, float *dbi,
                                  float *dbh_n, float *partial, int32_t R, int32_t H, int32_t accumulate_ln,
                                  void *stream) {
    return msat_gru_ln_bwd_g4f(dy, ldy, g4, ldg, hprev, ldp, ln_scale, dGi, lddi, dGh, lddh, dhprev, lddp, dln_scale,
                               dln_bias, dbi, dbh_n, nullptr, 0, 0, nullptr, partial, R, H, accumulate_ln, stream);
}

extern "C" int msat_assemble_graph_batch(
    int32_t S, int32_t G, int32_t A, int32_t V, int32_t C, const int32_t *inst, const uint8_t *x, const float *svf,
    const uint16_t *pool, const int32_t *sample_bases, const int32_t *t_vgid, const int32_t *t_cgid,
    const int32_t *t_slots, const int32_t *t_ptr, const int32_t *t_inc, const int32_t *voff, const int32_t *coff,
    const int32_t *eoff, const int32_t *poff, const int32_t *gv, const int32_t *gc, float *vfeat, float *cfeat,
    float *cdeg, int32_t *slots, int32_t *ptr, int32_t *inc, int32_t *g_vbase, int32_t *g_nv, int32_t *g_cbase, int32_t *g_nc,
    int32_t Nv, int32_t nnz, void *stream) {
    MSAT_REQUIRE(inst && x && svf && pool && sample_bases && t_vgid && t_cgid && t_slots && t_ptr && t_inc && voff &&
                     coff && eoff && poff && gv && gc && vfeat && cfeat && slots && ptr && inc && g_vbase && g_nv &&
                     g_cbase && g_nc,
                 "NULL pointer");
    MSAT_REQUIRE(G >= 1 && G <= A + 1, "G must be 1 (critic only) or A+1");
    if (!S) return MSAT_OK;
    const AsmDbg dbg{dbg_extent(x, 1),       dbg_extent(svf, 4),     dbg_extent(pool, 8),    dbg_extent(t_vgid, 4),
                     dbg_extent(t_cgid, 4),  dbg_extent(t_slots, 4), dbg_extent(t_ptr, 4),   dbg_extent(t_inc, 4),
                     dbg_extent(vfeat, 4),   dbg_extent(cfeat, 4),   dbg_extent(cdeg, 4),    dbg_extent(slots, 4),
                     dbg_extent(ptr, 4),     dbg_extent(inc, 4),     dbg_extent(g_vbase, 4), dbg_extent(g_nv, 4),
                     dbg_extent(g_cbase, 4), dbg_extent(g_nc, 4)};
    hipLaunchKernelGGL(assemble_graph_batch_kernel, dim3(S), dim3(256), 0, (hipStream_t)stream, S, G, A, V, C, inst, x,
                       svf, reinterpret_cast<const uint64_t *>(pool), sample_bases, t_vgid, t_cgid, t_slots, t_ptr,
                       t_inc, voff, coff, eoff, poff, gv, gc, vfeat, cfeat, cdeg, slots, ptr, inc, g_vbase, g_nv, g_cbase,
                       g_nc, Nv, nnz, dbg);
    return check_launch("assemble_graph_batch_kernel");
}

extern "C" int msat_relu(float *x, size_t n, void *stream) {
    MSAT_REQUIRE(x, "NULL pointer");
    if (!n) return MSAT_OK;
    hipLaunchKernelGGL(relu_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, n);
    return check_launch("relu_fwd_kernel");
}

extern "C" int msat_relu_bwd(float *dy, const float *y, size_t n, void *stream) {
    MSAT_REQUIRE(dy && y, "NULL pointer");
    if (!n) return MSAT_OK;
    hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dy, y, n);
    return check_launch("relu_bwd_kernel");
}
