// Batched multi-agent SAT environment on gfx950.
//
// One workgroup (64 / 256 / 512 lanes by instance size, env_threads) owns one environment for the whole call:
//   1. assignment -> LDS bit words (one ballot per 64 vars), agents' flips as
//      LDS atomic XORs;
//   2. every clause evaluated once from the L2/MALL-resident packed pool
//      (8 B/clause), clause status -> LDS bit words by wave ballot, the
//      unsatisfied count by popcount of the same ballots;
//   3. done / reward / info, and (auto-reset) an in-place reset of done envs;
//   4. the instance's agent tables (relation + neighbour bits, built once per
//      pool instance) staged into LDS;
//   5. the env's (A, 2V+C) observation block streamed to HBM with 16 B stores,
//      every 4-element chunk assembled from two LDS words by bit extraction.
// The observation write is >90 % of a step's algorithmic bytes (SURVEY.md
// §8(d)); everything before it is sized to keep the obs pass a pure
// LDS-read -> 16 B store stream.
//
// Reference semantics (kongqg/marl-sat, src/envs/multi_agent_sat_env.py):
//   flip decode             :230-250
//   clause evaluation       :130-156   (literal l true iff l>0&&x=1 or l<0&&x=0)
//   done / reward / info    :256-284, :183-198 (sparse) / :201-223 (PBRS)
//   reset + masks           :158-181, :99-128
//   get_obs                 :345-398
//   rollout auto-reset      src/learners/mappo_gnn_sat_learner.py:422-464
#include <stdlib.h>

#include <algorithm>

#include "common.h"

namespace msat {

constexpr int kThreads = 256;

struct EnvParams {
    int B, V, C, K, A, M, D;
    int WV, WC;     // uint32 words per agent row of the nbr / rel tables (even: whole 64-bit ballots)
    int base, rem;  // agent i owns [i*base + min(i,rem), +base+(i<rem))
    int max_steps, action_mode, reward_mode, N;
    float r_clause, r_sat, gamma;
    int ablate;  // diagnostics only (MARLSAT_ABLATE): bits 0-1: 0 full, 1 constant obs, 2 no obs write;
                 // bit 2: disable the XCD-major env order
    // debug builds (MSAT_DCHECK): elements from each caller buffer's pointer to the end of its allocation
    // (dbg_extent); 0 in product builds
    long long dbg_obs, dbg_assign, dbg_sat, dbg_ntrue, dbg_actions;
    // reset queue (msat_env_state.reset_queue): 0 none; 1 this autoreset launch consumes the list the previous
    // one made and makes the next one's (launch B + rq_cap workgroups); 2 the launch clears the entries of the
    // envs it modifies (the other state-modifying calls)
    int rq_mode, rq_cap;
    uint32_t rq_serial;
};

enum : int { kModeReset = 0, kModeStep = 1, kModeStepAutoReset = 2, kModeObs = 3 };

// Reset queue (msat_env_state.reset_queue): pend[2][B] uint32 tokens.  The launch with serial s reads parity s & 1 --
// env b timed out now iff pend[s & 1][b] == rq_token(s), written by the previous launch -- and writes every entry of
// parity (s + 1) & 1 (rq_token(s + 1) for an env whose next step times out, else 0): never the same words within a
// launch.  The reset workgroups of launch s take the pending envs in index order: workgroup j the one of rank j,
// the env of rank r is covered iff r < cap (the others reset in their step workgroup).  Ranks come from a scan of
// the pending words (one round trip), so no counter, list or atomic is involved: a launch in which every env times
// out (a batch reset together, every max_steps launches) costs each env one scan of B words from L2.  Tokens have
// bit 31 set, so a zeroed queue lists nothing.
__host__ __device__ __forceinline__ uint32_t rq_token(uint32_t serial) { return 0x80000000u | (serial & 0x7FFFFFFFu); }
// ~B/512 envs time out per launch; a multiple of 8, so the reset workgroups (launched first) leave the step workgroups
// XCD placement as without them
__host__ __device__ __forceinline__ int rq_capacity(int B) { return (B / 256 + 8 + 7) & ~7; }
__host__ __device__ __forceinline__ size_t rq_words(int B) { return 2 * (size_t)B; }

__device__ __forceinline__ uint32_t *rq_pend(uint32_t *q, int B, int par) { return q + (size_t)par * B; }

// Wave 0 (all 64 lanes, uniform arguments) scans pend[0 .. B): lane l owns the contiguous words [W l, W l + W),
// W = ceil(B / 64) rounded up to 4 (16-byte loads).  Returns, in every lane, the number of entries equal to tok
// with index < lim; with want >= 0 also the index of the entry of rank want (-1 if fewer), in *sel.  Each lane keeps
// its matches as a bit mask (W <= 64, i.e. B <= 4096), so the selection needs no second read; larger batches
// re-read the owning lane's range.
__device__ __forceinline__ int rq_scan(const uint32_t *__restrict__ pend, int B, uint32_t tok, int lim, int want,
                                       int *sel) {
    const int lane = threadIdx.x & 63;
    const int W = ((B + 63) / 64 + 3) & ~3;
    const int lo = lane * W;
    int below = 0, mine = 0;
    uint64_t bits = 0;
    for (int i = 0; i < W; i += 4) {
        const int k = lo + i;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (k < B) v = *reinterpret_cast<const uint4 *>(pend + k);  // B % 4 == 0 (host-checked)
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool m = k + u < B && w[u] == tok;
            mine += m;
            below += m && k + u < lim;
            if (m && i + u < 64) bits |= 1ull << (i + u);
        }
    }
    int total_below = below;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) total_below += __shfl_xor(total_below, d, 64);
    if (want >= 0) {
        int incl = mine;  // inclusive prefix of mine over the lanes (index order), Hillis-Steele by shuffles
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int up = __shfl_up(incl, d, 64);
            if (lane >= d) incl += up;
        }
        const int excl = incl - mine;
        int found = -1;
        if (want >= excl && want < incl) {  // the rank-want entry is in this lane's range
            int r = want - excl;            // its rank among this lane's matches
            if (W <= 64) {
                uint64_t m = bits;
                for (; r > 0; --r) m &= m - 1;
                found = lo + __ffsll((unsigned long long)m) - 1;
            } else {
                for (int i = 0; i < W && found < 0; i += 4) {
                    const int k = lo + i;
                    if (k >= B) break;
                    const uint4 v = *reinterpret_cast<const uint4 *>(pend + k);
                    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                    for (int u = 0; u < 4 && found < 0; ++u)
                        if (k + u < B && w[u] == tok && r-- == 0) found = k + u;
                }
            }
        }
        const uint64_t has = __ballot(found >= 0);
        *sel = has ? __shfl(found, __ffsll((unsigned long long)has) - 1, 64) : -1;
    }
    return total_below;
}

__host__ __device__ __forceinline__ int agent_lo(const EnvParams &p, int i) { return i * p.base + (i < p.rem ? i : p.rem); }
__host__ __device__ __forceinline__ int agent_size(const EnvParams &p, int i) { return p.base + (i < p.rem ? 1 : 0); }

__device__ __forceinline__ int agent_of_var(const EnvParams &p, int v) {
    const int split = p.rem * (p.base + 1);
    if (v < split) return v / (p.base + 1);
    return p.rem + (v - split) / p.base;  // base > 0 whenever v >= split
}

// LDS image of one environment (all uint32 words).
struct EnvLds {
    uint32_t *x;    // [WV]    assignment bits
    uint32_t *sat;  // [WC]    clause-satisfied bits
    uint32_t *rel;  // [A*WC]  agent-clause relation bits of the env's instance
    uint32_t *nbr;  // [A*WV]  agent neighbour bits of the env's instance
    uint32_t *fm;   // [NW]    obs image: element is not -1   (NW = A*D/32 + 2)
    uint32_t *fx;   // [NW]    obs image: element value bit
    int *red;       // [16]    reduction / broadcast scratch
};

__host__ __device__ __forceinline__ int obs_image_words(const EnvParams &p) { return (p.A * p.D) / 32 + 2; }

__host__ __device__ __forceinline__ size_t env_lds_words(const EnvParams &p) {
    return (size_t)p.WV + p.WC + (size_t)p.A * (p.WC + p.WV) + 2 * (size_t)obs_image_words(p) + 16;
}

__device__ __forceinline__ EnvLds carve(uint32_t *smem, const EnvParams &p) {
    EnvLds l;
    l.x = smem;
    l.sat = l.x + p.WV;
    l.rel = l.sat + p.WC;
    l.nbr = l.rel + (size_t)p.A * p.WC;
    l.fm = l.nbr + (size_t)p.A * p.WV;
    l.fx = l.fm + obs_image_words(p);
    l.red = reinterpret_cast<int *>(l.fx + obs_image_words(p));
    return l;
}

__device__ __forceinline__ uint32_t bit(const uint32_t *w, int i) { return (w[i >> 5] >> (i & 31)) & 1u; }

// Assignment bytes -> LDS bit words, one ballot per 64 vars.  x0: this lane's byte of the first pass
// (var threadIdx.x, loaded early by the caller; any value where threadIdx.x >= V).
template <int T>
__device__ __forceinline__ void load_x_bits(const EnvParams &p, const EnvLds &l, const uint8_t *__restrict__ xg,
                                            uint32_t x0) {
    const int lane = threadIdx.x & 63;
    for (int v0 = threadIdx.x & ~63; v0 < p.WV * 32; v0 += T) {
        const int v = v0 + lane;
        const uint32_t xv = v0 == (int)(threadIdx.x & ~63) ? x0 : (v < p.V ? xg[v] : 0u);
        const uint64_t m = __ballot(v < p.V && (xv & 1u));
        if (lane < 2) l.x[(v0 >> 5) + lane] = (uint32_t)(m >> (32 * lane));
    }
}
template <int T>
__device__ __forceinline__ void load_x_bits(const EnvParams &p, const EnvLds &l, const uint8_t *__restrict__ xg) {
    load_x_bits<T>(p, l, xg, (int)threadIdx.x < p.V ? xg[threadIdx.x] : 0u);
}

// Prefetch depth (per lane) of the step path: pool-row words (covers C <= kPfClause*T
// clauses) and agent-table words, all issued right after problem_idx is known so the
// preamble costs ~2 dependent memory round trips instead of ~4.
constexpr int kPfClause = 4;
constexpr int kPfRel = 4;
constexpr int kPfNbr = 2;

// One 64-clause wave slice of the clause scan: c0 wave-uniform, w = this lane's pool word.
template <bool kPbrs>
__device__ __forceinline__ void clause_slice(const EnvParams &p, const EnvLds &l, int c0, uint64_t w,
                                             uint8_t *__restrict__ sat_g, uint8_t *__restrict__ ntrue_g, int &unsat,
                                             int &newly) {
    const int lane = threadIdx.x & 63;
    const int c = c0 + lane;
    uint32_t sat = 0, ntrue = 0, old = 0;
    const bool live = c < p.C;
    if (live) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint32_t lit = (uint32_t)(w >> (16 * j)) & 0xFFFFu;
            if (lit < MSAT_LIT_ABSENT) ntrue += (bit(l.x, (int)(lit >> 1)) ^ lit) & 1u;
        }
        sat = ntrue ? 1u : 0u;
        if (kPbrs) old = sat_g[c];
        if (sat_g) sat_g[c] = (uint8_t)sat;  // NULL: a step whose reset another workgroup does (reset queue)
        if (ntrue_g) ntrue_g[c] = (uint8_t)ntrue;
    }
    const uint64_t ms = __ballot(sat);
    if (lane < 2) l.sat[(c0 >> 5) + lane] = (uint32_t)(ms >> (32 * lane));
    unsat += __popcll(__ballot(live && !sat));
    if (kPbrs) newly += __popcll(__ballot(sat && !old));
}

// Evaluate every clause of pool row `pidx` against l.x: clause bits -> l.sat,
// bytes -> sat_g / ntrue_g, unsat count (and PBRS newly-satisfied) -> red[0] / red[1].
// The first NPF slices use the lane's prefetched pool words pw[].
template <int T, bool kPbrs, int NPF>
__device__ __forceinline__ void eval_clauses(const EnvParams &p, const EnvLds &l, const uint16_t *__restrict__ lits,
                                             int pidx, uint8_t *__restrict__ sat_g, uint8_t *__restrict__ ntrue_g,
                                             const uint64_t (&pw)[kPfClause]) {
    const uint64_t *prow = reinterpret_cast<const uint64_t *>(lits) + (size_t)pidx * p.C;
    const int lane = threadIdx.x & 63;
    int unsat = 0, newly = 0;  // wave-uniform
    const int cend = p.WC * 32;
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
        const int c0 = (threadIdx.x & ~63) + j * T;
        if (c0 < cend) clause_slice<kPbrs>(p, l, c0, pw[j], sat_g, ntrue_g, unsat, newly);
    }
    for (int c0 = (threadIdx.x & ~63) + NPF * T; c0 < cend; c0 += T) {
        const int c = c0 + lane;
        const uint64_t w = c < p.C ? prow[c] : 0ull;  // pool rows are shared by many envs: keep them cached
        clause_slice<kPbrs>(p, l, c0, w, sat_g, ntrue_g, unsat, newly);
    }
    if (lane == 0) {
        atomicAdd(&l.red[0], unsat);
        if (kPbrs) atomicAdd(&l.red[1], newly);
    }
}

// ---------------------------------------------------------------- obs pass --
// The env's (A, D) observation block as two flat bit images over its A*D
// elements: FM (element != -1) and FX (its 0/1 value).  Row i, element k
// (env:345-398): k < V own vars (FM = owned, FX = x), V <= k < V+C clause
// status (FM = rel_i, FX = sat), k >= V+C neighbour vars (FM = nbr_i, FX = x).
// Built once per env from the LDS bit words (OR of shifted source words), then
// every 16 B store is a funnel-shifted extraction at its flat bit offset: no
// row/region logic and no divergence in the store loop, for any (V, C, A).

__device__ __forceinline__ uint32_t low_mask(int n) { return n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u); }

__device__ __forceinline__ void or_bits(uint32_t *img, int dst, uint32_t bits) {
    if (!bits) return;
    const int w = dst >> 5, s = dst & 31;
    atomicOr(&img[w], bits << s);
    if (s) {
        const uint32_t hi = bits >> (32 - s);
        if (hi) atomicOr(&img[w + 1], hi);
    }
}

template <int T>
__device__ __forceinline__ void build_obs_images(const EnvParams &p, const EnvLds &l) {
    const int nwV = (p.V + 31) >> 5, nwC = (p.C + 31) >> 5;
    const int U = 2 * nwV + nwC;  // source words per row
    for (int t = threadIdx.x; t < p.A * U; t += T) {
        const int i = t / U;
        int s = t - i * U;
        int len, off;
        uint32_t m, x;
        if (s < nwV) {  // own vars
            len = min(32, p.V - 32 * s);
            const int lo = agent_lo(p, i) - 32 * s, hi = lo + agent_size(p, i);
            const int a = max(lo, 0), z = min(hi, 32);
            m = z > a ? (low_mask(z) & ~low_mask(a)) : 0u;
            x = l.x[s];
            off = 32 * s;
        } else if ((s -= nwV) < nwC) {  // clause status
            len = min(32, p.C - 32 * s);
            m = l.rel[i * p.WC + s];
            x = l.sat[s];
            off = p.V + 32 * s;
        } else {  // neighbour vars
            s -= nwC;
            len = min(32, p.V - 32 * s);
            m = l.nbr[i * p.WV + s];
            x = l.x[s];
            off = p.V + p.C + 32 * s;
        }
        const uint32_t keep = low_mask(len);
        const int dst = i * p.D + off;
        or_bits(l.fm, dst, m & keep);
        or_bits(l.fx, dst, x & m & keep);  // value bits only where the element is live
    }
}

__device__ __forceinline__ uint32_t bits_at(const uint32_t *img, int e) {
    const int w = e >> 5, s = e & 31;
    return (uint32_t)((((uint64_t)img[w + 1] << 32) | img[w]) >> s);
}

__device__ __forceinline__ int elem_val(uint32_t m, uint32_t x, int u) {
    return ((m >> u) & 1u) ? (int)((x >> u) & 1u) : -1;
}

template <typename ObsT>
struct ObsVec;
template <>
struct ObsVec<int32_t> {
    static constexpr int N = 4;
    __device__ static void store(int32_t *dst, uint32_t m, uint32_t x) {
        typedef int v4i __attribute__((ext_vector_type(4)));
        const v4i q = {elem_val(m, x, 0), elem_val(m, x, 1), elem_val(m, x, 2), elem_val(m, x, 3)};
        *reinterpret_cast<v4i *>(dst) = q;
    }
};
template <>
struct ObsVec<int8_t> {
    static constexpr int N = 16;
    __device__ static void store(int8_t *dst, uint32_t m, uint32_t x) {
        // byte u = m_u ? x_u : 0xFF  (-1)
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        v4u q;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            uint32_t word = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) word |= ((uint32_t)elem_val(m, x, 4 * w + u) & 0xFFu) << (8 * u);
            q[w] = word;
        }
        *reinterpret_cast<v4u *>(dst) = q;
    }
};

// Stream the env's (A, D) observation block from the bit images: unaligned head, 16 B body, tail.
template <int T, typename ObsT>
__device__ __forceinline__ void write_obs(const EnvParams &p, const EnvLds &l, ObsT *__restrict__ o) {
    constexpr int VEC = ObsVec<ObsT>::N;
    const int total = p.A * p.D;
    int head = (int)((reinterpret_cast<uintptr_t>(o) / sizeof(ObsT)) % VEC);
    head = head ? VEC - head : 0;
    head = min(head, total);
    for (int e = threadIdx.x; e < head; e += T) o[e] = (ObsT)elem_val(bits_at(l.fm, e), bits_at(l.fx, e), 0);
    const int nchunks = (total - head) / VEC;
    for (int q = threadIdx.x; q < nchunks; q += T) {
        const int e = head + q * VEC;
        ObsVec<ObsT>::store(o + e, bits_at(l.fm, e), bits_at(l.fx, e));
    }
    for (int e = head + nchunks * VEC + threadIdx.x; e < total; e += T)
        o[e] = (ObsT)elem_val(bits_at(l.fm, e), bits_at(l.fx, e), 0);
}

// ---------------------------------------------------------------- kernel ----
// XCD-major env order: blocks b and b+8 share an XCD (round-robin dispatch, speed only),
// so consecutive envs -- adjacent obs blocks in HBM -- are written through one XCD's L2.
__device__ __forceinline__ int xcd_major(int blk, int n, bool off) {
    return (!off && (n & 7) == 0) ? (blk & 7) * (n >> 3) + (blk >> 3) : blk;
}

// Workgroup barrier for LDS only: waits for this wave's LDS operations, not for its global stores
// (a __syncthreads() fence drains every outstanding store).  env_run never reads back global memory
// written by another thread of its workgroup.  (A persistent variant that walks several envs per
// workgroup to overlap one env's store drain with the next env's scan measured slower at every
// occupancy, 114-188 us vs 112 us at uf200 x 4096: the 8 resident workgroups per CU already overlap.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Diagnostic stamps (msat_step_out.clock_stamps, NULL in product calls: a wave-uniform branch at each
// point).  Per env, 8 words written by lane 0 of wave 0 (vector stores):
//   [0] shader-clock counter delta over the workgroup's run (s_memtime), [1] the 100 MHz real-time counter
//   delta (s_memrealtime): clock MHz = 100 [0] / [1];
//   [2] real time at the workgroup's start, [3..6] at four phase ends (3: assignment bits + flips in LDS,
//   i.e. the first global loads landed; 4: clause scan done; 5: agent tables staged; 6: obs bit images
//   built), [7] at the end, after wave 0's stores have drained (vmcnt(0)).
// Same CU, same wave: the ratio is the clock that CU ran at while it stepped this env, and the phase times
// are wave 0's view of the env's dependent chain.
struct ClockStamp {
    uint64_t *buf = nullptr;
    uint64_t t0 = 0, r0 = 0;
    __device__ __forceinline__ ClockStamp(uint64_t *stamps, int b) {
        if (stamps != nullptr) {
            t0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
            buf = stamps + 8 * (size_t)b;
        }
    }
    __device__ __forceinline__ void mark(int i) const {
        if (buf == nullptr) return;
        const uint64_t r = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) buf[2 + i] = i == 0 ? r0 : r;
    }
    __device__ __forceinline__ void finish() const {
        if (buf == nullptr) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x < 4) {
            const int i = threadIdx.x;
            buf[i == 3 ? 7 : i] = i == 0 ? t1 - t0 : i == 1 ? r1 - r0 : i == 2 ? r0 : r1;
        }
    }
};

// The prefetch of an instance's pool row and agent tables into this lane's registers (one round trip).
template <int T>
__device__ __forceinline__ void prefetch_instance(const EnvParams &p, const msat_pool &pool, int n,
                                                  uint64_t (&w)[kPfClause], uint32_t (&rl)[kPfRel],
                                                  uint32_t (&nb)[kPfNbr]) {
    // Branch-free: every lane loads a clamped (valid) address and zeroes what lies past the end.  Loads under a
    // branch leave the compiler's vmcnt bookkeeping unsure how many are in flight, so the first use of an
    // EARLIER load (the assignment byte) then waited for all of these (a whole round trip before the flips).
    const int tid = threadIdx.x;
    const uint64_t *prow = reinterpret_cast<const uint64_t *>(pool.lits) + (size_t)n * p.C;
    const uint32_t *rel_g = pool.rel + (size_t)n * p.A * p.WC;
    const uint32_t *nbr_g = pool.nbr + (size_t)n * p.A * p.WV;
    const int nrel = p.A * p.WC, nnbr = p.A * p.WV;
#pragma unroll
    for (int j = 0; j < kPfClause; ++j) {
        const int c = tid + j * T;
        const uint64_t v = prow[min(c, p.C - 1)];
        w[j] = c < p.C ? v : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kPfRel; ++j) {
        const int t = tid + j * T;
        const uint32_t v = rel_g[min(t, nrel - 1)];
        rl[j] = t < nrel ? v : 0u;
    }
#pragma unroll
    for (int j = 0; j < kPfNbr; ++j) {
        const int t = tid + j * T;
        const uint32_t v = nbr_g[min(t, nnbr - 1)];
        nb[j] = t < nnbr ? v : 0u;
    }
}

// The instance a reset of env b draws (env:158-162 via the rollout's reset, learner:426-436): the caller's index,
// or Philox word block 0 of (seed, ctr, env).
__device__ __forceinline__ int reset_instance(const EnvParams &p, const int32_t *__restrict__ new_pidx, uint64_t seed,
                                              uint64_t ctr, int b) {
    if (new_pidx != nullptr) return new_pidx[b];
    const uint4 r = reset_rng_block(seed, ctr, (uint32_t)b, 0u);
    return (int)(((uint64_t)r.x * (uint64_t)p.N) >> 32);
}

// The assignment a reset of env b draws into l.x: the caller's bytes, or word t = lane t % 4 of the Philox block
// 1 + t / 4 (128 vars per block).
template <int T>
__device__ __forceinline__ void reset_assignment(const EnvParams &p, const EnvLds &l,
                                                 const uint8_t *__restrict__ new_assign, uint64_t seed, uint64_t ctr,
                                                 int b) {
    if (new_assign != nullptr) {
        load_x_bits<T>(p, l, new_assign + (size_t)b * p.V);
        return;
    }
    for (int t = threadIdx.x; t < p.WV; t += T) {
        const uint4 r = reset_rng_block(seed, ctr, (uint32_t)b, 1u + (uint32_t)(t >> 2));
        const int lane = t & 3;
        uint32_t w = lane == 0 ? r.x : lane == 1 ? r.y : lane == 2 ? r.z : r.w;
        const int hi = p.V - 32 * t;
        if (hi < 32) w &= hi <= 0 ? 0u : ((1u << hi) - 1u);
        l.x[t] = w;
    }
}

// Stage instance pidx's agent tables in LDS (the first kPf* words from this lane's prefetch registers when pf),
// build the obs bit images and stream the env's (A, D) block.
template <typename ObsT, int T>
__device__ __forceinline__ void stage_and_write_obs(const EnvParams &p, const EnvLds &l, const msat_pool &pool,
                                                    int pidx, bool pf, const uint32_t (&prel)[kPfRel],
                                                    const uint32_t (&pnbr)[kPfNbr], ObsT *__restrict__ o,
                                                    const ClockStamp *cs) {
    const int tid = threadIdx.x;
    {
        const uint32_t *rel_g = pool.rel + (size_t)pidx * p.A * p.WC;
        const uint32_t *nbr_g = pool.nbr + (size_t)pidx * p.A * p.WV;
        int t0r = 0, t0n = 0;
        if (pf) {
#pragma unroll
            for (int j = 0; j < kPfRel; ++j)
                if (tid + j * T < p.A * p.WC) l.rel[tid + j * T] = prel[j];
#pragma unroll
            for (int j = 0; j < kPfNbr; ++j)
                if (tid + j * T < p.A * p.WV) l.nbr[tid + j * T] = pnbr[j];
            t0r = kPfRel * T;
            t0n = kPfNbr * T;
        }
        for (int t = t0r + tid; t < p.A * p.WC; t += T) l.rel[t] = rel_g[t];
        for (int t = t0n + tid; t < p.A * p.WV; t += T) l.nbr[t] = nbr_g[t];
        for (int t = tid; t < 2 * obs_image_words(p); t += T) l.fm[t] = 0u;  // fm, fx contiguous
    }
    lds_barrier();
    if (cs) cs->mark(3);
    if ((p.ablate & 3) == 0) {
        build_obs_images<T>(p, l);
        lds_barrier();
        if (cs) cs->mark(4);
        write_obs<T, ObsT>(p, l, o);
    } else {
        constexpr int VEC = ObsVec<ObsT>::N;
        const int n = (p.A * p.D) / VEC;
        for (int q = tid; q < n; q += T) ObsVec<ObsT>::store(o + q * VEC, 0u, 0u);
    }
}

// One environment (index b of its batch) advanced / reset / observed by one workgroup.
template <int MODE, typename ObsT, int T>
__device__ __forceinline__ void env_run(const EnvParams &p, const msat_pool &pool, const msat_env_state &st,
                                        const int32_t *__restrict__ actions, const uint8_t *__restrict__ reset_mask,
                                        const int32_t *__restrict__ new_pidx, const uint8_t *__restrict__ new_assign,
                                        uint64_t seed, uint64_t ctr, const msat_step_out &out, ObsT *__restrict__ obs,
                                        int b, uint32_t *smem, const ClockStamp &cs) {
    const EnvLds l = carve(smem, p);
    const int tid = threadIdx.x;
    if (MODE == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return;

    uint8_t *__restrict__ xg = st.assign + (size_t)b * p.V;
    uint8_t *__restrict__ sat_g = st.clause_sat + (size_t)b * p.C;
    uint8_t *__restrict__ ntrue_g = st.clause_ntrue ? st.clause_ntrue + (size_t)b * p.C : nullptr;
    if (tid < 16) l.red[tid] = 0;
    // reset queue: rq_fast = this autoreset launch consumes / produces it; rq_mode 2 = clear this env's entries
    const bool rq_fast = MODE == kModeStepAutoReset && p.rq_mode == 1;  // host: sparse reward, mode 0, A < 64
    if (MODE != kModeObs && p.rq_mode == 2 && tid == 0) {
        rq_pend(st.reset_queue, p.B, 0)[b] = 0u;
        rq_pend(st.reset_queue, p.B, 1)[b] = 0u;
    }

    bool do_reset = (MODE == kModeReset);
    // the per-lane loads that do not depend on problem_idx, issued together with it (one round trip): this
    // lane's action and its assignment byte of the first ballot pass (clamped indices, no branches), then
    // problem_idx, step and unsat.  (step / unsat are wave-uniform values the compiler moves to scalar registers
    // as soon as they are loaded, i.e. waits for them right there: issued behind problem_idx, that wait retires
    // the first round trip, which the prefetch needs anyway.  Issued behind the prefetch (round 5), it held the
    // assignment bits and the flips until the prefetch had landed too.)
    int step0 = 0, u_old = 0, a0 = 0;
    uint32_t x0 = 0;
    bool covered = false;
    // the reset-queue entry rides in the action load: lane A of wave 0 (mode 0, A < 64) reads it instead of a
    // duplicate action, so it costs no round trip of its own
    if (MODE != kModeReset) {
        if (MODE != kModeObs && p.action_mode == 0) {
            const int32_t *ap = actions + (size_t)b * p.A + min(tid, p.A - 1);
            if (rq_fast && tid == p.A)
                ap = reinterpret_cast<const int32_t *>(rq_pend(st.reset_queue, p.B, p.rq_serial & 1) + b);
            a0 = *ap;
        }
        x0 = xg[min(tid, p.V - 1)];
    }
    int pidx = st.problem_idx[b];
    if (MODE != kModeReset) {
        step0 = st.step[b];
        u_old = st.num_unsat[b];
    }
    // keep the first round trip's loads ahead of the prefetch (the scheduler sank the assignment byte below it,
    // and its first use then waited for the prefetch as well)
    __builtin_amdgcn_sched_barrier(0);
    if (MSAT_DEBUG_BUILD && tid == 0) {  // this env's rows of every caller buffer, and its pool row
        if (MODE != kModeReset) MSAT_DCHECK(pidx, p.N);
        MSAT_DCHECK((long long)(b + 1) * p.V - 1, p.dbg_assign);
        MSAT_DCHECK((long long)(b + 1) * p.C - 1, p.dbg_sat);
        if (ntrue_g) MSAT_DCHECK((long long)(b + 1) * p.C - 1, p.dbg_ntrue);
        if (obs) MSAT_DCHECK((long long)(b + 1) * p.A * p.D - 1, p.dbg_obs);
        if (MODE == kModeStep || MODE == kModeStepAutoReset)
            MSAT_DCHECK((long long)(b + 1) * p.A * (p.action_mode == 0 ? 1 : p.M) - 1, p.dbg_actions);
    }
    uint64_t pw[kPfClause];
    uint32_t prel[kPfRel], pnbr[kPfNbr];
    if (MODE != kModeReset) {
        // ---- then the loads that do: the instance's pool row and agent tables (second round trip) --------
        prefetch_instance<T>(p, pool, pidx, pw, prel, pnbr);
        __builtin_amdgcn_sched_barrier(0);
        // ---- assignment + the agents' flips (env:230-250) --------------------
        load_x_bits<T>(p, l, xg, x0);
        lds_barrier();
        cs.mark(1);
        if (MODE == kModeObs) {
            // get_obs only: no flips, no state update
        } else if (p.action_mode == 0) {
            if (rq_fast && tid < 64) {  // wave 0: is this env covered?  (read by every wave after the barrier)
                const uint32_t tok = rq_token(p.rq_serial);
                int cov = 0;
                if (__builtin_amdgcn_readlane(a0, p.A) == (int)tok) {  // pending: its rank among the pending envs
                    int unused;
                    cov = rq_scan(rq_pend(st.reset_queue, p.B, p.rq_serial & 1), p.B, tok, b, -1, &unused) < p.rq_cap;
                }
                if (tid == 0) l.red[3] = cov;
            }
            for (int i = tid; i < p.A; i += T) {
                const int a = i == tid ? a0 : actions[(size_t)b * p.A + i];
                const int n = agent_size(p, i);
                if (a >= n) continue;  // no-op index (and every action of a var-less agent)
                int s = a;
                if (s < 0) {
                    s += p.M;  // jnp negative-index normalisation
                    if (s < 0) {
                        if (p.reward_mode == MSAT_REWARD_SINGLE_DELTA) continue;  // x.at[a] scatter drops it
                        s = 0;                                                   // agent_vars gather clamps
                    }
                }
                if (s < n) {
                    const int v = agent_lo(p, i) + s;
                    atomicXor(&l.x[v >> 5], 1u << (v & 31));
                }
            }
        } else {
            for (int t = tid; t < p.A * p.M; t += T) {
                const int i = t / p.M, j = t - (t / p.M) * p.M;
                if (j < agent_size(p, i) && (actions[(size_t)b * p.A * p.M + t] & 1)) {
                    const int v = agent_lo(p, i) + j;
                    atomicXor(&l.x[v >> 5], 1u << (v & 31));
                }
            }
        }
        lds_barrier();
        // ---- clause scan of the stepped assignment (env:252-254); a covered env (a reset workgroup of this launch
        // resets it: it times out now, listed by the previous launch) leaves its clause state to that workgroup
        covered = rq_fast && l.red[3] != 0;
        uint8_t *const scan_sat = covered ? nullptr : sat_g;
        uint8_t *const scan_ntrue = covered ? nullptr : ntrue_g;
        if (MODE != kModeObs && p.reward_mode == MSAT_REWARD_PBRS)
            eval_clauses<T, true, kPfClause>(p, l, pool.lits, pidx, scan_sat, scan_ntrue, pw);
        else
            eval_clauses<T, false, kPfClause>(p, l, pool.lits, pidx, scan_sat, scan_ntrue, pw);
        lds_barrier();
        cs.mark(2);
        if (MODE != kModeObs && tid == 0) {
            const int u_new = l.red[0];
            const bool solved = (u_new == 0);
            // single-agent SatEnv (sat_env.py:106) tests the pre-increment step
            const bool done = solved || (p.reward_mode == MSAT_REWARD_SINGLE_DELTA ? step0 >= p.max_steps
                                                                                   : step0 + 1 >= p.max_steps);
            float r;
            if (p.reward_mode == MSAT_REWARD_SINGLE_DELTA) {
                // sat_env.py:86-101, f32 in the reference's order: ((u_prev - u_new) * 10 + bonus) + (-0.005)
                const float up = __fdiv_rn((float)u_old, (float)p.C), un = __fdiv_rn((float)u_new, (float)p.C);
                r = __fmul_rn(__fsub_rn(up, un), 10.0f);
                r = __fadd_rn(r, solved ? p.r_sat : 0.0f);
                r = __fadd_rn(r, -0.005f);
            } else if (p.reward_mode == MSAT_REWARD_PBRS) {
                const float pot_new = (float)(-u_new), pot_old = (float)(-u_old);
                const float r_pbrs = __fsub_rn(__fmul_rn(p.gamma, pot_new), pot_old);
                const float r_cl = __fmul_rn((float)l.red[1], p.r_clause);
                r = __fadd_rn(__fadd_rn(r_pbrs, r_cl), solved ? p.r_sat : 0.0f);
            } else {
                r = solved ? 1.0f : 0.0f;
            }
            out.reward[b] = r;
            out.done[b] = done ? 1 : 0;
            out.solved[b] = solved ? 1 : 0;
            if (out.num_unsat) out.num_unsat[b] = u_new;
            if (out.episode_step) out.episode_step[b] = step0 + 1;
            // a covered env times out now (the previous launch listed it at max_steps - 1): its reset happens in any
            // case, here and in its reset workgroup, so the state stays whole even for a misused queue
            MSAT_DCHECK(covered && !done ? 1 : 0, 1);
            const bool reset_now = (MODE == kModeStepAutoReset) && (done || covered);
            l.red[2] = reset_now ? 1 : 0;
            if (!reset_now) {
                st.num_unsat[b] = u_new;
                st.step[b] = step0 + 1;
                st.done[b] = done ? 1 : 0;
            }
            if (rq_fast) {  // list this env for the next launch if its next step times out
                const int next_step = reset_now ? 0 : step0 + 1;
                rq_pend(st.reset_queue, p.B, (p.rq_serial + 1) & 1)[b] =
                    next_step + 1 >= p.max_steps ? rq_token(p.rq_serial + 1u) : 0u;
            }
        }
        lds_barrier();
        do_reset = (l.red[2] != 0);
    }

    if (do_reset) {
        // ---- reset (env:158-181): new problem, new assignment ---------------
        pidx = reset_instance(p, new_pidx, seed, ctr, b);
        if (MSAT_DEBUG_BUILD && tid == 0) MSAT_DCHECK(pidx, p.N);  // the reset's pool row
        reset_assignment<T>(p, l, new_assign, seed, ctr, b);
        if (covered) {
            // the reset workgroup scans the new instance and writes its clause state, count and observation;
            // this one writes the fields it read: assignment, step, done, problem_idx
            lds_barrier();
            if (tid == 0) {
                st.step[b] = 0;
                st.done[b] = 0;
                st.problem_idx[b] = pidx;
            }
            for (int v = tid; v < p.V; v += T) xg[v] = (uint8_t)bit(l.x, v);
            return;
        }
        if (tid < 2) l.red[tid] = 0;  // red[2] (reset broadcast) may still be read by slower waves
        lds_barrier();
        eval_clauses<T, false, 0>(p, l, pool.lits, pidx, sat_g, ntrue_g, pw);
        lds_barrier();
        if (tid == 0) {
            st.num_unsat[b] = l.red[0];
            st.step[b] = 0;
            st.done[b] = 0;
            st.problem_idx[b] = pidx;
        }
    }
    if (MODE != kModeObs)
        for (int v = tid; v < p.V; v += T) xg[v] = (uint8_t)bit(l.x, v);
    if ((p.ablate & 3) == 2 || obs == nullptr) return;  // NULL obs: state-only step (single-agent SatEnv)
    // ---- the instance's agent tables (built once per pool instance), obs images, obs stores ----------------
    stage_and_write_obs<ObsT, T>(p, l, pool, pidx, (MODE != kModeReset) && !do_reset, prel, pnbr,
                                 obs + (size_t)b * p.A * p.D, &cs);
}

// A reset workgroup of an autoreset launch with a reset queue (rq_mode 1): the pending env of rank j, i.e. an env that
// times out in this launch.  It draws the env's new instance and assignment (the same draw as its step workgroup's),
// scans the new instance, and writes the clause state, the unsatisfied count and the observation; its step workgroup
// writes the transition outputs, the assignment, step, done and problem_idx.  Two dependent round trips: the
// pending words (wave 0's scan), then the pool row and agent tables.
template <typename ObsT, int T>
__device__ __forceinline__ void env_side_reset(const EnvParams &p, const msat_pool &pool, const msat_env_state &st,
                                               const int32_t *__restrict__ new_pidx,
                                               const uint8_t *__restrict__ new_assign, uint64_t seed, uint64_t ctr,
                                               ObsT *__restrict__ obs, int j, uint32_t *smem) {
    const EnvLds l = carve(smem, p);
    const int tid = threadIdx.x;
    if (tid < 64) {
        int b = -1;
        rq_scan(rq_pend(st.reset_queue, p.B, p.rq_serial & 1), p.B, rq_token(p.rq_serial), 0, j, &b);
        if (tid == 0) l.red[4] = b;
    }
    if (tid < 4) l.red[tid] = 0;
    lds_barrier();
    const int b = l.red[4];
    if (b < 0) return;  // fewer than j + 1 envs time out in this launch
    const int pidx = reset_instance(p, new_pidx, seed, ctr, b);
    if (MSAT_DEBUG_BUILD && tid == 0) MSAT_DCHECK(pidx, p.N);
    uint64_t pw[kPfClause];
    uint32_t prel[kPfRel], pnbr[kPfNbr];
    prefetch_instance<T>(p, pool, pidx, pw, prel, pnbr);
    reset_assignment<T>(p, l, new_assign, seed, ctr, b);
    lds_barrier();
    uint8_t *__restrict__ sat_g = st.clause_sat + (size_t)b * p.C;
    uint8_t *__restrict__ ntrue_g = st.clause_ntrue ? st.clause_ntrue + (size_t)b * p.C : nullptr;
    eval_clauses<T, false, kPfClause>(p, l, pool.lits, pidx, sat_g, ntrue_g, pw);
    lds_barrier();
    if (tid == 0) st.num_unsat[b] = l.red[0];
    if ((p.ablate & 3) == 2 || obs == nullptr) return;
    stage_and_write_obs<ObsT, T>(p, l, pool, pidx, true, prel, pnbr, obs + (size_t)b * p.A * p.D, nullptr);
}

template <int MODE, typename ObsT, int T>
__global__ void __launch_bounds__(T)
env_kernel(EnvParams p, msat_pool pool, msat_env_state st, const int32_t *__restrict__ actions,
           const uint8_t *__restrict__ reset_mask, const int32_t *__restrict__ new_pidx,
           const uint8_t *__restrict__ new_assign, uint64_t seed, uint64_t ctr, msat_step_out out,
           ObsT *__restrict__ obs) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    // the reset workgroups first (block ids 0 .. cap - 1: their chain starts with a scan of the pending marks, and a
    // place at the end of the dispatch order made them the launch's tail)
    const int side = (MODE == kModeStepAutoReset && p.rq_mode == 1) ? p.rq_cap : 0;
    if ((int)blockIdx.x < side) {
        env_side_reset<ObsT, T>(p, pool, st, new_pidx, new_assign, seed, ctr, obs, (int)blockIdx.x, smem);
        return;
    }
    const int b = xcd_major((int)blockIdx.x - side, p.B, p.ablate & 4);
    const ClockStamp cs(out.clock_stamps, b);
    env_run<MODE, ObsT, T>(p, pool, st, actions, reset_mask, new_pidx, new_assign, seed, ctr, out, obs, b, smem, cs);
    cs.finish();
}

// Ragged batches (BASELINE config 5): several size classes, each its own (V, C, A) batch with its own
// pool / state / obs, advanced by ONE launch (256-lane workgroups).  Blocks map to (class, env) with
// the classes laid out most expensive first (launch_groups).  Class g draws its resets from seed ^ group_seed(g), so it
// replays exactly as a single-class launch with that seed (group_seed(0) = 0).
struct EnvGroup {
    EnvParams p;
    msat_pool pool;
    msat_env_state st;
    const int32_t *actions;
    msat_step_out out;
    void *obs;
    int begin;  // first block of the class
    int gid;    // the class's index in the caller's arrays (selects its RNG stream)
};

struct EnvGroups {
    int G, total, ablate;
    EnvGroup g[MSAT_MAX_GROUPS];
};

__host__ __device__ __forceinline__ uint64_t group_seed(int g) { return (uint64_t)g * 0x9E3779B97F4A7C15ull; }

template <int MODE, typename ObsT, int T>
__global__ void __launch_bounds__(T)
env_group_kernel(EnvGroups gs, uint64_t seed, uint64_t ctr) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    // Blocks in dispatch order, the classes laid out most expensive first (launch_groups): no XCD-major
    // remap here -- it put whole classes on a few XCDs (1024 mixed envs: 29.3 -> 19.4 us without it)
    const int gb = blockIdx.x;
    int g = 0;
#pragma unroll
    for (int k = 1; k < MSAT_MAX_GROUPS; ++k)
        if (k < gs.G && gb >= gs.g[k].begin) g = k;
    const EnvGroup &e = gs.g[g];
    const ClockStamp cs(e.out.clock_stamps, gb - e.begin);
    env_run<MODE, ObsT, T>(e.p, e.pool, e.st, e.actions, nullptr, nullptr, nullptr, seed ^ group_seed(e.gid), ctr, e.out,
                        reinterpret_cast<ObsT *>(e.obs), gb - e.begin, smem, cs);
    cs.finish();
}

// ---------------------------------------------------------------- cold path --

__global__ void pool_pack_kernel(const int32_t *__restrict__ lits, int NC, int K, int V,
                                 uint16_t *__restrict__ pool, int32_t *__restrict__ err) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= NC) return;
    uint64_t w = 0;
#pragma unroll
    for (int j = 0; j < MSAT_LIT_SLOTS; ++j) {
        uint32_t code = MSAT_LIT_ABSENT;
        if (j < K) {
            const int lit = lits[(size_t)t * K + j];
            if (lit == 0) {
                code = MSAT_LIT_NULL;
            } else {
                const int a = lit < 0 ? -lit : lit;
                if (a > V) {
                    atomicOr(err, 1);
                    code = MSAT_LIT_NULL;
                } else {
                    code = ((uint32_t)(a - 1) << 1) | (lit < 0 ? 1u : 0u);
                }
            }
        }
        w |= (uint64_t)code << (16 * j);
    }
    reinterpret_cast<uint64_t *>(pool)[t] = w;
}

// Per-instance agent tables (env:99-128): rel[i][c] = clause c contains a var of
// agent i; nbr[i][v] = v appears in a clause related to i and is not i's.
__global__ void __launch_bounds__(kThreads)
agent_tables_kernel(EnvParams p, const uint16_t *__restrict__ lits, uint32_t *__restrict__ rel_g,
                    uint32_t *__restrict__ nbr_g) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *rel = smem;
    uint32_t *nbr = rel + (size_t)p.A * p.WC;
    const int n = blockIdx.x;
    for (int t = threadIdx.x; t < p.A * (p.WC + p.WV); t += kThreads) smem[t] = 0u;
    __syncthreads();
    const uint64_t *prow = reinterpret_cast<const uint64_t *>(lits) + (size_t)n * p.C;
    for (int c = threadIdx.x; c < p.C; c += kThreads) {
        const uint64_t w = prow[c];
        int vars[3], ags[3];
        bool nullLit = false;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint32_t lit = (uint32_t)(w >> (16 * j)) & 0xFFFFu;
            vars[j] = lit < MSAT_LIT_ABSENT ? (int)(lit >> 1) : -1;
            ags[j] = vars[j] >= 0 ? agent_of_var(p, vars[j]) : -1;
            nullLit |= (lit == MSAT_LIT_NULL);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (ags[j] < 0) continue;
            atomicOr(&rel[ags[j] * p.WC + (c >> 5)], 1u << (c & 31));
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                if (k == j || vars[k] < 0 || ags[k] == ags[j]) continue;
                atomicOr(&nbr[ags[j] * p.WV + (vars[k] >> 5)], 1u << (vars[k] & 31));
            }
        }
        if (nullLit && p.rem > 0) {
            // Reference quirk: literal 0 decodes to var index -1, equal to the -1 padding of
            // agent_vars rows, so the clause is "related" to every agent owning fewer than M vars.
            for (int i = p.rem; i < p.A; ++i) {
                atomicOr(&rel[i * p.WC + (c >> 5)], 1u << (c & 31));
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    if (vars[k] < 0 || ags[k] == i) continue;
                    atomicOr(&nbr[i * p.WV + (vars[k] >> 5)], 1u << (vars[k] & 31));
                }
            }
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < p.A * p.WC; t += kThreads) rel_g[(size_t)n * p.A * p.WC + t] = rel[t];
    for (int t = threadIdx.x; t < p.A * p.WV; t += kThreads) nbr_g[(size_t)n * p.A * p.WV + t] = nbr[t];
}

// Per-env materialisation of the reference's mask tensors (env:99-128, :160).
__global__ void __launch_bounds__(kThreads)
env_masks_kernel(EnvParams p, msat_pool pool, const int32_t *__restrict__ problem_idx, int32_t *__restrict__ acm,
                 int32_t *__restrict__ anm, int32_t *__restrict__ l2a) {
    const int b = blockIdx.x;
    const int pidx = problem_idx[b];
    const uint32_t *rel = pool.rel + (size_t)pidx * p.A * p.WC;
    const uint32_t *nbr = pool.nbr + (size_t)pidx * p.A * p.WV;
    if (acm)
        for (int t = threadIdx.x; t < p.A * p.C; t += kThreads) {
            const int i = t / p.C, c = t - i * p.C;
            acm[(size_t)b * p.A * p.C + t] = bit(rel + i * p.WC, c) ? 1 : -1;
        }
    if (anm)
        for (int t = threadIdx.x; t < p.A * p.V; t += kThreads) {
            const int i = t / p.V, v = t - i * p.V;
            anm[(size_t)b * p.A * p.V + t] = bit(nbr + i * p.WV, v) ? 1 : -1;
        }
    if (l2a) {
        const uint64_t *prow = reinterpret_cast<const uint64_t *>(pool.lits) + (size_t)pidx * p.C;
        const int last_agent = agent_of_var(p, p.V - 1);  // var2agent[-1] wraps to the last var
        for (int t = threadIdx.x; t < p.C * p.K; t += kThreads) {
            const int c = t / p.K, j = t - c * p.K;
            const uint32_t lit = (uint32_t)(prow[c] >> (16 * j)) & 0xFFFFu;
            l2a[(size_t)b * p.C * p.K + t] = lit == MSAT_LIT_NULL ? last_agent : agent_of_var(p, (int)(lit >> 1));
        }
    }
}

__global__ void clause_features_kernel(int BC, const uint8_t *__restrict__ sat,
                                       const uint8_t *__restrict__ ntrue, float *__restrict__ f) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= BC) return;
    f[3 * (size_t)t + 0] = (float)sat[t];
    f[3 * (size_t)t + 1] = (float)ntrue[t] / 3.0f;
    f[3 * (size_t)t + 2] = 1.0f;
}

__global__ void __launch_bounds__(kThreads)
static_var_features_kernel(const uint16_t *__restrict__ pool, int V, int C, float *__restrict__ f) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    int *deg = reinterpret_cast<int *>(smem);  // [2V]
    const int n = blockIdx.x;
    for (int t = threadIdx.x; t < 2 * V; t += kThreads) deg[t] = 0;
    __syncthreads();
    const uint64_t *prow = reinterpret_cast<const uint64_t *>(pool) + (size_t)n * C;
    for (int c = threadIdx.x; c < C; c += kThreads) {
        const uint64_t w = prow[c];
        for (int j = 0; j < 3; ++j) {
            const uint32_t lit = (uint32_t)(w >> (16 * j)) & 0xFFFFu;
            if (lit < MSAT_LIT_ABSENT) atomicAdd(&deg[2 * (lit >> 1) + (lit & 1)], 1);
        }
    }
    __syncthreads();
    for (int v = threadIdx.x; v < V; v += kThreads) {
        float *o = f + ((size_t)n * V + v) * 3;
        o[0] = (float)deg[2 * v] / (float)C;
        o[1] = (float)deg[2 * v + 1] / (float)C;
        o[2] = 0.0f;
    }
}

// ------------------------------------------------------- BC joint labels ----
// behavioral_cloning.py:54-100 (compute_joint_labels_parallel_greedy) for a batch: per env,
// delta[v] = unsat(x with v flipped) - unsat(x) for every var (one pass over the clauses: a clause
// changes status under the flip of v iff re-evaluating it with v flipped differs; duplicate vars in
// a clause are counted once, literal 0 stays false), then per agent the first local index with the
// smallest delta among strictly improving flips; label = that index if best < tau, else M (no-op).
__global__ void __launch_bounds__(kThreads)
bc_labels_kernel(EnvParams p, const uint16_t *__restrict__ lits, const int32_t *__restrict__ pidx,
                 const uint8_t *__restrict__ assign, float tau, int32_t *__restrict__ labels,
                 int32_t *__restrict__ deltas) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *xb = smem;                               // [WV] assignment bits
    int *dl = reinterpret_cast<int *>(smem + p.WV);    // [V]
    const int b = blockIdx.x, tid = threadIdx.x;
    const uint8_t *xg = assign + (size_t)b * p.V;
    for (int t = tid; t < p.WV; t += kThreads) {
        uint32_t w = 0;
        for (int k = 0; k < 32; ++k) {
            const int v = 32 * t + k;
            if (v < p.V && (xg[v] & 1u)) w |= 1u << k;
        }
        xb[t] = w;
    }
    for (int v = tid; v < p.V; v += kThreads) dl[v] = 0;
    __syncthreads();
    const uint64_t *prow = reinterpret_cast<const uint64_t *>(lits) + (size_t)pidx[b] * p.C;
    for (int c = tid; c < p.C; c += kThreads) {
        const uint64_t w = prow[c];
        int var[MSAT_LIT_SLOTS];
        bool val[MSAT_LIT_SLOTS];
        bool old = false;
#pragma unroll
        for (int j = 0; j < MSAT_LIT_SLOTS; ++j) {
            const uint32_t code = (uint32_t)(w >> (16 * j)) & 0xFFFFu;
            var[j] = code >= MSAT_LIT_ABSENT ? -1 : (int)(code >> 1);  // NULL / ABSENT: no variable, false
            val[j] = var[j] >= 0 && ((((xb[var[j] >> 5] >> (var[j] & 31)) & 1u) ^ (code & 1u)) != 0u);
            old = old || val[j];
        }
#pragma unroll
        for (int j = 0; j < MSAT_LIT_SLOTS; ++j) {
            const int v = var[j];
            if (v < 0) continue;
            bool dup = false;
#pragma unroll
            for (int k = 0; k < j; ++k) dup = dup || (var[k] == v);
            if (dup) continue;
            bool nw = false;
#pragma unroll
            for (int k = 0; k < MSAT_LIT_SLOTS; ++k) nw = nw || (var[k] >= 0 && (val[k] != (var[k] == v)));
            if (nw != old) atomicAdd(&dl[v], old ? 1 : -1);
        }
    }
    __syncthreads();
    if (deltas)
        for (int v = tid; v < p.V; v += kThreads) deltas[(size_t)b * p.V + v] = dl[v];
    for (int i = tid; i < p.A; i += kThreads) {
        int best = 0, bi = p.M;
        const int lo = agent_lo(p, i), n = agent_size(p, i);
        for (int j = 0; j < n; ++j) {
            const int d = dl[lo + j];
            if (d < best) {
                best = d;
                bi = j;
            }
        }
        labels[(size_t)b * p.A + i] = ((float)best < tau) ? bi : p.M;
    }
}

// single-agent SatEnv clause features [is_sat, is_unsat, 1] (sat_env.py:143-160)
__global__ void clause_sat_features_kernel(int BC, const uint8_t *__restrict__ sat, float *__restrict__ f) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= BC) return;
    const float s = (float)sat[t];
    f[3 * (size_t)t + 0] = s;
    f[3 * (size_t)t + 1] = 1.0f - s;
    f[3 * (size_t)t + 2] = 1.0f;
}

// ------------------------------------------------------------- host glue ----

static int make_params(const msat_env_desc *d, EnvParams *p) {
    MSAT_REQUIRE(d != nullptr, "desc is NULL");
    MSAT_REQUIRE(d->num_envs >= 0, "num_envs < 0");
    MSAT_REQUIRE(d->num_vars >= 1 && d->num_vars <= 32000, "num_vars %d out of [1,32000]", d->num_vars);
    MSAT_REQUIRE(d->num_clauses >= 1, "num_clauses %d < 1", d->num_clauses);
    MSAT_REQUIRE(d->clause_width >= 1 && d->clause_width <= 3, "clause_width %d out of [1,3]", d->clause_width);
    MSAT_REQUIRE(d->num_agents >= 1 && d->num_agents <= 1000, "num_agents %d out of [1,1000]", d->num_agents);
    MSAT_REQUIRE(d->action_mode == 0 || d->action_mode == 1, "action_mode %d", d->action_mode);
    MSAT_REQUIRE(d->reward_mode >= 0 && d->reward_mode <= 2, "reward_mode %d", d->reward_mode);
    MSAT_REQUIRE(d->obs_dtype == MSAT_OBS_I32 || d->obs_dtype == MSAT_OBS_I8, "obs_dtype %d", d->obs_dtype);
    MSAT_REQUIRE(d->num_problems >= 1, "num_problems %d < 1", d->num_problems);
    p->B = d->num_envs;
    p->V = d->num_vars;
    p->C = d->num_clauses;
    p->K = d->clause_width;
    p->A = d->num_agents;
    p->base = p->V / p->A;
    p->rem = p->V % p->A;
    p->M = p->base + (p->rem > 0 ? 1 : 0);
    MSAT_REQUIRE(d->max_vars_per_agent == p->M, "max_vars_per_agent %d != ceil(V/A)=%d",
                 d->max_vars_per_agent, p->M);
    p->WV = 2 * ((p->V + 63) / 64);
    p->WC = 2 * ((p->C + 63) / 64);
    p->D = 2 * p->V + p->C;
    p->max_steps = d->max_steps;
    p->action_mode = d->action_mode;
    p->reward_mode = d->reward_mode;
    p->N = d->num_problems;
    p->r_clause = d->r_clause;
    p->r_sat = d->r_sat;
    p->gamma = d->gamma;
    const char *ab = getenv("MARLSAT_ABLATE");
    p->ablate = ab ? atoi(ab) : 0;
    p->dbg_obs = p->dbg_assign = p->dbg_sat = p->dbg_ntrue = p->dbg_actions = 0;
    p->rq_mode = 0;
    p->rq_cap = rq_capacity(p->B);
    p->rq_serial = 0;
    return MSAT_OK;
}

// The reset-queue role of a launch on state st (EnvParams::rq_mode): the autoreset step of the sparse reward mode
// consumes and produces it; every other state-modifying launch clears the entries of the envs it touches.
static int set_reset_queue(EnvParams *p, const msat_env_state *st, int mode) {
    p->rq_mode = 0;
    if (st->reset_queue == nullptr || mode == kModeObs) return MSAT_OK;
    MSAT_REQUIRE((reinterpret_cast<uintptr_t>(st->reset_queue) & 15) == 0, "reset_queue must be 16-byte aligned");
    if (MSAT_DEBUG_BUILD)
        MSAT_REQUIRE(dbg_extent(st->reset_queue, 4) >= (long long)rq_words(p->B),
                     "MSAT_DEBUG: reset_queue smaller than msat_reset_queue_words(%d)", p->B);
    p->rq_serial = st->reset_serial;
    // the fast path reads an env's entry in its action load (mode 0, A < 64) and scans the entries 16 bytes at a time
    p->rq_mode = (mode == kModeStepAutoReset && p->reward_mode == MSAT_REWARD_SPARSE && p->action_mode == 0 &&
                  p->A < 64 && p->B % 4 == 0) ? 1 : 2;
    return MSAT_OK;
}

// debug builds: the extents of the launch's caller buffers (EnvParams::dbg_*)
static void set_dbg_extents(EnvParams *p, const msat_env_state *st, const int32_t *actions, const void *obs,
                            int obs_dtype) {
    if (!MSAT_DEBUG_BUILD) return;
    p->dbg_obs = dbg_extent(obs, obs_dtype == MSAT_OBS_I32 ? 4 : 1);
    p->dbg_assign = dbg_extent(st->assign, 1);
    p->dbg_sat = dbg_extent(st->clause_sat, 1);
    p->dbg_ntrue = dbg_extent(st->clause_ntrue, 1);
    p->dbg_actions = dbg_extent(actions, 4);
}

static int check_state(const msat_env_state *st) {
    MSAT_REQUIRE(st != nullptr, "state is NULL");
    MSAT_REQUIRE(st->assign && st->clause_sat && st->num_unsat && st->step && st->done && st->problem_idx,
                 "a required state pointer is NULL");
    return MSAT_OK;
}

static int check_pool(const msat_pool *pool) {
    MSAT_REQUIRE(pool != nullptr && pool->lits && pool->rel && pool->nbr, "pool (lits/rel/nbr) is NULL");
    return MSAT_OK;
}

// Workgroup size of the single-class env kernel: one wave per env for small instances (more envs
// resident per CU: the per-env chain of dependent memory round trips, not bandwidth, bounds them),
// 512 lanes for large ones (A * D >= 16384: uf200), 256 otherwise.  MARLSAT_ENV_THREADS (64 / 128 / 256 / 512) overrides.
static int env_threads(const EnvParams &p) {
    static const int forced = [] {
        const char *e = getenv("MARLSAT_ENV_THREADS");
        const int v = e ? atoi(e) : 0;
        return v == 64 || v == 128 || v == 256 || v == 512 ? v : 0;
    }();
    if (forced) return forced;
    // Fewer lanes per env as the batch grows (more envs resident per CU), more while each env's chain bounds the
    // launch (a few envs per CU).  uf50: x 1024 7.57 us at 128 vs 7.86 at 64, 7.88 at 256; x 2048 9.86 at 64 vs 10.1
    // at 128; x 4096 14.1 at 64 vs 16.6 at 128.  uf100: x 1024 11.0 at 256 vs 11.6 at 128, 14.6 at 64; x 2048 15.3 at
    // 128 vs 16.6 at 256; x 4096 25.8 at 128 vs 26.3 at 256.  uf200 x 4096: 107 at 512 vs 109 at 256, 142 at 64
    // (profiles/r06/r06t_*, r06u_*, r06w_*, r06x_*)
    const long n = (long)p.A * p.D;
    if (n >= 16384) return 512;
    if (n > 4096) return p.B <= 1024 ? 256 : 128;
    return p.B <= 1024 ? 128 : 64;
}

template <int MODE>
static int launch_env(const EnvParams &p, const msat_env_desc *d, const msat_pool *pool,
                      const msat_env_state *st, const int32_t *actions, const uint8_t *mask,
                      const int32_t *npidx, const uint8_t *nassign, uint64_t seed, uint64_t ctr,
                      const msat_step_out *out, void *obs, hipStream_t s) {
    const size_t lds = env_lds_words(p) * 4;
    MSAT_REQUIRE(lds <= 160 * 1024, "env needs %zu B of LDS (> 160 KiB)", lds);
    msat_step_out o{};
    if (out) o = *out;
    if (p.B == 0) return MSAT_OK;
    const int T = env_threads(p);
    EnvParams pd = p;  // + the buffer extents in debug builds, the reset queue's role
    set_dbg_extents(&pd, st, actions, obs, d->obs_dtype);
    if (int rc = set_reset_queue(&pd, st, MODE)) return rc;
    // the reset workgroups of a queue-consuming launch come first (block ids 0 .. cap - 1)
    const int grid = p.B + (pd.rq_mode == 1 ? pd.rq_cap : 0);
#define MSAT_ENV_LAUNCH(TT)                                                                                        \
    if (d->obs_dtype == MSAT_OBS_I32)                                                                              \
        hipLaunchKernelGGL((env_kernel<MODE, int32_t, TT>), dim3(grid), dim3(TT), lds, s, pd, *pool, *st, actions, \
                           mask, npidx, nassign, seed, ctr, o, (int32_t *)obs);                                    \
    else                                                                                                           \
        hipLaunchKernelGGL((env_kernel<MODE, int8_t, TT>), dim3(grid), dim3(TT), lds, s, pd, *pool, *st, actions,  \
                           mask, npidx, nassign, seed, ctr, o, (int8_t *)obs);
    if (T == 64) {
        MSAT_ENV_LAUNCH(64)
    } else if (T == 128) {
        MSAT_ENV_LAUNCH(128)
    } else if (T == 512) {
        MSAT_ENV_LAUNCH(512)
    } else {
        MSAT_ENV_LAUNCH(256)
    }
#undef MSAT_ENV_LAUNCH
    return check_launch("env_kernel");
}

template <int MODE>
static int launch_groups(int G, const msat_env_desc *descs, const msat_pool *pools, const msat_env_state *states,
                         const int32_t *const *actions, uint64_t seed, uint64_t ctr, const msat_step_out *outs,
                         void *const *obs, hipStream_t s) {
    MSAT_REQUIRE(G >= 1 && G <= MSAT_MAX_GROUPS, "num_groups %d out of [1,%d]", G, MSAT_MAX_GROUPS);
    MSAT_REQUIRE(descs && pools && states && obs, "NULL group arrays");
    MSAT_REQUIRE(MODE == kModeReset || (actions && outs), "NULL actions / outs");
    EnvGroups gs{};
    gs.G = G;
    size_t lds = 0;
    int total = 0;
    // block layout: classes by descending per-env obs size (A * D), so the longest envs are dispatched
    // first and the small ones fill in behind them (stable for equal sizes)
    int order[MSAT_MAX_GROUPS];
    long cost[MSAT_MAX_GROUPS];
    for (int g = 0; g < G; ++g) {
        order[g] = g;
        cost[g] = (long)descs[g].num_agents * (2L * descs[g].num_vars + descs[g].num_clauses);
    }
    std::stable_sort(order, order + G, [&](int x, int y) { return cost[x] > cost[y]; });
    for (int pos = 0; pos < G; ++pos) {
        const int g = order[pos];
        EnvGroup &e = gs.g[pos];
        e.gid = g;
        int rc = make_params(&descs[g], &e.p);
        if (rc) return rc;
        e.begin = total;
        if (e.p.B == 0) continue;  // empty class: no blocks (its pointers may be NULL)
        if ((rc = check_state(&states[g])) || (rc = check_pool(&pools[g]))) return rc;
        MSAT_REQUIRE(descs[g].obs_dtype == descs[0].obs_dtype, "groups must share obs_dtype");
        MSAT_REQUIRE(obs[g], "NULL obs for group %d", g);
        e.pool = pools[g];
        e.st = states[g];
        e.actions = MODE == kModeReset ? nullptr : actions[g];
        if (MODE != kModeReset) {
            MSAT_REQUIRE(e.actions && outs[g].reward && outs[g].done && outs[g].solved, "NULL step I/O, group %d", g);
            e.out = outs[g];
        }
        e.obs = obs[g];
        set_dbg_extents(&e.p, &e.st, e.actions, e.obs, descs[g].obs_dtype);
        // the grouped launch keeps every reset in its step workgroup: it only clears the queue's entries
        if ((rc = set_reset_queue(&e.p, &e.st, MODE))) return rc;
        if (e.p.rq_mode == 1) e.p.rq_mode = 2;
        total += e.p.B;
        lds = std::max(lds, env_lds_words(e.p) * 4);
        gs.ablate = e.p.ablate;
    }
    MSAT_REQUIRE(lds <= 160 * 1024, "env needs %zu B of LDS (> 160 KiB)", lds);
    gs.total = total;
    if (total == 0) return MSAT_OK;
    // workgroup size: 512 lanes for small batches (<= 2048 envs: the launch is bound by one large env's
    // latency; mixed 1024: 15.7 vs 16.9 us), 256 otherwise (mixed 8192: 91.5-96.9 vs 105.5 us on
    // 512); MARLSAT_ENV_GROUP_THREADS (256 / 512 / 1024) overrides
    static const int forced = [] {
        const char *e = getenv("MARLSAT_ENV_GROUP_THREADS");
        const int v = e ? atoi(e) : 0;
        return v == 256 || v == 512 || v == 1024 ? v : 0;
    }();
    const int gT = forced ? forced : (total <= 2048 ? 512 : 256);
#define MSAT_GROUP_LAUNCH(TT)                                                                                      \
    if (descs[0].obs_dtype == MSAT_OBS_I32)                                                                        \
        hipLaunchKernelGGL((env_group_kernel<MODE, int32_t, TT>), dim3(total), dim3(TT), lds, s, gs, seed, ctr);   \
    else                                                                                                           \
        hipLaunchKernelGGL((env_group_kernel<MODE, int8_t, TT>), dim3(total), dim3(TT), lds, s, gs, seed, ctr);
    if (gT == 1024) {
        MSAT_GROUP_LAUNCH(1024)
    } else if (gT == 512) {
        MSAT_GROUP_LAUNCH(512)
    } else {
        MSAT_GROUP_LAUNCH(256)
    }
#undef MSAT_GROUP_LAUNCH
    return check_launch("env_group_kernel");
}

}  // namespace msat

using namespace msat;

extern "C" int msat_env_reset_grouped(int32_t num_groups, const msat_env_desc *descs, const msat_pool *pools,
                                      const msat_env_state *states, uint64_t seed, uint64_t rng_counter,
                                      void *const *obs, void *stream) {
    return launch_groups<kModeReset>(num_groups, descs, pools, states, nullptr, seed, rng_counter, nullptr, obs,
                                     (hipStream_t)stream);
}

extern "C" int msat_env_step_grouped(int32_t num_groups, const msat_env_desc *descs, const msat_pool *pools,
                                     const msat_env_state *states, const int32_t *const *actions, int32_t autoreset,
                                     uint64_t seed, uint64_t rng_counter, const msat_step_out *outs, void *const *obs,
                                     void *stream) {
    if (autoreset)
        return launch_groups<kModeStepAutoReset>(num_groups, descs, pools, states, actions, seed, rng_counter, outs,
                                                 obs, (hipStream_t)stream);
    return launch_groups<kModeStep>(num_groups, descs, pools, states, actions, seed, rng_counter, outs, obs,
                                    (hipStream_t)stream);
}

extern "C" size_t msat_reset_queue_words(int32_t num_envs) { return num_envs < 0 ? 0 : rq_words(num_envs); }

extern "C" int msat_pool_pack(const int32_t *lits, int32_t num_problems, int32_t num_clauses,
                              int32_t clause_width, int32_t num_vars, uint16_t *pool,
                              int32_t *err_flag, void *stream) {
    MSAT_REQUIRE(lits && pool && err_flag, "NULL pointer");
    MSAT_REQUIRE(clause_width >= 1 && clause_width <= 3, "clause_width %d out of [1,3]", clause_width);
    MSAT_REQUIRE(num_problems >= 0 && num_clauses >= 1, "bad pool dims");
    const int NC = num_problems * num_clauses;
    if (NC == 0) return MSAT_OK;
    hipLaunchKernelGGL(pool_pack_kernel, dim3((NC + 255) / 256), dim3(256), 0, (hipStream_t)stream, lits,
                       NC, clause_width, num_vars, pool, err_flag);
    return check_launch("pool_pack_kernel");
}

extern "C" int msat_pool_agent_tables(const msat_env_desc *desc, const uint16_t *lits, uint32_t *rel, uint32_t *nbr,
                                      void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    MSAT_REQUIRE(lits && rel && nbr, "NULL pointer");
    const size_t lds = (size_t)p.A * (p.WC + p.WV) * 4;
    MSAT_REQUIRE(lds <= 160 * 1024, "agent tables need %zu B of LDS (> 160 KiB)", lds);
    hipLaunchKernelGGL(agent_tables_kernel, dim3(p.N), dim3(kThreads), lds, (hipStream_t)stream, p, lits, rel, nbr);
    return check_launch("agent_tables_kernel");
}

extern "C" int msat_env_reset(const msat_env_desc *desc, const msat_pool *pool,
                              const msat_env_state *state, const uint8_t *reset_mask,
                              const int32_t *new_problem_idx, const uint8_t *new_assign,
                              uint64_t seed, uint64_t rng_counter, void *obs, void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if (p.B == 0) return MSAT_OK;
    if ((rc = check_state(state)) || (rc = check_pool(pool))) return rc;
    return launch_env<kModeReset>(p, desc, pool, state, nullptr, reset_mask, new_problem_idx, new_assign,
                                  seed, rng_counter, nullptr, obs, (hipStream_t)stream);
}

extern "C" int msat_env_step(const msat_env_desc *desc, const msat_pool *pool,
                             const msat_env_state *state, const int32_t *actions, int32_t autoreset,
                             const int32_t *new_problem_idx, const uint8_t *new_assign, uint64_t seed,
                             uint64_t rng_counter, const msat_step_out *out, void *obs, void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if (p.B == 0) return MSAT_OK;
    if ((rc = check_state(state)) || (rc = check_pool(pool))) return rc;
    MSAT_REQUIRE(actions, "NULL actions");
    MSAT_REQUIRE(out && out->reward && out->done && out->solved, "NULL step outputs");
    if (autoreset)
        return launch_env<kModeStepAutoReset>(p, desc, pool, state, actions, nullptr, new_problem_idx,
                                              new_assign, seed, rng_counter, out, obs, (hipStream_t)stream);
    return launch_env<kModeStep>(p, desc, pool, state, actions, nullptr, nullptr, nullptr, seed,
                                 rng_counter, out, obs, (hipStream_t)stream);
}

extern "C" int msat_env_obs(const msat_env_desc *desc, const msat_pool *pool, const msat_env_state *state,
                            void *obs, void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if (p.B == 0) return MSAT_OK;
    if ((rc = check_state(state)) || (rc = check_pool(pool))) return rc;
    MSAT_REQUIRE(obs, "NULL obs");
    return launch_env<kModeObs>(p, desc, pool, state, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, obs,
                                (hipStream_t)stream);
}

extern "C" int msat_env_masks(const msat_env_desc *desc, const msat_pool *pool,
                              const msat_env_state *state, int32_t *agent_clause_masks,
                              int32_t *agent_neighbor_masks, int32_t *literal_to_agent_idx,
                              void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if ((rc = check_state(state)) || (rc = check_pool(pool))) return rc;
    if (p.B == 0) return MSAT_OK;
    hipLaunchKernelGGL(env_masks_kernel, dim3(p.B), dim3(kThreads), 0, (hipStream_t)stream, p, *pool,
                       state->problem_idx, agent_clause_masks, agent_neighbor_masks, literal_to_agent_idx);
    return check_launch("env_masks_kernel");
}

extern "C" int msat_clause_features(const msat_env_desc *desc, const msat_env_state *state,
                                    float *clause_features, void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    MSAT_REQUIRE(state && state->clause_sat && state->clause_ntrue && clause_features,
                 "clause_features needs clause_sat, clause_ntrue and an output");
    const int BC = p.B * p.C;
    if (BC == 0) return MSAT_OK;
    hipLaunchKernelGGL(clause_features_kernel, dim3((BC + 255) / 256), dim3(256), 0, (hipStream_t)stream, BC,
                       state->clause_sat, state->clause_ntrue, clause_features);
    return check_launch("clause_features_kernel");
}

extern "C" int msat_bc_greedy_labels(const msat_env_desc *desc, const uint16_t *lits, const int32_t *problem_idx,
                                     const uint8_t *assign, float tau, int32_t *labels, int32_t *deltas,
                                     void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if (p.B == 0) return MSAT_OK;
    MSAT_REQUIRE(lits && problem_idx && assign && labels, "NULL pointer");
    const size_t lds = ((size_t)p.WV + p.V) * 4;
    MSAT_REQUIRE(lds <= 160 * 1024, "bc labels need %zu B of LDS", lds);
    hipLaunchKernelGGL(bc_labels_kernel, dim3(p.B), dim3(kThreads), lds, (hipStream_t)stream, p, lits, problem_idx,
                       assign, tau, labels, deltas);
    return check_launch("bc_labels_kernel");
}

extern "C" int msat_clause_sat_features(const msat_env_desc *desc, const msat_env_state *state,
                                        float *clause_features, void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    MSAT_REQUIRE(state && state->clause_sat && clause_features, "NULL pointer");
    const int BC = p.B * p.C;
    if (BC == 0) return MSAT_OK;
    hipLaunchKernelGGL(clause_sat_features_kernel, dim3((BC + 255) / 256), dim3(256), 0, (hipStream_t)stream, BC,
                       state->clause_sat, clause_features);
    return check_launch("clause_sat_features_kernel");
}

extern "C" int msat_static_var_features(const uint16_t *pool, int32_t num_problems, int32_t num_vars,
                                        int32_t num_clauses, float *var_features, void *stream) {
    MSAT_REQUIRE(pool && var_features, "NULL pointer");
    MSAT_REQUIRE(num_vars >= 1 && num_vars <= 32000 && num_clauses >= 1, "bad dims");
    if (num_problems == 0) return MSAT_OK;
    hipLaunchKernelGGL(static_var_features_kernel, dim3(num_problems), dim3(kThreads),
                       (size_t)num_vars * 8, (hipStream_t)stream, pool, num_vars, num_clauses, var_features);
    return check_launch("static_var_features_kernel");
}
