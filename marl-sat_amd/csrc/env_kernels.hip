// Batched multi-agent SAT environment on gfx950.
//
// One workgroup (256 threads = 4 waves) owns one environment for the whole
// call: it stages the env's variables in LDS (assignment bit + owning agent,
// 2 B/var), evaluates every clause once from the L2/MALL-resident packed
// problem pool (8 B/clause: 4 x uint16 literal codes), reduces the
// unsatisfied count with wave shuffles, optionally resets the env in place
// (auto-reset) and finally streams the env's (A, 2V+C) observation block to
// HBM with 16-byte stores.  The observation write is >90 % of the algorithmic
// bytes of a step, so everything before it is organised to
// leave the obs pass a pure LDS-read -> 16 B store stream.
//
// Reference semantics (kongqg/marl-sat, src/envs/multi_agent_sat_env.py):
//   flip decode             :230-250
//   clause evaluation       :130-156   (literal l true iff l>0&&x=1 or l<0&&x=0)
//   done / reward / info    :256-284, :183-198 (sparse) / :201-223 (PBRS)
//   reset + masks           :158-181, :99-128
//   get_obs                 :345-398
//   rollout auto-reset      src/learners/mappo_gnn_sat_learner.py:422-464
#include "common.h"

namespace msat {

constexpr int kThreads = 256;
constexpr uint32_t kNoAgent = 0x3FFu;

struct EnvParams {
    int B, V, C, K, A, M, W, D;
    int base, rem;  // agent i owns [i*base + min(i,rem), +base+(i<rem))
    int max_steps, action_mode, reward_mode, N;
    float r_clause, r_sat, gamma;
};

enum : int { kModeReset = 0, kModeStep = 1, kModeStepAutoReset = 2, kModeObs = 3 };

__device__ __forceinline__ int agent_lo(const EnvParams &p, int i) { return i * p.base + min(i, p.rem); }
__device__ __forceinline__ int agent_size(const EnvParams &p, int i) { return p.base + (i < p.rem ? 1 : 0); }

__device__ __forceinline__ int agent_of_var(const EnvParams &p, int v) {
    const int split = p.rem * (p.base + 1);
    if (v < split) return v / (p.base + 1);
    return p.rem + (v - split) / p.base;  // base > 0 whenever v >= split
}

// LDS image of one environment.
struct EnvLds {
    uint32_t *clinfo;  // [C]   a0 | a1<<10 | a2<<20 | nullLit<<30 | sat<<31
    uint32_t *nbr;     // [A*W] neighbour bits
    int *red;          // [16]  reduction / broadcast scratch
    uint16_t *vinfo;   // [V]   agent | x<<15
};

__device__ __forceinline__ EnvLds carve(unsigned char *smem, const EnvParams &p) {
    EnvLds l;
    l.clinfo = reinterpret_cast<uint32_t *>(smem);
    l.nbr = l.clinfo + p.C;
    l.red = reinterpret_cast<int *>(l.nbr + p.A * p.W);
    l.vinfo = reinterpret_cast<uint16_t *>(l.red + 16);
    return l;
}

// Evaluate every clause of pool row `pidx` against the assignment in LDS.
// Writes clinfo, clause_sat (and ntrue), accumulates the unsat count (and,
// for PBRS, newly-satisfied count) into red[0] / red[1]; when `build_nbr`,
// ORs the neighbour bits of every agent related to each clause.
template <bool kPbrs, bool kBuildNbr>
__device__ __forceinline__ void eval_clauses(const EnvParams &p, const EnvLds &l,
                                             const uint16_t *__restrict__ pool, int pidx,
                                             uint8_t *__restrict__ sat_g, uint8_t *__restrict__ ntrue_g) {
    const uint64_t *prow = reinterpret_cast<const uint64_t *>(pool) + (size_t)pidx * p.C;
    int unsat = 0, newly = 0;
    for (int c = threadIdx.x; c < p.C; c += kThreads) {
        const uint64_t w = prow[c];  // pool rows are shared by many envs: keep them cached
        uint32_t info = 0, nullLit = 0;
        int ntrue = 0;
        int vars[3];
        uint32_t ags[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint32_t lit = (uint32_t)(w >> (16 * j)) & 0xFFFFu;
            uint32_t ag = kNoAgent;
            int var = -1;
            if (lit < MSAT_LIT_ABSENT) {
                var = (int)(lit >> 1);
                const uint32_t vi = l.vinfo[var];
                ntrue += (int)(((vi >> 15) ^ lit) & 1u);
                ag = vi & kNoAgent;
            } else if (lit == MSAT_LIT_NULL) {
                nullLit = 1;
            }
            vars[j] = var;
            ags[j] = ag;
            info |= ag << (10 * j);
        }
        const uint32_t sat = ntrue > 0 ? 1u : 0u;
        info |= (nullLit << 30) | (sat << 31);
        l.clinfo[c] = info;
        if (kPbrs) newly += (int)(sat & (sat_g[c] ^ 1u));
        sat_g[c] = (uint8_t)sat;
        if (ntrue_g) ntrue_g[c] = (uint8_t)ntrue;
        unsat += (int)(sat ^ 1u);
        if (kBuildNbr) {
            // vars of a related clause that the agent does not own are its neighbours (env:115-126)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                if (ags[j] == kNoAgent) continue;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    if (k == j || vars[k] < 0 || ags[k] == ags[j]) continue;
                    atomicOr(&l.nbr[ags[j] * p.W + (vars[k] >> 5)], 1u << (vars[k] & 31));
                }
            }
            if (nullLit && p.rem > 0) {
                // Reference quirk: literal 0 decodes to var index -1, which equals the -1
                // padding of agent_vars rows, so the clause is "related" to every agent
                // that owns fewer than M vars (agents i >= rem).
                for (int i = p.rem; i < p.A; ++i) {
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        if (vars[k] < 0 || ags[k] == (uint32_t)i) continue;
                        atomicOr(&l.nbr[i * p.W + (vars[k] >> 5)], 1u << (vars[k] & 31));
                    }
                }
            }
        }
    }
    unsat = wave_sum_i32(unsat);
    if (kPbrs) newly = wave_sum_i32(newly);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&l.red[0], unsat);
        if (kPbrs) atomicAdd(&l.red[1], newly);
    }
}

// One observation element (env:345-398): own vars | clause status | neighbour vars.
__device__ __forceinline__ int obs_value(const EnvParams &p, const EnvLds &l, int i, int k) {
    if (k < p.V) {
        const int lo = agent_lo(p, i);
        return (k >= lo && k < lo + agent_size(p, i)) ? (int)(l.vinfo[k] >> 15) : -1;
    }
    k -= p.V;
    if (k < p.C) {
        const uint32_t info = l.clinfo[k];
        const uint32_t ui = (uint32_t)i;
        const bool small = (p.rem > 0) && (i >= p.rem);
        const bool rel = ((info & kNoAgent) == ui) | (((info >> 10) & kNoAgent) == ui) |
                         (((info >> 20) & kNoAgent) == ui) | (small && ((info >> 30) & 1u));
        return rel ? (int)(info >> 31) : -1;
    }
    k -= p.C;
    const bool nb = (l.nbr[i * p.W + (k >> 5)] >> (k & 31)) & 1u;
    return nb ? (int)(l.vinfo[k] >> 15) : -1;
}

template <typename ObsT>
struct ObsVec;
template <>
struct ObsVec<int32_t> {
    static constexpr int N = 4;
    __device__ static void store(int32_t *dst, const int (&v)[4]) {
        typedef int v4i __attribute__((ext_vector_type(4)));
        const v4i q = {v[0], v[1], v[2], v[3]};
        __builtin_nontemporal_store(q, reinterpret_cast<v4i *>(dst));
    }
};
template <>
struct ObsVec<int8_t> {
    static constexpr int N = 16;
    __device__ static void store(int8_t *dst, const int (&v)[16]) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            w[q] = ((uint32_t)(v[4 * q] & 0xFF)) | ((uint32_t)(v[4 * q + 1] & 0xFF) << 8) |
                   ((uint32_t)(v[4 * q + 2] & 0xFF) << 16) | ((uint32_t)(v[4 * q + 3] & 0xFF) << 24);
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const v4u q4 = {w[0], w[1], w[2], w[3]};
        __builtin_nontemporal_store(q4, reinterpret_cast<v4u *>(dst));
    }
};

// Stream the env's (A, D) observation block: unaligned head, 16 B body, tail.
template <typename ObsT>
__device__ __forceinline__ void write_obs(const EnvParams &p, const EnvLds &l, ObsT *__restrict__ o) {
    constexpr int VEC = ObsVec<ObsT>::N;
    const int total = p.A * p.D;
    int head = (int)((reinterpret_cast<uintptr_t>(o) / sizeof(ObsT)) % VEC);
    head = head ? VEC - head : 0;
    head = min(head, total);
    for (int e = threadIdx.x; e < head; e += kThreads) {
        const int i = e / p.D;
        o[e] = (ObsT)obs_value(p, l, i, e - i * p.D);
    }
    const int nchunks = (total - head) / VEC;
    for (int q = threadIdx.x; q < nchunks; q += kThreads) {
        const int e = head + q * VEC;
        int i = e / p.D;
        int k = e - i * p.D;
        int v[VEC];
#pragma unroll
        for (int u = 0; u < VEC; ++u) {
            v[u] = obs_value(p, l, i, k);
            if (++k == p.D) {
                k = 0;
                ++i;
            }
        }
        ObsVec<ObsT>::store(o + e, v);
    }
    for (int e = head + nchunks * VEC + threadIdx.x; e < total; e += kThreads) {
        const int i = e / p.D;
        o[e] = (ObsT)obs_value(p, l, i, e - i * p.D);
    }
}

template <int MODE, typename ObsT>
__global__ void __launch_bounds__(kThreads)
env_kernel(EnvParams p, const uint16_t *__restrict__ pool, msat_env_state st,
           const int32_t *__restrict__ actions, const uint8_t *__restrict__ reset_mask,
           const int32_t *__restrict__ new_pidx, const uint8_t *__restrict__ new_assign,
           uint64_t seed, uint64_t ctr, msat_step_out out, ObsT *__restrict__ obs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const EnvLds l = carve(smem, p);
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    if (MODE == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return;

    uint8_t *__restrict__ xg = st.assign + (size_t)b * p.V;
    uint8_t *__restrict__ sat_g = st.clause_sat + (size_t)b * p.C;
    uint8_t *__restrict__ ntrue_g = st.clause_ntrue ? st.clause_ntrue + (size_t)b * p.C : nullptr;
    if (tid < 16) l.red[tid] = 0;

    bool do_reset = (MODE == kModeReset);
    if (MODE != kModeReset) {
        // ---- load assignment + apply the agents' flips (env:230-250) ----------
        for (int v = tid; v < p.V; v += kThreads)
            l.vinfo[v] = (uint16_t)(agent_of_var(p, v) | ((xg[v] & 1u) << 15));
        __syncthreads();
        if (MODE == kModeObs) {
            // get_obs only: no flips, no state update
        } else if (p.action_mode == 0) {
            for (int i = tid; i < p.A; i += kThreads) {
                const int a = actions[(size_t)b * p.A + i];
                const int n = agent_size(p, i);
                if (a >= n) continue;  // no-op index (and every action of a var-less agent)
                int s = a;
                if (s < 0) s = max(s + p.M, 0);  // jnp index normalisation + clamp
                if (s < n) l.vinfo[agent_lo(p, i) + s] ^= 0x8000u;
            }
        } else {
            for (int t = tid; t < p.A * p.M; t += kThreads) {
                const int i = t / p.M, j = t - (t / p.M) * p.M;
                if (j < agent_size(p, i) && (actions[(size_t)b * p.A * p.M + t] & 1))
                    l.vinfo[agent_lo(p, i) + j] ^= 0x8000u;
            }
        }
        __syncthreads();
        // ---- clause scan of the stepped assignment (env:252-254) ------------
        const int pidx = st.problem_idx[b];
        if (MODE != kModeObs && p.reward_mode == MSAT_REWARD_PBRS)
            eval_clauses<true, false>(p, l, pool, pidx, sat_g, ntrue_g);
        else
            eval_clauses<false, false>(p, l, pool, pidx, sat_g, ntrue_g);
        __syncthreads();
        if (MODE != kModeObs && tid == 0) {
            const int u_new = l.red[0];
            const int step0 = st.step[b];
            const bool solved = (u_new == 0);
            const bool done = solved || (step0 + 1 >= p.max_steps);
            float r;
            if (p.reward_mode == MSAT_REWARD_PBRS) {
                const float pot_new = (float)(-u_new), pot_old = (float)(-st.num_unsat[b]);
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
            const bool reset_now = (MODE == kModeStepAutoReset) && done;
            l.red[2] = reset_now ? 1 : 0;
            if (!reset_now) {
                st.num_unsat[b] = u_new;
                st.step[b] = step0 + 1;
                st.done[b] = done ? 1 : 0;
            }
        }
        __syncthreads();
        do_reset = (l.red[2] != 0);
    }

    if (do_reset) {
        // ---- reset (env:158-181): new problem, new assignment, masks --------
        int pidx;
        if (new_pidx != nullptr) {
            pidx = new_pidx[b];
        } else {
            const uint4 r = reset_rng_block(seed, ctr, (uint32_t)b, 0u);
            pidx = (int)(((uint64_t)r.x * (uint64_t)p.N) >> 32);
        }
        for (int v = tid; v < p.V; v += kThreads) {
            uint32_t x;
            if (new_assign != nullptr) {
                x = new_assign[(size_t)b * p.V + v] & 1u;
            } else {
                const uint4 r = reset_rng_block(seed, ctr, (uint32_t)b, 1u + (uint32_t)(v >> 7));
                const int lane = (v >> 5) & 3;
                const uint32_t wsel = lane == 0 ? r.x : lane == 1 ? r.y : lane == 2 ? r.z : r.w;
                x = (wsel >> (v & 31)) & 1u;
            }
            l.vinfo[v] = (uint16_t)(agent_of_var(p, v) | (x << 15));
        }
        for (int t = tid; t < p.A * p.W; t += kThreads) l.nbr[t] = 0u;
        if (tid < 2) l.red[tid] = 0;  // red[2] (reset broadcast) may still be read by slower waves
        __syncthreads();
        eval_clauses<false, true>(p, l, pool, pidx, sat_g, ntrue_g);
        __syncthreads();
        if (tid == 0) {
            st.num_unsat[b] = l.red[0];
            st.step[b] = 0;
            st.done[b] = 0;
            st.problem_idx[b] = pidx;
        }
        uint32_t *nbr_g = st.nbr_mask + (size_t)b * p.A * p.W;
        for (int t = tid; t < p.A * p.W; t += kThreads) nbr_g[t] = l.nbr[t];
    } else {
        const uint32_t *nbr_g = st.nbr_mask + (size_t)b * p.A * p.W;
        for (int t = tid; t < p.A * p.W; t += kThreads) l.nbr[t] = nbr_g[t];
    }
    for (int v = tid; v < p.V; v += kThreads) xg[v] = (uint8_t)(l.vinfo[v] >> 15);
    __syncthreads();
    write_obs<ObsT>(p, l, obs + (size_t)b * p.A * p.D);
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

// Per-env materialisation of the reference's mask tensors (env:99-128, :160).
__global__ void __launch_bounds__(kThreads)
env_masks_kernel(EnvParams p, const uint16_t *__restrict__ pool, msat_env_state st,
                 int32_t *__restrict__ acm, int32_t *__restrict__ anm, int32_t *__restrict__ l2a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const EnvLds l = carve(smem, p);
    const int b = blockIdx.x;
    for (int v = threadIdx.x; v < p.V; v += kThreads) l.vinfo[v] = (uint16_t)agent_of_var(p, v);
    const uint32_t *nbr_g = st.nbr_mask + (size_t)b * p.A * p.W;
    for (int t = threadIdx.x; t < p.A * p.W; t += kThreads) l.nbr[t] = nbr_g[t];
    __syncthreads();
    const uint64_t *prow = reinterpret_cast<const uint64_t *>(pool) + (size_t)st.problem_idx[b] * p.C;
    const int last_agent = agent_of_var(p, p.V - 1);  // var2agent[-1] wraps to the last var
    for (int c = threadIdx.x; c < p.C; c += kThreads) {
        const uint64_t w = prow[c];
        uint32_t info = 0, nullLit = 0;
        for (int j = 0; j < 3; ++j) {
            const uint32_t lit = (uint32_t)(w >> (16 * j)) & 0xFFFFu;
            uint32_t ag = kNoAgent;
            if (lit < MSAT_LIT_ABSENT) ag = l.vinfo[lit >> 1];
            if (lit == MSAT_LIT_NULL) nullLit = 1;
            info |= ag << (10 * j);
            if (l2a && j < p.K)
                l2a[((size_t)b * p.C + c) * p.K + j] = (lit == MSAT_LIT_NULL) ? last_agent : (int)ag;
        }
        l.clinfo[c] = info | (nullLit << 30);
    }
    __syncthreads();
    if (acm) {
        for (int t = threadIdx.x; t < p.A * p.C; t += kThreads) {
            const int i = t / p.C, c = t - (t / p.C) * p.C;
            const uint32_t info = l.clinfo[c], ui = (uint32_t)i;
            const bool small = (p.rem > 0) && (i >= p.rem);
            const bool rel = ((info & kNoAgent) == ui) | (((info >> 10) & kNoAgent) == ui) |
                             (((info >> 20) & kNoAgent) == ui) | (small && ((info >> 30) & 1u));
            acm[(size_t)b * p.A * p.C + t] = rel ? 1 : -1;
        }
    }
    if (anm) {
        for (int t = threadIdx.x; t < p.A * p.V; t += kThreads) {
            const int i = t / p.V, v = t - (t / p.V) * p.V;
            anm[(size_t)b * p.A * p.V + t] = ((l.nbr[i * p.W + (v >> 5)] >> (v & 31)) & 1u) ? 1 : -1;
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
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
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

// ------------------------------------------------------------- host glue ----

static int make_params(const msat_env_desc *d, EnvParams *p) {
    MSAT_REQUIRE(d != nullptr, "desc is NULL");
    MSAT_REQUIRE(d->num_envs >= 0, "num_envs < 0");
    MSAT_REQUIRE(d->num_vars >= 1 && d->num_vars <= 32000, "num_vars %d out of [1,32000]", d->num_vars);
    MSAT_REQUIRE(d->num_clauses >= 1, "num_clauses %d < 1", d->num_clauses);
    MSAT_REQUIRE(d->clause_width >= 1 && d->clause_width <= 3, "clause_width %d out of [1,3]", d->clause_width);
    MSAT_REQUIRE(d->num_agents >= 1 && d->num_agents <= 1000, "num_agents %d out of [1,1000]", d->num_agents);
    MSAT_REQUIRE(d->action_mode == 0 || d->action_mode == 1, "action_mode %d", d->action_mode);
    MSAT_REQUIRE(d->reward_mode == 0 || d->reward_mode == 1, "reward_mode %d", d->reward_mode);
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
    p->W = (p->V + 31) / 32;
    p->D = 2 * p->V + p->C;
    p->max_steps = d->max_steps;
    p->action_mode = d->action_mode;
    p->reward_mode = d->reward_mode;
    p->N = d->num_problems;
    p->r_clause = d->r_clause;
    p->r_sat = d->r_sat;
    p->gamma = d->gamma;
    return MSAT_OK;
}

static size_t env_lds_bytes(const EnvParams &p) {
    return (size_t)p.C * 4 + (size_t)p.A * p.W * 4 + 16 * 4 + (((size_t)p.V * 2 + 15) & ~(size_t)15);
}

static int check_state(const msat_env_state *st) {
    MSAT_REQUIRE(st != nullptr, "state is NULL");
    MSAT_REQUIRE(st->assign && st->clause_sat && st->num_unsat && st->step && st->done &&
                     st->problem_idx && st->nbr_mask,
                 "a required state pointer is NULL");
    return MSAT_OK;
}

template <int MODE>
static int launch_env(const EnvParams &p, const msat_env_desc *d, const uint16_t *pool,
                      const msat_env_state *st, const int32_t *actions, const uint8_t *mask,
                      const int32_t *npidx, const uint8_t *nassign, uint64_t seed, uint64_t ctr,
                      const msat_step_out *out, void *obs, hipStream_t s) {
    const size_t lds = env_lds_bytes(p);
    MSAT_REQUIRE(lds <= 160 * 1024, "env needs %zu B of LDS (> 160 KiB)", lds);
    msat_step_out o{};
    if (out) o = *out;
    if (p.B == 0) return MSAT_OK;
    if (d->obs_dtype == MSAT_OBS_I32)
        hipLaunchKernelGGL((env_kernel<MODE, int32_t>), dim3(p.B), dim3(kThreads), lds, s, p, pool, *st,
                           actions, mask, npidx, nassign, seed, ctr, o, (int32_t *)obs);
    else
        hipLaunchKernelGGL((env_kernel<MODE, int8_t>), dim3(p.B), dim3(kThreads), lds, s, p, pool, *st,
                           actions, mask, npidx, nassign, seed, ctr, o, (int8_t *)obs);
    return check_launch("env_kernel");
}

}  // namespace msat

using namespace msat;

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

extern "C" int msat_env_reset(const msat_env_desc *desc, const uint16_t *pool,
                              const msat_env_state *state, const uint8_t *reset_mask,
                              const int32_t *new_problem_idx, const uint8_t *new_assign,
                              uint64_t seed, uint64_t rng_counter, void *obs, void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if ((rc = check_state(state))) return rc;
    MSAT_REQUIRE(pool && obs, "NULL pool/obs");
    return launch_env<kModeReset>(p, desc, pool, state, nullptr, reset_mask, new_problem_idx, new_assign,
                                  seed, rng_counter, nullptr, obs, (hipStream_t)stream);
}

extern "C" int msat_env_step(const msat_env_desc *desc, const uint16_t *pool,
                             const msat_env_state *state, const int32_t *actions, int32_t autoreset,
                             const int32_t *new_problem_idx, const uint8_t *new_assign, uint64_t seed,
                             uint64_t rng_counter, const msat_step_out *out, void *obs, void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if ((rc = check_state(state))) return rc;
    MSAT_REQUIRE(pool && obs && actions, "NULL pool/obs/actions");
    MSAT_REQUIRE(out && out->reward && out->done && out->solved, "NULL step outputs");
    if (autoreset)
        return launch_env<kModeStepAutoReset>(p, desc, pool, state, actions, nullptr, new_problem_idx,
                                              new_assign, seed, rng_counter, out, obs, (hipStream_t)stream);
    return launch_env<kModeStep>(p, desc, pool, state, actions, nullptr, nullptr, nullptr, seed,
                                 rng_counter, out, obs, (hipStream_t)stream);
}

extern "C" int msat_env_obs(const msat_env_desc *desc, const uint16_t *pool, const msat_env_state *state,
                            void *obs, void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if ((rc = check_state(state))) return rc;
    MSAT_REQUIRE(pool && obs, "NULL pool/obs");
    return launch_env<kModeObs>(p, desc, pool, state, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, obs,
                                (hipStream_t)stream);
}

extern "C" int msat_env_masks(const msat_env_desc *desc, const uint16_t *pool,
                              const msat_env_state *state, int32_t *agent_clause_masks,
                              int32_t *agent_neighbor_masks, int32_t *literal_to_agent_idx,
                              void *stream) {
    EnvParams p;
    int rc = make_params(desc, &p);
    if (rc) return rc;
    if ((rc = check_state(state))) return rc;
    MSAT_REQUIRE(pool, "NULL pool");
    if (p.B == 0) return MSAT_OK;
    hipLaunchKernelGGL(env_masks_kernel, dim3(p.B), dim3(kThreads), env_lds_bytes(p), (hipStream_t)stream, p,
                       pool, *state, agent_clause_masks, agent_neighbor_masks, literal_to_agent_idx);
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

extern "C" int msat_static_var_features(const uint16_t *pool, int32_t num_problems, int32_t num_vars,
                                        int32_t num_clauses, float *var_features, void *stream) {
    MSAT_REQUIRE(pool && var_features, "NULL pointer");
    MSAT_REQUIRE(num_vars >= 1 && num_vars <= 32000 && num_clauses >= 1, "bad dims");
    if (num_problems == 0) return MSAT_OK;
    hipLaunchKernelGGL(static_var_features_kernel, dim3(num_problems), dim3(kThreads),
                       (size_t)num_vars * 8, (hipStream_t)stream, pool, num_vars, num_clauses, var_features);
    return check_launch("static_var_features_kernel");
}
