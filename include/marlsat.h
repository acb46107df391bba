/*
 * marlsat.h — C-ABI of libmarlsat.so, the MI355X (gfx950) implementation of the
 * marl-sat data-parallel hot path: the batched multi-agent SAT environment
 * (reset / step / auto-reset / local observations) and the MAPPO rollout math
 * around it (GAE + advantage normalisation).
 *
 * Every pointer is a DEVICE pointer owned by the caller (torch tensors on the
 * Python side); dims are passed explicitly; the stream is the last argument and
 * every call only enqueues work on it (no implicit device synchronisation, no
 * allocation on the hot path).  Return value: 0 on success, negative on error
 * (MSAT_EBADARG / MSAT_EHIP); msat_last_error() returns a thread-local message.
 *
 * Reference interfaces replaced (paths relative to kongqg/marl-sat):
 *   msat_pool_pack           <- jnp.abs(clauses)-1 literal decoding shared by
 *                               src/envs/multi_agent_sat_env.py:135-144 and :100
 *   msat_pool_agent_tables   <- _compute_observation_maps  src/envs/multi_agent_sat_env.py:99-128
 *                               (hoisted from every reset to once per pool instance)
 *   msat_env_reset           <- SATEnv.reset               src/envs/multi_agent_sat_env.py:158-181
 *                               (+ _compute_observation_maps :99-128, get_obs :345-398)
 *   msat_env_step            <- SATEnv.step_env            src/envs/multi_agent_sat_env.py:225-284
 *                               (flip decode :230-250, _calculate_satisfaction_explicit
 *                               :130-156, _calculate_rewards :183-198 / PBRS :201-223)
 *                               autoreset=1 additionally replaces the rollout's
 *                               reset-all-then-where-select  src/learners/mappo_gnn_sat_learner.py:422-464
 *   msat_env_obs             <- SATEnv.get_obs              src/envs/multi_agent_sat_env.py:345-398
 *   msat_env_masks           <- SATState.agent_clause_masks / agent_neighbor_masks /
 *                               literal_to_agent_idx        src/envs/multi_agent_sat_env.py:160-161
 *   msat_clause_features     <- SATDataWrapper._calculate_dynamic_clause_features
 *                               src/learners/mappo_gnn_sat_learner.py:176-195
 *   msat_static_var_features <- SATDataWrapper._state_to_gnn_input degrees
 *                               src/learners/mappo_gnn_sat_learner.py:150-164
 *   msat_gae                 <- _calculate_gae + global normalisation
 *                               src/learners/mappo_gnn_sat_learner.py:504-532
 */
#ifndef MARLSAT_H
#define MARLSAT_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSAT_OK 0
#define MSAT_EBADARG (-1)
#define MSAT_EHIP (-2)
#define MSAT_ECOMM (-3)

/* packed literal codes (uint16 per literal slot, clause rows padded to 4 slots) */
#define MSAT_LIT_NULL 0xFFFFu   /* literal value 0 in the int32 input: always false,  */
                                /* and (reference quirk) "matches" padded agent slots */
#define MSAT_LIT_ABSENT 0xFFFEu /* padding slot beyond the clause width: inert        */
#define MSAT_LIT_SLOTS 4

/* obs element type */
#define MSAT_OBS_I32 0 /* reference dtype (jnp.int32)                */
#define MSAT_OBS_I8 1  /* same values {-1,0,1}, 4x fewer bytes        */

/* reward modes */
#define MSAT_REWARD_SPARSE 0 /* active reference reward: 1.0 on solve else 0 (env:183-198) */
#define MSAT_REWARD_PBRS 1   /* commented reference variant (env:201-223)                  */
#define MSAT_REWARD_SINGLE_DELTA 2 /* single-agent SatEnv (src/envs/sat_env.py:77-118): f32     */
                                   /* ((u_prev - u_new) * 10 + r_sat * solved) - 0.005, u =      */
                                   /* unsat/C; done = solved || step >= max_steps (pre-increment) */

/* Static description of one batch of environments (all envs share V, C, K, A). */
typedef struct msat_env_desc {
    int32_t num_envs;           /* B */
    int32_t num_vars;           /* V  (<= 32000) */
    int32_t num_clauses;        /* C */
    int32_t clause_width;       /* K  (1..3) */
    int32_t num_agents;         /* A  (<= 1000); contiguous partition, first V%A agents get V/A+1 vars */
    int32_t max_vars_per_agent; /* M = ceil(V/A) */
    int32_t max_steps;          /* MAX_STEPS */
    int32_t action_mode;        /* 0 single-flip Discrete(M+1), 1 multi-flip MultiDiscrete([2]*M) */
    int32_t reward_mode;        /* MSAT_REWARD_* */
    int32_t obs_dtype;          /* MSAT_OBS_* */
    int32_t num_problems;       /* N instances in the device problem pool */
    float r_clause;             /* PBRS only */
    float r_sat;                /* PBRS only */
    float gamma;                /* PBRS only */
} msat_env_desc;

/* Device problem pool: packed literals + per-instance agent tables.  The tables
 * depend only on the instance and the agent partition (the reference recomputes
 * them on every reset, env:99-128), so they are built once per pool. */
typedef struct msat_pool {
    const uint16_t *lits; /* (N,C,4)  packed literal codes                          */
    const uint32_t *rel;  /* (N,A,WC) agent-clause relation bits, WC = 2*ceil(C/64) */
    const uint32_t *nbr;  /* (N,A,WV) agent neighbour-var bits,  WV = 2*ceil(V/64)  */
} msat_pool;

/* Device-resident batch state (structure of arrays, leading dim B). */
typedef struct msat_env_state {
    uint8_t *assign;      /* (B,V)   variable_assignments in {0,1}           */
    uint8_t *clause_sat;  /* (B,C)   clauses_satisfied_status                */
    uint8_t *clause_ntrue;/* (B,C)   #true literals per clause (nullable)    */
    int32_t *num_unsat;   /* (B,)    num_unsatisfied                         */
    int32_t *step;        /* (B,)    step                                    */
    uint8_t *done;        /* (B,)    done (every agent shares it)            */
    int32_t *problem_idx; /* (B,)    row of the problem pool this env solves */
    /* Reset queue (nullable; msat_reset_queue_words(B) zeroed uint32 words, 16-byte aligned, owned by the state like
     * the arrays above): each msat_env_step(autoreset=1) launch marks the envs whose NEXT step times out (their step
     * counter reaches max_steps - 1; the reference's timed_out, env:256-260), and the next launch resets the first
     * B/256 + 8 of them (rounded up to a multiple of 8; in index order) in workgroups of their own, beside the step workgroups, instead of serially
     * behind their step (their step workgroup then writes only the transition outputs, the assignment, step, done
     * and problem_idx).  Results are identical with or without it.  Used by the sparse reward mode with mode-0
     * actions and fewer than 64 agents (B a multiple of 4); the other state-modifying calls clear the entries of the
     * envs they touch.  A caller that writes the state arrays directly must zero the queue (or pass NULL).
     * reset_serial: the launch's serial, +1 per msat_env_step(autoreset=1) call on this state; a launch uses the
     * marks only if the previous launch on the state had serial reset_serial - 1. */
    uint32_t *reset_queue;
    uint32_t reset_serial;
} msat_env_state;

/* uint32 words of a msat_env_state.reset_queue for B envs. */
size_t msat_reset_queue_words(int32_t num_envs);

/* Step outputs that are NOT state (they describe the transition that was taken). */
typedef struct msat_step_out {
    float *reward;          /* (B,)  team reward (identical for every agent)        */
    uint8_t *done;          /* (B,)  dones["__all__"] of the step (pre-reset)        */
    uint8_t *solved;        /* (B,)  infos["solved"]                                 */
    int32_t *num_unsat;     /* (B,)  infos["num_unsatisfied"]  (nullable)            */
    int32_t *episode_step;  /* (B,)  infos["episode_step"]     (nullable)            */
    /* Diagnostics, not reference state (nullable; NULL in every product call): per env 8 words from
     * its workgroup's wave 0 -- [0] shader-clock counter delta (s_memtime) and [1] 100 MHz real-time
     * counter delta over the workgroup's run (clock MHz = 100 * [0] / [1]); [2] real time at its
     * start, [3..6] at the end of four phases (assignment in LDS, clause scan, agent tables staged,
     * obs bit images built; 0 where a phase does not run), [7] at its end after its stores drained.
     * bench.py reads it for the clock and the phase breakdown of its env steps. */
    uint64_t *clock_stamps; /* (B,8) */
} msat_step_out;

const char *msat_last_error(void);
int msat_version(void); /* 3: msat_env_state carries reset_queue / reset_serial (version 2 had neither), 2:
                         * msat_step_out carries clock_stamps (version 1 had no such field) */

/* Pack an int32 literal tensor (N,C,K) (signed, 1-based, 0 = null literal) into
 * the device pool layout uint16 (N,C,4).  Literals with |l| > V set *err_flag
 * (device int32, caller zeroes it) to 1. */
int msat_pool_pack(const int32_t *lits, int32_t num_problems, int32_t num_clauses,
                   int32_t clause_width, int32_t num_vars, uint16_t *pool,
                   int32_t *err_flag, void *stream);

/* Build the per-instance agent tables of a packed pool for desc's partition
 * (desc->num_problems rows): rel (N,A,WC) and nbr (N,A,WV) uint32 bit words.
 * Reproduces _compute_observation_maps (env:99-128) incl. the literal-0 quirk. */
int msat_pool_agent_tables(const msat_env_desc *desc, const uint16_t *lits,
                           uint32_t *rel, uint32_t *nbr, void *stream);

/* Reset the envs with reset_mask[b] != 0 (NULL: all envs).
 * new_problem_idx (B,) and new_assign (B,V) are explicit inputs for exact-parity
 * runs; when NULL they are drawn from the counter-based RNG (Philox4x32-10 keyed
 * by seed, counter=(rng_counter, env)).  Writes every state field of the reset
 * envs (step=0, done=0) and their observations obs (B,A,D), D = 2V+C. */
int msat_env_reset(const msat_env_desc *desc, const msat_pool *pool,
                   const msat_env_state *state, const uint8_t *reset_mask,
                   const int32_t *new_problem_idx, const uint8_t *new_assign,
                   uint64_t seed, uint64_t rng_counter, void *obs, void *stream);

/* One batched SATEnv.step_env.  actions: (B,A) int32 (mode 0) or (B,A,M) int32
 * (mode 1, values 0/1: MultiDiscrete([2]*m); the state keeps one bit per variable, so bit 0
 * is applied — the reference's integer XOR with other values (env:246-250) leaves non-binary
 * assignments, and the Python facade rejects such actions before the call).  autoreset=0: pure step_env (state/obs are the stepped ones).
 * autoreset=1: the rollout's auto-reset — envs whose step is done are reset
 * (problem index / assignment from the explicit arrays or the RNG, exactly as
 * msat_env_reset) and state/obs hold the post-reset values, while `out` holds
 * the pre-reset reward/done/info of the step, as in the reference rollout. */
int msat_env_step(const msat_env_desc *desc, const msat_pool *pool,
                  const msat_env_state *state, const int32_t *actions,
                  int32_t autoreset, const int32_t *new_problem_idx,
                  const uint8_t *new_assign, uint64_t seed, uint64_t rng_counter,
                  const msat_step_out *out, void *obs, void *stream);

/* Ragged batches (BASELINE config 5: mixed uf50/uf100/uf200): up to MSAT_MAX_GROUPS size
 * classes, each a homogeneous batch with its own desc / pool / state / obs / actions / outs,
 * advanced by ONE kernel launch (no padding to the largest instance; the reference cannot
 * mix sizes at all, runner:118 jnp.stack).  Resets draw from the counter RNG only, class g
 * keyed by seed ^ (g * 0x9E3779B97F4A7C15) -- bit-identical to msat_env_reset / msat_env_step
 * of that class alone with that seed.  All classes share obs_dtype. */
#define MSAT_MAX_GROUPS 8
int msat_env_reset_grouped(int32_t num_groups, const msat_env_desc *descs, const msat_pool *pools,
                           const msat_env_state *states, uint64_t seed, uint64_t rng_counter,
                           void *const *obs, void *stream);
int msat_env_step_grouped(int32_t num_groups, const msat_env_desc *descs, const msat_pool *pools,
                          const msat_env_state *states, const int32_t *const *actions, int32_t autoreset,
                          uint64_t seed, uint64_t rng_counter, const msat_step_out *outs, void *const *obs,
                          void *stream);

/* obs may be NULL in msat_env_reset / msat_env_step: state-only update, no observation write
 * (the single-agent SatEnv observes the GNN input instead, src/envs/sat_env.py:120-166). */

/* Behavioural-cloning joint labels: compute_joint_labels_parallel_greedy
 * (src/runners/behavioral_cloning.py:54-100) for B envs (desc->num_envs) given explicit
 * problem_idx (B,) into the packed pool lits and assignments (B,V) u8: per agent, the first
 * local var index whose single flip lowers the unsatisfied-clause count the most, if that
 * delta < tau, else the no-op index M.  labels (B,A) int32; deltas (B,V) int32 (nullable) =
 * unsat(x with v flipped) - unsat(x). */
int msat_bc_greedy_labels(const msat_env_desc *desc, const uint16_t *lits, const int32_t *problem_idx,
                          const uint8_t *assign, float tau, int32_t *labels, int32_t *deltas, void *stream);

/* Single-agent SatEnv clause features [is_sat, is_unsat, 1] (B,C,3) (src/envs/sat_env.py:143-160). */
int msat_clause_sat_features(const msat_env_desc *desc, const msat_env_state *state,
                             float *clause_features, void *stream);

/* SATEnv.get_obs (env:345-398) of the current state, without changing it. */
int msat_env_obs(const msat_env_desc *desc, const msat_pool *pool,
                 const msat_env_state *state, void *obs, void *stream);

/* Materialise the reference's per-env static mask tensors (cold path):
 * agent_clause_masks (B,A,C) int32 +-1, agent_neighbor_masks (B,A,V) int32 +-1,
 * literal_to_agent_idx (B,C,K) int32.  Any output pointer may be NULL. */
int msat_env_masks(const msat_env_desc *desc, const msat_pool *pool,
                   const msat_env_state *state, int32_t *agent_clause_masks,
                   int32_t *agent_neighbor_masks, int32_t *literal_to_agent_idx,
                   void *stream);

/* Dynamic clause features (B,C,3) float32 = [is_sat, ntrue/3, 1]. */
int msat_clause_features(const msat_env_desc *desc, const msat_env_state *state,
                         float *clause_features, void *stream);

/* Static variable features (N,V,3) float32 = [deg+/C, deg-/C, 0] per pool row. */
int msat_static_var_features(const uint16_t *pool, int32_t num_problems,
                             int32_t num_vars, int32_t num_clauses,
                             float *var_features, void *stream);

/* GAE over a (T,B) rollout + global normalisation over all T*B entries.
 * reward: team reward with row stride reward_stride (elements) per (t,b)
 * (reward[...,0] of the reference's (T,B,A) reward; stride 1 for a (T,B) tensor).
 * done: (T,B) uint8.  value: (T,B).  last_val: (B,).
 * gamma_lambda is GAMMA*GAE_LAMBDA rounded once to float32 (the reference
 * multiplies the two Python floats before the fp32 arithmetic).
 * advantages/targets: (T,B) outputs (advantages normalised when normalize!=0,
 * targets = raw advantages + value).  workspace: >= msat_gae_workspace_bytes(T,B)
 * bytes; after the call workspace holds (double) the mean and the std+1e-8 used. */
size_t msat_gae_workspace_bytes(int32_t T, int32_t B);
int msat_gae(int32_t T, int32_t B, const float *reward, int32_t reward_stride,
             const uint8_t *done, const float *value, const float *last_val,
             float gamma, float gamma_lambda, int32_t normalize, float *advantages,
             float *targets, void *workspace, void *stream);

/* Global-normalisation pieces for multi-GPU GAE (the reference normalises over ALL
 * T*B advantages, learner:529-532): per-rank moments (fp64 sum, sum of squares;
 * workspace >= 2*1024 doubles), all-reduced by the caller, then x = (x - mean)/std. */
int msat_moments(const float *x, size_t n, double *out2, void *workspace, void *stream);
int msat_standardize(float *x, size_t n, float mean, float stdv, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* MARLSAT_H */
