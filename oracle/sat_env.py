"""NumPy restatement of the reference multi-agent SAT environment — TEST INFRASTRUCTURE.

Restates, vectorised over a leading env axis B, the algorithm of
``src/envs/multi_agent_sat_env.py`` (kongqg/marl-sat @ 2025-10-31) and the
global-state features of ``SATDataWrapper`` (``src/learners/mappo_gnn_sat_learner.py``)
and ``create_static_graph`` (``src/utils/graph_constructor.py``), including the
reference's quirks (literal 0 -> var index -1, which JAX/NumPy gathers wrap to
the last variable and which "matches" the -1 padding of ``agent_vars``).

It is the checker for the HIP kernels and the timed CPU baseline of bench.py
(same algorithm as the reference: full clause rescan, dense int32 obs,
mask recomputation on every reset).  Never imported by the product path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace
from typing import Dict, List, Optional

import numpy as np


def find_factors(n: int) -> List[int]:
    """env:286-293."""
    out = set()
    for i in range(1, int(math.sqrt(n)) + 1):
        if n % i == 0:
            out.add(i)
            out.add(n // i)
    return sorted(out)


def create_agent_groups(num_vars: int, vars_per_agent: Optional[int]) -> Dict[str, List[int]]:
    """env:294-338 — contiguous groups; the first V % A agents get one extra var."""
    if vars_per_agent is not None:
        num_agents = math.ceil(num_vars / vars_per_agent)
    else:
        cands = [f for f in find_factors(num_vars) if 4 <= f <= 4]
        num_agents = num_vars // max(cands) if cands else max(2, int(math.sqrt(num_vars)))
    base, rem = divmod(num_vars, num_agents)
    groups, cur = {}, 0
    for i in range(num_agents):
        size = base + 1 if i < rem else base
        groups[f"agent_{i}"] = list(range(cur, cur + size))
        cur += size
    return groups


@dataclass
class OracleState:
    """SATState (env:13-24) with a leading env axis."""

    variable_assignments: np.ndarray  # (B,V) int32
    clauses_satisfied_status: np.ndarray  # (B,C) bool
    num_unsatisfied: np.ndarray  # (B,) int32
    step: np.ndarray  # (B,) int32
    done: np.ndarray  # (B,A) bool
    clauses: np.ndarray  # (B,C,K) int32
    agent_clause_masks: np.ndarray  # (B,A,C) int32 +-1
    agent_neighbor_masks: np.ndarray  # (B,A,V) int32 +-1
    literal_to_agent_idx: np.ndarray  # (B,C,K) int32


class OracleSATEnv:
    def __init__(self, num_vars, num_clauses, max_steps, vars_per_agent=None, action_mode=0,
                 r_clause=0.02, r_sat=1.0, gamma=0.99, reward_mode=0):
        self.num_vars, self.num_clauses, self.max_steps = num_vars, num_clauses, max_steps
        self.action_mode, self.reward_mode = action_mode, reward_mode
        self.r_clause, self.r_sat, self.gamma = r_clause, r_sat, gamma
        self.agent_groups = create_agent_groups(num_vars, vars_per_agent)
        self.agents = list(self.agent_groups)
        self.num_agents = len(self.agents)
        self.max_vars_per_agent = max(len(v) for v in self.agent_groups.values())
        A, M, V = self.num_agents, self.max_vars_per_agent, num_vars
        # env:61-67
        self.agent_vars = np.full((A, M), -1, dtype=np.int32)
        self.action_mask = np.zeros((A, M), dtype=bool)
        for i, a in enumerate(self.agents):
            g = self.agent_groups[a]
            self.agent_vars[i, : len(g)] = g
            self.action_mask[i, : len(g)] = True
        # env:92-97
        self.variable_to_agent_idx = np.full((V,), -1, dtype=np.int32)
        for i, a in enumerate(self.agents):
            self.variable_to_agent_idx[self.agent_groups[a]] = i
        self.own = np.zeros((A, V), dtype=bool)
        for i, a in enumerate(self.agents):
            self.own[i, self.agent_groups[a]] = True
        self.obs_dim = 2 * V + num_clauses  # env:340-343

    # ------------------------------------------------------------ masks ----
    def observation_maps(self, clauses: np.ndarray):
        """env:99-128 -> agent_clause_masks (B,A,C), agent_neighbor_masks (B,A,V), both +-1."""
        vidx = np.abs(clauses).astype(np.int64) - 1  # (B,C,K); literal 0 -> -1
        B, C, K = vidx.shape
        V = self.num_vars
        # matches[b,i,c] = any_{j,k} vidx[b,c,j] == agent_vars[i,k]  (-1 == padded -1 counts)
        related = np.zeros((B, self.num_agents, C), dtype=bool)
        for j in range(K):
            related |= (vidx[:, None, :, j, None] == self.agent_vars[None, :, None, :]).any(-1)
        acm = np.where(related, 1, -1).astype(np.int32)
        # vars appearing in a related clause (the -1 entries match no var in arange(V))
        occ = np.zeros((B, C, V), dtype=np.float32)
        bb, cc = np.meshgrid(np.arange(B), np.arange(C), indexing="ij")
        for j in range(K):
            vj = vidx[:, :, j]
            ok = vj >= 0
            occ[bb[ok], cc[ok], vj[ok]] = 1.0
        rel_var = np.matmul(related.astype(np.float32), occ) > 0  # (B,A,C)@(B,C,V)
        nbr = rel_var & ~self.own[None]
        anm = np.where(nbr, 1, -1).astype(np.int32)
        return acm, anm

    def literal_to_agent(self, clauses: np.ndarray) -> np.ndarray:
        """env:160 — var2agent[|l|-1]; literal 0 wraps to the last var."""
        return self.variable_to_agent_idx[np.abs(clauses) - 1]

    # ---------------------------------------------------- satisfaction ----
    @staticmethod
    def satisfaction(x: np.ndarray, clauses: np.ndarray):
        """env:130-156 -> (status (B,C) bool, num_unsat (B,) int32)."""
        vidx = np.abs(clauses) - 1
        B = x.shape[0]
        vals = x[np.arange(B)[:, None, None], vidx]  # negative index wraps like the JAX gather
        truth = ((clauses > 0) & (vals == 1)) | ((clauses < 0) & (vals == 0))
        status = truth.any(axis=-1)
        return status, (~status).sum(axis=-1).astype(np.int32)

    @staticmethod
    def num_true_literals(x: np.ndarray, clauses: np.ndarray) -> np.ndarray:
        vidx = np.abs(clauses) - 1
        vals = x[np.arange(x.shape[0])[:, None, None], vidx]
        truth = ((clauses > 0) & (vals == 1)) | ((clauses < 0) & (vals == 0))
        return truth.sum(axis=-1).astype(np.int32)

    # ------------------------------------------------------------ reset ----
    def reset(self, clauses: np.ndarray, x: np.ndarray):
        """env:158-181 with the assignment given explicitly (no JAX RNG here)."""
        clauses = np.asarray(clauses, dtype=np.int32)
        x = np.asarray(x, dtype=np.int32)
        B = clauses.shape[0]
        acm, anm = self.observation_maps(clauses)
        status, nun = self.satisfaction(x, clauses)
        st = OracleState(
            variable_assignments=x, clauses_satisfied_status=status, num_unsatisfied=nun,
            step=np.zeros((B,), np.int32), done=np.zeros((B, self.num_agents), bool), clauses=clauses,
            agent_clause_masks=acm, agent_neighbor_masks=anm,
            literal_to_agent_idx=self.literal_to_agent(clauses),
        )
        return self.get_obs(st), st

    # ------------------------------------------------------------- step ----
    def decode_flips(self, x: np.ndarray, actions: np.ndarray) -> np.ndarray:
        """env:230-250 -> new assignment (B,V) int32."""
        B, V = x.shape
        A, M = self.num_agents, self.max_vars_per_agent
        actions = np.asarray(actions, dtype=np.int64)
        if self.action_mode == 0:
            n = self.action_mask.sum(-1)[None, :]  # (1,A)
            is_noop = actions >= n
            safe = np.minimum(actions, n - 1)
            safe = np.where(safe < 0, safe + M, safe)  # jnp index normalisation
            safe = np.clip(safe, 0, M - 1)  # out-of-bound gathers clamp
            var = self.agent_vars[np.arange(A)[None, :], safe]
            var = np.where(is_noop, -1, var)
            flip = np.zeros((B, V), np.int32)
            bb, aa = np.nonzero(var >= 0)
            np.add.at(flip, (bb, var[bb, aa]), 1)  # one_hot(-1) == 0
            return np.logical_xor(x, flip).astype(np.int32)
        new = x.copy()
        ia, ja = np.nonzero(self.action_mask)
        vv = self.agent_vars[ia, ja]
        new[:, vv] = x[:, vv] ^ actions[:, ia, ja].astype(np.int32)
        return new

    def step(self, state: OracleState, actions: np.ndarray):
        """env:225-284 -> (obs, next_state, reward (B,), done (B,), info dict)."""
        x1 = self.decode_flips(state.variable_assignments, actions)
        status, nun = self.satisfaction(x1, state.clauses)
        solved = nun == 0
        timed_out = state.step + 1 >= self.max_steps
        done = solved | timed_out
        nxt = replace(state, variable_assignments=x1, clauses_satisfied_status=status, num_unsatisfied=nun,
                      step=state.step + 1, done=np.repeat(done[:, None], self.num_agents, 1))
        reward = self.rewards(state, nxt, solved)
        info = {"solved": solved, "num_unsatisfied": nun, "episode_step": state.step + 1}
        return self.get_obs(nxt), nxt, reward, done, info

    def rewards(self, state: OracleState, nxt: OracleState, solved: np.ndarray) -> np.ndarray:
        if self.reward_mode == 0:  # env:183-198 (active)
            return np.where(solved, 1.0, 0.0).astype(np.float32)
        # env:201-223 (commented PBRS variant), fp32 arithmetic in reference order
        g = np.float32(self.gamma)
        r_pbrs = g * (-nxt.num_unsatisfied).astype(np.float32) - (-state.num_unsatisfied).astype(np.float32)
        newly = (nxt.clauses_satisfied_status & ~state.clauses_satisfied_status).astype(np.float32).sum(-1)
        r_cl = newly.astype(np.float32) * np.float32(self.r_clause)
        r_s = np.where(solved, np.float32(self.r_sat), np.float32(0.0))
        return ((r_pbrs + r_cl) + r_s).astype(np.float32)

    def step_autoreset(self, state: OracleState, actions, new_clauses, new_x):
        """learner:418-464 — step, reset ALL envs, where(done) select (the reference rollout)."""
        obs, nxt, reward, done, info = self.step(state, actions)
        obs_r, st_r = self.reset(new_clauses, new_x)
        sel = lambda old, new: np.where(done.reshape(done.shape + (1,) * (old.ndim - 1)), new, old)
        merged = OracleState(**{f: sel(getattr(nxt, f), getattr(st_r, f)) for f in nxt.__dataclass_fields__})
        return sel(obs, obs_r), merged, reward, done, info

    # -------------------------------------------------------------- obs ----
    def get_obs(self, state: OracleState) -> np.ndarray:
        """env:345-398 -> (B,A,D) int32."""
        x = state.variable_assignments[:, None, :]  # (B,1,V)
        own = np.where(self.own[None], x, -1)
        cl = np.where(state.agent_clause_masks == 1,
                      np.where(state.clauses_satisfied_status[:, None, :] == 1, 1, 0), -1)
        nb = np.where(state.agent_neighbor_masks != -1, state.agent_neighbor_masks * x, -1)
        return np.concatenate([own, cl, nb], axis=-1).astype(np.int32)

    # ------------------------------------------------ wrapper features ----
    def clause_features(self, state: OracleState) -> np.ndarray:
        """learner:176-195 -> (B,C,3) float32 [is_sat, #true/3, 1]."""
        n = self.num_true_literals(state.variable_assignments, state.clauses)
        is_sat = state.clauses_satisfied_status.astype(np.float32)
        return np.stack([is_sat, n.astype(np.float32) / np.float32(3.0), np.ones_like(is_sat)], -1)

    def static_graph(self, clauses: np.ndarray):
        """graph_constructor.py:93-114 -> A_pos, A_neg (B,V,C) float32 (duplicates add)."""
        clauses = np.asarray(clauses)
        B, C, K = clauses.shape
        V = self.num_vars
        vidx = np.abs(clauses) - 1
        A_pos = np.zeros((B, V, C), np.float32)
        A_neg = np.zeros((B, V, C), np.float32)
        bb = np.broadcast_to(np.arange(B)[:, None, None], clauses.shape)
        cc = np.broadcast_to(np.arange(C)[None, :, None], clauses.shape)
        np.add.at(A_pos, (bb, vidx, cc), (clauses > 0).astype(np.float32))
        np.add.at(A_neg, (bb, vidx, cc), (clauses < 0).astype(np.float32))
        return A_pos, A_neg

    def static_var_features(self, clauses: np.ndarray) -> np.ndarray:
        """learner:150-164 -> (B,V,3) float32 [deg+/C, deg-/C, 0]."""
        A_pos, A_neg = self.static_graph(clauses)
        C = np.asarray(clauses).shape[1]
        pos = A_pos.sum(-1, keepdims=True) / np.float32(C)
        neg = A_neg.sum(-1, keepdims=True) / np.float32(C)
        return np.concatenate([pos, neg, np.zeros_like(pos)], -1).astype(np.float32)
