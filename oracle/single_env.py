"""NumPy restatement of the single-agent SatEnv and the BC label generator -- TEST INFRASTRUCTURE.

* ``OracleSatEnv``: src/envs/sat_env.py:24-179 (one agent flips one variable per step,
  Discrete(V); delta reward ``(u(s) - u(s')) * 10 + c_bonus * [sat] - 0.005`` with
  u = unsat/C in float32, done = sat or step >= max_steps with the PRE-increment step,
  obs = GNN input with clause features [sat, unsat, 1]); vectorised over a leading env axis.
* ``compute_joint_labels_parallel_greedy``: src/runners/behavioral_cloning.py:54-100, literal
  (per agent, per valid local index: copy, flip, full re-evaluation through
  ``OracleSATEnv.satisfaction``, keep the first strictly better delta; label it if < tau).
Never imported by the product path.
"""
from __future__ import annotations

import numpy as np

from .sat_env import OracleSATEnv


def unsat_ratio(x: np.ndarray, clauses: np.ndarray) -> np.ndarray:
    """sat_env.py:168-175 (dense A_pos/A_neg products == literal evaluation) -> float32 (B,)."""
    sat, nun = OracleSATEnv.satisfaction(x, clauses)
    C = clauses.shape[-2]
    return (nun.astype(np.float32) / np.float32(C)).astype(np.float32)


class OracleSatEnv:
    def __init__(self, num_vars, num_clauses, max_clause_len=3, c_bonus=1.0, alpha=1.0, max_steps=128):
        self.num_vars, self.num_clauses = num_vars, num_clauses
        self.c_bonus, self.max_steps = np.float32(c_bonus), max_steps

    def reset(self, clauses: np.ndarray, x: np.ndarray):
        x = np.asarray(x, np.int32)
        return {"x": x.copy(), "step": np.zeros(x.shape[0], np.int32), "u": unsat_ratio(x, clauses),
                "clauses": clauses}

    def step(self, st, actions: np.ndarray):
        """sat_env.py:77-118 (a in [-V, V) flips var a mod V; other indices are dropped by the scatter)."""
        x = st["x"].copy()
        a = np.asarray(actions).astype(np.int64)
        a = np.where(a < 0, a + self.num_vars, a)  # x.at[a]: one negative wrap, then out-of-range drops
        ok = (a >= 0) & (a < self.num_vars)
        rows = np.nonzero(ok)[0]
        x[rows, a[ok]] = 1 - x[rows, a[ok]]
        u_new = unsat_ratio(x, st["clauses"])
        delta = (st["u"] - u_new).astype(np.float32)
        r = (delta * np.float32(10.0)).astype(np.float32)
        is_sat = u_new == np.float32(0.0)
        r = (r + np.where(is_sat, self.c_bonus, np.float32(0.0)).astype(np.float32)).astype(np.float32)
        r = (r + np.float32(-0.005)).astype(np.float32)
        done = is_sat | (st["step"] >= self.max_steps)
        nxt = {"x": x, "step": st["step"] + 1, "u": u_new, "clauses": st["clauses"]}
        return nxt, r, done

    def clause_features(self, st) -> np.ndarray:
        sat, _ = OracleSATEnv.satisfaction(st["x"], st["clauses"])
        s = sat.astype(np.float32)
        return np.stack([s, 1.0 - s, np.ones_like(s)], -1)


def compute_joint_labels_parallel_greedy(env: OracleSATEnv, clauses: np.ndarray, assignments: np.ndarray,
                                         tau: float) -> np.ndarray:
    """behavioral_cloning.py:54-100 for ONE env (clauses (C,K), assignments (V,))."""
    cl = clauses[None]
    _, base = env.satisfaction(assignments[None].astype(np.int32), cl)
    base = int(base[0])
    labels = []
    for i in range(env.num_agents):
        valid_local = np.flatnonzero(env.action_mask[i])
        glob = env.agent_vars[i][valid_local]
        best_delta, best = 0.0, env.max_vars_per_agent
        for j, g in enumerate(glob):
            t = assignments.astype(np.int32).copy()
            t[g] ^= 1
            _, nu = env.satisfaction(t[None], cl)
            d = float(int(nu[0]) - base)
            if d < best_delta:
                best_delta, best = d, int(valid_local[j])
        labels.append(best if best_delta < tau else env.max_vars_per_agent)
    return np.array(labels, dtype=np.int32)
