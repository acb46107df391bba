"""NumPy restatement of the MAPPO rollout math — TEST INFRASTRUCTURE.

GAE + normalisation: src/learners/mappo_gnn_sat_learner.py:504-532 (fp32, the
reference's operation order); schedules: :534-560 and
src/runners/mappo_runner.py:171-200.
"""
from __future__ import annotations

import numpy as np


def gae(reward_team, value, done, last_val, gamma: float, gae_lambda: float):
    """Reverse scan over T (learner:506-526) -> (advantages, targets) float32 (T,B)."""
    r = np.asarray(reward_team, np.float32)
    v = np.asarray(value, np.float32)
    d = np.asarray(done).astype(np.int32)
    g = np.float32(gamma)
    gl = np.float32(gamma * gae_lambda)  # python-float product, then weak-typed to f32
    T = r.shape[0]
    adv = np.zeros_like(r)
    a = np.zeros_like(np.asarray(last_val, np.float32))
    nv = np.asarray(last_val, np.float32)
    for t in range(T - 1, -1, -1):
        nd = (1 - d[t]).astype(np.float32)
        delta = (r[t] + (g * nv) * nd) - v[t]
        a = delta + (gl * nd) * a
        adv[t] = a
        nv = v[t]
    return adv, adv + v


def normalize(adv):
    """learner:529-532 — global (population) standardisation, computed in float64 then applied in f32."""
    a64 = np.asarray(adv, np.float64)
    mean = a64.mean()
    std = a64.std() + 1e-8
    return ((np.asarray(adv, np.float32) - np.float32(mean)) / np.float32(std)).astype(np.float32), mean, std


def ent_coef(update_idx, cfg):
    """learner:534-558."""
    if not cfg.get("ANNEAL_ENT", False):
        return float(cfg["ENT_COEF"])
    n = cfg["NUM_UPDATES"]
    start, end = cfg["ENT_COEF"], cfg.get("ENT_COEF_END", 0.0)
    s_upd = n * (1.0 - cfg.get("ANNEAL_ENT_FRAC", 0.333))
    frac = min(1.0, max(0.0, (update_idx - s_upd) / (n - s_upd)))
    return start - (start - end) * frac if update_idx >= s_upd else start


def learning_rate(count, cfg):
    """mappo_runner.py:171-193 — optax.linear_schedule over Adam step counts."""
    if not cfg.get("ANNEAL_LR", False):
        return cfg.get("LEARNING_RATE", 3e-4)
    n = cfg.get("NUM_UPDATES", 1)
    lr0 = cfg.get("LEARNING_RATE", 3e-4) * cfg.get("LR_START_FACTOR", 1.0)
    lr1 = cfg.get("LR_END_FLOOR", 1e-5)
    frac = 1.0 - min(max(count, 0), n) / n
    return (lr0 - lr1) * frac + lr1
