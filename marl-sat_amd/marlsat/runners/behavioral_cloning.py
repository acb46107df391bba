"""Behavioural-cloning data producer -- drop-in for the data side of src/runners/behavioral_cloning.py.

* ``load_expert_data(cnf_dir, sol_dir)`` (behavioral_cloning.py:29-50): ``<name>.sol`` files
  (first line: signed DIMACS model or 0/1 values; negatives become 0) paired with
  ``<name>.cnf``;
* ``compute_joint_labels_parallel_greedy(env, clauses, assignments, tau)`` (:54-100): the
  reference signature for one env, and ``compute_joint_labels`` for a whole batch -- both run
  ``msat_bc_greedy_labels`` (one workgroup per env evaluates every single-variable flip in one
  clause pass; the reference re-evaluates the formula once per candidate flip);
* ``preprocess(...)`` (:103-151): NUM_SAMPLES_PER_EXPERT corrupted copies of every expert
  solution (CORRUPTION_LEVEL distinct variables flipped), labelled with TAU_IMPROVE; the
  result is saved as ``.npz`` (instance ids, assignments, labels) -- the global GNN input is
  re-derived on the device from (instance, assignment), as in the MAPPO learner.
The BC training loop itself is outside this path.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import SATEnv, _lib
from ..envs.multi_agent_sat_env import ProblemPool
from ..utils.data_parser import clauses_array, load_cnf_problems


def load_expert_data(cnf_dir: str, sol_dir: str) -> List[Dict[str, np.ndarray]]:
    problems = {p["name"]: p for p in load_cnf_problems(cnf_dir)}
    out = []
    for sol in sorted(f for f in os.listdir(sol_dir) if f.endswith(".sol")):
        name = sol[: -len(".sol")] + ".cnf"
        if name not in problems:
            continue
        with open(os.path.join(sol_dir, sol)) as f:
            vals = [int(v) for v in f.readline().split()]
        out.append({"name": name, "problem_clauses": clauses_array(problems[name]),
                    "expert_solution": np.array([max(0, v) for v in vals], dtype=np.int32)})
    return out


def compute_joint_labels(env: SATEnv, pool: ProblemPool, problem_idx, assignments, tau: float = 0.0,
                         return_deltas: bool = False):
    """Batched labels (B, A) int32 (device): per agent the best single flip among its variables
    (local index) if it lowers the unsatisfied count by more than -tau, else the no-op index M."""
    dev = env.device
    pidx = torch.as_tensor(problem_idx, device=dev).to(torch.int32).contiguous()
    x = torch.as_tensor(assignments, device=dev).to(torch.uint8).contiguous()
    B = pidx.numel()
    if x.shape != (B, env.num_vars):
        raise ValueError(f"assignments must be (B, V) = ({B}, {env.num_vars})")
    labels = torch.empty((B, env.num_agents), dtype=torch.int32, device=dev)
    deltas = torch.empty((B, env.num_vars), dtype=torch.int32, device=dev) if return_deltas else None
    _lib.check(_lib.lib.msat_bc_greedy_labels(env._desc(B, pool), pool.packed.data_ptr(), pidx.data_ptr(),
                                              x.data_ptr(), float(tau), labels.data_ptr(), _lib.ptr(deltas),
                                              _lib.stream_ptr(dev)), "msat_bc_greedy_labels")
    return (labels, deltas) if return_deltas else labels


def compute_joint_labels_parallel_greedy(env: SATEnv, clauses: np.ndarray, assignments: np.ndarray,
                                         tau: float) -> np.ndarray:
    """behavioral_cloning.py:54-100 signature: one env's (C, K) clauses and (V,) assignment -> (A,) labels."""
    pool = env.make_pool(np.asarray(clauses, dtype=np.int32)[None])
    lab = compute_joint_labels(env, pool, [0], np.asarray(assignments)[None], tau)
    return lab[0].cpu().numpy()


def corrupt(solutions: np.ndarray, num_samples: int, level: int, seed: int = 0) -> np.ndarray:
    """(N, V) expert solutions -> (N * num_samples, V): `level` distinct variables flipped per copy
    (behavioral_cloning.py:121-124; numpy RNG instead of jax.random.choice)."""
    rng = np.random.default_rng(seed)
    N, V = solutions.shape
    out = np.repeat(solutions.astype(np.uint8), num_samples, axis=0)
    for r in range(out.shape[0]):
        out[r, rng.choice(V, size=min(level, V), replace=False)] ^= 1
    return out


def preprocess(expert_data: List[Dict[str, np.ndarray]], env: SATEnv, config: Optional[dict] = None,
               save_path: Optional[str] = None, seed: int = 0) -> Dict[str, np.ndarray]:
    bc = (config or {}).get("bc_training", {}) or {}
    S = int(bc.get("NUM_SAMPLES_PER_EXPERT", 5))
    level = int(bc.get("CORRUPTION_LEVEL", 3))
    tau = float(bc.get("TAU_IMPROVE", 0.0))
    clauses = np.stack([e["problem_clauses"] for e in expert_data])
    sols = np.stack([e["expert_solution"][: env.num_vars] for e in expert_data])
    pool = env.make_pool(clauses)
    x = corrupt(sols, S, level, seed)
    pidx = np.repeat(np.arange(len(expert_data), dtype=np.int32), S)
    labels = compute_joint_labels(env, pool, pidx, x, tau).cpu().numpy()
    data = {"problem_idx": pidx, "assignments": x, "labels": labels, "clauses": clauses}
    if save_path:
        np.savez_compressed(save_path, **data)
    return data
