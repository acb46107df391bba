"""Single-agent SAT environment -- batched drop-in for src/envs/sat_env.py ``SatEnv``.

One agent (``agent_0``) flips one variable per step (``Discrete(num_vars)``):
  * reward  ``(u(s) - u(s')) * 10 + c_bonus * [sat] - 0.005``, u = unsatisfied / C (f32, the
    reference's operation order, sat_env.py:86-101);
  * done    ``sat or step >= max_steps`` with the step BEFORE the increment (sat_env.py:106);
  * obs     ``{"agent_0": GNNInput}`` with clause features ``[is_sat, is_unsat, 1]``
            (sat_env.py:120-166) -- the GNN input, not a local observation vector.

It runs on the multi-agent env kernel with one agent owning every variable
(``MSAT_REWARD_SINGLE_DELTA``, no observation write): the same fused flip + clause
scan, so a step costs one launch over the whole batch.  ``alpha`` and
``max_clause_len`` are accepted for API compatibility (the reference stores and
never uses them).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .. import _lib
from ..random import as_key
from .multi_agent_sat_env import ProblemPool, SATEnv, SATState
from .spaces import Box, Discrete


@dataclass
class SatGNNInput:
    """graph_constructor.GNNInput of the single-agent env (batched); dense adjacency on demand."""

    static_var_features: torch.Tensor  # (B,V,3)
    assignment: torch.Tensor  # (B,V)
    clause_features: torch.Tensor  # (B,C,3) [sat, unsat, 1]
    _state: SATState

    @property
    def A_pos(self) -> torch.Tensor:
        from ..learners.mappo_gnn_sat_learner import GNNInput

        return GNNInput(self.static_var_features, self.assignment, self.clause_features, self._state).A_pos

    @property
    def A_neg(self) -> torch.Tensor:
        from ..learners.mappo_gnn_sat_learner import GNNInput

        return GNNInput(self.static_var_features, self.assignment, self.clause_features, self._state).A_neg


class SatEnv:
    """Batched single-agent SatEnv (sat_env.py:24-179)."""

    def __init__(self, num_vars, num_clauses, max_clause_len=3, c_bonus=1.0, alpha=1.0, max_steps=128, device=None):
        self.num_agents = 1
        self.agents = ["agent_0"]
        self.num_vars, self.num_clauses = int(num_vars), int(num_clauses)
        self.max_clause_len, self.c_bonus, self.alpha, self.max_steps = max_clause_len, float(c_bonus), alpha, max_steps
        self.observation_spaces = {a: Box(-np.inf, np.inf, (1,)) for a in self.agents}
        self.action_spaces = {a: Discrete(self.num_vars) for a in self.agents}
        self._env = SATEnv(self.num_vars, self.num_clauses, max_steps, vars_per_agent=self.num_vars, action_mode=0,
                           r_sat=self.c_bonus, reward_mode=_lib.REWARD_SINGLE_DELTA, device=device)
        self.device = self._env.device

    @property
    def name(self) -> str:
        return "SATEnv"

    @property
    def agent_classes(self) -> dict:
        return {"agents": self.agents}

    def action_space(self, agent: str):
        return self.action_spaces[agent]

    def observation_space(self, agent: str):
        return self.observation_spaces[agent]

    # ------------------------------------------------------------------------
    def _pool(self, cnf_problem) -> ProblemPool:
        if isinstance(cnf_problem, ProblemPool):
            return cnf_problem
        cl = cnf_problem["clauses"] if isinstance(cnf_problem, dict) else cnf_problem
        return self._env.make_pool(np.asarray(cl, dtype=np.int32) if not torch.is_tensor(cl) else cl)

    def reset(self, key, cnf_problem, *, assignments=None) -> Tuple[Dict[str, SatGNNInput], SATState]:
        """sat_env.py:47-68: one env per problem (a (C,K) clause list or a batch (B,C,K) / ProblemPool),
        uniformly random initial assignment (or the explicit ``assignments``)."""
        pool = self._pool(cnf_problem)
        B = pool.num_problems
        idx = torch.arange(B, dtype=torch.int32, device=self.device)
        _, st = self._env.reset_from_pool(pool, B, as_key(key), problem_idx=idx, assignments=assignments,
                                          with_obs=False)
        return self.get_obs(st), st

    def step_env(self, key, state: SATState, actions, *, inplace: bool = False):
        """sat_env.py:70-118 -> (obs, state, rewards, dones, {})."""
        a = actions[self.agents[0]] if isinstance(actions, dict) else actions
        a = torch.as_tensor(a, device=self.device).to(torch.int32).reshape(-1, 1).contiguous()
        nxt = state if inplace else state.clone()
        _, out = self._env.step_raw(nxt, a, autoreset=False, key=key, with_obs=False)
        done = out["done"].bool()
        return self.get_obs(nxt), nxt, {self.agents[0]: out["reward"]}, {self.agents[0]: done, "__all__": done}, {}

    def get_obs(self, state: SATState) -> Dict[str, SatGNNInput]:
        B = state.num_envs
        f = torch.empty((B, self.num_clauses, 3), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib.msat_clause_sat_features(self._env._desc(B, state.pool), state._c(), f.data_ptr(),
                                                     _lib.stream_ptr(self.device)), "msat_clause_sat_features")
        svf = state.pool.static_var_features()[state.problem_idx.long()]
        return {self.agents[0]: SatGNNInput(svf, state.variable_assignments, f, state)}

    def get_unsat_clause_mask(self, state: SATState) -> torch.Tensor:
        """sat_env.py:120-126: True where a clause is unsatisfied."""
        return state.clauses_satisfied_status == 0

    def unsat_ratio_from_assignment(self, state: SATState) -> torch.Tensor:
        """sat_env.py:168-175 for the state's current assignment: float32 (B,)."""
        u = state.num_unsatisfied.to(torch.float32)
        return u / torch.full_like(u, float(self.num_clauses))  # tensor divisor: correctly rounded quotient
