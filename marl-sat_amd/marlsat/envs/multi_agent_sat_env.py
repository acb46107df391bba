"""Batched multi-agent SAT environment — jaxmarl ``MultiAgentEnv``-shaped facade.

Drop-in for ``SATEnv`` / ``SATState`` of the reference
(``src/envs/multi_agent_sat_env.py:13-412``): same constructor arguments,
attributes, agent partition, spaces and ``reset`` / ``step_env`` / ``get_obs``
signatures and return structures.  Differences, all deliberate:

* every array carries a leading env axis B (the reference is vmapped by its
  caller, ``mappo_runner.py:137`` / ``learner:418``); a 2-D ``(C,K)`` problem is
  treated as B=1;
* arrays are torch device tensors; the per-agent dicts are views into one
  ``(B, A, D)`` observation tensor (``ObsDict.tensor``) and one ``(B,)`` reward;
* ``key`` is ``marlsat.random.Key`` (Philox seed + counter) or an int seed;
  JAX threefry streams cannot be reproduced, so exact-parity callers pass
  ``assignments=`` / ``problem_idx=`` explicitly;
* the compute runs in hand-written HIP kernels (``libmarlsat.so``); there is
  no CPU path.  ``variable_assignments`` is stored as uint8 (values {0,1}).
"""
from __future__ import annotations

import ctypes
import os
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import _lib
from ..random import Key, as_key
from .spaces import Box, Discrete, MultiDiscrete


def _find_factors(n: int) -> List[int]:
    """env:286-293."""
    fs = set()
    for i in range(1, int(math.isqrt(n)) + 1):
        if n % i == 0:
            fs.update((i, n // i))
    return sorted(fs)


def create_agent_groups(num_vars: int, vars_per_agent: Optional[int]) -> Dict[str, List[int]]:
    """Contiguous variable groups, identical to ``SATEnv._create_agent_groups`` (env:294-338)."""
    if vars_per_agent is not None:
        num_agents = math.ceil(num_vars / vars_per_agent)
    else:
        sizes = [f for f in _find_factors(num_vars) if f == 4]  # ideal_min_size == ideal_max_size == 4
        num_agents = num_vars // sizes[-1] if sizes else max(2, int(math.sqrt(num_vars)))
    base, rem = divmod(num_vars, num_agents)
    groups, start = {}, 0
    for i in range(num_agents):
        n = base + (1 if i < rem else 0)
        groups[f"agent_{i}"] = list(range(start, start + n))
        start += n
    return groups


class ObsDict(dict):
    """{agent: (B, D) view} with the backing (B, A, D) tensor in ``.tensor``."""

    def __init__(self, agents: List[str], tensor: torch.Tensor):
        super().__init__((a, tensor[:, i, :]) for i, a in enumerate(agents))
        self.tensor = tensor


class ProblemPool:
    """Device-resident problem pool: int32 literals (N,C,K) + packed uint16 (N,C,4).

    Replaces the stacked ``problems['clauses']`` pytree (``mappo_runner.py:114-118``).
    """

    def __init__(self, clauses, num_vars: int, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        t = torch.as_tensor(np.asarray(clauses) if not torch.is_tensor(clauses) else clauses)
        if t.dim() == 2:
            t = t.unsqueeze(0)
        if t.dim() != 3:
            raise ValueError(f"problem clauses must be (N,C,K), got {tuple(t.shape)}")
        self.clauses = t.to(device=dev, dtype=torch.int32).contiguous()
        _lib.require_device(self.clauses, "problem pool")
        self.num_problems, self.num_clauses, self.clause_width = self.clauses.shape
        self.num_vars = num_vars
        self.packed = torch.empty((self.num_problems, self.num_clauses, 4), dtype=torch.int16, device=dev)
        err = torch.zeros((1,), dtype=torch.int32, device=dev)
        _lib.check(
            _lib.lib.msat_pool_pack(self.clauses.data_ptr(), self.num_problems, self.num_clauses,
                                    self.clause_width, num_vars, self.packed.data_ptr(), err.data_ptr(),
                                    _lib.stream_ptr(dev)),
            "msat_pool_pack",
        )
        if int(err.item()) != 0:
            raise ValueError(f"problem pool has a literal with |l| > num_vars={num_vars}")
        self._svf = None
        self._tables = {}  # num_agents -> (rel (N,A,WC), nbr (N,A,WV)) int32 bit words

    def agent_tables(self, env: "SATEnv"):
        """Per-instance relation / neighbour bit tables for env's agent partition
        (_compute_observation_maps, env:99-128, hoisted from every reset to once per pool)."""
        key = env.num_agents
        if key not in self._tables:
            WC = 2 * ((self.num_clauses + 63) // 64)
            WV = 2 * ((self.num_vars + 63) // 64)
            rel = torch.empty((self.num_problems, env.num_agents, WC), dtype=torch.int32, device=self.device)
            nbr = torch.empty((self.num_problems, env.num_agents, WV), dtype=torch.int32, device=self.device)
            desc = env._desc(0, self)
            _lib.check(_lib.lib.msat_pool_agent_tables(ctypes.byref(desc), self.packed.data_ptr(), rel.data_ptr(),
                                                       nbr.data_ptr(), _lib.stream_ptr(self.device)),
                       "msat_pool_agent_tables")
            self._tables[key] = (rel, nbr)
        return self._tables[key]

    def c(self, env: "SATEnv") -> _lib.PoolC:
        rel, nbr = self.agent_tables(env)
        return _lib.PoolC(self.packed.data_ptr(), rel.data_ptr(), nbr.data_ptr())

    @property
    def device(self):
        return self.clauses.device

    def static_var_features(self) -> torch.Tensor:
        """(N,V,3) float32 [deg+/C, deg-/C, 0] (learner:150-164); computed once per pool."""
        if self._svf is None:
            self._svf = torch.empty((self.num_problems, self.num_vars, 3), dtype=torch.float32, device=self.device)
            _lib.check(_lib.lib.msat_static_var_features(self.packed.data_ptr(), self.num_problems, self.num_vars,
                                                         self.num_clauses, self._svf.data_ptr(),
                                                         _lib.stream_ptr(self.device)),
                       "msat_static_var_features")
        return self._svf


# MARLSAT_RESET_QUEUE=0: states without a reset queue (every reset in its step workgroup; A/B runs only)
RESET_QUEUE = os.environ.get("MARLSAT_RESET_QUEUE", "1") != "0"


@dataclass
class SATState:
    """``SATState`` (env:13-24) as device SoA tensors with a leading env axis."""

    variable_assignments: torch.Tensor  # (B,V) uint8
    clauses_satisfied_status: torch.Tensor  # (B,C) uint8 (bool values)
    clause_ntrue: torch.Tensor  # (B,C) uint8   #true literals (wrapper feature)
    num_unsatisfied: torch.Tensor  # (B,) int32
    step: torch.Tensor  # (B,) int32
    env_done: torch.Tensor  # (B,) uint8
    problem_idx: torch.Tensor  # (B,) int32
    pool: ProblemPool
    env: "SATEnv" = field(repr=False)
    _masks: Optional[tuple] = field(default=None, repr=False)
    # msat_env_state.reset_queue (include/marlsat.h): each autoreset step lists the envs whose next step times
    # out, and the next one resets them in workgroups of their own; reset_serial counts those launches.  Not
    # reference state: results are identical without it.  Code that writes the arrays above directly must call
    # invalidate_reset_queue().
    reset_queue: Optional[torch.Tensor] = field(default=None, repr=False)
    reset_serial: int = field(default=0, repr=False)

    @property
    def num_envs(self) -> int:
        return self.variable_assignments.shape[0]

    @property
    def done(self) -> torch.Tensor:
        """(B,A) bool — every agent shares the env's done (env:270)."""
        return self.env_done.bool()[:, None].expand(-1, self.env.num_agents)

    @property
    def clauses(self) -> torch.Tensor:
        return self.pool.clauses[self.problem_idx.long()]

    @property
    def action_mask(self) -> torch.Tensor:
        return self.env.action_mask

    def _materialise_masks(self):
        if self._masks is None:
            e = self.env
            B = self.num_envs
            dev = self.variable_assignments.device
            acm = torch.empty((B, e.num_agents, e.num_clauses), dtype=torch.int32, device=dev)
            anm = torch.empty((B, e.num_agents, e.num_vars), dtype=torch.int32, device=dev)
            l2a = torch.empty((B, e.num_clauses, self.pool.clause_width), dtype=torch.int32, device=dev)
            _lib.check(_lib.lib.msat_env_masks(e._desc(B, self.pool), self.pool.c(e), self._c(),
                                               acm.data_ptr(), anm.data_ptr(), l2a.data_ptr(), _lib.stream_ptr(dev)),
                       "msat_env_masks")
            self._masks = (acm, anm, l2a)
        return self._masks

    @property
    def agent_clause_masks(self) -> torch.Tensor:
        return self._materialise_masks()[0]

    @property
    def agent_neighbor_masks(self) -> torch.Tensor:
        return self._materialise_masks()[1]

    @property
    def literal_to_agent_idx(self) -> torch.Tensor:
        return self._materialise_masks()[2]

    def _c(self) -> _lib.EnvStateC:
        return _lib.EnvStateC(
            self.variable_assignments.data_ptr(), self.clauses_satisfied_status.data_ptr(),
            self.clause_ntrue.data_ptr(), self.num_unsatisfied.data_ptr(), self.step.data_ptr(),
            self.env_done.data_ptr(), self.problem_idx.data_ptr(), _lib.ptr(self.reset_queue),
            self.reset_serial & 0xFFFFFFFF,
        )

    def invalidate_reset_queue(self) -> None:
        """Forget the listed timed-out envs (after writing state arrays directly, e.g. bench.py's staggered
        episode counters): the next autoreset step resets every env in its own workgroup and lists afresh."""
        if self.reset_queue is not None:
            self.reset_queue.zero_()

    def clone(self) -> "SATState":
        return SATState(
            self.variable_assignments.clone(), self.clauses_satisfied_status.clone(), self.clause_ntrue.clone(),
            self.num_unsatisfied.clone(), self.step.clone(), self.env_done.clone(), self.problem_idx.clone(),
            self.pool, self.env, reset_queue=None if self.reset_queue is None else self.reset_queue.clone(),
            reset_serial=self.reset_serial,
        )

    def replace(self, **kw) -> "SATState":
        """flax ``struct.replace`` analogue (shallow).  The result has no reset queue (its arrays may be
        other tensors than the ones the queue describes)."""
        d = {f: getattr(self, f) for f in self.__dataclass_fields__ if f not in ("_masks", "reset_queue", "reset_serial")}
        d.update(kw)
        return SATState(**d)


class SATEnv:
    """Batched drop-in for ``SATEnv`` (env:28-412)."""

    def __init__(self, num_vars, num_clauses, max_steps: int, vars_per_agent: Optional[int] = None,
                 action_mode: int = 0, r_clause: float = 0.02, r_sat: float = 1.0, gamma: float = 0.99, *,
                 reward_mode: int = _lib.REWARD_SPARSE, obs_dtype=torch.int32, device=None):
        self.num_vars = int(num_vars)
        self.num_clauses = int(num_clauses)
        self.agent_groups = create_agent_groups(self.num_vars, vars_per_agent)
        self.agents = list(self.agent_groups.keys())
        self.num_agents = len(self.agents)
        self.agent_to_idx = {a: i for i, a in enumerate(self.agents)}
        self.r_clause, self.r_sat, self.gamma = float(r_clause), float(r_sat), float(gamma)
        self.action_mode = int(action_mode)
        self.reward_mode = int(reward_mode)
        self.max_vars_per_agent = max(len(v) for v in self.agent_groups.values())
        self.max_steps = int(max_steps)
        if obs_dtype not in (torch.int32, torch.int8):
            raise ValueError("obs_dtype must be torch.int32 (reference) or torch.int8")
        self.obs_dtype = obs_dtype
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        A, M = self.num_agents, self.max_vars_per_agent
        av = np.full((A, M), -1, dtype=np.int32)
        am = np.zeros((A, M), dtype=bool)
        for i, a in enumerate(self.agents):
            g = self.agent_groups[a]
            av[i, : len(g)] = g
            am[i, : len(g)] = True
        self.agent_vars = torch.from_numpy(av).to(self.device)
        self.action_mask = torch.from_numpy(am).to(self.device)
        v2a = np.full((self.num_vars,), -1, dtype=np.int32)
        for i, a in enumerate(self.agents):
            v2a[self.agent_groups[a]] = i
        self.variable_to_agent_idx = torch.from_numpy(v2a).to(self.device)
        if self.action_mode == 0:
            self.action_spaces = {a: Discrete(M + 1) for a in self.agents}
        else:
            self.action_spaces = {a: MultiDiscrete([2] * M) for a in self.agents}
        self.obs_dim = 2 * self.num_vars + self.num_clauses  # env:340-343
        self.observation_spaces = {a: Box(-1, 1, (self.obs_dim,)) for a in self.agents}

    # ------------------------------------------------------------ props ----
    @property
    def name(self) -> str:
        return "SATEnv"

    def action_space(self, agent: str):
        return self.action_spaces[agent]

    def observation_space(self, agent: str):
        return self.observation_spaces[agent]

    # ---------------------------------------------------------- plumbing ----
    def _desc(self, num_envs: int, pool: ProblemPool) -> _lib.EnvDesc:
        if pool.num_clauses != self.num_clauses or pool.num_vars != self.num_vars:
            raise ValueError(f"pool is V={pool.num_vars}, C={pool.num_clauses}; env is V={self.num_vars}, "
                             f"C={self.num_clauses}")
        return _lib.EnvDesc(
            num_envs, self.num_vars, self.num_clauses, pool.clause_width, self.num_agents, self.max_vars_per_agent,
            self.max_steps, self.action_mode, self.reward_mode,
            _lib.OBS_I32 if self.obs_dtype == torch.int32 else _lib.OBS_I8, pool.num_problems,
            self.r_clause, self.r_sat, self.gamma,
        )

    def make_pool(self, problem_clauses) -> ProblemPool:
        return ProblemPool(problem_clauses, self.num_vars, self.device)

    def alloc_state(self, num_envs: int, pool: ProblemPool) -> SATState:
        dev = self.device
        B, V, C = num_envs, self.num_vars, self.num_clauses
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)
        return SATState(z((B, V), torch.uint8), z((B, C), torch.uint8), z((B, C), torch.uint8), z((B,), torch.int32),
                        z((B,), torch.int32), z((B,), torch.uint8), z((B,), torch.int32), pool, self,
                        reset_queue=z((int(_lib.lib.msat_reset_queue_words(B)),), torch.int32) if RESET_QUEUE else None)

    def alloc_obs(self, num_envs: int) -> torch.Tensor:
        return torch.empty((num_envs, self.num_agents, self.obs_dim), dtype=self.obs_dtype, device=self.device)

    def _actions_tensor(self, actions, B: int) -> torch.Tensor:
        if isinstance(actions, dict):  # learner:131 jnp.stack([actions[a] for a in agents])
            actions = torch.stack([torch.as_tensor(actions[a], device=self.device) for a in self.agents], dim=1)
        a = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        want = (B, self.num_agents) if self.action_mode == 0 else (B, self.num_agents, self.max_vars_per_agent)
        if tuple(a.shape) != want:
            raise ValueError(f"actions must have shape {want}, got {tuple(a.shape)}")
        return a

    def _refuse_nonbinary(self, actions, B: int) -> torch.Tensor:
        """env:246-250 XORs the raw integer: a mode-1 action of 2 or -1 leaves a non-binary assignment
        (both polarities false in the clause scan).  MultiDiscrete([2]*m) never samples one, and the device
        state keeps one bit per variable, so the reference-API entry points refuse such actions (one
        device reduction + sync; the raw ``step_raw`` / ``stepper`` paths apply bit 0 unchecked)."""
        a = self._actions_tensor(actions, B)
        if self.action_mode == 1 and a.numel() and bool(((a != 0) & (a != 1)).any()):
            raise ValueError("action_mode 1 actions must be 0 or 1 (MultiDiscrete([2] * max_vars_per_agent))")
        return a

    # ------------------------------------------------------------ reset ----
    def reset_from_pool(self, pool: ProblemPool, num_envs: int, key=None, *, problem_idx=None, assignments=None,
                        state: Optional[SATState] = None, reset_mask=None, obs: Optional[torch.Tensor] = None,
                        with_obs: bool = True):
        """Reset (all or masked) envs onto pool rows; returns (obs (B,A,D), state). In place when state given.
        with_obs=False: state only (obs is None, nothing written)."""
        k = as_key(key)
        if state is None:
            state = self.alloc_state(num_envs, pool)
        if obs is None and with_obs:
            obs = self.alloc_obs(num_envs)
        pidx = None
        if problem_idx is not None:
            pidx = torch.as_tensor(problem_idx, device=self.device).to(torch.int32).contiguous()
            if pidx.shape != (num_envs,):
                raise ValueError("problem_idx must be (B,)")
            if int(pidx.min()) < 0 or int(pidx.max()) >= pool.num_problems:
                raise ValueError("problem_idx out of range")
        x = None
        if assignments is not None:
            x = torch.as_tensor(assignments, device=self.device).to(torch.uint8).contiguous()
            if x.shape != (num_envs, self.num_vars):
                raise ValueError(f"assignments must be (B,V)=({num_envs},{self.num_vars})")
        m = None
        if reset_mask is not None:
            m = torch.as_tensor(reset_mask, device=self.device).to(torch.uint8).contiguous()
        _lib.check(_lib.lib.msat_env_reset(self._desc(num_envs, pool), pool.c(self), state._c(), _lib.ptr(m),
                                           _lib.ptr(pidx), _lib.ptr(x), k.seed, k.counter, _lib.ptr(obs),
                                           _lib.stream_ptr(self.device)),
                   "msat_env_reset")
        state._masks = None
        return obs, state

    def reset(self, problem_clauses, key=None, *, assignments=None) -> Tuple[ObsDict, SATState]:
        """env:158-181 — one env per row of ``problem_clauses`` (B,C,K)."""
        pool = problem_clauses if isinstance(problem_clauses, ProblemPool) else self.make_pool(problem_clauses)
        B = pool.num_problems
        idx = torch.arange(B, dtype=torch.int32, device=self.device)
        obs, state = self.reset_from_pool(pool, B, key, problem_idx=idx, assignments=assignments)
        return ObsDict(self.agents, obs), state

    # ------------------------------------------------------------- step ----
    def _step_out(self, B: int):
        dev = self.device
        return {
            "reward": torch.empty((B,), dtype=torch.float32, device=dev),
            "done": torch.empty((B,), dtype=torch.uint8, device=dev),
            "solved": torch.empty((B,), dtype=torch.uint8, device=dev),
            "num_unsatisfied": torch.empty((B,), dtype=torch.int32, device=dev),
            "episode_step": torch.empty((B,), dtype=torch.int32, device=dev),
        }

    def step_raw(self, state: SATState, actions: torch.Tensor, *, autoreset: bool = False, key=None,
                 problem_idx=None, assignments=None, obs: Optional[torch.Tensor] = None, out=None,
                 with_obs: bool = True):
        """In-place batched step on device tensors; returns (obs, out-dict). The hot-loop entry point.
        with_obs=False: no observation write (obs is None)."""
        B = state.num_envs
        a = self._actions_tensor(actions, B)
        if obs is None and with_obs:
            obs = self.alloc_obs(B)
        if out is None:
            out = self._step_out(B)
        pidx = None if problem_idx is None else torch.as_tensor(problem_idx, device=self.device).to(torch.int32).contiguous()
        x = None if assignments is None else torch.as_tensor(assignments, device=self.device).to(torch.uint8).contiguous()
        k = as_key(key)
        so = _lib.StepOutC(out["reward"].data_ptr(), out["done"].data_ptr(), out["solved"].data_ptr(),
                           out["num_unsatisfied"].data_ptr(), out["episode_step"].data_ptr(),
                           _lib.stamps_ptr(out.get("clock_stamps"), B))
        _lib.check(_lib.lib.msat_env_step(self._desc(B, state.pool), state.pool.c(self), state._c(),
                                          a.data_ptr(), 1 if autoreset else 0, _lib.ptr(pidx), _lib.ptr(x), k.seed,
                                          k.counter, so, _lib.ptr(obs), _lib.stream_ptr(self.device)),
                   "msat_env_step")
        if autoreset:
            state.reset_serial += 1
        state._masks = None
        return obs, out

    def stepper(self, state: SATState, obs: torch.Tensor, out: dict, *, autoreset: bool = True, seed: int = 0):
        """Pre-bound in-place step for hot loops: ``f(actions, counter)`` launches one fused
        step (+ auto-reset) on the current stream with no per-call Python marshalling
        beyond the ctypes call itself.  ``actions`` must be a contiguous device int32 tensor."""
        B = state.num_envs
        desc = self._desc(B, state.pool)
        cst = state._c()
        # out["clock_stamps"] (optional, (B, 8) int64): the kernel's diagnostic clock stamps (bench.py)
        so = _lib.StepOutC(out["reward"].data_ptr(), out["done"].data_ptr(), out["solved"].data_ptr(),
                           out["num_unsatisfied"].data_ptr(), out["episode_step"].data_ptr(),
                           _lib.stamps_ptr(out.get("clock_stamps"), B))
        fn = _lib.lib.msat_env_step
        cpool = state.pool.c(self)
        obs_p, s = obs.data_ptr(), _lib.stream_ptr(self.device)
        ar = 1 if autoreset else 0
        want = (B, self.num_agents) if self.action_mode == 0 else (B, self.num_agents, self.max_vars_per_agent)
        dref, pref, sref, oref = ctypes.byref(desc), ctypes.byref(cpool), ctypes.byref(cst), ctypes.byref(so)

        def step(actions: torch.Tensor, counter: int) -> None:
            if actions.shape != want or actions.dtype != torch.int32:
                raise ValueError(f"actions must be int32 {want}")
            cst.reset_serial = state.reset_serial & 0xFFFFFFFF
            rc = fn(dref, pref, sref, actions.data_ptr(), ar, None, None, seed, counter, oref, obs_p, s)
            state._masks = None
            if rc:
                _lib.check(rc, "msat_env_step")
            if ar:
                state.reset_serial += 1

        step._keepalive = (desc, cpool, cst, so, state, obs, out)
        return step

    def step_env(self, key, state: SATState, actions, *, inplace: bool = False):
        """env:225-284 -> (obs, next_state, rewards, dones, infos). Functional unless ``inplace``."""
        actions = self._refuse_nonbinary(actions, state.num_envs)
        nxt = state if inplace else state.clone()
        obs, out = self.step_raw(nxt, actions, autoreset=False, key=key)
        done = out["done"].bool()
        rewards = {a: out["reward"] for a in self.agents}
        dones = {a: done for a in self.agents}
        dones["__all__"] = done
        infos = {"solved": out["solved"].bool(), "num_unsatisfied": out["num_unsatisfied"],
                 "episode_step": out["episode_step"]}
        return ObsDict(self.agents, obs), nxt, rewards, dones, infos

    def step(self, key, state: SATState, actions, *, inplace: bool = False, problem_idx=None, assignments=None):
        """jaxmarl ``MultiAgentEnv.step``: step_env + auto-reset of done envs onto random pool rows."""
        nxt = state if inplace else state.clone()
        actions = self._refuse_nonbinary(actions, state.num_envs)
        obs, out = self.step_raw(nxt, actions, autoreset=True, key=key, problem_idx=problem_idx,
                                 assignments=assignments)
        done = out["done"].bool()
        rewards = {a: out["reward"] for a in self.agents}
        dones = {a: done for a in self.agents}
        dones["__all__"] = done
        infos = {"solved": out["solved"].bool(), "num_unsatisfied": out["num_unsatisfied"],
                 "episode_step": out["episode_step"]}
        return ObsDict(self.agents, obs), nxt, rewards, dones, infos

    def get_obs(self, state: SATState) -> ObsDict:
        """env:345-398."""
        B = state.num_envs
        obs = self.alloc_obs(B)
        _lib.check(_lib.lib.msat_env_obs(self._desc(B, state.pool), state.pool.c(self), state._c(),
                                         obs.data_ptr(), _lib.stream_ptr(self.device)),
                   "msat_env_obs")
        return ObsDict(self.agents, obs)

    def clause_features(self, state: SATState) -> torch.Tensor:
        """(B,C,3) float32 [is_sat, #true/3, 1] — SATDataWrapper._calculate_dynamic_clause_features (learner:176-195)."""
        B = state.num_envs
        f = torch.empty((B, self.num_clauses, 3), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib.msat_clause_features(self._desc(B, state.pool), state._c(), f.data_ptr(),
                                                 _lib.stream_ptr(self.device)),
                   "msat_clause_features")
        return f

    def _calculate_satisfaction_explicit(self, variable_assignments, clauses):
        """env:130-156 for one or many envs -> (status bool, num_unsat); runs on the device."""
        cl = torch.as_tensor(np.asarray(clauses) if not torch.is_tensor(clauses) else clauses)
        x = torch.as_tensor(np.asarray(variable_assignments) if not torch.is_tensor(variable_assignments)
                            else variable_assignments)
        single = cl.dim() == 2
        if single:
            cl, x = cl.unsqueeze(0), x.reshape(1, -1)
        pool = ProblemPool(cl, self.num_vars, self.device)
        B = pool.num_problems
        _, st = self.reset_from_pool(pool, B, problem_idx=torch.arange(B, device=self.device), assignments=x)
        status, nun = st.clauses_satisfied_status.bool(), st.num_unsatisfied
        return (status[0], nun[0]) if single else (status, nun)
