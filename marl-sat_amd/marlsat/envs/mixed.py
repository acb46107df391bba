"""Ragged (mixed-size) batches: several SATEnv size classes advanced by ONE launch.

BASELINE.json config 5 ("mixed-size batch uf50/uf100/uf200, 8192 envs"): the reference
cannot express it (every env of a vmapped batch shares V, C and the agent partition,
runner:118 ``jnp.stack``; padding to the largest instance would be needed).  Here each
size class keeps its native layout -- its own desc, problem pool, SoA state and (B_g, A_g,
D_g) observation tensor -- and ``msat_env_step_grouped`` advances all classes in one
kernel launch, so no padded bytes are read or written and small classes still fill the
GPU together.

RNG: class g draws its resets with seed ^ group_seed(g) (group_seed(0) = 0), so each class
replays bit-exactly as its own SATEnv with that seed (tests/test_env_gpu.py).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import torch

from .. import _lib
from ..random import as_key
from .multi_agent_sat_env import ObsDict, ProblemPool, SATEnv, SATState

_MASK64 = (1 << 64) - 1


def group_seed(g: int) -> int:
    return (g * 0x9E3779B97F4A7C15) & _MASK64


class MixedSATEnv:
    """A list of SATEnv size classes sharing action_mode / reward_mode / obs_dtype / device."""

    def __init__(self, classes: Sequence[SATEnv]):
        if not 1 <= len(classes) <= _lib.MAX_GROUPS:
            raise ValueError(f"1..{_lib.MAX_GROUPS} size classes supported, got {len(classes)}")
        c0 = classes[0]
        for c in classes:
            if (c.action_mode, c.reward_mode, c.obs_dtype, c.device) != (c0.action_mode, c0.reward_mode,
                                                                           c0.obs_dtype, c0.device):
                raise ValueError("size classes must share action_mode, reward_mode, obs_dtype and device")
        self.classes = list(classes)
        self.G = len(classes)
        self.device = c0.device

    # --------------------------------------------------------------- setup ----
    def _arrays(self, pools: Sequence[ProblemPool], sizes: Sequence[int], states: Sequence[SATState],
                obs: Sequence[torch.Tensor]):
        G = self.G
        descs = (_lib.EnvDesc * G)(*[c._desc(b, p) for c, b, p in zip(self.classes, sizes, pools)])
        cpools = (_lib.PoolC * G)(*[p.c(c) for c, p in zip(self.classes, pools)])
        cst = (_lib.EnvStateC * G)(*[s._c() for s in states])
        cobs = (ctypes.c_void_p * G)(*[o.data_ptr() for o in obs])
        return descs, cpools, cst, cobs

    def reset(self, pools: Sequence[ProblemPool], num_envs: Sequence[int], key=None):
        """Reset every env of every class onto RNG-drawn rows of its class pool.

        Returns (obs list of (B_g, A_g, D_g), state list)."""
        if len(pools) != self.G or len(num_envs) != self.G:
            raise ValueError("one pool and one env count per size class")
        k = as_key(key)
        states = [c.alloc_state(int(b), p) for c, b, p in zip(self.classes, num_envs, pools)]
        obs = [c.alloc_obs(int(b)) for c, b in zip(self.classes, num_envs)]
        descs, cpools, cst, cobs = self._arrays(pools, num_envs, states, obs)
        _lib.check(_lib.lib.msat_env_reset_grouped(self.G, descs, cpools, cst, k.seed, k.counter, cobs,
                                                   _lib.stream_ptr(self.device)), "msat_env_reset_grouped")
        return obs, states

    def alloc_outs(self, states: Sequence[SATState]):
        return [c._step_out(s.num_envs) for c, s in zip(self.classes, states)]

    # ---------------------------------------------------------------- step ----
    def stepper(self, states: Sequence[SATState], obs: Sequence[torch.Tensor], outs: Sequence[dict], *,
                autoreset: bool = True, seed: int = 0):
        """Pre-bound grouped step: ``f(actions_list, counter)`` launches one kernel for every class.
        ``actions_list[g]`` is a contiguous device int32 (B_g, A_g) (mode 0) tensor."""
        G = self.G
        sizes = [s.num_envs for s in states]
        descs, cpools, cst, cobs = self._arrays([s.pool for s in states], sizes, states, obs)
        couts = (_lib.StepOutC * G)(*[
            _lib.StepOutC(o["reward"].data_ptr(), o["done"].data_ptr(), o["solved"].data_ptr(),
                          o["num_unsatisfied"].data_ptr(), o["episode_step"].data_ptr(),
                          _lib.stamps_ptr(o.get("clock_stamps"), b)) for o, b in zip(outs, sizes)])
        cact = (ctypes.c_void_p * G)()
        fn = _lib.lib.msat_env_step_grouped
        s = _lib.stream_ptr(self.device)
        ar = 1 if autoreset else 0
        wants = [(b, c.num_agents) if c.action_mode == 0 else (b, c.num_agents, c.max_vars_per_agent)
                 for c, b in zip(self.classes, sizes)]

        def step(actions: Sequence[torch.Tensor], counter: int) -> None:
            for g in range(G):
                a = actions[g]
                if tuple(a.shape) != wants[g] or a.dtype != torch.int32:
                    raise ValueError(f"actions[{g}] must be int32 {wants[g]}")
                cact[g] = a.data_ptr()
            rc = fn(G, descs, cpools, cst, cact, ar, seed, counter, couts, cobs, s)
            for st in states:
                st._masks = None
            if rc:
                _lib.check(rc, "msat_env_step_grouped")

        step._keepalive = (descs, cpools, cst, cobs, couts, cact, states, obs, outs)
        return step

    def step_raw(self, states: Sequence[SATState], actions: Sequence, *, autoreset: bool = True, key=None,
                 obs: Optional[Sequence[torch.Tensor]] = None, outs: Optional[Sequence[dict]] = None):
        """In place on every class; returns (obs list, outs list)."""
        k = as_key(key)
        if obs is None:
            obs = [c.alloc_obs(s.num_envs) for c, s in zip(self.classes, states)]
        if outs is None:
            outs = self.alloc_outs(states)
        acts = [c._actions_tensor(a, s.num_envs) for c, a, s in zip(self.classes, actions, states)]
        self.stepper(states, obs, outs, autoreset=autoreset, seed=k.seed)(acts, k.counter)
        return obs, outs

    def obs_dicts(self, obs: Sequence[torch.Tensor]) -> List[ObsDict]:
        return [ObsDict(c.agents, o) for c, o in zip(self.classes, obs)]
