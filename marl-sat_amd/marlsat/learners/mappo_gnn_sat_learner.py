"""MAPPO train cycle on the device — drop-in for ``make_train_cycle`` /
``SATDataWrapper`` / ``GNN_ActorCritic`` of src/learners/mappo_gnn_sat_learner.py.

One ``train_cycle(runner_state, update_idx)`` is the reference's jitted
``_train_cycle`` (:382-729):
  1. rollout of NUM_STEPS batched steps (:383-494): actor + critic forward on the
     current global states, Categorical sampling, fused env step with the
     rollout's auto-reset (done envs redraw a pool instance + assignment);
  2. bootstrap value, GAE and global advantage normalisation (:497-532);
  3. UPDATE_EPOCHS x (T*B / MINIBATCH_SIZE) PPO minibatch steps (:563-659), each a
     gradient over the whole minibatch (micro-batched to bound activation memory,
     exact: gradients of per-sample terms add) followed by one Adam step;
  4. the reference's metrics dict (:661-719).
Transitions store (instance id, assignment) instead of the dense GNN input
(the reference's dense A_pos/A_neg per transition is ~2.9 TB at
uf200 x 4096 x 512); the global state is re-derived on the device when needed.
Multi-GPU: one process per GPU with its own env shard; the flat gradient is
all-reduced (RCCL via torch.distributed) before every Adam step and the
advantage moments / metric sums once per cycle.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np
import torch

from .. import _lib
from ..envs.multi_agent_sat_env import ObsDict, ProblemPool, SATEnv, SATState
from ..random import Key, as_key, split
from .collectives import allreduce_grads, allreduce_sums, global_moments, world_size
from .gnn import GNNActorCritic
from .graphs import DeviceTemplates, GraphBatch, assemble, batch_totals, build_templates
from .ops import gae as device_gae

L_ = _lib.lib
NO_BAD_STEP = 2 ** 31 - 1  # msat_adam_checked's "no non-finite update" value


# ------------------------------------------------------------ schedules ----
def learning_rate_at(count: int, config: dict) -> float:
    """mappo_runner.py:171-193: optax.linear_schedule over Adam step counts (else constant)."""
    if not config.get("ANNEAL_LR", False):
        return float(config.get("LEARNING_RATE", 3e-4))
    n = config.get("NUM_UPDATES", 1)
    lr0 = config.get("LEARNING_RATE", 3e-4) * config.get("LR_START_FACTOR", 1.0)
    lr1 = config.get("LR_END_FLOOR", 1e-5)
    frac = 1.0 - min(max(count, 0), n) / n
    return (lr0 - lr1) * frac + lr1


def ent_coef_at(update_idx: int, config: dict) -> float:
    """learner:534-558."""
    if not config.get("ANNEAL_ENT", False):
        return float(config["ENT_COEF"])
    n = config["NUM_UPDATES"]
    c0, c1 = config["ENT_COEF"], config.get("ENT_COEF_END", 0.0)
    start = n * (1.0 - config.get("ANNEAL_ENT_FRAC", 0.333))
    if update_idx < start:
        return float(c0)
    frac = min(1.0, max(0.0, (update_idx - start) / (n - start)))
    return float(c0 - (c0 - c1) * frac)


# ------------------------------------------------------------- wrapper ----
@dataclass
class GNNInput:
    """graph_constructor.GNNInput (batched).  The dense adjacency is materialised on demand."""

    static_var_features: torch.Tensor  # (B,V,3)
    assignment: torch.Tensor  # (B,V)
    clause_features: torch.Tensor  # (B,C,3)
    _state: SATState = field(repr=False)

    def _dense(self, sign: int) -> torch.Tensor:
        st = self._state
        cl = st.clauses.long()  # (B,C,K)
        B, C, K = cl.shape
        V = st.env.num_vars
        A = torch.zeros((B, V, C), dtype=torch.float32, device=cl.device)
        keep = (cl > 0) if sign > 0 else (cl < 0)
        b = torch.arange(B, device=cl.device)[:, None, None].expand_as(cl)[keep]
        c = torch.arange(C, device=cl.device)[None, :, None].expand_as(cl)[keep]
        v = (cl.abs() - 1)[keep]
        A.index_put_((b, v, c), torch.ones_like(v, dtype=torch.float32), accumulate=True)
        return A

    @property
    def A_pos(self) -> torch.Tensor:
        return self._dense(+1)

    @property
    def A_neg(self) -> torch.Tensor:
        return self._dense(-1)


@dataclass
class GNNWrapperState:
    env_state: SATState


class SATDataWrapper:
    """learner:93-195 — adds the GNN global state to every reset / step (batched)."""

    def __init__(self, env: SATEnv):
        self._env = env

    def __getattr__(self, name):  # JaxMARLWrapper attribute delegation
        return getattr(self._env, name)

    def _global_state(self, st: SATState) -> GNNInput:
        svf = st.pool.static_var_features()[st.problem_idx.long()]
        return GNNInput(svf, st.variable_assignments, self._env.clause_features(st), st)

    def reset(self, problem_clauses, key=None, *, assignments=None):
        obs, st = self._env.reset(problem_clauses, key, assignments=assignments)
        return (obs, self._global_state(st)), GNNWrapperState(st)

    def step(self, key, state: GNNWrapperState, actions):
        obs, st, reward, done, info = self._env.step_env(key, state.env_state, actions)
        return (obs, self._global_state(st)), GNNWrapperState(st), reward, done, info


# -------------------------------------------------------------- learner ----
@dataclass
class RunnerState:
    env_state: SATState
    obs: torch.Tensor  # (B,A,D) last local obs
    rng: Key
    rollout_counter: int = 0


class MAPPOLearner:
    """Device implementation of make_train_cycle's _train_cycle (see module docstring)."""

    def __init__(self, config: dict, env: SATEnv, network: GNNActorCritic, pool: ProblemPool,
                 dist=None, micro_bytes: Optional[float] = None):
        self.cfg = dict(config)
        self.env, self.net, self.pool = env, network, pool
        self.dist = dist
        self.world = world_size(dist)
        self.device = env.device
        self.B = int(config["NUM_ENVS"])
        self.T = int(config["NUM_STEPS"])
        self.MB = int(config["MINIBATCH_SIZE"])
        N = self.T * self.B
        if N % self.MB:
            raise ValueError(f"NUM_STEPS*NUM_ENVS={N} must be divisible by MINIBATCH_SIZE={self.MB} (learner:582-592)")
        self.n_minibatches = N // self.MB
        self.tpl = DeviceTemplates(build_templates(pool.clauses.cpu().numpy(), env.num_vars, env.num_agents),
                                   env.num_agents, self.device)
        H, L = network.H, network.L
        rows = self.tpl.mean_full_rows
        # saved activations per sample (encode tape, fp32, per message step): var rows Hp, Hn, NV, two
        # G4 tapes = 12H, clause rows Hc, GIN, G4 = 7H (bounded by 12H), plus ~24H of transients
        per_sample_train = 4.0 * L * rows * 12 * H + 4.0 * rows * 24 * H
        per_sample_infer = 4.0 * rows * 24 * H
        budget = micro_bytes if micro_bytes is not None else float(config.get("MICROBATCH_BYTES", 240e9))
        cap = max(1, min(self.MB, int(budget // per_sample_train)))
        self.micro = -(-self.MB // -(-self.MB // cap))  # equal micro-batches, none above the budget
        self.chunk = max(1, min(self.B, int(budget // per_sample_infer)))
        self.A, self.M = env.num_agents, env.max_vars_per_agent
        self.mode = env.action_mode
        self.svf = pool.static_var_features()
        # parity instrumentation: a list makes ppo_update record, per Adam step, the minibatch rows,
        # the parameters it started from, the (all-reduced) gradient and the learning rate
        self.trace: Optional[list] = None
        self._alloc()

    def _alloc(self):
        T, B, V, A, M, dev = self.T, self.B, self.env.num_vars, self.A, self.M, self.device
        act_shape = (T, B, A) if self.mode == 0 else (T, B, A, M)
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)
        self.tr = {
            "pidx": z((T, B), torch.int32), "x": z((T, B, V), torch.uint8), "action": z(act_shape, torch.int32),
            "log_prob": z(act_shape, torch.float32), "value": z((T, B), torch.float32),
            "reward": z((T, B), torch.float32), "done": z((T, B), torch.uint8), "solved": z((T, B), torch.uint8),
            "num_unsatisfied": z((T, B), torch.int32), "episode_step": z((T, B), torch.int32),
        }
        self.adv = z((T, B), torch.float32)
        self.targets = z((T, B), torch.float32)
        self.last_val = z((B,), torch.float32)
        self.mom_ws = z((2 * 1024 + 2,), torch.float64)
        self.moments = z((2,), torch.float64)
        # fail-loud guard: the smallest Adam count whose update left a parameter non-finite (INT32_MAX: none)
        self.first_bad = torch.full((1,), NO_BAD_STEP, dtype=torch.int32, device=dev)

    # ------------------------------------------------------------ helpers ----
    def init_runner_state(self, key) -> RunnerState:
        """mappo_runner.py:288-303: B envs reset onto uniformly drawn training problems."""
        k = as_key(key)
        k_reset, k_run = split(k, 2)
        obs, st = self.env.reset_from_pool(self.pool, self.B, k_reset)
        return RunnerState(st, obs, k_run, 0)

    def _batch(self, pidx: torch.Tensor, x: torch.Tensor, critic_only: bool = False, totals=None) -> GraphBatch:
        return assemble(self.tpl, self.pool.packed, self.svf, pidx.contiguous(), x.contiguous(), critic_only, totals)

    def policy(self, st: SATState, key: Key, greedy: bool = False, critic: bool = True):
        """Actor (+ critic) on the current states (learner:391-403): actions, log_probs, values.
        greedy: argmax actions (evaluate_policy, runner:38-46); critic=False skips the value head."""
        B = st.num_envs
        A, M = self.A, self.M
        act = torch.empty((B, A) if self.mode == 0 else (B, A, M), dtype=torch.int32, device=self.device)
        logp = torch.empty(act.shape, dtype=torch.float32, device=self.device)
        val = torch.empty((B,), dtype=torch.float32, device=self.device)
        W = M + 1 if self.mode == 0 else 2
        for c, b0 in enumerate(range(0, B, self.chunk)):
            b1 = min(B, b0 + self.chunk)
            gb = self._batch(st.problem_idx[b0:b1], st.variable_assignments[b0:b1])
            logits, value, _ = self.net.forward(gb, critic=critic)
            if critic:
                val[b0:b1] = value
            rows = logits.numel() // W
            _lib.check(L_.msat_sample_actions(logits.data_ptr(), rows, W, 1 if greedy else 0, key.seed,
                                              (key.counter << 16) + c, act[b0:b1].data_ptr(), logp[b0:b1].data_ptr(),
                                              _lib.stream_ptr(self.device)), "msat_sample_actions")
        return act, logp, val

    def critic_values(self, pidx: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        n = pidx.shape[0]
        out = torch.empty((n,), dtype=torch.float32, device=self.device)
        step = self.chunk * (self.A + 1)  # critic-only samples are ~A+1 times smaller
        for b0 in range(0, n, step):
            b1 = min(n, b0 + step)
            _, v, _ = self.net.forward(self._batch(pidx[b0:b1], x[b0:b1], critic_only=True), actor=False)
            out[b0:b1] = v
        return out

    # ------------------------------------------------------------- rollout ----
    def rollout(self, rs: RunnerState) -> RunnerState:
        tr, env = self.tr, self.env
        out_views = [{k: tr[k][t] for k in ("reward", "done", "solved", "num_unsatisfied", "episode_step")}
                     for t in range(self.T)]
        for t in range(self.T):
            st = rs.env_state
            tr["pidx"][t].copy_(st.problem_idx)
            tr["x"][t].copy_(st.variable_assignments)
            rs.rng, k_act, k_env = (lambda ks: (ks[0], ks[1], ks[2]))(split(rs.rng, 3))
            act, logp, val = self.policy(st, k_act)
            tr["action"][t].copy_(act)
            tr["log_prob"][t].copy_(logp)
            tr["value"][t].copy_(val)
            obs, _ = env.step_raw(st, tr["action"][t], autoreset=True, key=k_env, obs=rs.obs, out=out_views[t])
            rs.rollout_counter += 1
        return rs

    # ----------------------------------------------------------------- GAE ----
    def compute_advantages(self, rs: RunnerState):
        self.last_val.copy_(self.critic_values(rs.env_state.problem_idx, rs.env_state.variable_assignments))
        c = self.cfg
        device_gae(self.tr["reward"], self.tr["value"], self.tr["done"], self.last_val, c["GAMMA"], c["GAE_LAMBDA"],
                   normalize=False, out=(self.adv, self.targets))
        n = self.adv.numel()
        _lib.check(L_.msat_moments(self.adv.data_ptr(), n, self.moments.data_ptr(), self.mom_ws.data_ptr(),
                                   _lib.stream_ptr(self.device)), "msat_moments")
        mean, std = global_moments(self.moments, n, self.dist)
        _lib.check(L_.msat_standardize(self.adv.data_ptr(), n, mean, std, _lib.stream_ptr(self.device)),
                   "msat_standardize")

    # ------------------------------------------------------------- update ----
    def minibatch_grad(self, idx: torch.Tensor, ent: float, sums: torch.Tensor, mb_size: int) -> None:
        """net.grads = d(loss)/d(params) of the PPO loss (learner:597-645) over the flat transition rows
        ``idx``; ``sums`` (3,) fp64 accumulates (value, actor, entropy) row sums.  Loss means divide by
        ``mb_size`` (the minibatch size), so micro-batch gradients add up to the minibatch's."""
        c, net, dev = self.cfg, self.net, self.device
        A, M = self.A, self.M
        idx = idx.to(torch.int32)
        net.grads.zero_()
        # every micro-batch's row totals from one device -> host read per minibatch (assemble would
        # otherwise read each batch's totals back, and the GPU idled while the host caught up)
        bounds = list(range(0, idx.numel(), self.micro)) + [idx.numel()]
        sizes = batch_totals(self.tpl, self.tr["pidx"].reshape(-1).index_select(0, idx.long()), bounds)
        for m0, m1, tot in zip(bounds[:-1], bounds[1:], sizes):
            mi = idx[m0:m1]
            S = mi.numel()
            pidx, x, act, olp, g_, vold, tg = self.gather_rows(mi)
            gb = self._batch(pidx, x, totals=tot)
            logits, value, state = net.forward(gb, save=True)
            dlog = torch.empty_like(logits)
            dval = torch.empty_like(value)
            rows = torch.empty((2 * S * A + S,), device=dev)
            _lib.check(L_.msat_ppo_loss(
                logits.data_ptr(), S, A, M, self.mode, net.base, net.rem, act.data_ptr(), olp.data_ptr(),
                g_.data_ptr(), value.data_ptr(), vold.data_ptr(), tg.data_ptr(), float(c["CLIP_EPS"]),
                float(c["VF_CLIP"]), ent, float(c["VF_COEF"]), mb_size, dlog.data_ptr(), dval.data_ptr(),
                rows.data_ptr(), sums.data_ptr(), _lib.stream_ptr(dev)), "msat_ppo_loss")
            net.backward(gb, state, dlog, dval)
            del state

    def gather_rows(self, idx: torch.Tensor):
        """The transition rows ``idx`` (int32, device) of the flat (T*B) buffers, in one launch
        (msat_gather_rows): (pidx, x, action, log_prob, advantage, value, target)."""
        S, dev = idx.numel(), self.device
        srcs = [self.tr["pidx"], self.tr["x"], self.tr["action"], self.tr["log_prob"], self.adv, self.tr["value"],
                self.targets]
        outs = [torch.empty((S,) + tuple(t.shape[2:]), dtype=t.dtype, device=dev) for t in srcs]
        n = len(srcs)
        src = (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs])
        dst = (ctypes.c_void_p * n)(*[t.data_ptr() for t in outs])
        rb = (ctypes.c_int32 * n)(*[t[0, 0].numel() * t.element_size() for t in srcs])
        _lib.check(L_.msat_gather_rows(idx.data_ptr(), S, n, src, dst, rb, _lib.stream_ptr(dev)), "msat_gather_rows")
        return outs

    def permutation(self, generator: torch.Generator) -> torch.Tensor:
        """A pseudo-random permutation of the T*B transition rows (learner:576), keyed from the host
        generator's stream and drawn on the device (msat_permutation)."""
        N = self.T * self.B
        seed = int(torch.randint(0, 2 ** 62, (1,), generator=generator))
        perm = torch.empty((N,), dtype=torch.int32, device=self.device)
        _lib.check(L_.msat_permutation(N, seed, 0, perm.data_ptr(), _lib.stream_ptr(self.device)), "msat_permutation")
        return perm

    def ppo_update(self, update_idx: int, generator: torch.Generator):
        c, net, dev = self.cfg, self.net, self.device
        N, MB, E = self.T * self.B, self.MB, int(c["UPDATE_EPOCHS"])
        ent = ent_coef_at(update_idx, c)
        losses = torch.zeros((E, self.n_minibatches, 3), dtype=torch.float64, device=dev)
        A, M = self.A, self.M
        n_ent = MB * A * (M if self.mode == 1 else 1)
        for e in range(E):
            perm = self.permutation(generator)
            for k in range(self.n_minibatches):
                idx = perm[k * MB:(k + 1) * MB]
                self.minibatch_grad(idx, ent, losses[e, k], MB)
                scale = allreduce_grads(net.grads, self.dist)
                lr = learning_rate_at(net.adam_count, c)
                if self.trace is not None:
                    self.trace.append({"idx": idx.cpu(), "params": net.params.clone(),
                                       "grads": net.grads.clone() * scale, "lr": lr})
                net.adam_step(lr, grad_scale=scale, first_bad=self.first_bad)
        self.check_finite()
        # per-minibatch means over the UNION minibatch (learner:708-719 reports each minibatch's loss
        # triple over the whole minibatch): the row sums of every rank are added once per cycle, then
        # divided by the union's row counts (every rank's slice has MB rows)
        allreduce_sums(losses, self.dist)
        w = self.world
        losses[..., 0] /= MB * w
        losses[..., 1] /= MB * A * w
        losses[..., 2] /= n_ent * w
        return losses, ent

    def check_finite(self) -> None:
        """One read per cycle of the Adam guard (msat_adam_checked): raise instead of carrying non-finite
        parameters into the next cycle (the loop of mappo_runner.py:313-317 would train on NaN silently, as
        the reference does)."""
        bad = int(self.first_bad.item())
        if bad != NO_BAD_STEP:
            self.first_bad.fill_(NO_BAD_STEP)
            raise FloatingPointError(
                f"MAPPO: Adam step {bad} left non-finite parameters.  A known cause: a pool instance with a variable "
                f"in no clause -- assigned 0, that variable is a constant LayerNorm row at zero-initialised biases and "
                f"its gradient grows ~1000x per message-passing layer past fp32 range, in the reference as here "
                f"(tests/test_isolated_variable.py; filter the pool with generate_problem_pool(skip_isolated=True) or "
                f"utils.generate_cnf_dataset.has_isolated_variable)")

    # ------------------------------------------------------------ metrics ----
    def metrics(self, losses, ent):
        tr, dev = self.tr, self.device
        N = self.T * self.B
        vpred = self.critic_values(tr["pidx"].reshape(N), tr["x"].reshape(N, -1))
        out = torch.empty((11,), dtype=torch.float64, device=dev)
        # out[0..9) = sums over the transitions (msat_cycle_metrics), then the env and row counts
        _lib.check(L_.msat_cycle_metrics(N, tr["reward"].data_ptr(), tr["done"].data_ptr(), tr["solved"].data_ptr(),
                                         tr["num_unsatisfied"].data_ptr(), tr["episode_step"].data_ptr(),
                                         self.targets.data_ptr(), vpred.data_ptr(), out.data_ptr(),
                                         _lib.stream_ptr(dev)), "msat_cycle_metrics")
        out[9] = float(self.B)
        out[10] = float(N)
        allreduce_sums(out, self.dist)
        o = out.tolist()
        s = [o[0], o[9], o[1], o[2], o[3], o[4]]  # reward, envs, done, solved, unsat*done, steps*solved
        t1, t2, d1, d2, n = o[5], o[6], o[7], o[8], o[10]
        var_t = t2 / n - (t1 / n) ** 2
        var_d = d2 / n - (d1 / n) ** 2
        lc = losses.cpu().numpy()
        return {
            "mean_episodic_return": s[0] / s[1],
            "solve_rate": s[3] / max(s[2], 1.0),
            "avg_unsatisfied_clauses": s[4] / max(s[2], 1.0),
            "avg_steps_to_solve": s[5] / max(s[3], 1.0),
            "explained_variance": 1.0 - var_d / max(var_t, 1e-8),
            "epoch_value_losses": lc[..., 0],
            "epoch_actor_losses": lc[..., 1],
            "epoch_entropies": lc[..., 2],
            "current_ent_coef": ent,
        }

    def train_cycle(self, rs: RunnerState, update_idx: int, generator: torch.Generator):
        rs = self.rollout(rs)
        self.compute_advantages(rs)
        losses, ent = self.ppo_update(update_idx, generator)
        return rs, self.metrics(losses, ent)


def make_train_cycle(config, env: SATEnv, network: GNNActorCritic, pool: ProblemPool, dist=None):
    """learner:381-732 — returns (learner, train_cycle(runner_state, update_idx, generator))."""
    learner = MAPPOLearner(config, env, network, pool, dist=dist)
    return learner, learner.train_cycle


# reference class name (learner:198)
GNN_ActorCritic = GNNActorCritic
