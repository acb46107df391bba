"""Multi-rank semantics of the learner's exchanges on CPU (gloo, world_size 2).

The device learner meets the other ranks only through marlsat/learners/collectives.py
(SURVEY.md §8(e)); these tests run exactly those functions on CPU tensors:
  * global advantage moments == the single-process normalisation of the union
    (learner:530-532);
  * SUM all-reduce of per-rank gradients x grad_scale (1/world) == the gradient of the
    union minibatch of the reference loss (oracle torch network, float64), and one Adam
    step from it == Adam on the union gradient;
  * metric sums add across ranks;
  * torchrun-style init from the environment.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _union_batch(n, seed=0):
    from oracle import net as onet
    from oracle.sat_env import OracleSATEnv
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    V, C, vpa = 12, 40, 4
    pool = generate_problem_pool(V, C, 5, size_id=13)
    ora = OracleSATEnv(V, C, 5, vars_per_agent=vpa)
    rng = np.random.default_rng(seed)
    pidx = rng.integers(0, 5, n)
    x = rng.integers(0, 2, (n, V)).astype(np.int32)
    _, st = ora.reset(pool[pidx], x)
    Ap, An = onet.dense_graph(pool[pidx], V)
    A, M = ora.num_agents, ora.max_vars_per_agent
    b = {"svf": torch.from_numpy(ora.static_var_features(pool[pidx])).double(),
         "x": torch.from_numpy(x.astype(np.float64)), "cf": torch.from_numpy(ora.clause_features(st)).double(),
         "A_pos": Ap, "A_neg": An,
         "action": torch.from_numpy(rng.integers(0, M + 1, (n, A))),
         "log_prob": torch.from_numpy(rng.normal(-1.5, 0.3, (n, A))),
         "value": torch.from_numpy(rng.normal(0, 0.5, n)),
         "targets": torch.from_numpy(rng.normal(0, 1, n)),
         "gae": torch.from_numpy(rng.normal(0, 1, n))}
    av = torch.from_numpy(ora.agent_vars.astype(np.int64))
    am = torch.from_numpy(ora.action_mask)
    return b, av, am, A, M


def _grads(P, batch, av, am):
    from oracle import net as onet

    cfg = {"CLIP_EPS": 0.2, "VF_CLIP": 0.2, "ENT_COEF": 0.01, "VF_COEF": 0.5}
    Pk = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    total, _, _, _ = onet.ppo_loss(Pk, 2, batch, cfg, av, am, 0)
    total.backward()
    return torch.cat([(Pk[k].grad if Pk[k].grad is not None else torch.zeros_like(Pk[k])).reshape(-1)
                      for k in sorted(Pk)])


def _worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from marlsat.learners import collectives as co
    from oracle import mappo as om
    from oracle import net as onet

    dist = co.init_from_env("gloo")
    assert dist is not None and co.world_size(dist) == world
    try:
        # ---- global advantage moments
        adv_all = (np.random.default_rng(5).normal(1.0, 3.0, (world, 6, 7))).astype(np.float32)
        loc = torch.from_numpy(adv_all[rank].astype(np.float64)).reshape(-1)
        mean, std = co.global_moments(torch.stack([loc.sum(), (loc * loc).sum()]), loc.numel(), dist)
        _, rmean, rstd = om.normalize(adv_all)
        assert abs(mean - rmean) <= 1e-12 * max(1.0, abs(rmean)) and abs(std - rstd) <= 1e-12 * rstd

        # ---- gradient all-reduce == union-minibatch gradient; Adam step on it
        n = 4 * world
        batch, av, am, A, M = _union_batch(n)
        P = onet.init_params(onet.param_shapes(16, 2, A, M, 0), seed=3)
        lo, hi = rank * n // world, (rank + 1) * n // world
        mine = {k: v[lo:hi] for k, v in batch.items()}
        g = _grads(P, mine, av, am)
        scale = co.allreduce_grads(g, dist)
        assert scale == 1.0 / world
        g_mean = g * scale
        g_union = _grads(P, batch, av, am)
        err = (g_mean - g_union).abs().max().item()
        assert err <= 1e-12 * max(1.0, g_union.abs().max().item()), err
        flat = lambda d: torch.cat([d[k].reshape(-1) for k in sorted(d)])
        z = {k: torch.zeros_like(v) for k, v in P.items()}
        keys, sizes = sorted(P), [P[k].numel() for k in sorted(P)]
        unflat = lambda v: {k: t.reshape(P[k].shape) for k, t in zip(keys, torch.split(v, sizes))}
        p1, _ = onet.adam_update(P, unflat(g_mean), {"count": 0, "m": z, "v": z}, 1e-3)
        p2, _ = onet.adam_update(P, unflat(g_union), {"count": 0, "m": z, "v": z}, 1e-3)
        assert (flat(p1) - flat(p2)).abs().max().item() <= 1e-9
        # every rank ends with identical parameters
        pv = flat(p1)
        pmax = pv.clone()
        dist.all_reduce(pmax, op=dist.ReduceOp.MAX)
        assert torch.equal(pv, pmax)

        # ---- metric sums
        s = torch.tensor([rank + 1.0, 2.0 * rank], dtype=torch.float64)
        co.allreduce_sums(s, dist)
        assert s.tolist() == [sum(r + 1.0 for r in range(world)), sum(2.0 * r for r in range(world))]
    finally:
        dist.destroy_process_group()


def test_collectives_world2_gloo():
    mp.spawn(_worker, args=(WORLD, _free_port()), nprocs=WORLD, join=True)


def test_single_rank_is_identity():
    from marlsat.learners import collectives as co

    g = torch.arange(5.0)
    assert co.allreduce_grads(g, None) == 1.0 and torch.equal(g, torch.arange(5.0))
    mean, std = co.global_moments(torch.tensor([10.0, 30.0], dtype=torch.float64), 5, None)
    assert mean == 2.0 and abs(std - (np.sqrt(6.0 - 4.0) + 1e-8)) < 1e-15
