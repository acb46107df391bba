"""Worker of tests/test_dist_learner_gpu.py (not collected by pytest).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tests/dist_learner_worker.py OUTDIR

Every rank builds the same union transition set (T x B_UNION envs, deterministic), keeps its
column shard of B_UNION / world envs, runs the device learner's advantage normalisation and
PPO update with ``dist`` set (learners/collectives.py: global moments, gradient all-reduce per
minibatch) and writes its trace (minibatch rows, parameters before and all-reduced gradient of
every Adam step, final parameters, normalised advantages) to OUTDIR/rank<r>.pt.  World 1 (called
in-process by the test) is the union run.
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for p in (ROOT, os.path.join(ROOT, "marl-sat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

V, C, VPA, H, L = 20, 91, 10, 64, 2
T, B_UNION, N_POOL = 4, 8, 6
CFG = dict(NUM_STEPS=T, NUM_UPDATES=10, UPDATE_EPOCHS=2, LEARNING_RATE=1e-3, GAMMA=0.99, GAE_LAMBDA=0.95,
           CLIP_EPS=0.12, ENT_COEF=0.01, VF_COEF=0.5, VF_CLIP=0.5, ANNEAL_LR=True, LR_START_FACTOR=1.0,
           LR_END_FLOOR=2e-5, action_mode=0)


def union_transitions(A, M):
    rng = np.random.default_rng(2024)
    return {
        "pidx": rng.integers(0, N_POOL, (T, B_UNION)).astype(np.int32),
        "x": rng.integers(0, 2, (T, B_UNION, V)).astype(np.uint8),
        "action": rng.integers(0, M + 1, (T, B_UNION, A)).astype(np.int32),
        "log_prob": rng.normal(-2.3, 0.3, (T, B_UNION, A)).astype(np.float32),
        "value": rng.normal(0.0, 0.5, (T, B_UNION)).astype(np.float32),
        "reward": (rng.random((T, B_UNION)) < 0.2).astype(np.float32),
        "done": (rng.random((T, B_UNION)) < 0.25).astype(np.uint8),
        "last_pidx": rng.integers(0, N_POOL, B_UNION).astype(np.int32),
        "last_x": rng.integers(0, 2, (B_UNION, V)).astype(np.uint8),
    }


def run(rank: int, world: int, dist=None, minibatches_per_rank: int = 2):
    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner, RunnerState
    from marlsat.random import PRNGKey
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    Bl = B_UNION // world
    cfg = dict(CFG, NUM_ENVS=Bl, MINIBATCH_SIZE=T * Bl // minibatches_per_rank)
    pool = generate_problem_pool(V, C, N_POOL, size_id=5)
    env = SATEnv(V, C, max_steps=8, vars_per_agent=VPA, device=dev)
    A, M = env.num_agents, env.max_vars_per_agent
    net = GNNActorCritic(H, L, A, M, 0, V, device=dev, seed=9)
    learner = MAPPOLearner(cfg, env, net, env.make_pool(pool), dist=dist)
    u = union_transitions(A, M)
    cols = slice(rank * Bl, (rank + 1) * Bl)
    for k in ("pidx", "x", "action", "log_prob", "value", "reward", "done"):
        learner.tr[k].copy_(torch.from_numpy(np.ascontiguousarray(u[k][:, cols])).to(dev))
    obs, st = env.reset_from_pool(learner.pool, Bl, problem_idx=u["last_pidx"][cols], assignments=u["last_x"][cols])
    learner.compute_advantages(RunnerState(st, obs, PRNGKey(0)))
    learner.trace = []
    losses, _ = learner.ppo_update(0, torch.Generator().manual_seed(100 + rank))
    torch.cuda.synchronize()
    return {"trace": [{k: (v.cpu() if torch.is_tensor(v) else v) for k, v in r.items()} for r in learner.trace],
            "final": net.params.cpu(), "adv": learner.adv.cpu(), "targets": learner.targets.cpu(),
            "losses": losses.cpu(), "learner": learner}


def main():
    import torch.distributed as dist

    out = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group(os.environ.get("MARLSAT_DIST_BACKEND", "gloo"))
    res = run(rank, world, dist)
    res.pop("learner")
    torch.save(res, os.path.join(out, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
