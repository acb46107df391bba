"""Worker of tests/test_dist_learner_gpu.py::test_two_rank_train_cycles_keep_replicas_identical (not collected).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tests/dist_replica_worker.py OUTDIR H [workload envs T L micro_gb cycles]

Each rank runs the bench's path -- its own env shard and rollout RNG, two full train cycles
(MAPPOLearner.train_cycle: rollout, GAE with global moments, PPO minibatches with the gradient
all-reduce before every Adam step) -- at GNN width H (128 takes the fp16x2 / bf16x3 kernels, 64 the
fp32 ones) and records, per Adam step, the parameters it started from and the all-reduced gradient.
Replicas must stay bitwise identical (learner:647-650 is one optimizer on one parameter set).
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for p in (ROOT, os.path.join(ROOT, "marl-sat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def _debug_hooks(learner, rank):
    import marlsat.learners.mappo_gnn_sat_learner as ML

    say = lambda *a: print(f"[rank{rank}]", *a, file=sys.stderr, flush=True)
    fin = lambda t: bool(torch.isfinite(t.float()).all())
    gm = ML.global_moments

    def moments(sums, n, d):
        m = gm(sums, n, d)
        say("moments local", sums.tolist(), "n", n, "-> mean/std", m)
        return m
    ML.global_moments = moments
    ro, mg = learner.rollout, learner.minibatch_grad

    def rollout(rs):
        rs = ro(rs)
        say("rollout finite", {k: fin(v) for k, v in learner.tr.items() if v.is_floating_point()})
        return rs

    def minibatch_grad(idx, ent, sums, mb):
        mg(idx, ent, sums, mb)
        g = learner.net.grads
        say("local grad finite", fin(g), "adv finite", fin(learner.adv), "sums", sums.tolist(),
            "nonfinite", int((~torch.isfinite(g)).sum()))
    learner.rollout, learner.minibatch_grad = rollout, minibatch_grad


def main():
    import torch.distributed as dist

    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner
    from marlsat.random import PRNGKey
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    out, H = sys.argv[1], int(sys.argv[2])
    os.makedirs(out, exist_ok=True)
    rank = int(os.environ["RANK"])
    dist.init_process_group(os.environ.get("MARLSAT_DIST_BACKEND", "gloo"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sizes = {"uf50-218": (50, 218, 10), "uf100-430": (100, 430, 10), "uf200-860": (200, 860, 8)}
    wl = sys.argv[3] if len(sys.argv) > 3 else "uf50-218"
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    T = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    L = int(sys.argv[6]) if len(sys.argv) > 6 else 2
    micro_gb = float(sys.argv[7]) if len(sys.argv) > 7 else 240.0
    cycles = int(sys.argv[8]) if len(sys.argv) > 8 else 2
    V, C, vpa = sizes[wl]
    cfg = dict(NUM_ENVS=B, NUM_STEPS=T, UPDATE_EPOCHS=2, MINIBATCH_SIZE=B * T // 4, NUM_UPDATES=10, LEARNING_RATE=3e-4,
               ANNEAL_LR=True, LR_START_FACTOR=1.0, LR_END_FLOOR=1e-5, GAMMA=0.99, GAE_LAMBDA=0.95, CLIP_EPS=0.2,
               ENT_COEF=0.01, VF_COEF=0.5, VF_CLIP=0.2, GNN_HIDDEN_DIM=H, GNN_NUM_MESSAGE_PASSING_STEPS=L,
               action_mode=0, MICROBATCH_BYTES=micro_gb * 1e9)
    if os.environ.get("REPLICA_BENCH_ENV") == "1":  # bench.py's env and pool: 512-step episodes, 1024 instances
        size_id = {"uf50-218": 1, "uf100-430": 2, "uf200-860": 3}[wl]
        env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa, device=dev)
        pool = env.make_pool(generate_problem_pool(V, C, 1024, size_id=size_id, skip_isolated=True))
    else:
        env = SATEnv(V, C, max_steps=16, vars_per_agent=vpa, device=dev)
        pool = env.make_pool(generate_problem_pool(V, C, 32, size_id=1))
    net = GNNActorCritic(H, L, env.num_agents, env.max_vars_per_agent, 0, V, device=dev, seed=0)
    learner = MAPPOLearner(cfg, env, net, pool, dist=dist)
    if os.environ.get("REPLICA_DEBUG") == "1":  # per-step finiteness report (stderr)
        _debug_hooks(learner, rank)
    so = rank + int(os.environ.get("REPLICA_SEED_OFFSET", "0"))  # run rank k's shard alone: offset k at world 1
    rs = learner.init_runner_state(PRNGKey(77 + so))
    gen = torch.Generator().manual_seed(99 + so)
    p0 = net.params.clone()
    learner.trace = []
    if os.environ.get("REPLICA_BENCH_FLOW") == "1":  # bench.py's mappo_bench: 1-epoch warm-up, 4-epoch cycle, ktimer
        learner.cfg["UPDATE_EPOCHS"] = 1
        rs, _ = learner.train_cycle(rs, 0, gen)
        learner.cfg["UPDATE_EPOCHS"] = 4
        GNNActorCritic.ktimer = {} if os.environ.get("REPLICA_KTIMER", "1") == "1" else None
        rs, _ = learner.train_cycle(rs, 1, gen)
        GNNActorCritic.ktimer = None
    else:
        for u in range(cycles):
            rs, _ = learner.train_cycle(rs, u, gen)
    torch.cuda.synchronize()
    big = B * T >= 4096
    if big:  # keep checksums only: (fp64 sum, first 8 values) per tensor
        ck = lambda t: torch.cat([t.double().sum().reshape(1), t[:8].double()]).cpu()
        learner.trace = [{"params": ck(r["params"]), "grads": ck(r["grads"])} for r in learner.trace]
    ck64 = lambda t: float(t.double().sum()) if t.is_floating_point() else int(t.long().sum())
    bufs = {k: ck64(v) for k, v in learner.tr.items()}
    bufs["adv"] = ck64(learner.adv)
    torch.save({"init": p0.cpu(), "final": net.params.cpu(), "bufs": bufs,
                "trace": [{"params": r["params"].cpu(), "grads": r["grads"].cpu()} for r in learner.trace]},
               os.path.join(out, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
