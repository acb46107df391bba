"""Probe (not collected): the bench's MAPPO leg at one rank with a per-Adam-step trace; reports the first step
whose gradient or parameters are not finite, and which parameter tensors.  usage:
    python tests/probe_mappo_finite.py [workload] [envs] [T] [micro_gb]"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from marlsat import SATEnv  # noqa: E402
from marlsat.learners import params as Pm  # noqa: E402
from marlsat.learners.gnn import GNNActorCritic  # noqa: E402
from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner  # noqa: E402
from marlsat.random import PRNGKey  # noqa: E402
from marlsat.utils.generate_cnf_dataset import generate_problem_pool  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "uf200-860"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
T = int(sys.argv[3]) if len(sys.argv) > 3 else 1
gb = float(sys.argv[4]) if len(sys.argv) > 4 else 240.0
V, C, vpa, _, sid = bench.WORKLOADS[wl]
torch.cuda.set_device(0)
cfg = dict(NUM_ENVS=B, NUM_STEPS=T, UPDATE_EPOCHS=4, MINIBATCH_SIZE=B * T // 4, NUM_UPDATES=1000, LEARNING_RATE=3e-4,
           ANNEAL_LR=True, LR_START_FACTOR=1.0, LR_END_FLOOR=1e-5, GAMMA=0.99, GAE_LAMBDA=0.95, CLIP_EPS=0.2,
           ENT_COEF=0.01, VF_COEF=0.5, VF_CLIP=0.2, GNN_HIDDEN_DIM=128, GNN_NUM_MESSAGE_PASSING_STEPS=16,
           action_mode=0, MICROBATCH_BYTES=gb * 1e9)
env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa)
pool = env.make_pool(generate_problem_pool(V, C, 1024, size_id=sid))
net = GNNActorCritic(128, 16, env.num_agents, env.max_vars_per_agent, 0, V, device=env.device, seed=0)
learner = MAPPOLearner(cfg, env, net, pool)
rs = learner.init_runner_state(PRNGKey(77))
gen = torch.Generator().manual_seed(99)
print("micro", learner.micro, "init finite", bool(torch.isfinite(net.params).all()), flush=True)
for cyc in range(2):
    learner.trace = []
    rs = learner.rollout(rs)
    lp = learner.tr["log_prob"]
    print(f"cycle {cyc} rollout: log_prob finite {bool(torch.isfinite(lp).all())}, value finite "
          f"{bool(torch.isfinite(learner.tr['value']).all())}", flush=True)
    learner.compute_advantages(rs)
    print(f"  adv finite {bool(torch.isfinite(learner.adv).all())}", flush=True)
    losses, ent = learner.ppo_update(cyc, gen)
    for s, rec in enumerate(learner.trace):
        gfin = torch.isfinite(rec["grads"])
        pfin = torch.isfinite(rec["params"])
        if not (bool(gfin.all()) and bool(pfin.all())):
            tree = Pm.to_flax(gfin.float().cpu().numpy(), net.H, net.L, net.A, net.M, net.mode, net.E)
            bad = [k for k, v in tree.items() if (v < 1).any()]
            print(f"  Adam step {s}: grads finite {bool(gfin.all())} params finite {bool(pfin.all())}; "
                  f"non-finite gradient tensors: {bad[:12]}", flush=True)
            break
    else:
        print(f"  all {len(learner.trace)} Adam steps finite; losses {losses.cpu().tolist()}", flush=True)
    print("  params finite after cycle", bool(torch.isfinite(net.params).all()), flush=True)
