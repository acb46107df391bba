"""Probe (not collected): two fresh learners with the same seeds, one after the other in one process:
rollout buffers, advantages and the first minibatch gradient must be bitwise equal.
usage: probe_flow_determinism.py [workload] [envs] [T]"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from marlsat import SATEnv  # noqa: E402
from marlsat.learners.gnn import GNNActorCritic  # noqa: E402
from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner, ent_coef_at  # noqa: E402
from marlsat.random import PRNGKey  # noqa: E402
from marlsat.utils.generate_cnf_dataset import generate_problem_pool  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "uf200-860"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
T = int(sys.argv[3]) if len(sys.argv) > 3 else 1
V, C, vpa, _, sid = bench.WORKLOADS[wl]
torch.cuda.set_device(0)


def run():
    cfg = dict(NUM_ENVS=B, NUM_STEPS=T, UPDATE_EPOCHS=1, MINIBATCH_SIZE=B * T // 4, NUM_UPDATES=1000,
               LEARNING_RATE=3e-4, ANNEAL_LR=True, LR_START_FACTOR=1.0, LR_END_FLOOR=1e-5, GAMMA=0.99, GAE_LAMBDA=0.95,
               CLIP_EPS=0.2, ENT_COEF=0.01, VF_COEF=0.5, VF_CLIP=0.2, GNN_HIDDEN_DIM=128,
               GNN_NUM_MESSAGE_PASSING_STEPS=16, action_mode=0, MICROBATCH_BYTES=100e9)
    env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa)
    pool = env.make_pool(generate_problem_pool(V, C, 1024, size_id=sid))
    net = GNNActorCritic(128, 16, env.num_agents, env.max_vars_per_agent, 0, V, device=env.device, seed=0)
    lr = MAPPOLearner(cfg, env, net, pool)
    rs = lr.init_runner_state(PRNGKey(77))
    out = {}
    for t in range(2):
        rs = lr.rollout(rs)
        out.update({f"c{t}_{k}": v.clone() for k, v in lr.tr.items()})
        lr.compute_advantages(rs)
        out[f"c{t}_adv"] = lr.adv.clone()
        perm = lr.permutation(torch.Generator().manual_seed(5))
        sums = torch.zeros(3, dtype=torch.float64, device="cuda")
        lr.minibatch_grad(perm[:lr.MB], ent_coef_at(0, cfg), sums, lr.MB)
        out[f"c{t}_grads"] = net.grads.clone()
        net.adam_step(3e-4)
    torch.cuda.synchronize()
    return out


a = run()
b = run()
for k in a:
    x, y = a[k], b[k]
    same = torch.equal(x, y) if x.is_floating_point() is False else bool(((x == y) | (x.isnan() & y.isnan())).all())
    if not same:
        n = int((x != y).sum())
        print("DIFF", k, "elements", n, "of", x.numel(), flush=True)
print("compared", len(a), "buffers", flush=True)
