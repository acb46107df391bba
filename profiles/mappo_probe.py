"""MAPPO network throughput probe at BASELINE sizes (diagnostic).

Times, with HIP events, (a) the rollout policy forward (actor + critic, no tape) and
(b) one training micro-batch forward(save) + PPO loss + backward, and reports samples/s,
matmul TFLOP/s (2MNK of every GEMM issued) and the fraction of the fp32 MFMA peak."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import numpy as np
import torch
from marlsat import SATEnv, _lib
from marlsat.learners.gnn import GNNActorCritic
from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner
from marlsat.random import PRNGKey
from marlsat.utils.generate_cnf_dataset import generate_problem_pool

wl = sys.argv[1] if len(sys.argv) > 1 else "uf200"
S_roll = int(sys.argv[2]) if len(sys.argv) > 2 else 256
S_train = int(sys.argv[3]) if len(sys.argv) > 3 else 32
phases = sys.argv[4].split(",") if len(sys.argv) > 4 else ["rollout", "train"]
V, C, vpa, sid = {"uf20": (20, 91, 10, 0), "uf50": (50, 218, 10, 1), "uf100": (100, 430, 10, 2),
                  "uf200": (200, 860, 8, 3)}[wl]
H, L = 128, 16
pool = generate_problem_pool(V, C, 64, size_id=sid)
env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa)
net = GNNActorCritic(H, L, env.num_agents, env.max_vars_per_agent, 0, V, device="cuda")
cfg = dict(NUM_ENVS=S_roll, NUM_STEPS=1, MINIBATCH_SIZE=S_roll, UPDATE_EPOCHS=1, GAMMA=0.99, GAE_LAMBDA=0.95,
           CLIP_EPS=0.1, VF_CLIP=0.5, ENT_COEF=0.01, VF_COEF=0.5, LEARNING_RATE=1e-4)
lr = MAPPOLearner(cfg, env, net, env.make_pool(pool), micro_bytes=1e15)
rs = lr.init_runner_state(PRNGKey(0))
st = rs.env_state

def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        GNNActorCritic.flops = 0
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3)
    return min(ts), GNNActorCritic.flops

res = {"workload": wl, "H": H, "L": L, "A": env.num_agents}
if "rollout" in phases:
  t, fl = timed(lambda: lr.policy(st, PRNGKey(1)))
  res["rollout_forward"] = {"samples": S_roll, "s": t, "samples_per_s": S_roll / t, "tflops": fl / t / 1e12,
                          "frac_fp32_mfma_peak": fl / t / 157.3e12}
# training samples: the rollout states, tiled when S_train exceeds the rollout batch
rep = -(-S_train // st.num_envs)
pidx = st.problem_idx.repeat(rep)[:S_train].contiguous()
x = st.variable_assignments.repeat(rep, 1)[:S_train].contiguous()
def train_step():
    gb = lr._batch(pidx, x)
    logits, value, state = net.forward(gb, save=True)
    dl = torch.randn_like(logits).nan_to_num_(0.0) * 1e-3
    dl = torch.where(torch.isfinite(logits), dl, torch.zeros_like(dl))
    dv = torch.randn_like(value) * 1e-3
    net.backward(gb, state, dl.contiguous(), dv.contiguous())
if "train" in phases:
  t, fl = timed(train_step, reps=2)
  res["train_fwd_bwd"] = {"samples": S_train, "s": t, "samples_per_s": S_train / t, "tflops": fl / t / 1e12,
                        "frac_fp32_mfma_peak": fl / t / 157.3e12, "rows_per_sample": lr.tpl.mean_full_rows}
print(json.dumps(res, indent=1))
