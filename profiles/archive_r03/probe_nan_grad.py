"""Probe (not collected): the first PPO minibatch of the bench's uf200 flow on rank 1's shard (seed offset 1),
world 1 -- which parameter gradients come out non-finite, under the precision path MARLSAT_PRECISION selects.
With PROBE_CALLS=1 the backward's C-ABI calls are wrapped and the first call after which net.grads holds a
non-finite value is reported."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlsat import SATEnv, _lib  # noqa: E402
from marlsat.learners import gnn as G  # noqa: E402
from marlsat.learners import params as Pm  # noqa: E402
from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner  # noqa: E402
from marlsat.random import PRNGKey  # noqa: E402
from marlsat.utils.generate_cnf_dataset import generate_problem_pool  # noqa: E402

so = int(os.environ.get("PROBE_SEED_OFFSET", "1"))
V, C, vpa, B = 200, 860, 8, 4096
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
cfg = dict(NUM_ENVS=B, NUM_STEPS=1, UPDATE_EPOCHS=1, MINIBATCH_SIZE=B // 4, NUM_UPDATES=1000, LEARNING_RATE=3e-4,
           ANNEAL_LR=True, LR_START_FACTOR=1.0, LR_END_FLOOR=1e-5, GAMMA=0.99, GAE_LAMBDA=0.95, CLIP_EPS=0.2,
           ENT_COEF=0.01, VF_COEF=0.5, VF_CLIP=0.2, GNN_HIDDEN_DIM=128, GNN_NUM_MESSAGE_PASSING_STEPS=16,
           action_mode=0, MICROBATCH_BYTES=100e9)
env = SATEnv(V, C, max_steps=512, vars_per_agent=vpa, device=dev)
npool = generate_problem_pool(V, C, 1024, size_id=3)
pool = env.make_pool(npool)
net = G.GNNActorCritic(128, 16, env.num_agents, env.max_vars_per_agent, 0, V, device=dev, seed=0)
learner = MAPPOLearner(cfg, env, net, pool, dist=None)
rs = learner.init_runner_state(PRNGKey(77 + so))
gen = torch.Generator().manual_seed(99 + so)
rs = learner.rollout(rs)
learner.compute_advantages(rs)
perm = learner.permutation(gen)
idx = perm[:learner.MB]
fin = lambda t: bool(torch.isfinite(t).all())

calls = []
if os.environ.get("PROBE_CALLS") == "1":
    names = [n for n in dir(G.L_) if n.startswith("msat_")]
    orig = {n: getattr(G.L_, n) for n in names}

    def wrap(n):
        f = orig[n]

        def w(*a):
            rc = f(*a)
            torch.cuda.synchronize()
            calls.append((n, fin(net.grads), [x for x in a if isinstance(x, int) and abs(x) < 1 << 24][:8]))
            return rc
        return w
    for n in names:
        setattr(G.L_, n, wrap(n))

sums = torch.zeros(3, dtype=torch.float64, device=dev)
learner.minibatch_grad(idx, 0.01, sums, idx.numel())
torch.cuda.synchronize()
print("precision", G.PRECISION, "sums", sums.tolist(), "grads finite", fin(net.grads), flush=True)
g = Pm.to_flax(net.grads.cpu().numpy(), net.H, net.L, net.A, net.M, net.mode, net.E)
for name, t in g.items():
    bad = ~np.isfinite(t)
    if bad.any():
        print(f"  {name} {t.shape}: {int(bad.sum())} non-finite, finite max |g| {np.abs(t[~bad]).max() if (~bad).any() else 0:.3e}")
if calls:
    first = next((i for i, c in enumerate(calls) if not c[1]), None)
    print("calls", len(calls), "first non-finite after", first)
    if first is not None:
        for c in calls[max(0, first - 6):first + 2]:
            print("   ", c)


if os.environ.get("PROBE_BISECT") == "1":
    # smallest offending sample: halve the row set while a half still gives a non-finite gradient
    rows = idx.clone()
    while rows.numel() > 1:
        h = rows.numel() // 2
        for part in (rows[:h], rows[h:]):
            learner.micro = part.numel()
            learner.minibatch_grad(part, 0.01, torch.zeros(3, dtype=torch.float64, device=dev), part.numel())
            if not fin(net.grads):
                rows = part
                break
        else:
            print("both halves finite at", rows.numel(), "rows", flush=True)
            break
    print("offending rows", rows.tolist(), flush=True)
    r = int(rows[0])
    inst = learner.tr["pidx"].reshape(-1)[r].item()
    xs = learner.tr["x"].reshape(-1, V)[r].cpu().numpy().astype(np.uint8)
    print("instance", inst, "x ones", int(xs.sum()), flush=True)
    from oracle import net as onet
    from oracle.sat_env import OracleSATEnv
    ora = OracleSATEnv(V, C, 512, vars_per_agent=vpa)
    _, ost = ora.reset(npool[[inst]], xs[None].astype(np.int32))
    Ap, An = onet.dense_graph(npool[[inst]], V)
    args = (torch.from_numpy(ora.static_var_features(npool[[inst]])).double(), torch.from_numpy(xs[None]).double(),
            torch.from_numpy(ora.clause_features(ost)).double(), Ap, An)
    P = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in net.to_flax().items()}
    av = torch.from_numpy(ora.agent_vars.astype(np.int64))
    am = torch.from_numpy(ora.action_mask)
    lnv = []
    ln0 = onet._ln

    def ln(P_, k, x, eps=1e-6):
        m = x.mean(-1, keepdim=True)
        v = torch.clamp((x * x).mean(-1, keepdim=True) - m * m, min=0.0)
        lnv.append((k, float(v.min()), int((v < 1e-4).sum())))
        return ln0(P_, k, x, eps)
    onet._ln = ln
    ref_l = onet.actor_logits(P, 16, *args, av, am, 0)
    ref_v = onet.critic(P, 16, *args)
    onet._ln = ln0
    worst = sorted(lnv, key=lambda t: t[1])[:8]
    print("oracle LN calls", len(lnv), "smallest row variances (layer, var, rows<1e-4):", worst, flush=True)
    g2 = torch.Generator().manual_seed(5)
    wl = torch.randn(ref_l.shape, generator=g2, dtype=torch.float64)
    wl = torch.where(torch.isfinite(ref_l), wl, torch.zeros_like(wl))
    wv = torch.randn(ref_v.shape, generator=g2, dtype=torch.float64)
    obj = (torch.where(torch.isfinite(ref_l), ref_l, torch.zeros_like(ref_l)) * wl).sum() + (ref_v * wv).sum()
    obj.backward()
    mx = {k: float(p.grad.abs().max()) for k, p in P.items() if p.grad is not None}
    top = sorted(mx.items(), key=lambda t: -t[1])[:6]
    print("oracle fp64 grad max |g| (top):", top, flush=True)
