"""Probe (not collected): which launch makes dF row 2H + 1 (the clause cell's n- count row) differ between
repetitions under GPU contention.  Wraps the backward's C-ABI calls to snapshot that row after each one."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlsat import SATEnv, _lib  # noqa: E402
from marlsat.learners import gnn as G  # noqa: E402
from marlsat.learners.graphs import DeviceTemplates, assemble, build_templates  # noqa: E402
from marlsat.utils.generate_cnf_dataset import generate_problem_pool  # noqa: E402

sync = os.environ.get("PROBE_SYNC", "1") == "1"
V, C, vpa, S = 200, 860, 8, 64
torch.cuda.set_device(0)
pool = generate_problem_pool(V, C, 64, size_id=3)
env = SATEnv(V, C, max_steps=16, vars_per_agent=vpa)
dpool = env.make_pool(pool)
net = G.GNNActorCritic(128, 16, env.num_agents, env.max_vars_per_agent, 0, V, device="cuda", seed=0)
tpl = DeviceTemplates(build_templates(pool, V, env.num_agents), env.num_agents, "cuda")
rng = np.random.default_rng(0)
inst = torch.from_numpy(rng.integers(0, 64, S).astype(np.int32)).cuda()
x = torch.from_numpy(rng.integers(0, 2, (S, V)).astype(np.uint8)).cuda()
snaps = []
names = ["msat_gru_ln_bwd_g4fe", "msat_gemm_h2_dual", "msat_gemm_wgrad_h2_dual", "msat_clause_gather2",
         "msat_var_gather2", "msat_gemm_f64acc", "msat_colsum", "msat_gemm_wgrad", "msat_gemm_wgrad_rot"]
orig = {n: getattr(_lib.lib, n) for n in names}


def wrap(n):
    f = orig[n]

    def w(*a):
        rc = f(*a)
        if sync:
            torch.cuda.synchronize()
        snaps.append((n, net._gF[257].clone() if net._gF is not None else None))
        return rc
    return w


g = torch.Generator(device="cuda").manual_seed(1)
ref = None
for r in range(8):
    b = assemble(tpl, dpool.packed, dpool.static_var_features(), inst, x)
    logits, value, state = net.forward(b, save=True)
    if r == 0:
        wl = torch.randn(logits.shape, device="cuda", generator=g)
        wl = torch.where(torch.isfinite(logits), wl, torch.zeros_like(wl)).contiguous()
        wv = torch.randn(value.shape, device="cuda", generator=g).contiguous()
    net.grads.zero_()
    snaps = []
    for n in names:
        setattr(G.L_, n, wrap(n))
    net.backward(b, state, wl, wv)
    for n in names:
        setattr(G.L_, n, orig[n])
    torch.cuda.synchronize()
    cur = [(n, s.cpu() if s is not None else None) for n, s in snaps]
    if ref is None:
        ref = cur
        print("calls", len(cur), flush=True)
        continue
    # compare from the first GRU backward on (the encoder backward zeroes dF before it; earlier snapshots hold the
    # previous repetition's final dF)
    i0 = next(i for i, (n, _) in enumerate(ref) if n == "msat_gru_ln_bwd_g4fe")
    first = next(((i, n) for i, ((n, s), (_, t)) in enumerate(zip(cur, ref))
                  if i >= i0 and s is not None and not torch.equal(s, t)), None)
    if first:
        i, n = first
        d = (cur[i][1] != ref[i][1]).nonzero().flatten()
        print(f"rep {r}: row 257 first differs after call {i} ({n}, previous {cur[i - 1][0] if i else None}); "
              f"columns {d.tolist()[:40]}", flush=True)
    else:
        print(f"rep {r}: identical", flush=True)
