"""Probe (not collected): run-to-run determinism of the device network.  The same graph batch (uf200 or
uf100 samples, H = 128, L = 16) through forward + backward REPS times in one process; every output and
every gradient tensor must be bitwise equal across repetitions.  Prints the first differing tensor and
how many elements differ.  usage: probe_determinism.py [V] [S] [reps] [precision]"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlsat import SATEnv  # noqa: E402
from marlsat.learners import params as Pm  # noqa: E402
from marlsat.learners.gnn import GNNActorCritic  # noqa: E402
from marlsat.learners.graphs import DeviceTemplates, assemble, build_templates  # noqa: E402
from marlsat.utils.generate_cnf_dataset import generate_problem_pool  # noqa: E402

V = int(sys.argv[1]) if len(sys.argv) > 1 else 200
S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
sizes = {50: (218, 10), 100: (430, 10), 200: (860, 8)}
C, vpa = sizes[V]
torch.cuda.set_device(0)
pool = generate_problem_pool(V, C, 64, size_id=3)
env = SATEnv(V, C, max_steps=16, vars_per_agent=vpa)
A, M = env.num_agents, env.max_vars_per_agent
dpool = env.make_pool(pool)
net = GNNActorCritic(128, 16, A, M, 0, V, device="cuda", seed=0)
tpl = DeviceTemplates(build_templates(pool, V, A), A, "cuda")
rng = np.random.default_rng(0)
inst = torch.from_numpy(rng.integers(0, 64, S).astype(np.int32)).cuda()
x = torch.from_numpy(rng.integers(0, 2, (S, V)).astype(np.uint8)).cuda()
g = torch.Generator(device="cuda").manual_seed(1)
ref = None
for r in range(reps):
    b = assemble(tpl, dpool.packed, dpool.static_var_features(), inst, x)
    logits, value, state = net.forward(b, save=True)
    if r == 0:
        wl = torch.randn(logits.shape, device="cuda", generator=g)
        wl = torch.where(torch.isfinite(logits), wl, torch.zeros_like(wl)).contiguous()
        wv = torch.randn(value.shape, device="cuda", generator=g).contiguous()
    net.grads.zero_()
    net.backward(b, state, wl, wv)
    torch.cuda.synchronize()
    out = {"logits": logits.clone(), "value": value.clone(), "grads": net.grads.clone(), "cdeg": b.cdeg.clone(),
           "vfeat": b.vfeat.clone(), "slots": b.slots.clone().float(), "gF": net._gF.clone()}
    fin = {k: bool(torch.isfinite(torch.where(torch.isinf(v) & (k == "logits"), torch.zeros_like(v), v)).all())
           for k, v in out.items()}
    if ref is None:
        ref = out
        print("rep 0 finite", fin, "rows", b.Nv, b.Nc, flush=True)
        continue
    diffs = {k: int((~((out[k] == ref[k]) | (torch.isnan(out[k]) & torch.isnan(ref[k])))).sum()) for k in out}
    line = f"rep {r}: differing elements {diffs}; finite {fin}"
    if diffs["gF"]:
        line += " gF rows " + str((out["gF"] != ref["gF"]).any(1).nonzero().flatten()[:12].tolist())
    if diffs["grads"]:
        d = (out["grads"] != ref["grads"]).float().cpu().numpy()
        tree = Pm.to_flax(d, net.H, net.L, net.A, net.M, net.mode, net.E)
        line += " tensors " + str([k for k, v in tree.items() if v.any()][:8])
    print(line, flush=True)
