"""Probe (test infrastructure, not collected): per-message-step error of the device encoder's
states against the float64 oracle on critic-only (full) graphs, per kernel path, next to the
float32 CPU oracle (reference order).  python tests/probe_fold_error.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-sat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import net as onet  # noqa: E402
from oracle.sat_env import OracleSATEnv  # noqa: E402


def oracle_states(P, L, svf, x, cf, Ap, An):
    out = []
    for l in range(1, L + 1):
        out.append(onet.encoder(P, l, svf, x, cf, Ap, An))
    return out


def main():
    from marlsat import SATEnv
    from marlsat.learners.gnn import GNNActorCritic
    from marlsat.learners.graphs import DeviceTemplates, assemble, build_templates
    from marlsat.utils.generate_cnf_dataset import generate_problem_pool

    torch.cuda.set_device(0)
    V, C, vpa, H, L, S = 50, 218, 10, 128, 16, 8
    pool = generate_problem_pool(V, C, 4, size_id=7)
    env = SATEnv(V, C, 10, vars_per_agent=vpa)
    A, M = env.num_agents, env.max_vars_per_agent
    dpool = env.make_pool(pool)
    net = GNNActorCritic(H, L, A, M, 0, V, device="cuda", seed=4)
    tpl = DeviceTemplates(build_templates(pool, V, A), A, "cuda")
    rng = np.random.default_rng(0)
    inst = rng.integers(0, 4, S).astype(np.int32)
    x = rng.integers(0, 2, (S, V)).astype(np.uint8)
    b = assemble(tpl, dpool.packed, dpool.static_var_features(), torch.from_numpy(inst).cuda(),
                 torch.from_numpy(x).cuda(), critic_only=True)
    assert b.Nv == S * V and b.Nc == S * C
    ora = OracleSATEnv(V, C, 10, vars_per_agent=vpa)
    _, ost = ora.reset(pool[inst], x.astype(np.int32))
    Ap, An = onet.dense_graph(pool[inst], V)
    args = (torch.from_numpy(ora.static_var_features(pool[inst])).double(), torch.from_numpy(x).double(),
            torch.from_numpy(ora.clause_features(ost)).double(), Ap, An)
    tree = net.to_flax()
    P64 = {k: torch.tensor(v, dtype=torch.float64) for k, v in tree.items()}
    P32 = {k: torch.tensor(v, dtype=torch.float32) for k, v in tree.items()}
    with torch.no_grad():
        ref = oracle_states(P64, L, *args)
        r32 = oracle_states(P32, L, *(a.float() for a in args))
    steps = [1, 2, 4, 8, 16]
    err = lambda a, r: float((a.double() - r).abs().max())
    print("cpu fp32 ref-order", [(l, "%.2e" % err(r32[l - 1][0], ref[l - 1][0]), "%.2e" % err(r32[l - 1][2], ref[l - 1][2]))
                                 for l in steps])
    for name, (fuse, x3, x3r) in {"x3r(default)": (True, True, True), "x3": (True, True, False),
                                  "fused-fp32": (True, False, False), "ref-order": (False, False, False)}.items():
        GNNActorCritic.fuse_phi, GNNActorCritic.use_x3, GNNActorCritic.use_gru_x3 = fuse, x3, x3
        GNNActorCritic.use_gru_x3r = x3r
        with torch.no_grad():
            _, _, state = net.forward(b, actor=False, save=True)
        Hp, Hn, Hc, tape, _ = state
        got = [(t.Hp, t.Hn, t.Hc) for t in tape[1:]] + [(Hp, Hn, Hc)]
        row = []
        for l in steps:
            gp = got[l - 1][0].cpu().reshape(S, V, H)
            gc = got[l - 1][2].cpu().reshape(S, C, H)
            row.append((l, "%.2e" % err(gp, ref[l - 1][0]), "%.2e" % err(gc, ref[l - 1][2])))
        print(f"device {name:14s}", row)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
