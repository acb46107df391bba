"""Attribution of the train-cycle test's device gradient error to kernel families, at FIXED parameters
(verdict r05 item 1).  The switch probe (parity_switch_probe.py) changes a kernel family for the whole cycle, so
step 1 then starts from other parameters and every comparison is a new draw; here every configuration computes
the gradient of the same minibatch from the same parameters (a dump written by tests/test_mappo_gpu.py with
MARLSAT_PARITY_DUMP set), and profiles/parity_orderings.py-style CPU analysis compares each with the oracle.

    python profiles/parity_attrib.py <dump.npz> <step> <out.npz>          (GPU)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-sat_amd"), os.path.join(ROOT, "profiles")):
    sys.path.insert(0, p)

from marlsat import SATEnv, _lib  # noqa: E402
from marlsat.learners import gnn  # noqa: E402
from marlsat.learners.gnn import GNNActorCritic  # noqa: E402
from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner, ent_coef_at  # noqa: E402
from marlsat.utils.generate_cnf_dataset import generate_problem_pool  # noqa: E402
from parity_orderings import cfg_of  # noqa: E402

# label: switches on top of the fp16x2 default (class attributes of GNNActorCritic; "_wgrad" sets the library's
# weight-gradient path)
CASES = {
    "default": {},
    "gru_x3": {"use_gru_h2": False},
    "dgrad_x3": {"use_dgrad_h2": False},
    "wgrad_x3": {"use_wgrad_h2": False, "_wgrad": "bf16x3"},
    "planes0": {"use_planes": False},
    "bf16x3": {"use_gru_h2": False, "use_dgrad_h2": False, "use_wgrad_h2": False, "_wgrad": "bf16x3"},
    "fp32": dict(gnn.path_switches("fp32"), _wgrad="fp32"),
    "fp32_fold": dict(gnn.path_switches("fp32"), fuse_phi=True, _wgrad="fp32"),
}


def main():
    path, s, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    d = np.load(path)
    V, C, vpa, H, L, mode, T, B, MB, E = (int(v) for v in d["shape"])
    cfg = cfg_of(d["shape"])
    pool = generate_problem_pool(V, C, 5, size_id=12, skip_isolated=True)  # the test's pool
    env = SATEnv(V, C, max_steps=2, vars_per_agent=vpa, action_mode=mode)
    A, M = env.num_agents, env.max_vars_per_agent
    net = GNNActorCritic(H, L, A, M, mode, V, device="cuda", seed=4)
    lr = MAPPOLearner(cfg, env, net, env.make_pool(pool))
    tr = lr.tr
    tr["pidx"].copy_(torch.from_numpy(d["pidx"].reshape(T, B).astype(np.int32)))
    tr["x"].copy_(torch.from_numpy(d["x_raw"].reshape(T, B, V).astype(np.uint8)))
    tr["action"].copy_(torch.from_numpy(d["full_action"].reshape(tr["action"].shape).astype(np.int32)))
    tr["log_prob"].copy_(torch.from_numpy(d["full_log_prob"].reshape(tr["log_prob"].shape).astype(np.float32)))
    tr["value"].copy_(torch.from_numpy(d["full_value"].reshape(tr["value"].shape).astype(np.float32)))
    lr.adv.copy_(torch.from_numpy(d["full_gae"].reshape(T, B).astype(np.float32)))
    lr.targets.copy_(torch.from_numpy(d["full_targets"].reshape(T, B).astype(np.float32)))
    idx = torch.from_numpy(d[f"idx_{s}"].astype(np.int32)).cuda()
    params = torch.from_numpy(d[f"params_{s}"]).cuda()
    ent = ent_coef_at(0, cfg)
    res = {}
    want = os.environ.get("ATTRIB_CASES")  # a comma-separated subset of CASES (default: all)
    for label, sw in CASES.items():
        if want and label not in want.split(","):
            continue
        saved = {k: getattr(GNNActorCritic, k) for k in sw if not k.startswith("_")}
        code = int(_lib.lib.msat_get_precision())
        try:
            for k, v in sw.items():
                if not k.startswith("_"):
                    setattr(GNNActorCritic, k, v)
            if "_wgrad" in sw:
                _lib.check(_lib.lib.msat_set_precision(gnn.PRECISION_CODES[sw["_wgrad"]]), "msat_set_precision")
            net.params.copy_(params)
            sums = torch.zeros(3, dtype=torch.float64, device="cuda")
            lr.minibatch_grad(idx, ent, sums, MB)
            torch.cuda.synchronize()
            res[label] = net.grads.cpu().numpy().copy()
            same = np.array_equal(res[label], d[f"grads_{s}"]) if label == "default" else None
            print(f"{label}: grads computed{'' if same is None else f', bitwise equal to the dumped default: {same}'}",
                  flush=True)
        finally:
            for k, v in saved.items():
                setattr(GNNActorCritic, k, v)
            _lib.check(_lib.lib.msat_set_precision(code), "msat_set_precision")
    np.savez(out, **res)


if __name__ == "__main__":
    main()
