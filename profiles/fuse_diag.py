import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "marl-sat_amd"), os.path.join(R, "tests")]
import numpy as np, torch
from test_gnn_gpu import _setup, CASES
from oracle import net as onet
from marlsat.learners.gnn import GNNActorCritic
for case in CASES:
    for fuse in (True, False):
        GNNActorCritic.fuse_phi = fuse
        V, C, vpa, H, L, S, mode = case
        net, b, P, batch, av, am, A, M = _setup(V, C, vpa, H, L, S, mode)
        logits, value, state = net.forward(b, save=True)
        rl = onet.actor_logits(P, L, batch["svf"], batch["x"], batch["cf"], batch["A_pos"], batch["A_neg"], av, am, mode).detach().numpy()
        rv = onet.critic(P, L, batch["svf"], batch["x"], batch["cf"], batch["A_pos"], batch["A_neg"]).detach().numpy()
        lg = logits.cpu().numpy().astype(np.float64); fin = np.isfinite(rl)
        el = np.abs(lg[fin] - rl[fin]); ev = np.abs(value.cpu().numpy() - rv)
        print(case, fuse, "logit maxerr %.3g max|ref| %.3g maxrel %.3g | value maxerr %.3g max|ref| %.3g" % (
            el.max(), np.abs(rl[fin]).max(), (el / np.abs(rl[fin])).max(), ev.max(), np.abs(rv).max()))
