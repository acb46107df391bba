"""Probe (test infrastructure, not collected by pytest): error of the device GNN forward /
backward against the float64 oracle at the reference depth (H=128, L=16), next to the error
of the same oracle evaluated in float32 on the CPU (the reference's own arithmetic class).

    python tests/probe_parity_depth.py > gpurun_out/parity_depth.txt
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-sat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import net as onet  # noqa: E402
from tests.test_gnn_gpu import _setup  # noqa: E402


def stats(dev, ref):
    dev = np.asarray(dev, np.float64)
    ref = np.asarray(ref, np.float64)
    fin = np.isfinite(ref)
    d, r = dev[fin], ref[fin]
    err = np.abs(d - r)
    rel = err / np.maximum(np.abs(r), 1e-30)
    return dict(max_rel=float(rel.max()), norm=float(err.max() / max(np.abs(r).max(), 1e-30)),
                n_fail_1e5=int((err > 1e-5 * np.abs(r)).sum()), n=int(r.size),
                p99_rel=float(np.quantile(rel, 0.99)), min_abs_ref=float(np.abs(r).min()))


def run(case, paths, own_init=False):
    V, C, vpa, H, L, S, mode = case
    from marlsat.learners.gnn import GNNActorCritic
    net, b, P, batch, av, am, A, M = _setup(V, C, vpa, H, L, S, mode)
    if own_init:  # the learner's own parameter init (params.init_flat) instead of the oracle's
        fresh = GNNActorCritic(H, L, A, M, mode, V, device="cuda", seed=4)
        net.params.copy_(fresh.params)
        P = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in net.to_flax().items()}
    args = (batch["svf"], batch["x"], batch["cf"], batch["A_pos"], batch["A_neg"])
    ref_l = onet.actor_logits(P, L, *args, av, am, mode)
    ref_v = onet.critic(P, L, *args)
    P32 = {k: v.detach().float() for k, v in P.items()}
    a32 = tuple(a.float() for a in args)
    with torch.no_grad():
        l32 = onet.actor_logits(P32, L, *a32, av, am, mode)
        v32 = onet.critic(P32, L, *a32)
    print(f"case {case} own_init={own_init}")
    print("  cpu-fp32 oracle  logits", stats(l32.numpy(), ref_l.detach().numpy()))
    print("  cpu-fp32 oracle  value ", stats(v32.numpy(), ref_v.detach().numpy()))
    g = torch.Generator().manual_seed(3)
    wl = torch.randn(ref_l.shape, generator=g, dtype=torch.float64)
    wl = torch.where(torch.isfinite(ref_l), wl, torch.zeros_like(wl))
    wv = torch.randn(ref_v.shape, generator=g, dtype=torch.float64)
    obj = (torch.where(torch.isfinite(ref_l), ref_l, torch.zeros_like(ref_l)) * wl).sum() + (ref_v * wv).sum()
    obj.backward()
    for name, (fuse, x3, x3r) in paths.items():
        GNNActorCritic.fuse_phi, GNNActorCritic.use_x3, GNNActorCritic.use_gru_x3 = fuse, x3, x3
        GNNActorCritic.use_gru_x3r = x3r
        logits, value, state = net.forward(b, save=True)
        print(f"  device[{name}] logits", stats(logits.cpu().numpy(), ref_l.detach().numpy()))
        print(f"  device[{name}] value ", stats(value.cpu().numpy(), ref_v.detach().numpy()))
        net.grads.zero_()
        net.backward(b, state, wl.float().cuda().contiguous(), wv.float().cuda().contiguous())
        got = net.to_flax(grads=True)
        worst = []
        for k, p in P.items():
            ref = p.grad.numpy() if p.grad is not None else np.zeros(p.shape)
            s = stats(got[k], ref)
            worst.append((s["norm"], k, s["p99_rel"]))
        worst.sort(reverse=True)
        print(f"  device[{name}] grads worst norm-err", [(f"{a:.2e}", k, f"p99rel {c:.2e}") for a, k, c in worst[:4]])
        sys.stdout.flush()


if __name__ == "__main__":
    torch.cuda.set_device(0)
    if len(sys.argv) > 1 and sys.argv[1] == "paths":
        paths = {"default": (True, True, True), "fused-fp32": (True, False, False),
                 "ref-order-x3": (False, True, True), "fp32-ref-order": (False, False, False)}
        for own in (True, False):
            run((50, 218, 10, 128, 16, 8, 0), paths, own_init=own)
        sys.exit(0)
    paths = {"default": (True, True, True), "fp32-ref-order": (False, False, False)}
    for case in [(20, 91, 10, 128, 2, 3, 0), (50, 218, 10, 128, 16, 4, 0), (100, 430, 10, 128, 16, 2, 0),
                 (16, 60, 4, 128, 16, 3, 1)]:
        run(case, paths)
