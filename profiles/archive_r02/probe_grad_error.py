"""Probe (test infrastructure, not collected): per-tensor gradient error / fp32-CPU-oracle error at
L = 16 (uf50 case of tests/test_gnn_gpu.py::test_depth16_matches_oracle) per kernel path and
weight-gradient reduction.  python tests/probe_grad_error.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-sat_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import net as onet  # noqa: E402
from tests.test_gnn_gpu import _fp32_yardstick, _setup  # noqa: E402


def main():
    from marlsat.learners.gnn import GNNActorCritic

    torch.cuda.set_device(0)
    V, C, vpa, H, L, S, mode = 50, 218, 10, 128, 16, 4, 0
    net, b, P, batch, av, am, A, M = _setup(V, C, vpa, H, L, S, mode, seed=11)
    args = (batch["svf"], batch["x"], batch["cf"], batch["A_pos"], batch["A_neg"])
    ref_l = onet.actor_logits(P, L, *args, av, am, mode)
    ref_v = onet.critic(P, L, *args)
    g = torch.Generator().manual_seed(5)
    wl = torch.randn(ref_l.shape, generator=g, dtype=torch.float64)
    wl = torch.where(torch.isfinite(ref_l), wl, torch.zeros_like(wl))
    wv = torch.randn(ref_v.shape, generator=g, dtype=torch.float64)
    ((torch.where(torch.isfinite(ref_l), ref_l, torch.zeros_like(ref_l)) * wl).sum() + (ref_v * wv).sum()).backward()
    _, _, y_g = _fp32_yardstick(P, L, args, av, am, mode, wl, wv)
    prev = None
    for name, (fuse, x3, x3r, skinny) in {"default-fold32": (True, True, True, "1"),
                                          "f64-fwd-only": (True, True, True, "1"), "f64-bwd-only": (True, True, True, "1"),
                                          "default": (True, True, True, "1"), "default-again": (True, True, True, "1"),
                                          "x3-not-r": (True, True, False, "1"),
                                          "fused-fp32-gemm-x3-gru": (True, False, True, "1"),
                                          "fused-fp32": (True, False, False, "1"),
                                          "ref-order": (False, False, False, "1")}.items():
        os.environ["MARLSAT_WGRAD_SKINNY"] = skinny
        GNNActorCritic.fuse_phi, GNNActorCritic.use_x3, GNNActorCritic.use_gru_x3 = fuse, x3, x3
        GNNActorCritic.use_gru_x3r = x3r
        os.environ["MARLSAT_FOLD_F64"] = {"default-fold32": "0", "f64-fwd-only": "bwd", "f64-bwd-only": "fwd"}.get(name, "1")
        if name == "fused-fp32-gemm-x3-gru":
            GNNActorCritic.use_x3, GNNActorCritic.use_gru_x3 = False, True
        logits, value, state = net.forward(b, save=True)
        rl = ref_l.detach().numpy()
        fin = np.isfinite(rl)
        print(name, "logits norm err %.2e" % (np.abs(logits.cpu().numpy()[fin] - rl[fin]).max() / np.abs(rl[fin]).max()))
        net.grads.zero_()
        net.backward(b, state, wl.float().cuda().contiguous(), wv.float().cuda().contiguous())
        got = net.to_flax(grads=True)
        if prev is not None and name == "default-again":
            print("default run-to-run identical:", all(np.array_equal(prev[k], got[k]) for k in got))
        prev = got
        rows = []
        for k, p in P.items():
            ref = p.grad.numpy() if p.grad is not None else np.zeros(p.shape)
            e32 = np.abs(y_g[k] - ref).max()
            rows.append((float(np.abs(got[k] - ref).max() / max(e32, 1e-300)), k,
                         float(np.abs(ref).max()), float(e32)))
        rows.sort(reverse=True)
        print(name, [(f"{r:.2f}", k, f"max|g| {m:.1e} e32 {e:.1e}") for r, k, m, e in rows[:6]])
        sys.stdout.flush()


if __name__ == "__main__":
    main()
